"""CPU oracle — test infrastructure only (see dsp_oracle.py header)."""
