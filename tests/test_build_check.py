"""Build check of the shipped libmsdsp.so (CPU only: reads the gfx950 code objects, runs nothing).

Round 5's one GPU fault was a build whose live Welch kernel called an out-of-line
numpy pairwise sum with a generic pointer to LDS.  With `#pragma unroll 2` on the leaf loop the
compiler displaced the loop pointer to `base - 64` and folded +128 .. +240 into the flat loads'
offsets; a flat instruction picks LDS / scratch / global from the address register alone, so for the
wave whose segment sat at LDS offset 0 the load left the LDS aperture
(HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION).  The shipped code keeps that pattern out structurally:

* no function of the library holds a flat memory instruction (LDS data is read with ds_*, global data
  with global_*; out-of-line code takes global pointers typed as such, np_reduce.h);
* only the listed kernels call out-of-line functions;
* the hot kernels use no scratch, and no kernel uses a dynamic stack.
"""
import os
import shutil

import pytest

from conftest import ROOT
from tools import kernel_resources as kr

SO = os.path.join(ROOT, "meteor-scatter_amd", "meteorgpu", "libmsdsp.so")

pytestmark = pytest.mark.skipif(not (os.path.exists(SO) and shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump")),
                                reason="libmsdsp.so or the ROCm LLVM tools are missing")

# kernels allowed to call out-of-line device functions (each callee is held to zero flat instructions
# below): the live scan's two event handlers (one call per meteor)
CALLERS = ("live_seg_scan_kernel", "live_seg_emit_kernel")

# the hot kernels of the benchmarked paths (C3, C5, live): no scratch at all
NO_SCRATCH = ("stft1024_kernel", "block_band_i8_kernel", "block_i8_kernel", "block_db_kernel", "detect_kernel",
              "welch_bands_kernel", "iq_band_delta_kernel", "scan_kernel", "frame_kernel", "live_over_kernel",
              "live_history_kernel", "welch_i8_kernel", "welch_i8_bands_kernel", "live_seg_init_kernel",
              "live_seg_link_kernel")


@pytest.fixture(scope="module")
def audit():
    return kr.audit(SO)


@pytest.fixture(scope="module")
def functions():
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(kr.code_objects(SO)):
            path = os.path.join(td, f"co{k}.o")
            open(path, "wb").write(co)
            for name, r in kr._function_instructions(path).items():
                out[name] = r
    return out


def test_code_objects_found(audit):
    assert len(audit) > 100, "expected every kernel of the library"
    for name in ("stft1024_kernel", "cstft4096_kernel", "welch_bands_kernel", "detect_kernel"):
        assert any(name in k for k in audit), name


def test_no_flat_memory_instructions(functions):
    bad = {k: r["flat"] for k, r in functions.items() if r["flat"]}
    assert not bad, f"generic-pointer (flat) accesses: {bad}"


def test_calls_only_where_listed(audit, functions):
    callers = {k for k, r in audit.items() if r["calls"]}
    assert all(any(f"{len(c)}{c}" in k for c in CALLERS) for k in callers), sorted(callers)
    assert not any(r.get("uses_dynamic_stack") for r in audit.values())


def test_hot_kernels_use_no_scratch(audit):
    # the Itanium-mangled name carries the identifier's length: "13detect_kernel" is not live_detect_kernel;
    # stft1024 only in its int16 form (the float32 forms spill at 128 VGPRs)
    hot = {k: r for k, r in audit.items() if any(f"{len(h)}{h}" in k for h in NO_SCRATCH)
           and not ("stft1024_kernel" in k and "stft1024_kernelIs" not in k)}
    assert len(hot) >= len(NO_SCRATCH) - 1
    bad = {k: r["private_segment_fixed_size"] for k, r in hot.items() if r["private_segment_fixed_size"]}
    assert not bad, bad


def test_c5_spectrogram_spill_bounded(audit):
    # cstft4096<int16> at 128 VGPRs (4 waves per SIMD) spills at most one register in the benchmarked
    # form; the generic instantiations stay under 96 B of scratch
    c5 = {k: r for k, r in audit.items() if "cstft4096_kernel" in k}
    assert c5
    assert max(r["private_segment_fixed_size"] for r in c5.values()) <= 96
