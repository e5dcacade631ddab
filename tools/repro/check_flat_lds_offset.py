#!/usr/bin/env python3
"""Compile tools/repro/flat_lds_offset.hip for gfx950 (CPU only) and report whether the compiler
still displaces the flat loop pointer below the object (`base - 64`, then `offset:128 ..`), the
pattern behind round 5's MEMORY_APERTURE_VIOLATION.  Never runs the kernel."""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "r.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                        "-S", os.path.join(HERE, "flat_lds_offset.hip"), "-o", asm], check=True)
        txt = open(asm).read()
    fn = txt[txt.index("_Z8pair_sumPKdll:"):txt.index(".Lfunc_end0")]
    neg = re.findall(r"s_mov_b64 (s\[\d+:\d+\]), (?:-64|0xffffffffffffffc0)", fn)
    movk = re.findall(r"s_movk_i32 (s\d+), 0xffc0", fn)
    offs = sorted({int(o) for o in re.findall(r"flat_load_dwordx4 v\[\d+:\d+\], v\[\d+:\d+\] offset:(\d+)", fn)})
    print(f"negative pointer displacement constants: {len(neg) + len(movk)}; flat_load_dwordx4 offsets: {offs}")
    hit = (neg or movk) and offs and max(offs) >= 128
    print("defect pattern present" if hit else "defect pattern not found")
    return 0


if __name__ == "__main__":
    sys.exit(main())
