"""Diagnostic (GPU): host→device copy rate from page-locked memory, one 690 MB copy (one WavDay
batch) and the same split into chunks, through libmsdsp's copy stream.  Not a test."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "meteor-scatter_amd"))
from meteorgpu import _lib  # noqa: E402
from meteorgpu.ingest import PinnedBuffer  # noqa: E402

ctx = _lib.Context(0)
nb = 120 * 2880000 * 2
h = PinnedBuffer(ctx, nb)
C.memset(h.ptr, 1, nb)
d = ctx.alloc(nb)
lib = ctx.lib
for chunks in (1, 4, 16):
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        step = nb // chunks
        for c in range(chunks):
            lib.msd_memcpy_h2d_async(ctx.h, C.c_void_p(d.ptr.value + c * step), C.c_void_p(h.ptr.value + c * step),
                                     C.c_size_t(step))
        lib.msd_copy_synchronize(ctx.h)
        best = min(best, time.perf_counter() - t0)
    print(f"SDMA={os.environ.get('HSA_ENABLE_SDMA', 'default')} chunks {chunks:2d}: {nb / best / 1e9:.1f} GB/s", flush=True)
