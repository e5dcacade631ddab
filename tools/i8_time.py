"""Time the exact C5 delta (msd_iq_delta64_dev: block_i8_kernel + frame_kernel) on its own, on a
3 h 192 kHz int16 I/Q shard of random samples resident in HBM, for library variants built by
tools/patch_build.sh (the bench's detector would reject a variant's garbage delta).

usage (GPU box): python3 tools/i8_time.py [TAG ...]   ("cur" = meteorgpu/libmsdsp.so)
Prints per variant the median of 10 timed calls, split into the two kernels."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(tag):
    sys.path.insert(0, os.path.join(ROOT, "meteor-scatter_amd"))
    import numpy as np
    import torch
    from meteorgpu import _lib, iq
    fs, N, hop, secs = 192000, 4096, 1024, int(os.environ.get("I8_SECONDS", "10800"))
    n = fs * secs + N - hop
    T = (n - N) // hop + 1
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(-3000, 3000, (2 * n,), dtype=torch.int16, device="cuda", generator=g)
    delta = torch.empty(T, dtype=torch.float64, device="cuda")
    ed = torch.empty(T, dtype=torch.float64, device="cuda")
    ctx = _lib.Context(0)
    band, noise = iq.iq_band_bins(N, fs, (950.0, 1050.0)), iq.iq_band_bins(N, fs, (-3050.0, -2950.0))
    r = np.array([[0, T]], np.int64)
    args = (ctx, x.data_ptr(), _lib.MSD_CI16, n, N, hop, float(fs), band, noise, r, delta.data_ptr(), ed.data_ptr())
    for _ in range(3):
        _lib.iq_delta64_dev(*args)
    ctx.synchronize()
    ms = []
    for _ in range(10):
        ctx.timing(True)
        ctx.timing_reset()
        _lib.iq_delta64_dev(*args)
        ctx.synchronize()
        ms.append(ctx.timing_get(_lib.K_REFINE)[0])
    ms.sort()
    print(f"{tag:10s} delta64 median {ms[5]:.4f} ms  min {ms[0]:.4f}  (T {T}, blocks {T + 3})", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(sys.argv[2])
        sys.exit(0)
    for t in sys.argv[1:] or ["cur"]:
        lib = (os.path.join(ROOT, "meteor-scatter_amd/meteorgpu", "libmsdsp.so") if t == "cur"
               else os.path.join(ROOT, "tools/ubench/bin", f"libmsdsp_{t}.so"))
        env = dict(os.environ, MSD_LIB_PATH=lib)
        rc = subprocess.run([sys.executable, __file__, "--one", t], env=env, timeout=300).returncode
        if rc:
            sys.exit(rc)
