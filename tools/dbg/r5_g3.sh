L=tools/ubench/bin/libmsdsp_pdold.so; C=meteor-scatter_amd/meteorgpu/libmsdsp.so; N=tools/ubench/bin/libmsdsp_nomean.so
tools/gpu.sh multi 'test t_c5 tests/test_iq.py tests/test_gpu_certify.py tests/test_gpu_stream.py tests/test_gpu_parity.py' 'py dcprec2 400 tools/dbg/dc_precision.py' "stft_ab ab_pd0 c5 8 $L $C" || exit 1
STFT_AB_FSUMS=1,1 tools/gpu.sh stft_ab ab_pd2 c5 8 $L $C || exit 1
tools/gpu.sh stft_ab ab_c3 c3 8 $L $C $N || exit 1
for ov in 0 4 8 16 32; do echo "== overlap $ov"; tools/gpu.sh c5 c5ov$ov 1 --c5-overlap $ov || exit 1; done
AB_ARGS='--c5-mode exact' tools/gpu.sh ab c5 2 pdold cur
tools/gpu.sh py mall 300 tools/dbg/mall_interleave.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for F in 262144 8192; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "block_i8|cstft" -d gpurun_out/mallpmc_$F -o p --output-format csv -- python3 tools/dbg/mall_interleave.py $F > gpurun_out/mallpmc_$F.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for F in (262144, 8192):
    tot = {}
    for f in glob.glob(f"gpurun_out/mallpmc_{F}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = "block_i8" if "block_i8" in r["Kernel_Name"] else "cstft"
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
    print(F, {k: f"{v * 1024 / 1e9:.3f} GB (FETCH_SIZE KB x 1024, before the x2 gfx950 correction)" for k, v in tot.items()})
PY
