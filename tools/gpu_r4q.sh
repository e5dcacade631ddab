# round 4: where the C5 exact step's host time goes (cProfile over a short bench run)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/r4q_c5.prof bench.py --workload c5 --c5-mode exact --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4q_c5.json 2> gpurun_out/r4q_c5.err &&
python3 -c "
import pstats; p = pstats.Stats('gpurun_out/r4q_c5.prof'); p.sort_stats('tottime').print_stats(30)" > gpurun_out/r4q_tottime.txt &&
python3 -c "
import pstats; p = pstats.Stats('gpurun_out/r4q_c5.prof'); p.sort_stats('cumulative').print_stats(60)" > gpurun_out/r4q_cum.txt && echo done
