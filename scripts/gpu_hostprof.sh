# Host-side profile (cProfile) of a short default bench: where the ~0.6-1.0 ms of host issue per
# step goes (the sampler threads are native and invisible here).
set -o pipefail
TAG=${1:-hostprof}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m cProfile -o gpurun_out/hostprof_$TAG.out bench.py --steps 200 --no-cpu-baseline \
    --no-traffic > gpurun_out/bench_hostprof_$TAG.json 2> gpurun_out/bench_hostprof_$TAG.err || exit 1
python - <<PY > gpurun_out/hostprof_$TAG.txt
import pstats
p = pstats.Stats("gpurun_out/hostprof_$TAG.out")
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
PY
echo done
