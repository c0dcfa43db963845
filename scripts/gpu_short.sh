# The driver's bench form (--steps 20 --warmup 5) three times, and the default once: how much the
# short timed window (≈ 33 ms) reads below the long one.
set -o pipefail
TAG=${1:-short}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_s20_${TAG}_$i.json \
      2>> gpurun_out/bench_s20_$TAG.err || exit 1
done
timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-traffic > gpurun_out/bench_s300_$TAG.json \
    2>> gpurun_out/bench_s20_$TAG.err || exit 1
echo done
