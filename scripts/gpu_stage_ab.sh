# A/B of the staging depth (--stage-ahead): end to end and gpu_step, A/B/A/B on one box.
set -o pipefail
TAG=${1:-sa}
mkdir -p gpurun_out
i=0
for SA in 1 2 1 2 3; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic --stage-ahead $SA \
      > gpurun_out/stage_${TAG}_$i.json 2> gpurun_out/stage_${TAG}_$i.err || exit 1
done
echo "exit 0"
