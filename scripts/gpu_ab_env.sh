# A/B of environment knobs on the default bench under rocprofv3 kernel stats. Usage: TAG "ENV1" "ENV2" ...
# (each argument: space-separated NAME=VALUE assignments, or "-" for none)
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
i=0
for ENVS in "$@"; do
  i=$((i+1))
  (
    [ "$ENVS" != "-" ] && export $ENVS
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ab_${TAG}_$i -o run -- \
        python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic --no-gpu-step \
        > $REPO/gpurun_out/ab_${TAG}_$i.json 2> $REPO/gpurun_out/ab_${TAG}_$i.err
  ) || { echo "failed $ENVS"; exit 1; }
  find /tmp/ab_${TAG}_$i -name "*kernel_stats.csv" -exec cp {} gpurun_out/ab_kstats_${TAG}_$i.csv \;
  echo "$i $ENVS" >> gpurun_out/ab_${TAG}_index.txt
done
echo "exit 0"
