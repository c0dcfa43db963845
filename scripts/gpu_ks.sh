# GPU box: per-kernel stats of the bench step under an env setting: bash scripts/gpu_ks.sh TAG [ENV=..]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks_$TAG -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-e2e > gpurun_out/ks_$TAG.json 2> gpurun_out/ks_$TAG.err
rc=$?
find /tmp/ks_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/ks_$TAG.csv \;
exit $rc
