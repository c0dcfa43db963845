# Standalone extraction kernels per variant (scripts/extract_probe.py) under rocprofv3 kernel stats:
# one process per variant (args: "tag:ENV=v,ENV=v"), REPS calls of each layer with and without the
# transpose, on an idle GPU.
set -o pipefail
TAG=${TAG:-lxp}
mkdir -p gpurun_out/lxp_$TAG
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp
for spec in "$@"; do
  name=${spec%%:*}; var=${spec#*:}
  VARIANTS="$var" REPS=${REPS:-50} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d /tmp/lxp_$name -o run -- python3 -u $REPO/scripts/extract_probe.py \
      > $REPO/gpurun_out/lxp_$TAG/$name.jsonl 2> $REPO/gpurun_out/lxp_$TAG/$name.err || exit 1
  find /tmp/lxp_$name -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/lxp_$TAG/kstats_$name.csv \;
done
echo "exit 0"
