# Extraction A/Bs: variants given as arguments, each "name:ENV=... --flag ..." (name = file tag).
# MODE=plain: bench runs for the rates (500 steps); MODE=prof: one rocprofv3 kernel-stats run per
# variant (300 steps) for the lx_* GPU time. TESTS=1 first runs the extraction GPU tests.
set -o pipefail
TAG=${TAG:-xl}
mkdir -p gpurun_out/xl_$TAG
export TMPDIR=/tmp
REPO=$(pwd)
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_extract.py tests/test_extract_full_gpu.py -m gpu -x -v \
      --timeout 120 --timeout-method thread > gpurun_out/xl_$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
fi
i=0
for spec in "$@"; do
  i=$((i+1))
  name=${spec%%:*}; rest=${spec#*:}
  envs=""; args=""
  for w in $rest; do case "$w" in -*) args="$args $w";; *) envs="$envs $w";; esac; done
  if [ "${MODE:-plain}" = "plain" ]; then
    env $envs timeout -k 10 300 python -u bench.py --steps 500 --no-cpu-baseline --no-traffic $args \
        > gpurun_out/xl_$TAG/bench_${i}_$name.json 2> gpurun_out/xl_$TAG/bench_${i}_$name.err || exit 1
  else
    (cd /tmp && env $envs timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/xl_$i -o run -- \
        python -u $REPO/bench.py --steps 300 --no-cpu-baseline --no-traffic --no-roofline $args \
        > $REPO/gpurun_out/xl_$TAG/prof_${i}_$name.json 2> $REPO/gpurun_out/xl_$TAG/prof_${i}_$name.err) || exit 1
    find /tmp/xl_$i -name "*kernel_stats.csv" -exec cp {} gpurun_out/xl_$TAG/kstats_${i}_$name.csv \;
  fi
done
echo "exit 0"
