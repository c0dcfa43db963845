# GPU box (round 2): parity tests, smoke, default bench, rocprofv3 kernel stats of the bench.
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
TAG=${1:-r2}
STEPS=${STEPS:-tests,smoke,bench,prof}
rc=0
run() { # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] start $name" >> gpurun_out/progress_$TAG.txt
  timeout -k 10 "$secs" "$@"
  local r=$?
  echo "[$(date +%T)] end $name rc=$r" >> gpurun_out/progress_$TAG.txt
  return $r
}
if [[ $STEPS == *tests* ]]; then
  run tests 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "tests rc=$?"; exit 1; }
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
      || { echo "smoke rc=$?"; exit 1; }
fi
if [[ $STEPS == *bench* ]]; then
  run bench 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
      || { echo "bench rc=$?"; exit 1; }
fi
if [[ $STEPS == *prof* ]]; then
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gnnprof/prof -o run -- \
      python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || rc=$?
  find /tmp/gnnprof/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$TAG.csv \;
fi
echo "exit $rc"
exit $rc
