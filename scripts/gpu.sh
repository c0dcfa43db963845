# One runner for every GPU-box call (replaces the round-1..4 one-off scripts/gpu_*.sh).
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failure ends the call (no GPU
# step runs after a failed, aborted or timed-out one). Outputs go to gpurun_out/*_TAG*.
#   tests[:PYTEST_K]     pytest -m gpu (optionally -k PYTEST_K; ',' in it means ' or ')
#   tfile:FILE[,FILE]    pytest -m gpu on the named test files only
#   smoke                __graft_entry__.smoke()
#   bench[:ARGS]         python bench.py ARGS (',' in ARGS means ' '), JSON line -> bench_TAG_N.json
#   envbench:ENV:ARGS    bench with ENV (NAME=V+NAME=V) — for A/B/A/B runs of knobs
#   kstats[:ARGS]        rocprofv3 --kernel-trace --stats of bench.py ARGS -> kstats_TAG_N.csv
#   ktrace[:ARGS]        rocprofv3 --kernel-trace (per dispatch, trimmed CSV) -> ktrace_TAG_N.csv
#   cpu1                 bench.py --cpu (BASELINE config 1 on the box's host)
#   self2                GNN_DIST_BACKEND=gloo bench.py --gpus 2 (self-launched ranks on the one GPU)
#   py:SCRIPT[:ARGS]     python SCRIPT ARGS (probes under scripts/)
#   envpy:ENV:SCRIPT[:ARGS]  the same with ENV (NAME=V+NAME=V)
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
n=0
sp() { echo "${1//,/ }"; }
for STEP in "$@"; do
  n=$((n+1))
  kind=${STEP%%:*}
  arg=""
  [ "$kind" != "$STEP" ] && arg=${STEP#*:}
  out=gpurun_out/${kind}_${TAG}_$n
  echo "[gpu.sh] step $n: $STEP ($(date +%T))"
  case $kind in
    tests)
      K=()
      [ -n "$arg" ] && K=(-k "${arg//,/ or }")
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${K[@]}" \
          > $out.log 2>&1; rc=$?; tail -3 $out.log ;;
    tfile)
      timeout -k 10 600 python -u -m pytest $(sp "$arg") -m gpu -x -v --timeout 200 --timeout-method thread \
          > $out.log 2>&1; rc=$?; tail -3 $out.log ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out.log 2>&1; rc=$?; cat $out.log ;;
    bench)
      timeout -k 10 500 python -u bench.py $(sp "$arg") > $out.json 2> $out.err; rc=$?
      python3 -c "import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);print('value',d['value'],'gpu_step',(d.get('gpu_step') or {}).get('value'))" 2>/dev/null ;;
    envbench)
      envs=${arg%%:*}; bargs=""; [ "$envs" != "$arg" ] && bargs=${arg#*:}
      env ${envs//+/ } timeout -k 10 500 python -u bench.py $(sp "$bargs") > $out.json 2> $out.err; rc=$?
      echo "$envs" > $out.env
      python3 -c "import json;d=json.loads(open('$out.json').read().strip().splitlines()[-1]);print('$envs','value',d['value'],'gpu_step',(d.get('gpu_step') or {}).get('value'))" 2>/dev/null ;;
    kstats|ktrace)
      mode="--kernel-trace --stats"; [ $kind = ktrace ] && mode="--kernel-trace"
      ( cd /tmp && timeout -k 10 500 rocprofv3 $mode --output-format csv -d /tmp/prof_${TAG}_$n -o run -- \
          python -u $REPO/bench.py $(sp "$arg") > $REPO/$out.json 2> $REPO/$out.err ); rc=$?
      if [ $kind = kstats ]; then
        find /tmp/prof_${TAG}_$n -name "*kernel_stats.csv" -exec cp {} $out.csv \;
      else
        f=$(find /tmp/prof_${TAG}_$n -name "*kernel_trace.csv" | head -1)
        [ -n "$f" ] && python3 - "$f" $out.csv <<'EOF'
import csv, sys
keep = ['Kernel_Name', 'Start_Timestamp', 'End_Timestamp', 'Grid_Size_X', 'Grid_Size_Y', 'Grid_Size_Z',
        'Workgroup_Size_X', 'Queue_Id', 'Stream_Id']
w = csv.DictWriter(open(sys.argv[2], 'w'), fieldnames=keep, extrasaction='ignore')
w.writeheader()
for row in csv.DictReader(open(sys.argv[1])):
    w.writerow({k: row.get(k, '') for k in keep})
EOF
      fi ;;
    cpu1)
      timeout -k 10 300 python -u bench.py --cpu --steps 30 --warmup 3 > $out.json 2> $out.err; rc=$? ;;
    self2)
      GNN_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 3 > $out.json 2> $out.err; rc=$? ;;
    py)
      script=${arg%%:*}; pargs=""; [ "$script" != "$arg" ] && pargs=${arg#*:}
      timeout -k 10 500 python -u $script $(sp "$pargs") > $out.log 2>&1; rc=$?; tail -5 $out.log ;;
    envpy)
      envs=${arg%%:*}; rest=${arg#*:}; script=${rest%%:*}; pargs=""; [ "$script" != "$rest" ] && pargs=${rest#*:}
      env ${envs//+/ } timeout -k 10 500 python -u $script $(sp "$pargs") > $out.log 2>&1; rc=$?
      echo "$envs" > $out.env; tail -5 $out.log ;;
    *)
      echo "unknown step $STEP"; rc=2 ;;
  esac
  echo "[gpu.sh] step $n: $STEP -> exit $rc ($(date +%T))"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
