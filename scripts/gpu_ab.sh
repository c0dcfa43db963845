# GPU box: gpu tests, then A/B bench runs (one argument per run: env settings and --bench-flags, "-" = defaults).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
fi
i=0
for spec in "$@"; do
  i=$((i+1))
  if [ "$spec" = "-" ]; then spec=""; fi
  envs=""; args=""
  for w in $spec; do case "$w" in -*) args="$args $w";; *) envs="$envs $w";; esac; done
  env $envs timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 10 --no-cpu-baseline --no-traffic ${BENCH_ARGS:---no-e2e} $args \
      > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { echo "bench $i failed"; exit 1; }
  echo "$i [$spec] $(python -c "import json,sys;d=json.loads(open('gpurun_out/bench_${TAG}_$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:round(v['avg_us'],1) for k,v in d['spmm_per_callsite'].items()})")"
done
