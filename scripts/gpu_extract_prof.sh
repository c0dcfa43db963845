# rocprofv3 kernel stats of the extraction probe (per-kernel durations). Usage: TAG [VARIANTS]
set -o pipefail
TAG=${1:-p}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/xprof_$TAG -o x -- \
    python -u $REPO/scripts/extract_probe.py > $REPO/gpurun_out/extract_prof_$TAG.json 2> $REPO/gpurun_out/extract_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/xprof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/extract_kstats_$TAG.csv \; 2>/dev/null
find /tmp/xprof_$TAG -name "*kernel_trace.csv" -exec cp {} gpurun_out/extract_ktrace_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
