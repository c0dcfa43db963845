# Per-dispatch kernel trace of a short default bench (rocprofv3 --kernel-trace, CSV kept): the
# durations of every call site, for the per-call breakdown that --stats averages away.
set -o pipefail
TAG=${1:-trace}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-traffic --gpu-step-batches 20 \
    > $REPO/gpurun_out/bench_trace_$TAG.json 2> $REPO/gpurun_out/bench_trace_$TAG.err
rc=$?
cd $REPO
f=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
r=csv.DictReader(open('$f'))
keep=['Kernel_Name','Start_Timestamp','End_Timestamp','Grid_Size_X','Grid_Size_Y','Grid_Size_Z','Workgroup_Size_X','Queue_Id','Stream_Id']
w=csv.DictWriter(open('gpurun_out/ktrace_$TAG.csv','w'),fieldnames=keep,extrasaction='ignore')
w.writeheader()
for row in r: w.writerow({k:row.get(k,'') for k in keep})
"
echo "exit $rc"
exit $rc
