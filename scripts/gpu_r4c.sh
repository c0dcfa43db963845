# Round-4 GPU pass c: kernel durations of the layer-2 probe (rocprofv3 kernel trace + stats) and
# the MFMA hybrid probe.
set -o pipefail
TAG=${1:-r4c}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_l2_$TAG -o run -- \
    python -u $REPO/scripts/spmm_layer2_probe.py --out $REPO/gpurun_out/layer2_probe_$TAG.json \
    > $REPO/gpurun_out/layer2_probe_$TAG.log 2>&1
rc=$?
cd $REPO
find /tmp/prof_l2_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_layer2_$TAG.csv \; 2>/dev/null
find /tmp/prof_l2_$TAG -name "*kernel_trace.csv" -exec cp {} gpurun_out/ktrace_layer2_$TAG.csv \; 2>/dev/null
[ $rc -eq 0 ] && timeout -k 10 400 python -u scripts/mfma_hybrid_probe.py --out gpurun_out/mfma_hybrid_$TAG.json \
    > gpurun_out/mfma_hybrid_$TAG.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
