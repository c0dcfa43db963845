# Extraction experiments: timing variants (GNN_LX_FLAGS / XU / XW) + one SQ PMC pass. Usage: TAG
set -o pipefail
TAG=${1:-e}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
VARIANTS="${VARIANTS:-GNN_LX_LDS=1;GNN_LX_LDS=0}" \
  timeout -k 10 300 python -u scripts/extract_probe.py > gpurun_out/extract_exp_$TAG.json 2> gpurun_out/extract_exp_$TAG.err && \
cd /tmp && REPS=3 timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d /tmp/pmc_$TAG -o p -- \
    python -u $REPO/scripts/extract_probe.py > $REPO/gpurun_out/extract_pmc_$TAG.log 2>&1
rc=$?
cd $REPO
find /tmp/pmc_$TAG -name "*counter_collection.csv" -exec cp {} gpurun_out/extract_pmc_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
