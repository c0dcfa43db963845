# GPU box: effective clock + MFMA busy of the layer GEMMs (rocprofv3 PMC, its own pass).
set -o pipefail
mkdir -p gpurun_out /tmp/gp
export TMPDIR=/tmp
VARIANTS=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES} \
    --output-format csv -d /tmp/gp/prof -o run -- python scripts/gemm_bench.py > gpurun_out/gemm_pmc.log 2>&1
rc=$?
find /tmp/gp/prof -name "*counter_collection.csv" -exec cp {} gpurun_out/gemm_pmc_counters.csv \;
find /tmp/gp/prof -name "*kernel_trace.csv" -exec cp {} gpurun_out/gemm_pmc_trace.csv \;
echo "exit $rc"
