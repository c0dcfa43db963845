set -o pipefail
mkdir -p gpurun_out /tmp/gp
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_tests.log 2>&1 || exit 1
for P in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVES"; do
  n=$(echo $P | cut -c1-8)
  VARIANTS=0 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d /tmp/gp/prof_$n -o run -- python scripts/gemm_bench.py > gpurun_out/gemm_pmc_$n.log 2>&1 || exit 2
  find /tmp/gp/prof_$n -name "*counter_collection.csv" -exec cp {} gpurun_out/gemm_pmc_counters_$n.csv \;
done
echo done
