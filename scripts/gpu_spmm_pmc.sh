# GPU box: SQ stall counters of the aggregation kernels on a dumped Reddit LADIES batch
# (scripts/spmm_microbench.py, default unit sizes), one rocprofv3 --pmc pass per counter set.
set -o pipefail
mkdir -p gpurun_out /tmp/sp
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-e2e \
    --dump-batch /tmp/sp/batch0.npz > gpurun_out/spmm_pmc_bench.json 2> gpurun_out/spmm_pmc_bench.err || exit 1
i=0
for P in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM" \
         "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d /tmp/sp/p$i -o run -- \
      python scripts/spmm_microbench.py /tmp/sp/batch0.npz --units 0 --reps 5 > gpurun_out/spmm_pmc_$i.log 2>&1 || exit 2
  find /tmp/sp/p$i -name "*counter_collection.csv" -exec cp {} gpurun_out/spmm_pmc_counters_$i.csv \;
done
echo done
