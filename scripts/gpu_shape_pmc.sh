# SQ counters of the access-shape microbenchmark vs the aggregation kernel on a cache-resident
# operand (scripts/shape_kernel_probe.py): instructions and wait cycles per byte. One pass per
# counter set, each under its own kill timeout.
set -o pipefail
mkdir -p gpurun_out/shape_pmc
export TMPDIR=/tmp
REPO=$(pwd)
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
B="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
cd /tmp
i=0
for C in "$A" "$B"; do
  i=$((i+1))
  PER_WAVE=1024 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d /tmp/spmc_shape_$i -o run -- \
      $REPO/scripts/bin/gather_shape 4096 16 4 > $REPO/gpurun_out/shape_pmc/shape_$i.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d /tmp/spmc_kern_$i -o run -- \
      python3 $REPO/scripts/shape_kernel_probe.py > $REPO/gpurun_out/shape_pmc/kern_$i.log 2>&1 || exit 1
  find /tmp/spmc_shape_$i -name "*counter_collection.csv" -exec cp {} $REPO/gpurun_out/shape_pmc/shape_$i.csv \;
  find /tmp/spmc_kern_$i -name "*counter_collection.csv" -exec cp {} $REPO/gpurun_out/shape_pmc/kern_$i.csv \;
done
echo "exit 0"
