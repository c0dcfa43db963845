# GPU box (1 GPU): rehearse the N=2 bench path with both ranks on cuda:0 (RCCL).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS:-} \
    > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err
rc=$?
tail -c 3000 gpurun_out/bench_dist2.json
echo "exit $rc"
