# Round 3: DP exchange + torch extension GPU tests, then the N=2 rehearsal on one GPU (gloo): the
# bench times the flat and the bucketed exchange (dp_exchange_ab). Usage: TAG
set -o pipefail
TAG=${1:-dp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dist_gpu.py tests/test_torch_ext.py -m gpu -x -v \
    --timeout 240 --timeout-method thread > gpurun_out/gputest_dp_$TAG.log 2>&1 && \
GNN_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 60 --warmup 5 --gpu-step-batches 30 \
    > gpurun_out/bench_dist2_$TAG.json 2> gpurun_out/bench_dist2_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
