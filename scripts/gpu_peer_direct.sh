# Peer rows read directly over IPC-mapped buffers (staging.PeerDirect): the GPU tests, then the
# N=2 bench rehearsal on one GPU (gloo) with each peer-row form; the final losses must agree.
set -o pipefail
TAG=${1:-pd}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v -k "peer" --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_peer_$TAG.log 2>&1 || exit 1
for PR in alltoall direct; do
  GNN_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 5 \
      --gpu-step-batches 20 --peer-rows $PR > gpurun_out/bench_dist2_${PR}_$TAG.json \
      2> gpurun_out/bench_dist2_${PR}_$TAG.err || exit 1
done
echo "exit 0"
