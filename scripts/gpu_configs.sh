# GPU box (1 GPU): the other BASELINE configs' single-GPU shapes, then the N=2 path rehearsed
# on one GPU (both ranks on cuda:0, gloo backend: RCCL refuses two ranks per GPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-cpu-baseline --no-traffic --no-e2e"
timeout -k 10 300 python bench.py --graph products $B > gpurun_out/cfg_products_sage.json 2> gpurun_out/cfg_products_sage.err && \
timeout -k 10 300 python bench.py --graph products --model gcn --sampler fastgcn $B > gpurun_out/cfg_products_gcn.json 2> gpurun_out/cfg_products_gcn.err && \
timeout -k 10 300 python bench.py --model gcn --sampler fastgcn $B > gpurun_out/cfg_reddit_gcn.json 2> gpurun_out/cfg_reddit_gcn.err && \
timeout -k 10 300 python bench.py --graph papers $B > gpurun_out/cfg_papers_sage.json 2> gpurun_out/cfg_papers_sage.err && \
GNN_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $B > gpurun_out/cfg_dist2.json 2> gpurun_out/cfg_dist2.err
rc=$?
echo "exit $rc"
