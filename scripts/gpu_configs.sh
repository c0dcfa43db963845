# GPU box (1 GPU): the other BASELINE configs' single-GPU shapes end to end (live sampling),
# then the N=2 path rehearsed on one GPU (both ranks on cuda:0, gloo backend: RCCL refuses two
# ranks per GPU). Usage: bash scripts/gpu_configs.sh TAG
set -o pipefail
T=gpurun_out/${1:-cfg}
mkdir -p $T
export TMPDIR=/tmp
B="--steps 100 --warmup 5 --no-cpu-baseline --no-traffic"
timeout -k 10 400 python bench.py --graph products $B > $T/products_sage.json 2> $T/products_sage.err && \
timeout -k 10 400 python bench.py --graph products --model gcn --sampler fastgcn $B > $T/products_gcn.json 2> $T/products_gcn.err && \
timeout -k 10 300 python bench.py --model gcn --sampler fastgcn $B > $T/reddit_gcn.json 2> $T/reddit_gcn.err && \
timeout -k 10 400 python bench.py --graph papers $B > $T/papers_sage.json 2> $T/papers_sage.err && \
GNN_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $B > $T/dist2.json 2> $T/dist2.err
rc=$?
echo "exit $rc"
exit $rc
