# Round-4 GPU pass b: the row kernel's tests, the layer-2 probe, the MFMA hybrid probe.
set -o pipefail
TAG=${1:-r4b}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gputest_spmm_$TAG.log 2>&1 && \
timeout -k 10 300 python -u scripts/spmm_layer2_probe.py --out gpurun_out/layer2_probe_$TAG.json \
    > gpurun_out/layer2_probe_$TAG.log 2>&1 && \
timeout -k 10 400 python -u scripts/mfma_hybrid_probe.py --out gpurun_out/mfma_hybrid_$TAG.json \
    > gpurun_out/mfma_hybrid_$TAG.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
