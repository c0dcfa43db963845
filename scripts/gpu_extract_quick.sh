# Quick GPU check of the LADIES extraction: parity tests + standalone probe (+ timing variants
# in $VARIANTS, e.g. "GNN_LX_LDS=0;GNN_LX_XU=16"). Usage: TAG
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract.py tests/test_extract_full_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_extract_$TAG.log 2>&1 && \
timeout -k 10 300 python -u scripts/extract_probe.py > gpurun_out/extract_probe_$TAG.json 2> gpurun_out/extract_probe_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
