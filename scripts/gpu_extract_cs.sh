# Standalone extraction probe per compaction slice count (GNN_LX_CS), after the parity tests.
set -o pipefail
TAG=${1:-cs}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract.py tests/test_extract_full_gpu.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_extract_$TAG.log 2>&1 || exit 1
for CS in 1 4 8 16 32; do
  GNN_LX_CS=$CS timeout -k 10 300 python -u scripts/extract_probe.py > gpurun_out/extract_probe_${TAG}_cs$CS.json \
      2> gpurun_out/extract_probe_${TAG}_cs$CS.err || exit 1
done
echo "exit 0"
