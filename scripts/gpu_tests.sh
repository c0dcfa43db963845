set -o pipefail
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "exit $?"
