set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
