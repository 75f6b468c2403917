set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_hierarchy.py tests/test_gpu_configs.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1
