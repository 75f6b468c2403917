set -o pipefail
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_distributed_loopback.py tests/test_gpu_hierarchy.py::test_c4_full_size_hierarchy_parity > $O/pytest.log 2>&1
