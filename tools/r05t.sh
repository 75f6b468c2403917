set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py > $O/pytest_sa.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_smoothing_variants.py tests/test_gpu_contract.py -k "gs or gauss or seidel or export or contract" > $O/pytest_gs.log 2>&1
