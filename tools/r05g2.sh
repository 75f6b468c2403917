set -o pipefail
O=gpurun_out/r05g2; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py tests/test_gpu_kernels.py tests/test_gpu_smoothing_variants.py tests/test_gpu_callers.py tests/test_gpu_coarse_pcg.py tests/test_gpu_preconditioner.py > $O/pytest.log 2>&1 ; echo "rc=$?" >> $O/pytest.log
timeout -k 10 600 python -u tools/pyamg_sa_bench.py --case poisson3d:216 --no-cpu --out $O/big.json > $O/big.log 2>&1
