set -o pipefail
O=gpurun_out/r05z3; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> $O/pytest_gpu.log
