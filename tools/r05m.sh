set -o pipefail
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "bellman or lloyd or modified" tests/test_gpu_configs.py::test_c2_reference_aggregation_parity > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/agg_agreement.py --no-oracle --out $O/agg.json > $O/agg.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-varcoef > $O/bench.json 2> $O/bench.err
