set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py::test_c2_reference_aggregation_parity tests/test_gpu_hierarchy.py::test_c4_full_size_hierarchy_parity > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/agg_agreement.py --out $O/agg.json > $O/agg.log 2>&1
