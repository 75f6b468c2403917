set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py::test_c2_reference_aggregation_parity tests/test_gpu_contract.py::test_dispatch_packet_timer tests/test_gpu_coarse_pcg.py::test_pcg_breakdown_is_reported > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/agg_agreement.py --out $O/agg_agreement.json > $O/agg.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-varcoef > $O/bench_ref_sorted.json 2> $O/bench_ref_sorted.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-varcoef --aggregation bellman_ford > $O/bench_canon.json 2> $O/bench_canon.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-varcoef --coarse-order seed > $O/bench_ref_seed.json 2> $O/bench_ref_seed.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --dist > $O/bench_dist1.json 2> $O/bench_dist1.err
