set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hierarchy.py -k "factored" > $O/pytest2.log 2>&1 ; \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-c3 --no-varcoef > $O/bench.json 2> $O/bench.err && \
bash tools/r05e.sh > $O/traces.log 2>&1
