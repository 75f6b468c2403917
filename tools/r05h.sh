set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_hierarchy.py -k "sorted_value_codes or exact_formats" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/vc_ab.py > $O/vc_ab.jsonl 2> $O/vc_ab.err
