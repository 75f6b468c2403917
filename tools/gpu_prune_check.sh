#!/bin/bash
# autotune pruning: hierarchy / config parity tests, then the default bench (setup_s.formats)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hierarchy.py tests/test_gpu_configs.py tests/test_gpu_distributed_loopback.py > gpurun_out/t_prune.log 2>&1 || { tail -30 gpurun_out/t_prune.log; exit 1; }
tail -2 gpurun_out/t_prune.log
timeout -k 10 600 python bench.py > gpurun_out/bench_prune.json 2> gpurun_out/bench_prune.err || { tail -20 gpurun_out/bench_prune.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_prune.json').read().splitlines()[0])
print(d['value'], d['ms_per_step'], d['setup_s'])
for l in d['format_autotune_us']:
    print({k: (v['chosen'], v.get('pruned')) for k, v in l.items()})
"
