set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u tools/bench_configs.py --steps 50 --done-ab --no-cpu --out $O/configs_done_ab.json > $O/configs.log 2>&1
