set -o pipefail
O=gpurun_out/r05z2; mkdir -p $O
timeout -k 10 600 python -u tools/bench_configs.py --steps 50 --cpu-cycles 5 --out $O/configs.json > $O/configs.log 2>&1 && \
OUT=$O/prof bash tools/gpu_prof_r05.sh > $O/prof.log 2>&1
