set -o pipefail
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u tools/bench_configs.py --steps 50 --cpu-cycles 5 --done-ab --out $O/configs.json > $O/configs.log 2>&1 && \
timeout -k 10 900 python -u tools/amg2v_farm_procs.py --procs 1,4,8,16 --grids 80 --out $O/amg2v_farm_procs.json > $O/farm.log 2>&1
