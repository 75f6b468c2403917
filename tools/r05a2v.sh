set -o pipefail
O=gpurun_out/r05a2v; mkdir -p $O
timeout -k 10 900 python -u tools/amg2v_large.py 256 512 768 1024 > $O/amg2v_large.jsonl 2> $O/err.log
