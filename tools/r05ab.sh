set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 600 python -u tools/amg2v_large.py 256 384 512 > $O/win.jsonl 2> $O/err1.log && \
MLAMG_GS_PREFER_RING=1 timeout -k 10 600 python -u tools/amg2v_large.py 256 384 512 > $O/ring.jsonl 2> $O/err2.log
