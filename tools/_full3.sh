set -u
bash tools/gpu_full.sh && bash tools/gpu_trace_main.sh
