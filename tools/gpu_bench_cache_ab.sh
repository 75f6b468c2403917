# default bench with the device allocation cache off / on / off / on (same box). Each GPU step
# has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  MLAMG_DEVICE_CACHE_MB=0 timeout -k 10 400 python bench.py > gpurun_out/bench_nocache_$i.json 2> gpurun_out/bench_nocache_$i.err || { tail -5 gpurun_out/bench_nocache_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_nocache_$i.json')); print('nocache', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  timeout -k 10 400 python bench.py > gpurun_out/bench_cache_$i.json 2> gpurun_out/bench_cache_$i.err || { tail -5 gpurun_out/bench_cache_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_cache_$i.json')); print('cache', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
