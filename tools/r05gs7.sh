set -o pipefail
O=gpurun_out/r05gs7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pyamg_sa.py tests/test_gpu_kernels.py tests/test_gpu_callers.py tests/test_gpu_smoothing_variants.py > $O/pytest.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe -o run -- python3 tools/gs_probe.py > $O/probe.log 2>&1 && \
timeout -k 10 900 python -u tools/pyamg_sa_bench.py --case poisson2d:1024 --case poisson3d:128 --out $O/pyamg_sa.json > $O/pyamg_sa.log 2>&1 ;
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete; du -sh $O
