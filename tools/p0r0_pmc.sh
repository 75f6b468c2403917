#!/bin/bash
# HBM traffic of the C4 level-0 prolongation / restriction kernels (sorted format, value codes):
# separate FETCH_SIZE and WRITE_SIZE rocprofv3 passes over tools/p0r0_driver.py. GPU box only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc_p0r0
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_p0r0/$c
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_p0r0/$c -o run \
    -- python tools/p0r0_driver.py > gpurun_out/pmc_p0r0/$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
echo done
