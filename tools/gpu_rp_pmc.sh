#!/bin/bash
# LDS / wait counters of the row-pair kernels on the C4 fine operator (window off / on)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/rp_pmc
for v in 0 1; do
  MLAMG_RP_WIN=$v timeout -k 10 120 python tools/rowpat_driver.py || exit 1
  MLAMG_RP_WIN=$v timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d gpurun_out/rp_pmc/w$v -o p -- python3 tools/rowpat_driver.py > gpurun_out/rp_pmc/w$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/rp_pmc/w$v.log; exit 1; }
  MLAMG_RP_WIN=$v timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT --output-format csv -d gpurun_out/rp_pmc/t$v -o p -- python3 tools/rowpat_driver.py > gpurun_out/rp_pmc/t$v.log 2>&1 || { echo "pmc2 $v failed"; tail -5 gpurun_out/rp_pmc/t$v.log; }
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob('gpurun_out/rp_pmc/[wt]?')):
    for f in glob.glob(d + '/*counter_collection.csv'):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if 'rowpair' in r['Kernel_Name']:
                acc[r['Counter_Name']].append(float(r['Counter_Value']))
        print(d, {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
