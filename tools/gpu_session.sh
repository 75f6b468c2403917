# ad-hoc GPU session (edited per experiment)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/p0_time.py 2>&1 | grep p0_time || exit 1
MLAMG_AP_NOPRE=1 timeout -k 10 200 python tools/p0_time.py 2>&1 | grep p0_time || exit 1
