#!/bin/bash
# GPU round: all gpu tests, smoke, then a bench with a short profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-full}
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -30 gpurun_out/${TAG}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -5 gpurun_out/${TAG}_smoke.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --json-out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -8 gpurun_out/${TAG}_bench.log
exit $rc
