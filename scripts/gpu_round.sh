#!/bin/bash
# Usage: bash scripts/gpu_round.sh <tag> "<pytest args>" "<bench cmd>"
# Runs GPU tests, then (only if the tests ended normally: exit 0 or 1) a benchmark command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; TESTS=$2; BENCH=${3:-}
export HSA_ENABLE_IPC_MODE_LEGACY=0
rc=0
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -m pytest $TESTS -q -rf > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"; tail -25 gpurun_out/${TAG}_tests.log
fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "stopping after abnormal test exit $rc"; exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 bash -c "$BENCH" > gpurun_out/${TAG}_bench.log 2>&1
  brc=$?
  echo "bench rc=$brc"; tail -60 gpurun_out/${TAG}_bench.log
  exit $brc
fi
exit $rc
