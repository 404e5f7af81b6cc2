#!/bin/bash
# Usage: bash scripts/gpu_step.sh <tag> <timeout_s> <cmd...>
# Runs one GPU step under its own time limit, output to gpurun_out/<tag>.log; prints the tail.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; T=$2; shift 2
timeout -k 10 "$T" "$@" > "gpurun_out/$TAG.log" 2>&1
rc=$?
echo "== $TAG rc=$rc"; tail -30 "gpurun_out/$TAG.log" | grep -v amdgpu.ids
exit $rc
