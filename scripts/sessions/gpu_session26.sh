#!/bin/bash
# GPU session 26 (round 3): (1) minimal-kernel attempt, full sequence: the packed complex twiddle multiply of the failing
# AFNO builds (two v_pk_mul_f32 op_sel:[0,1] products consumed 3 instructions later by two v_pk_fma_f32) on an
# LDS-loaded twiddle pair, co-resident workgroups; (2) fp32 FourCastNet step kernel table (rocprofv3 --kernel-trace --stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for m in "0 77448 2944 200 1" "2 77448 2944 200 1" "1 77448 2944 200 1" "0 16000 8192 200 1"; do
  timeout -k 10 120 ./diag_libs/opsel_lds_repro $m || { echo "repro ended abnormally"; exit 1; }
done
# (1b) the same with MFMA co-runner waves: 512-thread workgroups, waves 0-3 a dependent MFMA chain, waves 4-7 the check
for m in "0 77448 2944 200 2" "2 77448 2944 200 2" "1 77448 2944 200 2" "0 120000 2944 200 2"; do
  timeout -k 10 120 ./diag_libs/opsel_lds_repro2 $m || { echo "repro2 ended abnormally"; exit 1; }
done
PROF_TAG=_r3c timeout -k 10 700 bash scripts/prof_bench.sh > gpurun_out/s26_prof.txt 2>&1; rc=$?
head -30 gpurun_out/s26_prof.txt; exit $rc
