#!/bin/bash
# GPU session 27 (round 3): which packed-FP32 form goes wrong beside MFMA waves (scripts/diag/opsel_lds_repro.hip,
# built in the container): 512-thread workgroups, waves 0-3 a dependent MFMA chain, waves 4-7 one packed product per
# step on a global-loaded pair, in four forms (11: v_pk_mul op_sel:[0,1]; 12: v_pk_mul op_sel_hi:[1,0] on a v_mov'd
# copy = the shipped AFNO form; 13: v_pk_mul op_sel:[1,0] = src0 high half; 14: v_pk_fma op_sel:[0,1,0]); then the
# full AFNO sequence without (1) and with (2) MFMA co-runners again; 2 repeats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  for m in "1 77448 2944 200 11" "1 77448 2944 200 12" "1 77448 2944 200 13" "1 77448 2944 200 14" \
           "1 77448 2944 200 1" "1 77448 2944 200 2" "0 77448 2944 200 2"; do
    timeout -k 10 120 ./diag_libs/opsel_lds_repro3 $m || { echo "repro ended abnormally"; exit 1; }
  done
done
