#!/bin/bash
# Round 4, GPU session 16: FNO column kernels (forward pruned H transform, mixing + inverse H: 160 workgroups of
# 4 columns at 20 channels x 32 modes) as 2-column tiles (MI_DFT_FIXED_CFG=90,2: 320 workgroups) vs default, ABAB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
for r in 1 2; do
  TAILN=2 step r4s16_fno_def_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
  MI_DFT_FIXED_CFG=90,2 TAILN=2 step r4s16_fno_t2_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
  MI_DFT_FIXED_CFG=45,4 TAILN=2 step r4s16_fno_t4h_$r 200 python -u bench/bench_fno.py --amd-only --rounds 5
done
MI_DFT_FIXED_CFG=90,2 TAILN=3 step r4s16_fno_test_t2 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fno.py
# FNO tail setup: phase clocks without the G / rotation table loads (timing-only, variants/bin/fno_stamps_notab)
TAILN=8 step r4s16_stamps 120 ./variants/bin/fno_stamps
TAILN=8 step r4s16_stamps_notab 120 ./variants/bin/fno_stamps_notab
