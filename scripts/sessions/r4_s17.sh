#!/bin/bash
# Round 4, GPU session 17: FNO tail setup -- phase clocks with and without the G / rotation table loads
# (timing-only variants/bin/fno_stamps_notab: what computing the tables on the device could save at most).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
for r in 1 2; do
  TAILN=16 step r4s17_stamps_$r 120 ./variants/bin/fno_stamps
  TAILN=16 step r4s17_stamps_notab_$r 120 ./variants/bin/fno_stamps_notab
done
