#!/bin/bash
# GPU session 29 (round 3): radix-order A/B for rfft2/irfft2 720x1440 (MI_DFT_FFT_RADICES): default (1440 rows 5,6,6,8;
# 720 columns 8,9,10), columns 10,9,8 / 9,10,8, rows 8,6,6,5 -- DFT GPU tests under each, then bench_fft, 2 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "def:" "c1:720:10,9,8" "c2:720:9,10,8" "r1:1440:8,6,6,5"; do
  t=${v%%:*}; r=${v#*:}
  MI_DFT_FFT_RADICES="$r" timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_dft_gpu.py \
    > gpurun_out/s29_t_$t.log 2>&1 || { echo "tests $t failed"; tail -5 gpurun_out/s29_t_$t.log; exit 1; }
  echo "== $t tests: $(tail -1 gpurun_out/s29_t_$t.log)"
done
for rep in 1 2; do
  for v in "def:" "c1:720:10,9,8" "c2:720:9,10,8" "r1:1440:8,6,6,5"; do
    t=${v%%:*}; r=${v#*:}
    MI_DFT_FFT_RADICES="$r" timeout -k 10 300 python -u bench/bench_fft.py --rounds 10 > gpurun_out/s29_${t}_$rep.log 2>&1 || { echo "bench $t failed"; exit 1; }
    python3 -c "
import json
t=open('gpurun_out/s29_${t}_$rep.log').read(); j=json.loads(t[t.index('{'):t.rindex('}')+1])
print('$t rep $rep rfft2 %.2f irfft2 %.2f'%(j['amd_rfft2']['graph']['median_us'], j['amd_irfft2']['graph']['median_us']))"
  done
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s29_smoke.log 2>&1 || { tail -5 gpurun_out/s29_smoke.log; exit 1; }
tail -1 gpurun_out/s29_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s29_bench.log 2>&1 || { tail -5 gpurun_out/s29_bench.log; exit 1; }
tail -1 gpurun_out/s29_bench.log
