set -u
S=scripts/gpu_step.sh
export MI_DFT_LIB=ab/tune/_C.so
for u in 1 2 4 8 16; do
  MI_DFT_FNO_UPW=$u bash $S r6n_upw$u 200 python bench/fno_probe.py || exit $?
done
for w in 256 384 512; do
  MI_DFT_FNO_UPW=1 MI_DFT_FNO_WGS=$w bash $S r6n_wgs$w 200 python bench/fno_probe.py || exit $?
done
