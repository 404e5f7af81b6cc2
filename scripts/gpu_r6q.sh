set -u
S=scripts/gpu_step.sh
export MI_DFT_LIB=ab/tune/_C.so
for i in 1 2 3; do
  MI_DFT_FNO_UPW=4 bash $S r6q_u4_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_FNO_UPW=2 bash $S r6q_u2_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_FNO_UPW=1 MI_DFT_FNO_WGS=512 bash $S r6q_u1w512_$i 200 python bench/fno_probe.py || exit $?
  MI_DFT_FNO_UPW=1 MI_DFT_FNO_WGS=256 bash $S r6q_u1w256_$i 200 python bench/fno_probe.py || exit $?
done
