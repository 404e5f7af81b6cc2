set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for v in base occ4 bpf1; do
  if [ $v = base ]; then unset MI_DFT_LIB; else export MI_DFT_LIB=$PWD/ab/_C_$v.so; fi
  echo "== $v spec r$r"; timeout -k 10 120 python -u bench/bench_afno_spec.py
done; done
for v in base occ4 bpf1; do
  if [ $v = base ]; then unset MI_DFT_LIB; else export MI_DFT_LIB=$PWD/ab/_C_$v.so; fi
  echo "== $v bench"; timeout -k 10 300 python -u bench.py --no-fft | grep metric
done
