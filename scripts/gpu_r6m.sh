set -u
S=scripts/gpu_step.sh
for i in 1 2 3; do
  bash $S r6m_probe_$i 200 python -c "import importlib.util as u, json; s = u.spec_from_file_location('benchmain', 'bench.py'); m = u.module_from_spec(s); s.loader.exec_module(m); m.tdp.load_plugins(); print(json.dumps(m.time_fno_block_us()))" || exit $?
done
