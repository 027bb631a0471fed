#!/bin/bash
# A/B on one box: GPU tests on the in-tree library, then B=1 kernel times and the headline
# bench for each library named in LIBS (paths relative to the repo; I7M_LIB selects it).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for L in ${LIBS:-indy7_mpc_amd/lib/libindy7mpc.so}; do
  I7M_LIB=$PWD/$L timeout -k 10 200 python - <<'PY' 2>/dev/null || exit 2
import os, sys
sys.path.insert(0, '.')
from tools.small_batch_ab import run
for B in (1, 64):
    r = run(B, 32, {})
    print(os.environ['I7M_LIB'].split('/')[-1], 'B=%d' % B, r['kernels_us'], 'p50_ms', round(r['p50_ms'], 4))
PY
  I7M_LIB=$PWD/$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-config4 --no-config2 --steps 20 > gpurun_out/b.json 2>/dev/null || exit 3
  python -c "
import json; d=json.load(open('gpurun_out/b.json')); print('  B=4096', round(d['value']), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})"
done
