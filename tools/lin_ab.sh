#!/bin/bash
# A/B of library builds (indy7_mpc_amd/lib/variants/lib<NAME>.so, python __graft_entry__.py variant
# ...): per build, the linearisation/solver parity tests (TESTS=1) and tools/pipeline_ab.py
# (split pipeline) at several batch sizes.   LIBS="main head x" TAG=lin1 bash tools/lin_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for L in ${LIBS:-main}; do
  if [ $L = main ]; then LP=$PWD/indy7_mpc_amd/lib/libindy7mpc.so; else LP=$PWD/indy7_mpc_amd/lib/variants/lib$L.so; fi
  if [ "${TESTS:-0}" = 1 ]; then
    I7M_LIB=$LP timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_solver.py tests/test_gpu_wrench.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$L.log 2>&1 || { tail -30 $O/pytest_$L.log; exit 1; }
    echo "== $L tests: $(tail -1 $O/pytest_$L.log)"
  fi
  I7M_LIB=$LP timeout -k 10 300 python tools/pipeline_ab.py --modes split --batches ${BATCHES:-4096,256,64,1} --steps 30 > $O/ab_$L.jsonl 2>$O/ab_$L.err || { tail -5 $O/ab_$L.err; exit 2; }
  echo "== $L"; python -c "import sys,json; [print(d['B'], round(d['solves_per_s']), round(d['p50_h2h_ms'],4), d['kernels_us']) for d in map(json.loads, open(sys.argv[1]))]" $O/ab_$L.jsonl
done
