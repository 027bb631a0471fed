#!/bin/bash
# One GPU session of library A/Bs: the split-pipeline kernels per build (tools/lin_ab.sh), config 4
# per build (tools/config4_ab.py), then the GPU tests of the main build.
#   LIBS="main x" C4LIBS="main y" TAG=t bash tools/ab_session.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-abs}; mkdir -p $O
if [ -n "${LIBS:-}" ]; then
  LIBS="$LIBS" BATCHES=${BATCHES:-4096,1024,64,1} TAG=${TAG:-abs} bash tools/lin_ab.sh > $O/lin_ab.txt 2>&1 || { tail -20 $O/lin_ab.txt; exit 1; }
  cat $O/lin_ab.txt
fi
for L in ${C4LIBS:-}; do
  if [ $L = main ]; then LP=$PWD/indy7_mpc_amd/lib/libindy7mpc.so; else LP=$PWD/indy7_mpc_amd/lib/variants/lib$L.so; fi
  I7M_LIB=$LP timeout -k 10 300 python tools/config4_ab.py --steps 3 > $O/c4_$L.json 2> $O/c4_$L.err || { tail -20 $O/c4_$L.err; exit 2; }
  echo "== c4 $L"; python -c "import json,sys; d=json.load(open(sys.argv[1]))['fused']; print(round(d['solves_per_s']), d['ipm_iters_mean'], d['converged'], {k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})" $O/c4_$L.json
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  tail -15 $O/pytest.log
fi
