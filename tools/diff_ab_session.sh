#!/bin/bash
# One GPU session: bitwise tools/lib_diff.py of each variant in DIFFS against the reference variant
# REF, the split-pipeline A/B of LIBS (tools/lin_ab.sh), an environment A/B (VAR over VALUES,
# tools/env_ab.sh), config-4 A/B of C4LIBS, then the GPU tests.
#   REF=x DIFFS="main y" LIBS="x main" VAR=I7M_RIC_BC VALUES="7 15" C4LIBS="main z" TAG=t bash tools/diff_ab_session.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-dab}; mkdir -p $O
lp() { if [ $1 = main ]; then echo $PWD/indy7_mpc_amd/lib/libindy7mpc.so; else echo $PWD/indy7_mpc_amd/lib/variants/lib$1.so; fi; }
for L in ${REF:?} ${DIFFS:-}; do
  I7M_LIB=$(lp $L) timeout -k 10 300 python tools/lib_diff.py dump $O/d_$L.npz >> $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 3; }
done
for L in ${DIFFS:-}; do echo "== lib_diff $REF vs $L"; python tools/lib_diff.py cmp $O/d_$REF.npz $O/d_$L.npz | tee $O/lib_diff_$L.txt; done
if [ -n "${LIBS:-}" ]; then
  LIBS="$LIBS" BATCHES=${BATCHES:-4096,1024,64,1} TAG=${TAG:-dab} bash tools/lin_ab.sh > $O/lin_ab.txt 2>&1 || { tail -20 $O/lin_ab.txt; exit 4; }
  cat $O/lin_ab.txt
fi
if [ -n "${VAR:-}" ]; then
  VAR=$VAR VALUES="$VALUES" BATCHES=${BATCHES:-4096,2048,1024} TAG=${TAG:-dab} bash tools/env_ab.sh > $O/env_ab.txt 2>&1 || { tail -20 $O/env_ab.txt; exit 5; }
  cat $O/env_ab.txt
fi
for L in ${C4LIBS:-}; do
  I7M_LIB=$(lp $L) timeout -k 10 300 python tools/config4_ab.py --steps 3 > $O/c4_$L.json 2> $O/c4_$L.err || { tail -20 $O/c4_$L.err; exit 2; }
  echo "== c4 $L"; python -c "import json,sys; d=json.load(open(sys.argv[1]))['fused']; print(round(d['solves_per_s']), d['ipm_iters_mean'], d['converged'], {k: round(v['avg_us'], 1) for k, v in d['kernels'].items()})" $O/c4_$L.json
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  tail -15 $O/pytest.log
fi
