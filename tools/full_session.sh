#!/bin/bash
# One GPU session at the end of a change: GPU tests, bitwise lib_diff of variant $DIFF against the
# main build, the split-pipeline A/B of LIBS, then tools/gpu_round.sh's bench / profile steps.
#   DIFF=x LIBS="x main" TAG=r03c STEPS=bench,multi,trace,pmc,c4 bash tools/full_session.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
if [ -n "${DIFF:-}" ]; then
  I7M_LIB=$PWD/indy7_mpc_amd/lib/variants/lib$DIFF.so timeout -k 10 300 python tools/lib_diff.py dump $O/$DIFF.npz > $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 3; }
  timeout -k 10 300 python tools/lib_diff.py dump $O/main.npz >> $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 4; }
  python tools/lib_diff.py cmp $O/$DIFF.npz $O/main.npz | tee $O/lib_diff.txt
fi
if [ -n "${LIBS:-}" ]; then
  LIBS="$LIBS" BATCHES=${BATCHES:-4096,1024,64,1} TAG=${TAG:-full} bash tools/lin_ab.sh > $O/lin_ab.txt 2>&1 || { tail -20 $O/lin_ab.txt; exit 5; }
  cat $O/lin_ab.txt
fi
TAG=${TAG:-full} STEPS=${STEPS:-bench,multi,trace,pmc,c4} bash tools/gpu_round.sh > $O/round.txt 2>&1 || { tail -30 $O/round.txt; exit 6; }
head -c 1500 $O/bench.json
