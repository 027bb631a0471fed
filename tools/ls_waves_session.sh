#!/bin/bash
# Line-search waves per problem (I7M_LS_WAVES 1 | 4) by batch size (tools/env_ab.sh).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
VAR=I7M_LS_WAVES VALUES="1 4 1 4" BATCHES=${BATCHES:-1024,768,512,384} TAG=lsw bash tools/env_ab.sh > gpurun_out/lsw.txt 2>&1 || { tail -5 gpurun_out/lsw.txt; exit 1; }
cat gpurun_out/lsw.txt
