#!/bin/bash
# Riccati broadcast / two-wave selection A/B by batch size (tools/env_ab.sh over I7M_RIC_BC and I7M_RIC_W2).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
VAR=I7M_RIC_BC VALUES="2 3 2 3" BATCHES=128,64,1 TAG=bc3 bash tools/env_ab.sh > gpurun_out/bc3.txt 2>&1 || { tail -5 gpurun_out/bc3.txt; exit 1; }
cat gpurun_out/bc3.txt
I7M_RIC_BC=3 VAR=I7M_RIC_W2 VALUES="0 1 0 1" BATCHES=256,128,64,1 TAG=bc4 bash tools/env_ab.sh > gpurun_out/bc4.txt 2>&1 || { tail -5 gpurun_out/bc4.txt; exit 2; }
cat gpurun_out/bc4.txt
