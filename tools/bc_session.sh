#!/bin/bash
# Riccati broadcast / priority selection A/B by batch size (tools/env_ab.sh over I7M_RIC_BC).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
VAR=I7M_RIC_BC VALUES="${VALUES:-3 7 3 7}" BATCHES=${BATCHES:-768,512} TAG=bc5 bash tools/env_ab.sh > gpurun_out/bc5.txt 2>&1 || { tail -5 gpurun_out/bc5.txt; exit 1; }
cat gpurun_out/bc5.txt
