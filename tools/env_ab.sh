#!/bin/bash
# A/B of one environment switch over its values, on the split pipeline (tools/pipeline_ab.py):
#   VAR=I7M_RIC_BC VALUES="0 3" BATCHES=4096,256,1 TAG=x bash tools/env_ab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-envab}; mkdir -p $O
for v in ${VALUES:?}; do
  env ${VAR:?}=$v timeout -k 10 300 python tools/pipeline_ab.py --modes split --batches ${BATCHES:-4096,2048,1024,256,64,1} --steps 30 > $O/ab_$v.jsonl 2>$O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 2; }
  echo "== $VAR=$v"; python -c "import sys,json; [print(d['B'], round(d['solves_per_s']), round(d['p50_h2h_ms'],4), d['kernels_us']) for d in map(json.loads, open(sys.argv[1]))]" $O/ab_$v.jsonl
done
