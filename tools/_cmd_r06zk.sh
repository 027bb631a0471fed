#!/bin/bash
# round 6 session zk: SQ counters of the final ADMM kernels: config 3 (B = 4096, staggered ranges,
# k_admm_iter), B = 64 and B = 1 (k_admm_iter_res); plus FETCH/WRITE at B = 64.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zk; mkdir -p $O
cd /tmp
run() {  # name B counters...
  n=$1; B=$2; shift 2
  timeout -k 10 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o $n -- python $R/tools/admm_ab.py --B $B --chunks 0 --steps 1 > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 4; }
}
for B in 4096 64 1; do
  run p1_$B $B SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
  run p2_$B $B SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
  python $R/tools/pmc_admm.py $(ls $O/p1_$B/*counter_collection.csv) $(ls $O/p2_$B/*counter_collection.csv) > $O/pmc_$B.json
done
run p3_64 64 FETCH_SIZE
run p4_64 64 WRITE_SIZE
python -c "
import json
for B in (4096, 64, 1):
  d=json.load(open('$O/pmc_%d.json' % B))
  for k in d:
    if 'admm' in k: print(B, k, json.dumps({'per_wave': d[k]['per_wave'], 'frac': d[k]['frac_of_wave_cycles']}))
"
