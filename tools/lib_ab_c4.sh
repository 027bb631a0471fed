#!/bin/bash
# A/B of library builds on config 4 (B = 4096, N = 64, k_ipm_fused): LIBS="main head" TAG=x bash tools/lib_ab_c4.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG:-c4ab}; mkdir -p $O
for L in ${LIBS:-main}; do
  if [ $L = main ]; then LP=$PWD/indy7_mpc_amd/lib/libindy7mpc.so; else LP=$PWD/indy7_mpc_amd/lib/variants/lib$L.so; fi
  I7M_LIB=$LP timeout -k 10 300 python tools/config4_ab.py --modes fused --B ${B:-4096} --steps 2 > $O/c4_$L.json 2>$O/c4_$L.err || { tail -5 $O/c4_$L.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1]))['fused']; print(sys.argv[2], round(d['solves_per_s']), round(d['ms_per_step'],2), d['ipm_iters_mean'], {k:round(v['avg_us']) for k,v in d['kernels'].items()})" $O/c4_$L.json $L
done
