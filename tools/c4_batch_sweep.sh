set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/c4b; mkdir -p $O
for B in 512 1024 2048 4096; do
  timeout -k 10 300 python tools/config4_ab.py --modes fused --B $B --steps 2 > $O/c4_$B.json 2>$O/c4_$B.err || { tail -5 $O/c4_$B.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1]))['fused']; print(sys.argv[2], round(d['solves_per_s']), round(d['ms_per_step'],2), d['ipm_iters_mean'], {k:round(v['avg_us']) for k,v in d['kernels'].items()})" $O/c4_$B.json $B
done
