set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/s2; mkdir -p $O
for p in 2 3 2 3; do
  I7M_H2H_PIPE=$p timeout -k 10 300 python tools/h2h_ab.py --chunks 1,2,3,4,6 --reps 20 >> $O/h2h_ab.jsonl 2>> $O/h2h.err || { tail -20 $O/h2h.err; exit 1; }
done
I7M_H2H_PIPE=3 timeout -k 10 300 python tools/h2h_ab.py --chunks 2,3,4 --reps 20 --pinned >> $O/h2h_ab.jsonl 2>> $O/h2h.err || { tail -20 $O/h2h.err; exit 2; }
I7M_LIB=$PWD/indy7_mpc_amd/lib/variants/libbase.so timeout -k 10 300 python tools/lib_diff.py dump $O/base.npz > $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 3; }
timeout -k 10 300 python tools/lib_diff.py dump $O/main.npz >> $O/diff.log 2>&1 || { tail -20 $O/diff.log; exit 4; }
python tools/lib_diff.py cmp $O/base.npz $O/main.npz > $O/lib_diff.txt 2>&1
cat $O/lib_diff.txt
python -c "import json,sys; [print(d['pipe'], d['pinned'], d['h2h_chunks'], round(d['median_ms'],3), round(d['host_to_host_solves_per_s']/1e6,3), d['bit_identical_to_first']) for d in map(json.loads, open(sys.argv[1]))]" $O/h2h_ab.jsonl
