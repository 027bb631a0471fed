set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c4prof; mkdir -p $O; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 5; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/sq -o sq -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 6; }
echo done
