set -o pipefail
TAG=r02g bash tools/gpu_round.sh > gpurun_out/r02g.log 2>&1 || { tail -30 gpurun_out/r02g.log; exit 1; }
tail -3 gpurun_out/r02g/pytest_gpu.log
L=$PWD/indy7_mpc_amd/lib/libindy7mpc_diag.so
for B in 4096 64; do
I7M_LIB=$L timeout -k 10 200 python tools/timeline.py --B $B > gpurun_out/r02g/tl_$B.json 2> gpurun_out/r02g/tl_$B.err || { tail -20 gpurun_out/r02g/tl_$B.err; exit 2; }
grep kernel gpurun_out/r02g/tl_$B.err
done
I7M_LIB=$L timeout -k 10 200 python tools/timeline.py --B 4096 --N 64 --box > gpurun_out/r02g/tl_c4.json 2> gpurun_out/r02g/tl_c4.err || { tail -20 gpurun_out/r02g/tl_c4.err; exit 3; }
grep kernel gpurun_out/r02g/tl_c4.err
