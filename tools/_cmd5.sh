set -o pipefail
LIBS="main xpad0 main xpad0" BATCHES=4096,64 TAG=xpad bash tools/lin_ab.sh || exit 1
TAG=xpad_pmc bash tools/lds_pmc.sh || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > gpurun_out/xpad/pytest.log 2>&1 || { tail -30 gpurun_out/xpad/pytest.log; exit 3; }
tail -1 gpurun_out/xpad/pytest.log
