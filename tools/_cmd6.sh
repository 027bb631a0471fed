set -o pipefail
mkdir -p gpurun_out/w2
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread -k "two_wave or broadcast" > gpurun_out/w2/pytest.log 2>&1 || { tail -30 gpurun_out/w2/pytest.log; exit 1; }
tail -1 gpurun_out/w2/pytest.log
VAR=I7M_RIC_W2 VALUES="0 1 0 1" BATCHES=1,64,256,512,1024 TAG=w2 bash tools/env_ab.sh || exit 2
