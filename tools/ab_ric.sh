set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-config4 --steps 20 > gpurun_out/bench_new.json 2>/dev/null || exit 2
I7M_ABLATE=8 timeout -k 10 120 python bench.py --no-cpu-baseline --no-config4 --steps 20 > gpurun_out/bench_old.json 2>/dev/null || exit 3
python - <<'PY'
import json
for f in ("new","old"):
    d=json.load(open(f"gpurun_out/bench_{f}.json"))
    print(f, round(d["value"]), {k:round(v["avg_us"],1) for k,v in d["kernels"].items()})
PY
