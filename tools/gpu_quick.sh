#!/bin/bash
# Quick GPU check: full GPU test suite, then a short headline bench (no CPU leg, no config 4).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-config4 --steps 20 > gpurun_out/bench_quick.json 2>/dev/null || exit 2
python -c "
import json; d=json.load(open('gpurun_out/bench_quick.json'))
print(round(d['value']), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()}, 'b1', round(d['p50_latency_b1_ms'],4))"
