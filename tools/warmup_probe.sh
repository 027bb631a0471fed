#!/bin/bash
# Short-run vs steady-state bench on one box: the driver's --steps 20 --warmup 5 against a longer
# warm-up and a longer timed region (value only; the extras off).  profiles/r03_warmup_probe.txt
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/warm; mkdir -p $O
for a in "20 5" "20 100" "100 5" "20 5"; do
  set -- $a
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-config4 --no-config2 > $O/b_$1_$2.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],4))" $O/b_$1_$2.json $1 $2
done
