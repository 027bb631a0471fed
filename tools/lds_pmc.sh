#!/bin/bash
# LDS / MFMA counters of the config-3 kernels: rocprofv3 --list-avail, then one --pmc pass with the
# wanted counters this device has (at most 8 SQ).   TAG=x bash tools/lds_pmc.sh
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-ldspmc}; mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
WANT="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
HAVE=""; n=0
for c in $WANT; do
  if grep -qw "$c" $O/avail.txt && [ $n -lt 8 ]; then HAVE="$HAVE $c"; n=$((n+1)); fi
done
echo "counters:$HAVE"
[ -n "$HAVE" ] || exit 1
timeout -s KILL 90 rocprofv3 --pmc $HAVE --output-format csv -d $O/pmc -o lds -- python $R/tools/profile_kernels.py --steps 2 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 2; }
python - $O/pmc/lds_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", r.get("Kernel-Name", ""))
    for key in ("k_linearize", "k_riccati", "k_linesearch"):
        if key in k:
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[(key, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
