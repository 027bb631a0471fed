#!/bin/bash
# Copy one tools/gpu_round.sh session's summaries from gpurun_out/<TAG> into profiles/ under a
# round prefix and fold its PMC passes into profiles/pmc_traffic.json.
#   TAG=r02x ROUND=r02 bash tools/collect_round.sh
set -euo pipefail
cd "$(dirname "$0")/.."
I=gpurun_out/${TAG:?}; P=profiles; R=${ROUND:?}
cp $I/pytest_gpu.log $P/${R}_pytest_gpu.log
tail -1 $I/bench.json > $P/${R}_bench.json
cp $I/trace/run_kernel_stats.csv $P/${R}_kernel_stats.csv
cp $I/trace_summary.json $P/${R}_kernel_trace_summary.json
cp $I/sq_summary.json $P/${R}_sq_counters.json
cp $I/c4_trace/run_kernel_stats.csv $P/${R}_config4_kernel_stats.csv
cp $I/c4_trace_summary.json $P/${R}_config4_kernel_trace_summary.json
if [ -d $I/fused_trace ]; then
  cp $I/fused_trace/run_kernel_stats.csv $P/${R}_fused_kernel_stats.csv
  cp $I/fused_trace_summary.json $P/${R}_fused_kernel_trace_summary.json
fi
[ -f $I/bench_g2.json ] && tail -1 $I/bench_g2.json > $P/${R}_bench_g2_share.json
python tools/pmc_traffic.py $I/pmc_fetch/fetch_counter_collection.csv $I/pmc_write/write_counter_collection.csv --batch 4096 --N 32 > /dev/null
python tools/pmc_traffic.py $I/c4_fetch/fetch_counter_collection.csv $I/c4_write/write_counter_collection.csv --batch 4096 --N 64 > /dev/null
if [ -d $I/fused_fetch ]; then
  python tools/pmc_traffic.py $I/fused_fetch/fetch_counter_collection.csv $I/fused_write/write_counter_collection.csv --batch 4096 --N 32 > /dev/null
fi
echo collected $I into $P/${R}_*
