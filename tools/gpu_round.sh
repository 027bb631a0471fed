#!/bin/bash
# One GPU-box session: tests, bench, rocprof kernel trace, PMC passes. Every GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-run}
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
cat $O/bench.json
cd /tmp
# the bench command itself under the kernel tracer (no CPU leg / config 4, to keep it short)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py --no-cpu-baseline --no-config4 --no-config2 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 3; }
python $R/tools/trace_summary.py $O/trace/run_kernel_trace.csv --batch 4096 > $O/trace_summary.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python $R/tools/profile_kernels.py --steps 4 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python $R/tools/profile_kernels.py --steps 4 > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 5; }
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_sq -o sq -- python $R/tools/profile_kernels.py --steps 2 > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 6; }
python $R/tools/sq_summary.py $O/pmc_sq/sq_counter_collection.csv > $O/sq_summary.json
ls -R $O | head -40
