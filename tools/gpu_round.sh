#!/bin/bash
# One GPU-box session: tests, bench, rocprof kernel trace + PMC passes of the headline (config 3)
# and of config 4.  Every GPU step has its own time limit; the chain stops at the first failure.
#   TAG=r02 [STEPS=tests,bench,trace,pmc,c4,fused] bash tools/gpu_round.sh
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-run}
STEPS=${STEPS:-tests,bench,multi,trace,pmc,c4,fused}
mkdir -p $O
cd $R
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
if has bench; then
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
  cat $O/bench.json
fi
if has multi; then
  # bench.py --gpus 2 starting its own ranks, both on the one GPU (--share-devices rehearsal)
  timeout -k 10 300 python bench.py --gpus 2 --share-devices --steps 20 > $O/bench_g2.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 13; }
  cat $O/bench_g2.json
fi
cd /tmp
if has trace; then
  # the bench's own GPU work under the kernel tracer (no CPU leg / extras, to keep it short)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py --no-cpu-baseline --no-config4 --no-config2 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 3; }
  python $R/tools/trace_summary.py $O/trace/run_kernel_trace.csv --batch 4096 > $O/trace_summary.json
fi
if has pmc; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python $R/tools/profile_kernels.py --steps 4 > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 4; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python $R/tools/profile_kernels.py --steps 4 > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 5; }
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_sq -o sq -- python $R/tools/profile_kernels.py --steps 2 > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 6; }
  python $R/tools/sq_summary.py $O/pmc_sq/sq_counter_collection.csv > $O/sq_summary.json
fi
if has admm; then
  # config 3 in ADMM mode (B = 4096, N = 32, cold OSQP state per solve): trace + FETCH / WRITE of k_admm
  # per kernel over the whole batch (one range: I7M_ADMM_STAGGER=0), then the default schedule's
  # trace (two staggered ranges of 2048)
  export I7M_ADMM_STAGGER=0
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/admm_trace -o run -- python $R/tools/profile_kernels.py --admm --steps 2 --warmup 1 > $O/admm_trace.log 2>&1 || { tail -20 $O/admm_trace.log; exit 14; }
  python $R/tools/trace_summary.py $O/admm_trace/run_kernel_trace.csv --batch 4096 --N 32 > $O/admm_trace_summary.json
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/admm_fetch -o fetch -- python $R/tools/profile_kernels.py --admm --steps 1 --warmup 1 > $O/admm_fetch.log 2>&1 || { tail -20 $O/admm_fetch.log; exit 15; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/admm_write -o write -- python $R/tools/profile_kernels.py --admm --steps 1 --warmup 1 > $O/admm_write.log 2>&1 || { tail -20 $O/admm_write.log; exit 16; }
  unset I7M_ADMM_STAGGER
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/admm_trace_st -o run -- python $R/tools/profile_kernels.py --admm --steps 2 --warmup 1 > $O/admm_trace_st.log 2>&1 || { tail -20 $O/admm_trace_st.log; exit 17; }
  python $R/tools/trace_summary.py $O/admm_trace_st/run_kernel_trace.csv --batch 2048 --N 32 > $O/admm_trace_st_summary.json
fi
if has c4; then
  # config 4 (B = 4096, N = 64, box rows): trace + FETCH / WRITE of k_ipm_fused
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_trace -o run -- python $R/tools/profile_kernels.py --box --N 64 --steps 2 --warmup 1 > $O/c4_trace.log 2>&1 || { tail -20 $O/c4_trace.log; exit 7; }
  python $R/tools/trace_summary.py $O/c4_trace/run_kernel_trace.csv --batch 4096 --N 64 > $O/c4_trace_summary.json
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch -o fetch -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/c4_fetch.log 2>&1 || { tail -20 $O/c4_fetch.log; exit 8; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4_write -o write -- python $R/tools/profile_kernels.py --box --N 64 --steps 1 --warmup 1 > $O/c4_write.log 2>&1 || { tail -20 $O/c4_write.log; exit 9; }
fi
if has fused; then
  # the fused pipeline (k_sqp_fused, one launch per solve) at the bench shape: trace + FETCH / WRITE
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fused_trace -o run -- python $R/tools/profile_kernels.py --pipeline fused --steps 4 > $O/fused_trace.log 2>&1 || { tail -20 $O/fused_trace.log; exit 10; }
  python $R/tools/trace_summary.py $O/fused_trace/run_kernel_trace.csv --batch 4096 > $O/fused_trace_summary.json
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fused_fetch -o fetch -- python $R/tools/profile_kernels.py --pipeline fused --steps 2 > $O/fused_fetch.log 2>&1 || { tail -20 $O/fused_fetch.log; exit 11; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/fused_write -o write -- python $R/tools/profile_kernels.py --pipeline fused --steps 2 > $O/fused_write.log 2>&1 || { tail -20 $O/fused_write.log; exit 12; }
fi
ls -R $O | head -60
