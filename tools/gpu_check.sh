# GPU check: parity tests, then the default bench, then a rocprofv3 kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---cpu-baseline off} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 10 --warmup 2 > $R/gpurun_out/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof.log; exit 1; }
  head -8 $R/gpurun_out/prof/run_kernel_stats.csv | cut -c1-160
fi
