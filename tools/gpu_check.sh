set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --steps 10 --warmup 2 > $R/gpurun_out/prof1.log 2>&1 || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof1.log; exit 1; }
find $R/gpurun_out/prof1 -name "*stats*"
