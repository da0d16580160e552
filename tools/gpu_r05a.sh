# Round-5 first GPU call: the forced-native backward plan tests (ABI 7 group caps), then the
# default bench + per-shape kernel stats at HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05a}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "native" -v --timeout 300 --timeout-method thread > $OUT/native.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $OUT/native.log | sed 's/^tests\/test_gpu_parity.py:://' | head -60
tail -3 $OUT/native.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --train-steps 0 > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
python3 $R/tools/kernel_stats_by_shape.py $OUT/prof/run_kernel_trace.csv $OUT/kernel_stats_by_shape.csv || exit 1
echo R05A_OK
