set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/r04_v1; mkdir -p $OUT
DTA_TEST_LOG_DIR=$OUT timeout -k 10 840 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -40
tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --cpu-baseline off > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
