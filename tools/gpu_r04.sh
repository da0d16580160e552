# Round-4 GPU check: dQ parity first, the dq2 A/B, the full GPU suite, the default bench.
# Usage (on the GPU box): bash tools/gpu_r04.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/${1:-r04}; mkdir -p $OUT
DTA_DQ2=1 DTA_DKDV2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 120 --timeout-method thread -k "core_fwd_bwd or cfg2_full or reproducible" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log
if [ $rc -ne 0 ]; then echo "PARITY_FAILED rc=$rc"; grep -E "FAILED|Error|assert" $OUT/parity.log | head -20; exit 1; fi
if [ -n "$AB" ]; then
  DTA_DQ2=1 DTA_DKDV2=1 timeout -k 10 300 python tools/ab_kernels.py $AB --rounds 5 --reps 8 > $OUT/ab.json 2> $OUT/ab.err || { echo AB_FAILED; tail -20 $OUT/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab.json'))
for n,b in d['builds'].items(): print(n, {k: v for k, v in b.items() if 'ms' in k})"
fi
DTA_DQ2=${DQ2:-1} DTA_DKDV2=${DQ2:-1} DTA_TEST_LOG_DIR=$OUT timeout -k 10 840 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -40
tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
DTA_DQ2=${DQ2:-1} DTA_DKDV2=${DQ2:-1} timeout -k 10 300 python bench.py --cpu-baseline off > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
