# fp32 vs fp16 O_i (ABI 6 obr_dtype): kernel A/B at cfg2, then the full GPU suite and the bench.
# Usage (on the GPU box): bash tools/gpu_obr.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/${1:-r04_obr}; mkdir -p $OUT
for o in f32 f16 f32 f16; do
  timeout -k 10 200 python tools/ab_kernels.py base=lib/libdiffattn.so --obr $o --rounds 3 --reps 8 > $OUT/ab_$o.json 2> $OUT/ab_$o.err || { echo AB_FAILED; tail -5 $OUT/ab_$o.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/ab_$o.json')); print('$o', d['builds']['base']['median_ms'], d['builds']['base']['sum_median_ms'])"
done
DTA_TEST_LOG_DIR=$OUT timeout -k 10 840 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -20
tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
timeout -k 10 400 python bench.py --cpu-baseline off > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, 'train', d.get('train', {}).get('value'))"
