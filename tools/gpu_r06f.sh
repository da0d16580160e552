# Round-6 validation of the new defaults (seeded forward, |c_i|-folded dK/dV through lse_c,
# no PRE memset): the whole GPU suite, smoke, then the bench line (with the 1-rank RCCL
# hook leg of the cfg4 train step).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06f}
mkdir -p $OUT
DTA_TEST_LOG_DIR=$OUT timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -30
tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print(d['ms_per_step'], d['value'], d['kernels'])
print('train', d.get('train', {}).get('value'), d.get('train', {}).get('rccl_hooks_world1'))
print({k: v['core']['ms_per_step'] for k, v in d.get('configs', {}).items() if 'core' in v})"
echo R06F_OK
