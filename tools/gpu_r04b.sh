# Round-4 GPU check of the one-wave-per-SIMD kernels (attn_fwd3 / attn_dq2 / attn_dkdv2):
# parity with all three on, the A/B of builds in one process, SQ counters of the new kernels.
# Usage (on the GPU box): AB="base=lib/libdiffattn.so old=..." bash tools/gpu_r04b.sh <tag> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; OUT=gpurun_out/${1:-r04b}; mkdir -p $OUT
export DTA_FWD3=${FWD3:-1} DTA_DQ2=${DQ2:-1} DTA_DKDV2=${DKDV2:-1}
K=${2:-"core_fwd_bwd or cfg2_full or reproducible or padded_head or cfg5_control or forward_max_growth or large_logits"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_generality.py -v -x --timeout 120 --timeout-method thread -k "$K" > $OUT/parity.log 2>&1
rc=$?; tail -3 $OUT/parity.log
if [ $rc -ne 0 ]; then echo "PARITY_FAILED rc=$rc"; grep -E "FAILED|Error|assert" $OUT/parity.log | head -20; exit 1; fi
if [ -n "$AB" ]; then
  timeout -k 10 300 python tools/ab_kernels.py $AB --rounds 5 --reps 8 > $OUT/ab.json 2> $OUT/ab.err || { echo AB_FAILED; tail -20 $OUT/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab.json'))
for n,b in d['builds'].items(): print(n, {k: v for k, v in b.items() if 'ms' in k or 'diff' in k})"
fi
if [ -n "$SQ" ]; then
  mkdir -p $R/$OUT/sq; cd /tmp && export TMPDIR=/tmp
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/$OUT/sq/p$i -o run -- python3 $R/tools/ab_kernels.py base=lib/libdiffattn.so --rounds 1 --reps 2 > $R/$OUT/sq/p$i.log 2>&1 || { echo "PMC group $i failed"; tail -3 $R/$OUT/sq/p$i.log; exit 1; }
  done
  python3 $R/tools/pmc_sq.py $R/$OUT/sq/p* --json $R/$OUT/sq.json > $R/$OUT/sq.txt && tail -40 $R/$OUT/sq.txt
  cd $R
fi
if [ -n "$LNAB" ]; then
  cd $R && timeout -k 10 200 python tools/ab_ln.py $LNAB > $OUT/ab_ln.json 2> $OUT/ab_ln.err || { echo LNAB_FAILED; tail -5 $OUT/ab_ln.err; exit 1; }
  cat $OUT/ab_ln.json
fi
if [ -n "$FULL" ]; then
  cd $R && DTA_TEST_LOG_DIR=$OUT timeout -k 10 840 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/tests.log | head -20
  tail -2 $OUT/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
  timeout -k 10 400 python bench.py --cpu-baseline off > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, 'train', d.get('train', {}).get('value'), 'hbm', {k: v.get('GBps') for k, v in d.get('hbm_kernels', {}).items()})"
fi
if [ -n "$LNPROF" ]; then
  mkdir -p $R/$OUT/lnprof; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$OUT/lnprof -o run -- python3 $R/tools/ab_ln.py base=lib/libdiffattn.so > $R/$OUT/lnprof/log.txt 2>&1 || { echo LNPROF_FAILED; tail -5 $R/$OUT/lnprof/log.txt; exit 1; }
  cd $R; f=$(find $OUT/lnprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 $f | head -12
fi
if [ -n "$CFG3AB" ]; then
  cd $R
  for v in 0 1; do DTA_FWD3=$v timeout -k 10 200 python tools/ab_kernels.py base=lib/libdiffattn.so --shape 16,6,64,3,2048 --rounds 3 --reps 6 > $OUT/cfg3_fwd3_$v.json 2>/dev/null || { echo CFG3AB_FAILED; exit 1; }; done
  python3 -c "
import json
for v in (0, 1): print('cfg3 N=3 DTA_FWD3', v, json.load(open('$OUT/cfg3_fwd3_%d.json' % v))['builds']['base']['median_ms'])"
fi
