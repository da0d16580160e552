# Round-5: the LDS-bounced epilogues in all three attention kernels (HEAD tree) -- the full GPU
# suite, then a one-process A/B against the previous library (lib/libdiffattn_head.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05p}
mkdir -p $OUT
DTA_TEST_LOG_DIR=$OUT timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/tests.log | head; exit 1; fi
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048 4,16,128,2,8192; do
  timeout -k 10 300 python tools/ab_kernels.py old=lib/libdiffattn_head.so new=lib/libdiffattn.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_old'].items()})"
done
echo R05P_OK
