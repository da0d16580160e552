# Round-5: GPU suite at HEAD (N = 1 paired plans, SEQ forward, fp32 dV across groups), then
# a one-process A/B of the SEQ forward against the branch-split + combine forward (noseq).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -30
tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
for sh in 16,6,64,3,2048 16,6,64,4,2048 8,16,64,6,2048; do
  timeout -k 10 200 python tools/ab_kernels.py base=lib/libdiffattn.so noseq=lib/libdiffattn_noseq.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R05D_OK
