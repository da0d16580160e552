# Round-6: head sizes above 128 (the 16-bit head-size-256 plans) and the padded / group paths, then
# A/B of non-temporal bounced stores (nt1: fp32 O_i and dV sums, nt2: all) against base.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06i}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 240 --timeout-method thread \
  "tests/test_gpu_parity.py::test_core_large_head_sizes" "tests/test_gpu_parity.py::test_core_fwd_bwd" \
  tests/test_gpu_generality.py > $OUT/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -30
tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so nt1=lib/libdiffattn_nt1.so nt2=lib/libdiffattn_nt2.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], max(b['rel_diff_vs_base'].values()))"
done
echo R06I_OK
