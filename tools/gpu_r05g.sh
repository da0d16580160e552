# Round-5 A/B of the paired 32-key dQ plan for N = 3 at head size 64 (variant p3 =
# -DDTA_DQ_PAIR3=1) against HEAD; parity of the variant first (DTA_LIB).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05g}
mkdir -p $OUT
DTA_LIB=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib/libdiffattn_p3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropout.py -m gpu -q -k "3-64 or 3-32 or cfg3 or N3 or ndiff or large_logits or growth" --timeout 120 --timeout-method thread > $OUT/tests_p3.log 2>&1
rc=$?; tail -3 $OUT/tests_p3.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/tests_p3.log | head; exit 1; fi
for sh in 16,6,64,3,2048 8,16,64,3,4096; do
  timeout -k 10 200 python tools/ab_kernels.py head=lib/libdiffattn.so p3=lib/libdiffattn_p3.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R05G_OK
