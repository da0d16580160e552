# Round-5 epilogue-store experiments at cfg2 (and cfg3 N = 3 for the bounce):
#   bnc  = forward epilogue through an LDS bounce (whole-row store instructions), parity first
#   epi  = no output stores in any attention kernel, noob = no O_i stores (-DDTA_EPI_SKIP=1 / 2;
#          wrong results, timing only), nt = non-temporal epilogue stores (-DDTA_ATTN_NT=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05o}
mkdir -p $OUT
DTA_LIB=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib/libdiffattn_bnc.so timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/tests_bnc.log 2>&1
rc=$?; tail -3 $OUT/tests_bnc.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/tests_bnc.log | head; exit 1; fi
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so bnc=lib/libdiffattn_bnc.so epi=lib/libdiffattn_epi.so nt=lib/libdiffattn_nt.so noob=lib/libdiffattn_noob.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_head'].items()})"
done
echo R05O_OK
