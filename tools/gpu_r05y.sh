# Round-5: the sequential-branch forward issuing the next branch's Q rows and first ring stages
# before this branch's O_i / LSE stores (spf build) -- the GPU suite on it, then a one-process
# A/B against HEAD at the N >= 3 shapes that run it.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05y}
mkdir -p $OUT
DTA_LIB=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib/libdiffattn_spf.so timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/tests_spf.log 2>&1
rc=$?; tail -3 $OUT/tests_spf.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/tests_spf.log | head; exit 1; fi
for sh in 16,6,64,3,2048 16,6,64,4,2048 8,16,64,6,2048 8,16,64,2,4096; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so spf=lib/libdiffattn_spf.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_head'].items()})"
done
echo R05Y_OK
