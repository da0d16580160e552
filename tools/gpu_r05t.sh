# Round-5: the forward with paired query blocks (workgroup r runs blocks 2R-1-r and r; pb build)
# -- the full GPU suite on it, then a one-process A/B against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05t}
mkdir -p $OUT
DTA_LIB=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib/libdiffattn_pb.so timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 240 --timeout-method thread > $OUT/tests_pb.log 2>&1
rc=$?; tail -3 $OUT/tests_pb.log
if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/tests_pb.log | head; exit 1; fi
for sh in 8,16,64,2,4096 4,16,128,2,8192 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn_head.so pb=lib/libdiffattn_pb.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_head'].items()})"
done
echo R05T_OK
