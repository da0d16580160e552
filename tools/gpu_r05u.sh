# Round-5 A/B: the dQ softmax with its exps issued in groups of 4 / 2 ahead of their products
# (g4 / g2 = -DDTA_DQ_EXPG=4 / 2; the trans-use hazard puts an s_nop behind every exp used at once).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05u}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so g4=lib/libdiffattn_g4.so g2=lib/libdiffattn_g2.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_head'].items()})"
done
echo R05U_OK
