# Round-5 A/B of the N = 1 paired plan (DTA_PAIR_N1=1 variant vs base) on the shapes it touches:
# cfg3's branch-split forward (N = 3 / 4) and the control model (N = 1, dv = hs, cfg5).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
for sh in 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 200 python tools/ab_kernels.py base=lib/libdiffattn.so n1=lib/libdiffattn_n1.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
for sh in 1,32,128,1,32768 4,16,64,1,4096; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn.so n1=lib/libdiffattn_n1.so --shape $sh --dv $(echo $sh | cut -d, -f3) --rounds 3 --reps 3 > $OUT/ab_c$sh.json 2> $OUT/ab_c$sh.err || { echo "AB c$sh FAILED"; tail -5 $OUT/ab_c$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_c$sh.json'))
for n,b in d['builds'].items(): print('control $sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R05C_OK
