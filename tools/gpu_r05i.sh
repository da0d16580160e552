# Round-5 A/B: the bf16 attention unit built without -fno-slp-vectorize (packed fp32 VALU) against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05i}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 240 python tools/ab_kernels.py head=lib/libdiffattn.so slp=lib/libdiffattn_slp.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R05I_OK
