# Round-5 A/B: XCD groups of 8 (two groups at 16 pairs per XCD) against 4 at the cfg4 training
# shape (B 16 x H 8, T 2048) and cfg2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05zf}
mkdir -p $OUT
for sh in 16,8,64,2,2048 8,16,64,2,4096; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so l8=lib/libdiffattn_l8.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'])"
done
echo R05ZF_OK
