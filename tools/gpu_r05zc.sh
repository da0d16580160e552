# Round-5 A/B: two equal XCD groups between 8 and 16 pairs per XCD (lh build, DTA_LPT_HALVES)
# against HEAD (groups of 4), then the GPU suite on it.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05zc}
mkdir -p $OUT
for sh in 16,6,64,3,2048 16,6,64,4,2048 8,16,64,2,4096 1,16,128,2,32768; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so lh=lib/libdiffattn_lh.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'], {k: round(v, 6) for k, v in b['rel_diff_vs_head'].items()})"
done
echo R05ZC_OK
