# Round-5 A/B: the XCD group size of the longest-first dispatch (DTA_LPT_GROUP = 2 / 6 / 8
# against the default 4) re-measured on the round-5 kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05zb}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so l2=lib/libdiffattn_l2.so l6=lib/libdiffattn_l6.so l8=lib/libdiffattn_l8.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'])"
done
echo R05ZB_OK
