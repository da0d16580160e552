# Round-6 A/B: the XCD group size of the longest-first dispatch (DTA_LPT_GROUP 2 / 4 / 6 / 8)
# re-measured with the NT fp32 stores, step-interleaved, cfg2 and cfg3 N = 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06m}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py g4=lib/libdiffattn_g4.so g2=lib/libdiffattn_g2.so g6=lib/libdiffattn_g6.so g8=lib/libdiffattn_g8.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], max(b['rel_diff_vs_g4'].values()))"
done
echo R06M_OK
