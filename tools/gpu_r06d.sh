# Round-6 A/B: forward with Q pre-scaled and the S accumulators seeded with -m by one MFMA on
# the fixed-reference tiles (fseed: 191 -> 127 VALU per 64-key tile at cfg2), against the same
# reduced-config build of HEAD, step-interleaved; outputs compared with base.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06d}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so fseed=lib/libdiffattn_fseed.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b['rel_diff_vs_base'])"
done
echo R06D_OK
