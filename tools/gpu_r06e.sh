# Round-6 A/B: dK/dV with |c_i| folded into its probabilities through the lse_c seeds (cfold:
# 139 -> 123 VALU per step at cfg2), and cfold + the seeded forward (both), against the same
# reduced-config build with the fold compiled out (base0), step-interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06e}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base0=lib/libdiffattn_base0.so cfold=lib/libdiffattn_cfold.so both=lib/libdiffattn_both.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], {k: round(v, 5) for k, v in b['rel_diff_vs_base0'].items()})"
done
echo R06E_OK
