# Round-6 A/B: attn_dq writing the delta rows straight in the dK/dV grouping's encoding when one dQ
# launch holds every branch (DTA_DQ_KSTARTS=1) against the delta_rebase launch (0): cfg3 N = 3 (the
# 2 + 1 dK/dV groups), cfg2 as a control; then the GPU parity suite on the new default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06t}
mkdir -p $OUT
for sh in 16,6,64,3,2048 8,16,64,2,4096; do
  timeout -k 10 300 python tools/ab_kernels.py ks0=lib/libdiffattn_ks0.so ks1=lib/libdiffattn_ks1.so ks0b=lib/libdiffattn_ks0.so ks1b=lib/libdiffattn_ks1.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_ks0'))"
done
echo R06T_OK
