# Round-6 A/B: attn_dq's fp32 O_i reads non-temporal (ntl) on top of the NT bounced fp32 stores
# (base = the new default), against the old plain stores (nt0); step-interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06j}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py nt0=lib/libdiffattn_nt0.so base=lib/libdiffattn_base.so ntl=lib/libdiffattn_ntl.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], max(b['rel_diff_vs_nt0'].values()))"
done
echo R06J_OK
