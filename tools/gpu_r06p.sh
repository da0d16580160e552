# Round-6 A/B: the softmax / dS arithmetic of the three attention kernels as packed fp32 pairs
# (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32; DTA_FWD_PK, DTA_DQ_PK, DTA_DKDV_PK; second call: the forward only) against the
# scalar form, step-interleaved, cfg2 and cfg3 N = 3; outputs compared (bitwise equal expected).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06p}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so fpk=lib/libdiffattn_fpk.so base2=lib/libdiffattn_base.so fpk2=lib/libdiffattn_fpk.so base3=lib/libdiffattn_base.so fpk3=lib/libdiffattn_fpk.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R06P_OK
