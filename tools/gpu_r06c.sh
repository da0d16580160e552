# Round-6 A/B: transposed operand reads issued ahead of the softmax VALU -- dK/dV's Q_i^T (tkv),
# dQ's first d-block K_i^T (tq), the single-branch forward's first d-block V^T (tf) -- against
# the same reduced-config build of HEAD, step-interleaved (tools/ab_kernels.py --mode step).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06c}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so tkv=lib/libdiffattn_tkv.so tq=lib/libdiffattn_tq.so tf=lib/libdiffattn_tf.so --shape $sh --rounds 6 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], max(b['rel_diff_vs_base'].values()))"
done
echo R06C_OK
