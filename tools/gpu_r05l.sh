# Round-5 A/B of the backward branch-group caps at cfg3 (one library, ABI 7 caps per build name):
# N = 4 dQ native (the paired 32-key plan) vs groups of 2; N = 3 / 4 dK/dV native vs groups of 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05l}
mkdir -p $OUT
L=lib/libdiffattn.so
for sh in 16,6,64,4,2048 16,6,64,3,2048 8,16,64,4,4096; do
  timeout -k 10 240 python tools/ab_kernels.py def=$L q4=$L@4,0 k4=$L@0,4 --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], {k: round(v, 5) for k, v in b['rel_diff_vs_def'].items()})"
done
echo R05L_OK
