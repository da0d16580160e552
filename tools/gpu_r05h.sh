# Round-5 A/B at cfg2 and cfg3 of two tile-size variants against HEAD:
#   b32dq  = -DDTA_DQ_B32_N2=1  (paired N = 2 dQ with 32-key tiles)
#   b32fwd = -DDTA_FWD_BN32=1   (paired forward with 32-key tiles when Q rows stay in registers)
# Timing only; a variant that wins is adopted and then goes through the full parity suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05h}
mkdir -p $OUT
for sh in 8,16,64,2,4096 8,16,64,3,4096; do
  timeout -k 10 240 python tools/ab_kernels.py head=lib/libdiffattn.so b32dq=lib/libdiffattn_b32dq.so b32fwd=lib/libdiffattn_b32fwd.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R05H_OK
