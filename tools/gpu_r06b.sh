# Round-6 A/B + stamps: the dQ ring issued ahead of the delta prologue (early) against the same
# reduced-config build of HEAD (base), step-interleaved timing (tools/ab_kernels.py --mode step),
# then stamps of the forward, dQ and dK/dV loops (32-bit sums, no spills in the stamped dK/dV).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so early=lib/libdiffattn_early.so --shape $sh --rounds 6 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], max(b['rel_diff_vs_base'].values()))"
done
timeout -k 10 300 python tools/stamps.py lib/libdiffattn_stamps.so --shape 8,16,64,2,4096 > $OUT/stamps.json 2> $OUT/stamps.err || { echo STAMPS FAILED; tail -5 $OUT/stamps.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/stamps.json'))
for k,v in d.items(): print(k, v['share'])"
echo R06B_OK
timeout -k 10 900 python tools/bf16_dlambda_seeds.py --seeds 6 > $OUT/dlambda_seeds.json 2> $OUT/dlambda_seeds.err || { echo DLAMBDA FAILED; tail -5 $OUT/dlambda_seeds.err; exit 1; }
python3 -c "
import json; d=json.load(open(\"$OUT/dlambda_seeds.json\")); print({k:v for k,v in d.items() if k!=\"rows\"})"
echo R06B_DONE
