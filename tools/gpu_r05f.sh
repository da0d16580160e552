# Round-5 one-process A/B: the round-4 library (lib/libdiffattn_r04.so, a build of commit ce6f194)
# against HEAD on the attention core shapes (cfg2, cfg3 N = 3 / 4, cfg5) and the LayerNorm kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05f}
mkdir -p $OUT
timeout -k 10 120 python tools/ab_ln.py r04=lib/libdiffattn_r04.so head=lib/libdiffattn.so > $OUT/ab_ln.json 2> $OUT/ab_ln.err || { echo AB_LN_FAILED; tail -5 $OUT/ab_ln.err; exit 1; }
cat $OUT/ab_ln.json; echo
for sh in 8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048; do
  timeout -k 10 200 python tools/ab_kernels.py r04=lib/libdiffattn_r04.so head=lib/libdiffattn.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
timeout -k 10 300 python tools/ab_kernels.py r04=lib/libdiffattn_r04.so head=lib/libdiffattn.so --shape 1,16,128,2,32768 --rounds 3 --reps 2 > $OUT/ab_cfg5.json 2> $OUT/ab_cfg5.err || { echo "AB cfg5 FAILED"; tail -5 $OUT/ab_cfg5.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/ab_cfg5.json'))
for n,b in d['builds'].items(): print('cfg5', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
echo R05F_OK
