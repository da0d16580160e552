# Round-6 A/B: the attention unit built with -mllvm -amdgpu-use-amdgpu-trackers=1 (the scheduler register trackers) vs default,
# step-interleaved, cfg3 N = 3 and cfg2.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06v}
mkdir -p $OUT
for sh in 16,6,64,3,2048 8,16,64,2,4096; do
  timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn_base.so trk=lib/libdiffattn_trk.so base2=lib/libdiffattn_base.so trk2=lib/libdiffattn_trk.so --shape $sh --rounds 8 --reps 6 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'], b.get('rel_diff_vs_base'))"
done
echo R06V_OK
