# Round-5 A/B: dS packed ahead of the dQ product's transposed K reads (pk = -DDTA_DQ_PACKFIRST=1) against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05zg}
mkdir -p $OUT
for sh in 8,16,64,2,4096 16,6,64,3,2048; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so pk=lib/libdiffattn_pk.so --shape $sh --rounds 5 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['min_ms'], b['sum_median_ms'])"
done
echo R05ZG_OK
