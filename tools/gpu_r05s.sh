# Round-5 probe: per-workgroup fixed costs (prologue, epilogue drain) -- the same kernels at
# cfg2 and at twice T (half B: 2x the FLOPs, the same workgroup count, 2x the work each).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05s}
mkdir -p $OUT
for sh in 8,16,64,2,4096 4,16,64,2,8192 2,16,64,2,16384; do
  timeout -k 10 300 python tools/ab_kernels.py head=lib/libdiffattn.so --shape $sh --rounds 3 --reps 8 > $OUT/ab_$sh.json 2> $OUT/ab_$sh.err || { echo "AB $sh FAILED"; tail -5 $OUT/ab_$sh.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$sh.json'))
for n,b in d['builds'].items(): print('$sh', n, b['median_ms'], b['sum_median_ms'])"
done
echo R05S_OK
