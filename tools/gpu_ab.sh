# One GPU call of kernel A/B evidence: parity of the default build (test_gpu_parity), then
# tools/ab_kernels.py over BUILDS (name=lib/... pairs; default base + $VARIANT) at cfg2 and
# the cfg3 shapes, then any extra command in $EXTRA.   Usage: bash tools/gpu_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
  rc=$?; tail -2 $OUT/parity.log
  if [ $rc -ne 0 ]; then echo "PARITY_FAILED rc=$rc"; grep -E "FAILED|Error" $OUT/parity.log | head; exit 1; fi
fi
for shape in ${SHAPES:-8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048}; do
  timeout -k 10 300 python tools/ab_kernels.py $BUILDS --shape $shape --rounds ${ROUNDS:-5} --reps ${REPS:-8} > $OUT/ab_$shape.json 2> $OUT/ab_$shape.err || { echo "AB_FAILED $shape"; tail -20 $OUT/ab_$shape.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$OUT/ab_$shape.json'))
print('$shape', {n: (b['median_ms'], b['sum_median_ms'], max(b[k] for k in b if k.startswith('rel_diff')).__class__ and {kk: round(vv,4) for kk,vv in list(b.items())[-1][1].items()}) for n,b in d['builds'].items()})"
done
if [ -n "$EXTRA" ]; then eval "$EXTRA"; fi
echo GPU_AB_OK
