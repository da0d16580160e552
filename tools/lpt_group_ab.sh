# Dispatch-order A/B (DTA_LPT_GROUP builds): kernel times in one process (ab_kernels.py)
# at cfg2 and cfg3, then one rocprofv3 FETCH_SIZE pass per build over the cfg2 bench.
# Usage (GPU box): BUILDS="base=lib/libdiffattn.so g1=lib/libdiffattn_lg1.so ..." bash tools/lpt_group_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for shape in ${SHAPES:-8,16,64,2,4096 16,6,64,3,2048 16,6,64,4,2048}; do
  timeout -k 10 300 python tools/ab_kernels.py $BUILDS --shape $shape --rounds ${ROUNDS:-5} --reps ${REPS:-6} > $OUT/ab_$shape.json 2> $OUT/ab_$shape.err || { echo "AB_FAILED $shape"; tail -20 $OUT/ab_$shape.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/ab_$shape.json'))
print('$shape', {n: (b['median_ms'], b['sum_median_ms']) for n, b in d['builds'].items()})"
done
cd /tmp && export TMPDIR=/tmp
for b in $BUILDS; do
  name=${b%%=*}; lib=$R/differential_transformer_replication_amd/${b#*=}
  DTA_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$name -o run -- python3 $R/bench.py --cpu-baseline off --train-steps 0 --no-configs --no-hbm --steps 3 --warmup 1 > $OUT/fetch_$name.log 2>&1 || { echo "PMC_FAILED $name"; tail -5 $OUT/fetch_$name.log; exit 1; }
  python3 - <<EOF
import csv, glob, collections
v = collections.defaultdict(list)
for f in glob.glob('$OUT/fetch_$name/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        for k in ('attn_fwd', 'attn_dq', 'attn_dkdv'):
            if k + '_kernel' in r['Kernel_Name']:
                v[k].append(float(r['Counter_Value']))
print('$name', {k: round(sum(x) / len(x) * 2048 / 1e6, 1) for k, x in v.items()}, 'MB read per launch (FETCH_SIZE x2)')
EOF
done
echo LPT_AB_OK
