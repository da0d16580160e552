# Alternating decode-bench runs of two library builds (DTA_LIB), same box.
# Usage (on the GPU box): bash tools/ab_decode_lib.sh <tag> <libA> <libB> [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; A=$2; B=$3; R=${4:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do
  for v in A B; do
    L=$([ $v = A ] && echo "$A" || echo "$B")
    DTA_LIB=$L timeout -k 10 200 python bench.py --cpu-baseline off --mode decode --steps 50 --warmup 10 > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  done
done
