# Same-box A/B of training-step switches: alternating runs of the cfg4 train bench.
# Usage (on the GPU box): bash tools/ab_train.sh <tag> "ENV_A" "ENV_B" [rounds]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; A=$2; B=$3; R=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $R); do
  for v in A B; do
    E=$([ $v = A ] && echo "$A" || echo "$B")
    env $E timeout -k 10 300 python bench.py --cpu-baseline off --mode train --steps 8 --warmup 3 > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v$i.json')); print('$v', '$E', d['value'], d['ms_per_step'])"
  done
done
