# Round-6: the driver's bench command on the final build, repeated in one call (box variance within
# a box: first vs second run), plus the cfg2 host probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06q}
mkdir -p $OUT
for k in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$k.json 2> $OUT/bench_$k.err || { echo BENCH_FAILED; tail -20 $OUT/bench_$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$k.json')); print($k, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['configs']['cfg3_n3']['core']['ms_per_step'], d['train']['value'])"
done
echo R06Q_OK
