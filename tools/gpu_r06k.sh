# Round-6: same-box A/B of the cfg3 N = 3 and cfg4 training steps, this round's kernel defaults
# (new: |c_i| fold, NT fp32 stores) against both off (old), alternating processes (DTA_LIB).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06k}
mkdir -p $OUT
L=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib
for i in 1 2 3; do
  for v in old new; do
    DTA_LIB=$L/libdiffattn_$v.so timeout -k 10 300 python bench.py --cpu-baseline off --mode train --model ndiff --n-terms 3 --steps 10 --warmup 3 > $OUT/n3_$v$i.json 2> $OUT/n3_$v$i.err || { tail -5 $OUT/n3_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/n3_$v$i.json')); print('cfg3 n3', '$v', d['value'], d['ms_per_step'])"
  done
done
for i in 1 2; do
  for v in old new; do
    DTA_LIB=$L/libdiffattn_$v.so timeout -k 10 300 python bench.py --cpu-baseline off --mode train --steps 8 --warmup 3 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err || { tail -5 $OUT/c4_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_$v$i.json')); print('cfg4', '$v', d['value'], d['ms_per_step'])"
  done
done
echo R06K_OK
