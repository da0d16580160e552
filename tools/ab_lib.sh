# A/B of library variants over the cfg2 bench (interleaved rounds):
# VARIANTS names lib/libdiffattn_<v>.so builds; "base" is lib/libdiffattn.so.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib
for r in 1 2 3; do for v in base ${VARIANTS:-old}; do
  if [ $v = base ]; then f=$L/libdiffattn.so; else f=$L/libdiffattn_$v.so; fi
  DTA_LIB=$f timeout -k 10 120 python bench.py --cpu-baseline off > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "BENCH $v FAILED"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done; done
