# A/B of one environment switch over the cfg2 bench: VAR=name, values in VALS (interleaved rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|FAILED|error" gpurun_out/tests.log | head -20; exit 1; }
tail -1 gpurun_out/tests.log
fi
for m in $VALS; do
  env $VAR=$m timeout -k 10 120 python bench.py --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/ab_$m.json 2> gpurun_out/ab_$m.err || { echo "BENCH $m FAILED"; tail -5 gpurun_out/ab_$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$m.json')); print('$VAR=$m', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
