# A/B of K/V staging in the forward / dQ kernels (DTA_KV_STAGING): parity suite, then cfg2 bench per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|FAILED|error" gpurun_out/tests.log | head -20; exit 1; }
tail -1 gpurun_out/tests.log
for m in 1 0 1 0; do
  DTA_KV_STAGING=$m timeout -k 10 120 python bench.py --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/bench_kv$m.json 2> gpurun_out/bench_kv$m.err || { echo "BENCH $m FAILED"; tail -5 gpurun_out/bench_kv$m.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_kv$m.json')); print('kv_staging $m', d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
