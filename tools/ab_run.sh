# GPU parity tests (optional) then a one-process A/B of library builds.
# Usage (on the GPU box): TESTS="tests/..." bash tools/ab_run.sh <tag> name=lib/x.so name2=lib/y.so ...
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -15 $OUT/tests.log
  if [ $rc -ne 0 ]; then echo "TESTS_FAILED rc=$rc"; exit 1; fi
fi
timeout -k 10 300 python tools/ab_kernels.py "$@" --rounds ${ROUNDS:-5} --reps ${REPS:-8} ${SHAPE:+--shape $SHAPE} > $OUT/ab.json 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
