# Round measurements on one GPU: parity suite, then every BASELINE config's bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/meas
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { name=$1; shift; timeout -k 10 ${TL:-300} python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "BENCH $name FAILED"; tail -5 $O/$name.err; exit 1; }; echo "$name: $(head -c 400 $O/$name.json)"; }
[ -z "$SKIP_CFG2" ] && run cfg2 ${CFG2_ARGS:-}
run cfg5 --cpu-baseline off --batch 1 --heads 16 --head-size 128 --seq 32768 --control --steps 5 --warmup 2
run cfg3_n3 --cpu-baseline off --mode train --model ndiff --n-terms 3 --steps 6 --warmup 2
run cfg3_n4 --cpu-baseline off --mode train --model ndiff --n-terms 4 --steps 6 --warmup 2
run cfg4 --cpu-baseline off --mode train --steps 6 --warmup 2
