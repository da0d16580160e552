# GPU tests, then the cfg4 training step timed and profiled (kernel stats).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-train}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20; tail -2 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
timeout -k 10 300 python bench.py --cpu-baseline off --mode train --steps 8 --warmup 3 > $O/train.json 2> $O/train.err || { echo TRAIN_FAILED; tail -20 $O/train.err; exit 1; }
head -c 700 $O/train.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --mode train --steps 4 --warmup 2 > $O/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $O/prof.log; exit 1; }
echo PROF_OK
