# Round evidence: default bench (with CPU baseline), rocprofv3 kernel stats of the
# same command, and one --pmc pass each for FETCH_SIZE and WRITE_SIZE.
# Usage (on the GPU box): bash tools/profile_round.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --cpu-baseline off --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --cpu-baseline off --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -5 $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
