# cfg4 / cfg3 training step: rocprofv3 kernel trace of a few steps, summarised by kernel (no tests).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-trainprof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --mode train --steps 4 --warmup 2 > $O/prof4.log 2>&1 || { echo PROF4_FAILED; tail -20 $O/prof4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --mode train --model ndiff --n-terms 3 --steps 4 --warmup 2 > $O/prof3.log 2>&1 || { echo PROF3_FAILED; tail -20 $O/prof3.log; exit 1; }
head -25 $O/prof4/run_kernel_stats.csv | cut -c1-160
echo ---
head -25 $O/prof3/run_kernel_stats.csv | cut -c1-160
echo TRAINPROF_OK
