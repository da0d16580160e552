# cfg3 training step (N-diff, n_terms 3 and 4): bench lines standalone, then rocprofv3 kernel
# stats of each.   Usage (GPU box): bash tools/cfg3_prof.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cfg3}
mkdir -p $O
cd $R
for n in 3 4; do
  timeout -k 10 300 python bench.py --cpu-baseline off --mode train --model ndiff --n-terms $n --steps 6 --warmup 3 > $O/train_n$n.json 2> $O/train_n$n.err || { echo TRAIN_FAILED $n; tail -20 $O/train_n$n.err; exit 1; }
  head -c 300 $O/train_n$n.json; echo
done
cd /tmp && export TMPDIR=/tmp
for n in 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_n$n -o run --output-format csv -- python3 $R/bench.py --cpu-baseline off --mode train --model ndiff --n-terms $n --steps 3 --warmup 2 > $O/prof_n$n.log 2>&1 || { echo PROF_FAILED $n; tail -20 $O/prof_n$n.log; exit 1; }
  head -12 $O/prof_n$n/run_kernel_stats.csv | cut -c1-150
done
echo CFG3_OK
