# SQ counter passes (one rocprofv3 --pmc run per group) over the cfg2 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sq
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/sq/list.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/sq/p$i -o run -- python3 $R/bench.py --cpu-baseline off --steps 2 --warmup 1 > $R/gpurun_out/sq/p$i.log 2>&1 || { echo "PMC group $i failed: $grp"; tail -3 $R/gpurun_out/sq/p$i.log; exit 1; }
done
python3 $R/tools/pmc_sq.py $R/gpurun_out/sq/p*
