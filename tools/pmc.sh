# PMC passes (one rocprofv3 --pmc run per counter group, each under its own hard limit).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/list.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ|TCC|TCP|GRBM)_[A-Z0-9_]+" $R/gpurun_out/pmc/list.txt | sort -u > $R/gpurun_out/pmc/names.txt || true
wc -l $R/gpurun_out/pmc/names.txt
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/bench.py --cpu-baseline off --steps 3 --warmup 1 > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "PMC group $i failed: $grp"; tail -5 $R/gpurun_out/pmc/p$i.log; }
done
ls $R/gpurun_out/pmc
