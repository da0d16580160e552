set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab6
timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn.so preoff=lib/libdiffattn_preoff.so --rounds 5 --reps 8 > gpurun_out/ab6/ab.json 2> gpurun_out/ab6/ab.err || { tail -20 gpurun_out/ab6/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab6/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
timeout -k 10 300 python bench.py --cpu-baseline off --train-steps 0 --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['hbm_kernels']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ab6/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/ab6/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/ab6/prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/ab6/prof.log | cut -c1-300
head -25 $GRAFT_REPO_ROOT/gpurun_out/ab6/prof/run_kernel_stats.csv | cut -c1-180
