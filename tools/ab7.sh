set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab7
timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn.so pair=lib/libdiffattn_pair.so pairall=lib/libdiffattn_pairall.so --rounds 5 --reps 8 > gpurun_out/ab7/ab.json 2> gpurun_out/ab7/ab.err || { tail -20 gpurun_out/ab7/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab7/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
