set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab5
DTA_LIB=$PWD/differential_transformer_replication_amd/lib/libdiffattn_pipe32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "core_fwd_bwd or forced or sampled" > gpurun_out/ab5/t.log 2>&1
rc=$?; echo "tests pipe32 rc=$rc $(tail -1 gpurun_out/ab5/t.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn.so pipe32=lib/libdiffattn_pipe32.so pipe32q=lib/libdiffattn_pipe32q.so --rounds 5 --reps 8 > gpurun_out/ab5/ab.json 2> gpurun_out/ab5/ab.err || { tail -20 gpurun_out/ab5/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab5/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
