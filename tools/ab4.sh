set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab4
DTA_FWD_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "core_fwd_bwd or forced or sampled" > gpurun_out/ab4/t_pipe.log 2>&1
rc=$?; echo "tests pipe rc=$rc $(tail -1 gpurun_out/ab4/t_pipe.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python tools/ab_kernels.py base=lib/libdiffattn.so pipe=lib/libdiffattn_pipe.so --rounds 5 --reps 8 > gpurun_out/ab4/ab.json 2> gpurun_out/ab4/ab.err || { tail -20 gpurun_out/ab4/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab4/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'])"
DTA_FWD_PIPE=1 timeout -k 10 200 python tools/stamps.py lib/libdiffattn_stamps.so > gpurun_out/ab4/stamps.json 2> gpurun_out/ab4/stamps.err || { tail -20 gpurun_out/ab4/stamps.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab4/stamps.json')); print(json.dumps(d['fwd']))"
