set -o pipefail
cd $GRAFT_REPO_ROOT
L=differential_transformer_replication_amd/lib
mkdir -p gpurun_out/ab3
DTA_FWD_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modules.py -q -x --timeout 120 --timeout-method thread -k "core_fwd_bwd or forced or sampled or module_fp32 or tiny_model" > gpurun_out/ab3/t_pipe.log 2>&1
rc=$?; echo "tests pipe rc=$rc $(tail -1 gpurun_out/ab3/t_pipe.log)"; grep -E "FAILED|Error" gpurun_out/ab3/t_pipe.log | head -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
timeout -k 10 300 python tools/ab_kernels.py r1=lib/libdiffattn_r1.so base=lib/libdiffattn.so pipe=lib/libdiffattn_pipe.so --rounds 5 --reps 8 > gpurun_out/ab3/ab.json 2> gpurun_out/ab3/ab.err || { tail -20 gpurun_out/ab3/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab3/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
