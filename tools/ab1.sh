set -o pipefail
cd $GRAFT_REPO_ROOT
L=differential_transformer_replication_amd/lib
mkdir -p gpurun_out/ab1
for v in "" _pp _ppqk; do
  DTA_LIB=$PWD/$L/libdiffattn$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "core_fwd_bwd or forced or sampled" > gpurun_out/ab1/t$v.log 2>&1
  rc=$?; echo "tests$v rc=$rc $(tail -1 gpurun_out/ab1/t$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
done
timeout -k 10 300 python tools/ab_kernels.py r1=lib/libdiffattn_r1.so base=lib/libdiffattn.so qk=lib/libdiffattn_qk.so pp=lib/libdiffattn_pp.so ppqk=lib/libdiffattn_ppqk.so --rounds 5 --reps 8 > gpurun_out/ab1/ab.json 2> gpurun_out/ab1/ab.err || { tail -20 gpurun_out/ab1/ab.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab1/ab.json'))
for n,b in d['builds'].items(): print(n, b['median_ms'], b['sum_median_ms'], {k: '%.1e'%v for k,v in list(b.values())[3].items()})"
