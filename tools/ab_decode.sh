# A/B of decode-chunk library variants: parity tests then decode bench at three shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/differential_transformer_replication_amd/lib
for v in ${VARIANTS:-c512 c1024}; do
  DTA_LIB=$L/libdiffattn_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abd_$v.log 2>&1 || { echo "TESTS $v FAILED"; tail -20 gpurun_out/abd_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/abd_$v.log)"
done
for r in 1 2; do for v in base ${VARIANTS:-c512 c1024}; do
  if [ $v = base ]; then f=$L/libdiffattn.so; else f=$L/libdiffattn_$v.so; fi
  for shape in "--seq 4096" "--seq 32768" "--batch 1 --head-size 128 --seq 32768"; do
    DTA_LIB=$f timeout -k 10 120 python bench.py --mode decode --steps 50 --warmup 5 $shape > gpurun_out/abd.json 2> gpurun_out/abd.err || { echo "BENCH $v FAILED"; tail -5 gpurun_out/abd.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/abd.json')); print('$v', '$shape', d['roofline']['kernel_ms'], d['roofline']['achieved'])"
  done
done; done
