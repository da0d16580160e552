# One GPU call of round evidence: parity tests, the default bench line, a rocprofv3
# kernel trace of the same command, FETCH_SIZE / WRITE_SIZE passes, SQ counter passes.
# Usage (on the GPU box): bash tools/round_gpu.sh <tag> [skip-tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  # assertion failures (rc 1) are recorded and the evidence run continues; a crash,
  # abort or time limit (any other rc) ends the call
  DTA_TEST_LOG_DIR=$OUT timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/tests.log | head -30
  tail -3 $OUT/tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS_ABORTED rc=$rc"; exit 1; fi
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
PB="--cpu-baseline off --train-steps 0"
# counter passes: the cfg2 core only (PMC summaries are keyed by kernel family + shape)
PC="$PB --no-configs"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py $PB > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
head -14 $OUT/prof/run_kernel_stats.csv | cut -c1-200
# per-(kernel, grid) means: one instance serves several shapes in one bench process
python3 $R/tools/kernel_stats_by_shape.py $OUT/prof/run_kernel_trace.csv $OUT/kernel_stats_by_shape.csv || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $PC --steps 3 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $PC --steps 3 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -5 $OUT/pmc_write.log; exit 1; }
python3 $R/tools/pmc_summary.py $OUT $OUT/pmc_traffic.json B8_H16_hs64_N2_T4096_dv128 || exit 1
if [ -n "$SQ" ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq$i -o run -- python3 $R/bench.py $PC --no-hbm --steps 2 --warmup 1 > $OUT/sq$i.log 2>&1 || { echo "SQ group $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
  done
  LSHA=$(sha256sum $R/differential_transformer_replication_amd/lib/libdiffattn.so | cut -c1-16)
  python3 $R/tools/pmc_sq.py $OUT/sq1 $OUT/sq2 --json $OUT/sq.json --lib-sha $LSHA --shape B8_H16_hs64_N2_T4096_dv128 > $OUT/sq_summary.txt && cat $OUT/sq_summary.txt
fi
echo ROUND_GPU_OK
