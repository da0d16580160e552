# Decode-mode evidence: bench line, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes.
# Usage (on the GPU box): bash tools/profile_decode.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01_dec}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --mode decode --steps 5 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAILED; tail -5 $OUT/pmc_fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --mode decode --steps 5 --warmup 1 > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAILED; tail -5 $OUT/pmc_write.log; exit 1; }
echo DECODE_PMC_OK
