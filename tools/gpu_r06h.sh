# Round-6 evidence at HEAD: the whole GPU suite, bench line, rocprofv3 kernel stats, PMC traffic,
# SQ counters with the effective clock (tools/round_gpu.sh, SQ=1), stamps, smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r06h}
SQ=1 bash tools/round_gpu.sh $TAG || exit 1
OUT=gpurun_out/$TAG
timeout -k 10 300 python tools/stamps.py lib/libdiffattn_stamps.so --shape 8,16,64,2,4096 > $OUT/stamps.json 2> $OUT/stamps.err || { echo STAMPS FAILED; tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
echo R06H_OK
