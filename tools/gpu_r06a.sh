# Round-6 first GPU call: parity tests, bench line, rocprof stats, PMC traffic, SQ counters
# with the effective clock (tools/round_gpu.sh, SQ=1), then in-kernel stamps of the forward,
# dQ and dK/dV tile loops at cfg2 and cfg3 N = 3 (tools/stamps.py on a DTA_STAMPS=1 build).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r06a}
SQ=1 bash tools/round_gpu.sh $TAG || exit 1
OUT=gpurun_out/$TAG
for sh in 8,16,64,2,4096; do
  timeout -k 10 300 python tools/stamps.py lib/libdiffattn_stamps.so --shape $sh > $OUT/stamps_$sh.json 2> $OUT/stamps_$sh.err || { echo "STAMPS $sh FAILED"; tail -5 $OUT/stamps_$sh.err; exit 1; }
  cat $OUT/stamps_$sh.json
done
echo R06A_OK
