# Round-6 final evidence at HEAD: the whole GPU suite, the default bench line, rocprofv3 kernel
# stats, PMC FETCH / WRITE traffic, SQ counters with the effective clock (tools/round_gpu.sh SQ=1),
# stamps of the three tile loops (when a DTA_STAMPS=1 build is present), smoke, the decode bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r06z}
SQ=1 bash tools/round_gpu.sh $TAG || exit 1
OUT=gpurun_out/$TAG
[ ! -f differential_transformer_replication_amd/lib/libdiffattn_stamps.so ] || timeout -k 10 300 python tools/stamps.py lib/libdiffattn_stamps.so --shape 8,16,64,2,4096 > $OUT/stamps.json 2> $OUT/stamps.err || { echo STAMPS FAILED; tail -5 $OUT/stamps.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py --mode decode --steps 50 --warmup 10 > $OUT/decode.json 2> $OUT/decode.err || { echo DECODE_FAILED; tail -5 $OUT/decode.err; exit 1; }
tail -1 $OUT/decode.json
echo FINAL_OK
timeout -k 10 300 python tools/host_overhead_probe.py --shape 16,6,64,3,2048 > $OUT/host_probe_cfg3.json 2> $OUT/host_probe.err && cat $OUT/host_probe_cfg3.json
timeout -k 10 300 python tools/host_overhead_probe.py --shape 8,16,64,2,4096 > $OUT/host_probe_cfg2.json 2>> $OUT/host_probe.err && cat $OUT/host_probe_cfg2.json
echo PROBE_DONE
