# Round-6: the default bench line at HEAD with the committed r06z PMC / SQ profiles (roofline
# traffic and clock filled in), then the cfg3 / cfg4 training A/B of tools/gpu_r06k.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06l
timeout -k 10 600 python bench.py > gpurun_out/r06l/bench.json 2> gpurun_out/r06l/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/r06l/bench.err; exit 1; }
tail -1 gpurun_out/r06l/bench.json | cut -c1-400
bash tools/gpu_r06k.sh r06l || exit 1
echo R06L_OK
