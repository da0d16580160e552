set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
timeout -k 10 200 python tools/stamps.py lib/libdiffattn_stamps.so > gpurun_out/ab2/stamps.json 2> gpurun_out/ab2/stamps.err || { tail -20 gpurun_out/ab2/stamps.err; exit 1; }
cat gpurun_out/ab2/stamps.json
