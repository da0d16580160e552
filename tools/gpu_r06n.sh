# Round-6 A/B: the LayerNorm backward's ordered dw/db reduce in one launch (DTA_LN_REDUCE_ONE=1,
# default) against the two-launch reduce1 + reduce2; then the LN/rope GPU tests on the new build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06n}
mkdir -p $OUT
timeout -k 10 300 python tools/ab_ln.py red2=lib/libdiffattn_red2.so q8=lib/libdiffattn_q8.so q4=lib/libdiffattn_q4.so q2=lib/libdiffattn_q2.so q8b=lib/libdiffattn_q8.so red2b=lib/libdiffattn_red2.so > $OUT/ab_ln.json 2> $OUT/ab_ln.err || { echo AB FAILED; tail -5 $OUT/ab_ln.err; exit 1; }
cat $OUT/ab_ln.json
true

echo R06N_OK
