# Round-6 A/B: the LayerNorm backward's row prefetch depth (DTA_LN_BWD_PD 1 / 2 / 3 row groups in
# flight), then depths 3-5 and 384 workgroups (second call), cfg2 LN shape, one process, rounds interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06o}
mkdir -p $OUT
timeout -k 10 300 python tools/ab_ln.py pd1=lib/libdiffattn.so pd3=lib/libdiffattn_pd3.so pd4=lib/libdiffattn_pd4.so pd5=lib/libdiffattn_pd5.so pd3b384=lib/libdiffattn_pd3b384.so pd3b=lib/libdiffattn_pd3.so > $OUT/ab_ln.json 2> $OUT/ab_ln.err || { echo AB FAILED; tail -5 $OUT/ab_ln.err; exit 1; }
cat $OUT/ab_ln.json
echo R06O_OK
