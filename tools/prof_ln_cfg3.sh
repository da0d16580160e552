# Kernel traces of the LN / RoPE A/B command and of the cfg3 N=3 core, CSV stats.
# Usage (on the GPU box): bash tools/prof_ln_cfg3.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-r04_prof}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ln -o run -- python3 $R/tools/ab_ln.py base=lib/libdiffattn.so > $OUT/ln.log 2>&1 || { echo LN_PROF_FAILED; tail -5 $OUT/ln.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg3 -o run -- python3 $R/tools/ab_kernels.py base=lib/libdiffattn.so --shape 16,6,64,3,2048 --rounds 2 --reps 4 > $OUT/cfg3.log 2>&1 || { echo CFG3_PROF_FAILED; tail -5 $OUT/cfg3.log; exit 1; }
for d in ln cfg3; do echo "== $d"; f=$(find $OUT/$d -name "*kernel_stats.csv" | head -1); cut -d, -f1-7 $f | head -12 | cut -c1-200; done
