# SQ counter passes over the attention kernels of one core shape (tools/ab_kernels.py, one build).
# Usage (on the GPU box): bash tools/sq_shape.sh <tag> B,H,hs,N,T
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-sq_shape}; SHAPE=${2:-16,6,64,3,2048}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/tools/ab_kernels.py base=lib/libdiffattn.so --shape $SHAPE --rounds 1 --reps 2 > $OUT/p$i.log 2>&1 || { echo "PMC group $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/pmc_sq.py $OUT/p1 $OUT/p2 --json $OUT/sq.json > $OUT/sq.txt && tail -4 $OUT/sq.txt
