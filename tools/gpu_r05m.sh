# Round-5 SQ counters of the cfg3 N = 3 core at HEAD (sequential-branch forward, paired 32-key dQ,
# dK/dV in groups 2 + 1): the two counter groups of round_gpu.sh, each its own pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05m}
mkdir -p $OUT
A="--batch 16 --heads 6 --seq 2048 --n-terms 3 --no-configs --no-hbm --train-steps 0 --cpu-baseline off --steps 3 --warmup 1"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/sq$i -o run -- python3 $R/bench.py $A > $OUT/sq$i.log 2>&1 || { echo "SQ group $i failed"; tail -5 $OUT/sq$i.log; exit 1; }
done
python3 $R/tools/pmc_sq.py $OUT/sq1 $OUT/sq2 --json $OUT/sq.json > $OUT/sq_summary.txt && tail -8 $OUT/sq_summary.txt
echo R05M_OK
