# SQ / traffic counters of every kernel of tools/kbench.py (one preprocess + a few render steps).
set -u
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${T:-pmc2}; mkdir -p $O
bash tools/pmc_kbench.sh $O \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
  "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY" \
  "FETCH_SIZE" "WRITE_SIZE" || exit 1
python3 tools/pmc_summary.py $O k_sub_lists k_fine_count k_backward k_forward_s k_gather > $O/summary.txt 2>&1 || true
echo ALLDONE
