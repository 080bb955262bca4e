# SQ counters of the cell backward (in-tree) against the sub-cell backward (variants/bsub).
set -u
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/pmc_bsub; mkdir -p $O
C1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM"
C2="SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"
for v in base bsub; do
  if [ $v = base ]; then export PYTHONPATH=$GRAFT_REPO_ROOT/diff-gaussian-sampling_amd; else export PYTHONPATH=$GRAFT_REPO_ROOT/variants/bsub; fi
  i=0
  for pass in "$C1" "$C2"; do
    i=$((i+1))
    ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/$v/pass$i -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 3 --warmup 1 > $O/$v.pass$i.log 2>&1 ) || { echo "$v pass $i failed"; tail -5 $O/$v.pass$i.log; exit 1; }
  done
done
echo ALLDONE
