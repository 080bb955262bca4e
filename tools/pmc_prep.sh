set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcp; mkdir -p $OUT; cd /tmp
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/pass$i -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 1 --warmup 1 --prep 3 > $OUT/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pass$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/pmcp k_fine_count k_gather k_fine_fill k_geo_pack > gpurun_out/pmcp/summary.txt 2>&1; cat gpurun_out/pmcp/summary.txt
