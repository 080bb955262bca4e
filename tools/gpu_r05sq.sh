# Round-5 SQ counters of the render kernels (headline and --aniso 25), two passes each.
# Usage: bash tools/gpu_r05sq.sh TAG
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05sq}
mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/head "$P1" "$P2" || exit 1
python tools/pmc_summary.py $O/head > $O/head_summary.txt 2>&1
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --aniso 25" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/thin "$P1" "$P2" || exit 1
python tools/pmc_summary.py $O/thin > $O/thin_summary.txt 2>&1
echo ALLDONE
