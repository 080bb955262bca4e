# SQ counters of the render kernels (headline and thin fields), one rocprofv3 --pmc pass each.
# Usage: bash tools/gpu_pmc.sh TAG [COUNTERS...]
set -u
cd $GRAFT_REPO_ROOT
T=${1:-pmc}
shift || true
CNT=${*:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for A in 1 25; do
  ( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $CNT --output-format csv -d $GRAFT_REPO_ROOT/$O/a$A -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 2 --warmup 1 --aniso $A > $GRAFT_REPO_ROOT/$O/a$A.log 2>&1 ) || { echo "pmc aniso $A failed"; tail -5 $O/a$A.log; exit 1; }
done
echo done
