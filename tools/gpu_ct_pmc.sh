# SQ counters of the call-time kernels (tools/calltime_bench.py, one step).  Usage: bash tools/gpu_ct_pmc.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=$1
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc1 -o run -- python $GRAFT_REPO_ROOT/tools/calltime_bench.py --steps 1 > $GRAFT_REPO_ROOT/$O/pmc1.log 2>&1 || { echo pmc1 failed; tail -3 $GRAFT_REPO_ROOT/$O/pmc1.log; exit 1; }
cd $GRAFT_REPO_ROOT
python tools/pmc_summary.py $O/pmc1 2>&1 | grep -A9 "k_ref_" | head -40
