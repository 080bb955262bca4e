# SQ counters of the thin (--aniso 25) preprocess kernels (tools/kbench.py --prep 2).
# Usage: bash tools/gpu_prep_pmc.sh TAG [KBENCH ARGS]
set -u
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc1 -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 1 --warmup 1 --prep 2 "$@" > $GRAFT_REPO_ROOT/$O/pmc1.log 2>&1 || { echo pmc1 failed; tail -3 $GRAFT_REPO_ROOT/$O/pmc1.log; exit 1; }
echo done
