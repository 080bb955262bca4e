# One GPU call: tools/ab.py over env variants at one kbench workload.
# Usage: bash tools/gpu_abenv.sh TAG "KBENCH ARGS" VARIANTS...
set -u
cd $GRAFT_REPO_ROOT
T=$1; KA=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab.py --rounds 3 --kbench-args "$KA" "$@" > $O/ab.log 2>&1 || { echo ab failed; tail -5 $O/ab.log; exit 1; }
grep MEDIAN $O/ab.log
