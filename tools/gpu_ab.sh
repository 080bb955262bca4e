# One GPU call: tools/ab.py over variants at the thin (--aniso 25) workload and at the headline.
# Usage: bash tools/gpu_ab.sh TAG VARIANTS...
set -u
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 10 --warmup 2 --prep 6 --aniso 25" base "$@" > $O/ab_thin.log 2>&1 || { echo ab failed; tail -5 $O/ab_thin.log; exit 1; }
grep MEDIAN $O/ab_thin.log
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 20 --warmup 5 --prep 6" base "$@" > $O/ab_head.log 2>&1 || { echo ab failed; tail -5 $O/ab_head.log; exit 1; }
grep MEDIAN $O/ab_head.log
