# One GPU call: selected tests (-k), then tools/ab.py (thin and headline) over variants.
# Usage: bash tools/gpu_abt.sh TAG "PYTEST_K" VARIANTS...
set -u
cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -x -k "$K" > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 10 --warmup 2 --prep 4 --aniso 25" base "$@" > $O/ab_thin.log 2>&1 || { echo ab failed; tail -5 $O/ab_thin.log; exit 1; }
grep MEDIAN $O/ab_thin.log
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 20 --warmup 5 --prep 4" base "$@" > $O/ab_head.log 2>&1 || { echo ab failed; tail -5 $O/ab_head.log; exit 1; }
grep MEDIAN $O/ab_head.log
