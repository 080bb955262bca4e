# One GPU call: the -m gpu tests selected by -k (margins recorded).  Usage: bash tools/gpu_tests_k.sh TAG "K"
set -u
cd $GRAFT_REPO_ROOT
T=$1; K=$2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -x -k "$K" > $O/gpu_tests.log 2>&1
rc=$?
tail -15 $O/gpu_tests.log
exit $rc
