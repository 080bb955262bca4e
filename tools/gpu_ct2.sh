# Call-time path checks: its tests, then the kernel trace.  Usage: bash tools/gpu_ct2.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=$1
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -x -k "calltime or boundary or ctypes or plumbing or golden" > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_calltime.sh $T
