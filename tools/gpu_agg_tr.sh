# Transposed aggregate backward: GPU tests + bench.  Usage: bash tools/gpu_agg_tr.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03t}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_aggregate.py tests/test_gpu_ctypes.py -x -v --timeout 200 --timeout-method thread > $O/agg_tests.log 2>&1 || { echo "agg tests failed"; tail -40 $O/agg_tests.log; exit 1; }
tail -1 $O/agg_tests.log
timeout -k 10 300 python -u bench.py --op aggregate --steps 3 --warmup 1 --no-cpu > $O/agg.log 2>&1 || { echo agg failed; tail -5 $O/agg.log; exit 1; }
tail -1 $O/agg.log
DGS_AGG_TRANSPOSE=0 timeout -k 10 300 python -u bench.py --op aggregate --steps 3 --warmup 1 --no-cpu > $O/agg_atomic.log 2>&1 || { echo agg atomic failed; tail -5 $O/agg_atomic.log; exit 1; }
tail -1 $O/agg_atomic.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --op aggregate --steps 2 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
echo ALLDONE
