# One GPU call: the new / changed tests first, then the whole -m gpu suite, the headline bench
# and the 2-rank spatial rehearsal (gloo, both ranks on the one GPU).  Usage: bash tools/gpu_check.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_spatial.py tests/test_gpu_volume.py -x -v --timeout 300 --timeout-method thread > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -30 $O/new_tests.log; exit 1; }
tail -1 $O/new_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench2.log 2>&1 || { echo bench2 failed; tail -20 $O/bench2.log; exit 1; }
tail -1 $O/bench2.log > $O/bench2_rehearsal.json
echo ALLDONE
