# The bench line as the driver runs it (--steps 20 --warmup 5, CPU baselines included), and a
# 2-rank rehearsal on the one GPU (both ranks on cuda:0).  Usage: bash tools/gpu_settle.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r04s}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench2.log 2>&1 || { echo bench2 failed; tail -5 $O/bench2.log; exit 1; }
tail -1 $O/bench2.log
echo ALLDONE
