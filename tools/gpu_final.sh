# Round-end style refresh: GPU suite, smoke, bench (with CPU baselines), rocprof stats, PMC traffic,
# config 2, aggregate, 2-rank rehearsal, first-call diagnosis.  Usage: bash tools/gpu_final.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03z}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc FETCH_SIZE WRITE_SIZE || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
timeout -k 10 200 python -u bench.py --no-cpu --P 100000 --N 256000 --C 16 --steps 10 > $O/bench_config2.log 2>&1 && tail -1 $O/bench_config2.log > $O/bench_config2.json
timeout -k 10 400 python -u bench.py --op aggregate --steps 3 --warmup 1 > $O/bench_agg.log 2>&1 && tail -1 $O/bench_agg.log > $O/bench_agg.json
DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench2.log 2>&1 && tail -1 $O/bench2.log > $O/bench2_rehearsal.json
timeout -k 10 120 python -u tools/first_call.py tiny_first > $O/first_call_tiny.log 2>&1
timeout -k 10 120 python -u tools/first_call.py full > $O/first_call_full.log 2>&1
echo ALLDONE
