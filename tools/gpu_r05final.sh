# Round-5 final refresh at HEAD: the full -m gpu suite (margins), smoke, the bench line with CPU
# baselines, its kernel trace, the thin line and its trace, PMC traffic of both, the call-time
# and PIGS-graph lines.  Usage: bash tools/gpu_r05final.sh TAG [notests]
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r05z}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ "${2:-}" != "notests" ]; then
rm -f $O/margins.jsonl
DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
[ $rc -le 1 ] || exit $rc
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py --pigs-graph > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
grep '^{' $O/prof_bench.log | tail -1 > $O/bench_under_rocprof.json
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 && tail -1 $O/bench_aniso25.log > $O/bench_aniso25.json || { echo aniso failed; exit 1; }
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_thin -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu --aniso 25 > $GRAFT_REPO_ROOT/$O/prof_thin.log 2>&1 ) || { echo "rocprof thin failed"; exit 1; }
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc FETCH_SIZE WRITE_SIZE || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --aniso 25" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc_thin FETCH_SIZE WRITE_SIZE || { echo pmc thin failed; exit 1; }
python tools/pmc_summary.py $O/pmc_thin > $O/pmc_thin_summary.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --calltime --steps 5 --warmup 1 > $O/bench_calltime.log 2>&1 && tail -1 $O/bench_calltime.log > $O/bench_calltime.json || { echo calltime failed; exit 1; }
DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench2.log 2>&1 && tail -1 $O/bench2.log > $O/bench2_rehearsal.json
echo ALLDONE
