# Round-5 measurement refresh at HEAD: smoke, the bench line (with CPU baselines), its kernel
# trace, PMC traffic of the headline and of the thin (--aniso 25) workload, the thin, call-time
# and config-2 lines, and the 2-rank rehearsal.  Usage: bash tools/gpu_r05m.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r05m}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json; cat $O/bench.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu > $GRAFT_REPO_ROOT/$O/prof_bench.log 2>&1 ) || { echo "rocprof failed"; exit 1; }
tail -1 $O/prof_bench.log > $O/bench_under_rocprof.json
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc FETCH_SIZE WRITE_SIZE || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --aniso 25" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc_thin FETCH_SIZE WRITE_SIZE || { echo pmc thin failed; exit 1; }
python tools/pmc_summary.py $O/pmc_thin > $O/pmc_thin_summary.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 && tail -1 $O/bench_aniso25.log > $O/bench_aniso25.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_thin -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu --aniso 25 --steps 10 > $GRAFT_REPO_ROOT/$O/prof_thin.log 2>&1 ) || { echo "rocprof thin failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --calltime --steps 5 --warmup 1 > $O/bench_calltime.log 2>&1 && tail -1 $O/bench_calltime.log > $O/bench_calltime.json
timeout -k 10 200 python -u bench.py --no-cpu --P 100000 --N 256000 --C 16 --steps 10 > $O/bench_config2.log 2>&1 && tail -1 $O/bench_config2.log > $O/bench_config2.json
DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench2.log 2>&1 && tail -1 $O/bench2.log > $O/bench2_rehearsal.json
echo ALLDONE
