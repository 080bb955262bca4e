# Round-5 refresh of the lines that changed after a2c2e38 and of the off-headline paths: thin
# (--aniso 25) line + kernel trace + PMC, call-time line, config-2 line + PMC, the aggregation
# (config 5) and D = 3 lines.  Usage: bash tools/gpu_r05n.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r05n}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 && tail -1 $O/bench_aniso25.log > $O/bench_aniso25.json || { echo aniso failed; exit 1; }
cat $O/bench_aniso25.json | cut -c1-200
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_thin -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu --aniso 25 --steps 10 > $GRAFT_REPO_ROOT/$O/prof_thin.log 2>&1 ) || { echo "rocprof thin failed"; exit 1; }
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --aniso 25" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc_thin FETCH_SIZE WRITE_SIZE || { echo pmc thin failed; exit 1; }
python tools/pmc_summary.py $O/pmc_thin > $O/pmc_thin_summary.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --calltime --steps 5 --warmup 1 > $O/bench_calltime.log 2>&1 && tail -1 $O/bench_calltime.log > $O/bench_calltime.json || { echo calltime failed; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu --P 100000 --N 256000 --C 16 --steps 10 > $O/bench_config2.log 2>&1 && tail -1 $O/bench_config2.log > $O/bench_config2.json || { echo config2 failed; exit 1; }
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --P 100000 --N 256000 --C 16" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc_c2 FETCH_SIZE WRITE_SIZE || { echo pmc c2 failed; exit 1; }
python tools/pmc_summary.py $O/pmc_c2 > $O/pmc_c2_summary.txt 2>&1
timeout -k 10 400 python -u bench.py --op aggregate --steps 3 --warmup 1 > $O/bench_agg.log 2>&1 && tail -1 $O/bench_agg.log > $O/bench_agg.json || { echo agg failed; exit 1; }
timeout -k 10 300 python -u bench.py --op volume --grid3 64 --steps 3 --warmup 1 --no-cpu > $O/bench_vol64.log 2>&1 && tail -1 $O/bench_vol64.log > $O/bench_vol64.json || { echo vol failed; exit 1; }
echo ALLDONE
