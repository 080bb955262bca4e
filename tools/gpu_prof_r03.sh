# Round-3 profile refresh at HEAD: rocprof kernel stats of the bench, a kernel trace of warm
# preprocess calls, PMC traffic of the render kernels.  Usage: bash tools/gpu_prof_r03.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03p}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu > $O/prof_bench.log 2>&1 ) || { echo "rocprof bench failed"; tail -5 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profprep -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 1 --warmup 1 --prep 8 > $O/prof_prep.log 2>&1 ) || { echo "rocprof prep failed"; tail -5 $O/prof_prep.log; exit 1; }
tail -2 $O/prof_prep.log
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $O/pmc FETCH_SIZE WRITE_SIZE || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt | head -30
echo ALLDONE
