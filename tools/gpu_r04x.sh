# Steady-state check and PMC traffic at HEAD: the driver's bench command (warmup 5), the same
# after 60 warmup steps, a kernel trace of 80 steps (per-call durations over a long run), and
# FETCH_SIZE / WRITE_SIZE passes of the render kernels.  Usage: bash tools/gpu_r04x.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r04x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 5 > $O/bench_w5.log 2>&1 || { echo bench failed; tail -5 $O/bench_w5.log; exit 1; }
tail -1 $O/bench_w5.log
timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 60 > $O/bench_w60.log 2>&1 || { echo bench failed; tail -5 $O/bench_w60.log; exit 1; }
tail -1 $O/bench_w60.log
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/long -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 80 --warmup 5 > $GRAFT_REPO_ROOT/$O/long.log 2>&1 ) || { echo "rocprof long failed"; tail -5 $O/long.log; exit 1; }
grep '^{' $O/long.log | tail -1
PMC_ARGS="--steps 2 --warmup 1 --no-cpu" bash tools/pmc_passes.sh $GRAFT_REPO_ROOT/$O/pmc FETCH_SIZE WRITE_SIZE || { echo pmc failed; exit 1; }
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
head -30 $O/pmc_summary.txt
echo ALLDONE
