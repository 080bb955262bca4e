# rocprofv3 kernel trace + stats of the headline bench command (the summary behind the bench
# line's roofline), and the bench line itself.  Usage: bash tools/gpu_benchprof.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-bp}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/benchprof -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/benchprof.log 2>&1 ) || { echo "rocprof bench failed"; tail -5 $O/benchprof.log; exit 1; }
grep '^{' $O/benchprof.log | tail -1
echo done
