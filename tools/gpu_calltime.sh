# Kernel trace of the call-time path (tools/calltime_bench.py).  Usage: bash tools/gpu_calltime.sh TAG [ARGS]
set -u
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/calltime_bench.py "$@" > $O/ct.log 2>&1 || { echo ct failed; tail -5 $O/ct.log; exit 1; }
tail -1 $O/ct.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/tools/calltime_bench.py "$@" > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 ) || { echo "rocprof failed"; tail -3 $O/prof.log; exit 1; }
python - <<'PY'
import csv, glob, os
f = glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", os.environ.get("T_TAG", ""), "**", "run_kernel_stats.csv"), recursive=True)
PY
head -12 $O/prof/run_kernel_stats.csv | cut -c1-200
