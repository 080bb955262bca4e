# One GPU call for an iteration: a test subset (pytest -k EXPR), the headline and thin bench
# lines, and kernel traces of warm preprocess calls (headline and thin fields).
# Usage: bash tools/gpu_quick.sh TAG [PYTEST_K]
set -u
cd $GRAFT_REPO_ROOT
T=${1:-q}
K=${2:-radix or thin}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "$K" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 || { echo aniso failed; tail -5 $O/bench_aniso25.log; exit 1; }
tail -1 $O/bench_aniso25.log
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profprep -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 3 --warmup 1 --prep 8 > $GRAFT_REPO_ROOT/$O/prof_prep.log 2>&1 ) || { echo "rocprof prep failed"; tail -5 $O/prof_prep.log; exit 1; }
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profthin -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 3 --warmup 1 --prep 4 --aniso 25 > $GRAFT_REPO_ROOT/$O/prof_thin.log 2>&1 ) || { echo "rocprof thin failed"; tail -5 $O/prof_thin.log; exit 1; }
echo done
