# Full GPU suite, headline bench, rocprof kernel stats of the bench (render + a warm preprocess),
# config-2 bench.  Usage: bash tools/gpu_check2.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 10 --warmup 2 --prep 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 ) || { echo rocprof failed; tail -5 $O/prof.log; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu --P 100000 --N 256000 --C 16 --steps 10 > $O/bench_config2.log 2>&1 && tail -1 $O/bench_config2.log > $O/bench_config2.json
echo ALLDONE
