# Full GPU suite + SQ counters of the render and preprocess kernels (tools/kbench.py).  Usage: bash tools/gpu_pmc_fwd.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03f}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
T=$T/pmc bash tools/gpu_pmc2.sh > $O/pmc.log 2>&1 || { echo pmc failed; tail -5 $O/pmc.log; exit 1; }
cat $O/pmc/summary.txt | head -120
echo ALLDONE
