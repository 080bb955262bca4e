# Parity of the forward paths first, then A/B timing of the in-tree build against variants.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_multi.py tests/test_gpu_calltime.py tests/test_gpu_configs.py tests/test_gpu_spatial.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 700 python -u tools/ab.py --rounds 3 --kbench-args "--prep 7" ${AB:-base variants/head} > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
grep MEDIAN $O/ab.log
