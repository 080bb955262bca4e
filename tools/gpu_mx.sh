set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/mx; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_golden.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/ab.py --rounds 3 --kbench-args "--P 100000 --N 256000 --C 16" base variants/mx0 > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
grep MEDIAN $O/ab.log
