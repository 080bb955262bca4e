# A/B timing only (no tests): tools/ab.py over $AB (default: base vs variants/head).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab1; mkdir -p $O
timeout -k 10 700 python -u tools/ab.py --rounds 3 --kbench-args "--prep 7" ${AB:-base variants/head} > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
grep MEDIAN $O/ab.log
