# One GPU call: rerun the listed tests, a kernel trace of the thin (--aniso 25) preprocess, and an
# A/B of the thin binning against variants.  Usage: bash tools/gpu_r05b.sh TAG "PYTEST_K" VARIANTS...
set -u
cd $GRAFT_REPO_ROOT
T=$1; K=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
DGS_MARGINS=$O/margins.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
rc=$?
tail -8 $O/gpu_tests.log
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o thin -- python3 tools/kbench.py --steps 3 --warmup 1 --prep 4 --aniso 25 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
tail -2 $O/prof.log
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 10 --warmup 2 --prep 6 --aniso 25" base "$@" > $O/ab.log 2>&1 || { echo ab failed; tail -5 $O/ab.log; exit 1; }
tail -12 $O/ab.log
exit $rc
