# One GPU call: the -m gpu suite, A/B of variants (thin and headline), a thin kernel trace.
# Usage: bash tools/gpu_r05e.sh TAG VARIANTS...
set -u
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/margins.jsonl
DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -x > $O/gpu_tests.log 2>&1
rc=$?
tail -4 $O/gpu_tests.log
python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
if [ $# -gt 0 ]; then
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 10 --warmup 2 --prep 6 --aniso 25" base "$@" > $O/ab_thin.log 2>&1 || { echo ab failed; tail -5 $O/ab_thin.log; exit 1; }
grep MEDIAN $O/ab_thin.log
timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 20 --warmup 5 --prep 6" base "$@" > $O/ab_head.log 2>&1 || { echo ab failed; tail -5 $O/ab_head.log; exit 1; }
grep MEDIAN $O/ab_head.log
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o thin --output-format csv -- python3 tools/kbench.py --steps 3 --warmup 1 --prep 4 --aniso 25 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
tail -1 $O/prof.log
exit $rc
