# One GPU call: the whole -m gpu suite with margins recorded, the headline bench line (no CPU
# baselines) and a rocprof kernel trace of warm preprocess calls.  Usage: bash tools/gpu_r04.sh TAG [notests]
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
rc=0
if [ "${2:-}" != "notests" ]; then
  rm -f $O/margins.jsonl
  DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  tail -15 $O/gpu_tests.log
  python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
  echo "pytest rc=$rc"
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 120 python -u tools/first_call.py > $O/first_call.log 2>&1 || { echo first_call failed; tail -5 $O/first_call.log; exit 1; }
timeout -k 10 120 python -u tools/first_call.py --no-warmup >> $O/first_call.log 2>&1 || { echo first_call failed; tail -5 $O/first_call.log; exit 1; }
cat $O/first_call.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/profprep -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 3 --warmup 1 --prep 8 > $GRAFT_REPO_ROOT/$O/prof_prep.log 2>&1 ) || { echo "rocprof prep failed"; tail -5 $O/prof_prep.log; exit 1; }
tail -3 $O/prof_prep.log
exit $rc
