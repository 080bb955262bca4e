# One GPU call: the -m gpu suite (margins recorded; optional -k filter), the headline and thin
# (--aniso 25) bench lines.  Usage: bash tools/gpu_r05.sh TAG [PYTEST_K|notests]
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r05}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rc=0
if [ "${2:-}" != "notests" ]; then
  rm -f $O/margins.jsonl
  K=${2:-}
  DGS_MARGINS=$O/margins.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/gpu_tests.log 2>&1
  rc=$?
  tail -15 $O/gpu_tests.log
  python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
  echo "pytest rc=$rc"
  [ $rc -le 1 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 || { echo aniso failed; tail -5 $O/bench_aniso25.log; exit 1; }
tail -1 $O/bench_aniso25.log
exit $rc
