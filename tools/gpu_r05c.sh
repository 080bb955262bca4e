# One GPU call: the whole -m gpu suite (margins recorded), a kernel trace of the thin (--aniso 25)
# preprocess + render, and the headline / thin bench lines.  Usage: bash tools/gpu_r05c.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=$1
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/margins.jsonl
DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -x > $O/gpu_tests.log 2>&1
rc=$?
tail -8 $O/gpu_tests.log
python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o thin --output-format csv -- python3 tools/kbench.py --steps 3 --warmup 1 --prep 4 --aniso 25 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
tail -1 $O/prof.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { echo bench failed; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 || { echo aniso failed; tail -5 $O/bench_aniso25.log; exit 1; }
tail -1 $O/bench_aniso25.log
exit $rc
