# One GPU call: the whole -m gpu suite with every parity check's margin recorded
# (tests/helpers.close -> $DGS_MARGINS), folded into margins.json.  Usage: bash tools/gpu_margins.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
rm -f $O/margins.jsonl
DGS_MARGINS=$O/margins.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -25 $O/gpu_tests.log
python tools/margins_summary.py $O/margins.jsonl > $O/margins.json
echo "pytest rc=$rc"
exit $rc
