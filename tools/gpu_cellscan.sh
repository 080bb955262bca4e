# Fine-cell size scan at the headline (DGS_CELL_TARGET: mean samples per fine cell), settled bench
# lines.  Usage: bash tools/gpu_cellscan.sh TAG "130 150 175"
set -u
cd $GRAFT_REPO_ROOT
T=${1:-cs}
O=gpurun_out/$T
mkdir -p $O
for t in ${2:-130 150 175}; do
  DGS_CELL_TARGET=$t timeout -k 10 200 python -u bench.py --no-cpu --steps 20 --warmup 5 > $O/bench_$t.log 2>&1 || { echo "bench $t failed"; tail -5 $O/bench_$t.log; exit 1; }
  python3 -c "
import json,sys
j=json.loads(open('$O/bench_$t.log').read().strip().splitlines()[-1])
print('$t', round(j['ms_per_step'],4), j['kernels_ms'], 'prep', round(j['preprocess_ms'],4), 'total', round(j['total_ms_per_step_incl_preprocess'],4), 'cells', j['entries']['fine_cells'], 'E', j['entries']['fine_entries'])"
done
echo ALLDONE
