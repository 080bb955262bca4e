# Extra bench lines on one GPU: thin Gaussians (axis ratios to 25), the call-time path.
# Usage: bash tools/gpu_lines.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu --aniso 25 > $O/bench_aniso25.log 2>&1 || { echo aniso failed; tail -5 $O/bench_aniso25.log; exit 1; }
tail -1 $O/bench_aniso25.log > $O/bench_aniso25.json; cat $O/bench_aniso25.json
timeout -k 10 600 python -u bench.py --no-cpu --calltime --steps 5 > $O/bench_calltime.log 2>&1 || { echo calltime failed; tail -5 $O/bench_calltime.log; exit 1; }
tail -1 $O/bench_calltime.log > $O/bench_calltime.json; cat $O/bench_calltime.json
