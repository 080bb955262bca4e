# Aggregate backward ablations (DGS_AGG_EXPT) and the D = 3 256^3 lines.  Usage: bash tools/gpu_agg_vol.sh TAG
set -u
cd $GRAFT_REPO_ROOT
T=${1:-r03v}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --op aggregate --steps 3 --warmup 1 --no-cpu > $O/agg.log 2>&1 || { echo agg failed; tail -5 $O/agg.log; exit 1; }
tail -1 $O/agg.log
DGS_AGG_EXPT=1 timeout -k 10 300 python -u bench.py --op aggregate --steps 3 --warmup 1 --no-cpu > $O/agg_noscatter.log 2>&1 || { echo agg1 failed; exit 1; }
tail -1 $O/agg_noscatter.log
DGS_AGG_EXPT=3 timeout -k 10 300 python -u bench.py --op aggregate --steps 3 --warmup 1 --no-cpu > $O/agg_noscatter_nodt.log 2>&1 || { echo agg3 failed; exit 1; }
tail -1 $O/agg_noscatter_nodt.log
timeout -k 10 500 python -u bench.py --op volume --grid3 256 --steps 2 --warmup 1 --pre-reps 2 --no-cpu > $O/vol256_gaussian.log 2>&1 || { echo vol256 failed; tail -5 $O/vol256_gaussian.log; exit 1; }
tail -1 $O/vol256_gaussian.log
timeout -k 10 500 python -u bench.py --op volume --grid3 256 --function third --steps 2 --warmup 1 --pre-reps 2 --no-cpu > $O/vol256_third.log 2>&1 || { echo vol256 third failed; tail -5 $O/vol256_third.log; exit 1; }
tail -1 $O/vol256_third.log
echo ALLDONE
