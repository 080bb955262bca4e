# Secondary bench lines: D = 3 volume (128^3 third, 256^3 gaussian), aggregate (config 5).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${T:-benches3}; mkdir -p $O
timeout -k 10 300 python -u bench.py --op volume --function third --grid3 128 --steps 3 --warmup 1 --no-cpu > $O/vol128_third.log 2>&1 && tail -1 $O/vol128_third.log > $O/vol128_third.json || { echo vol128 failed; tail -5 $O/vol128_third.log; exit 1; }
timeout -k 10 300 python -u bench.py --op volume --function gaussian --grid3 256 --steps 3 --warmup 1 --no-cpu > $O/vol256.log 2>&1 && tail -1 $O/vol256.log > $O/vol256.json || { echo vol256 failed; tail -5 $O/vol256.log; exit 1; }
timeout -k 10 400 python -u bench.py --op aggregate --steps 3 --warmup 1 > $O/agg.log 2>&1 && tail -1 $O/agg.log > $O/agg.json || { echo agg failed; tail -5 $O/agg.log; exit 1; }
echo ALLDONE
