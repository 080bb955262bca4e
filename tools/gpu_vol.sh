# D = 3: the volume GPU tests, then the 128^3 third and 64^3 gaussian bench lines.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${T:-vol}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_volume.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --op volume --function third --grid3 128 --steps 3 --warmup 1 --no-cpu > $O/vol128_third.log 2>&1 && tail -1 $O/vol128_third.log > $O/vol128_third.json || { echo vol128 failed; tail -5 $O/vol128_third.log; exit 1; }
timeout -k 10 300 python -u bench.py --op volume --function gaussian --grid3 64 --steps 3 --warmup 1 --no-cpu > $O/vol64.log 2>&1 && tail -1 $O/vol64.log > $O/vol64.json || { echo vol64 failed; tail -5 $O/vol64.log; exit 1; }
python3 - <<'PY'
import json
for f in ["vol128_third", "vol64"]:
    d = json.load(open(f"gpurun_out/vol/{f}.json"))
    print(f, round(d["ms_per_step"], 1), d["phases_ms"], d["roofline"]["frac"])
PY
