# Graph-capture probes (tools/graph_probe2.py), safest first; stops at the first crash.
# Usage: bash tools/gpu_graph_probe.sh TAG
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gp}
mkdir -p $O
for sc in torch_recipe dgs_recipe torch_eager_then_capture dgs_eager_then_capture dgs_after_history; do
  timeout -k 10 120 python -u tools/graph_probe2.py $sc > $O/$sc.log 2>&1
  rc=$?
  echo "$sc rc=$rc: $(tail -1 $O/$sc.log)"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit 3;; esac
done
