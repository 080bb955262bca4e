# HIP calls inside a stream capture (tools/graph_probe3.py), safest first; stops at the first crash.
# Usage: bash tools/gpu_graph_probe3.sh TAG
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-gp3}
mkdir -p $O
for sc in plain memset malloc_only malloc_free raise_inside sync_inside; do
  timeout -k 10 120 python -u tools/graph_probe3.py $sc > $O/$sc.log 2>&1
  rc=$?
  echo "$sc rc=$rc: $(grep "$sc:" $O/$sc.log | tail -1)"
  case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; exit 0;; esac
done
