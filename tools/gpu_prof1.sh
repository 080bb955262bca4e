# rocprof kernel stats of kbench (render + warm preprocess) for the in-tree build, then A/B.
set -u
cd $GRAFT_REPO_ROOT
T=${T:-prof1}
O=gpurun_out/$T; mkdir -p $O
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python $GRAFT_REPO_ROOT/tools/kbench.py --steps 10 --warmup 2 --prep 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 ) || { echo rocprof failed; tail -5 $O/prof.log; exit 1; }
if [ -n "${AB:-}" ]; then
  timeout -k 10 700 python -u tools/ab.py --rounds 3 --kbench-args "--prep 7" $AB > $O/ab.log 2>&1 || { echo ab failed; tail -20 $O/ab.log; exit 1; }
  grep MEDIAN $O/ab.log
fi
echo ALLDONE
