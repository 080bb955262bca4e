#!/bin/bash
# PMC passes over tools/kbench.py (one rocprofv3 run per pass; at most 8 SQ counters a pass).
# usage: tools/pmc_kbench.sh OUTDIR "pass1 counters" "pass2 counters" ...
set -u
OUT=$1; shift
mkdir -p "$OUT"; cd /tmp
i=0
for pass in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- \
      python "$GRAFT_REPO_ROOT/tools/kbench.py" --steps 3 --warmup 1 > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
