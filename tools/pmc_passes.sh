#!/bin/bash
# Collects PMC counter passes for the bench workload (one rocprofv3 run per pass).
# usage: tools/pmc_passes.sh OUTDIR "pass1 counters" "pass2 counters" ...
# PMC_SCRIPT (default bench.py) and PMC_ARGS select the profiled python program.
set -u
OUT=$1; shift
mkdir -p "$OUT"; cd /tmp
i=0
for pass in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o run -- \
      python "$GRAFT_REPO_ROOT/${PMC_SCRIPT:-bench.py}" ${PMC_ARGS:---steps 2 --warmup 1 --no-cpu} > "$OUT/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
