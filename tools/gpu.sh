#!/bin/bash
# The one GPU-box runner (run through gpurun from the repo root; writes under gpurun_out/TAG).
# Round 6 folded the 43 one-off tools/gpu_*.sh lease scripts of rounds 1-5 into these steps;
# the old scripts are in git history (git log -- tools/gpu_r05final.sh ...).
#
#   bash tools/gpu.sh tests   TAG              pytest -m gpu (margins -> TAG/margins.json)
#   bash tools/gpu.sh smoke   TAG              __graft_entry__.smoke()
#   bash tools/gpu.sh bench   TAG [ARGS...]    one bench.py line (CPU baselines unless --no-cpu)
#   bash tools/gpu.sh prof    TAG [ARGS...]    rocprofv3 --kernel-trace --stats of bench.py --no-cpu ARGS
#   bash tools/gpu.sh pmc     TAG [ARGS...]    FETCH_SIZE / WRITE_SIZE passes (traffic.json input)
#   bash tools/gpu.sh sq      TAG [ARGS...]    the SQ issue / wait counters, two passes
#   bash tools/gpu.sh ab      TAG VARIANT...   tools/ab.py: headline and --aniso 25 medians
#   bash tools/gpu.sh graph   TAG              the graph-capture probes (tools/graph_probe2.py)
#   bash tools/gpu.sh final   TAG              the round's refresh, part 1: tests (margins) and smoke
#   bash tools/gpu.sh lines   TAG              part 2: every bench line (headline with the PIGS graph,
#                                              thin, config 2, call-time) with traces, PMC traffic, SQ
#                                              counters and the 2-rank rehearsal
# Every GPU step runs under its own timeout; the first failure ends the call.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CMD=$1; TAG=$2; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
R=$GRAFT_REPO_ROOT

step_tests() {
    rm -f "$O/margins.jsonl"
    DGS_MARGINS=$O/margins.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 \
        --timeout-method thread > "$O/gpu_tests.log" 2>&1
    local rc=$?
    tail -4 "$O/gpu_tests.log"
    python tools/margins_summary.py "$O/margins.jsonl" > "$O/margins.json"
    return $rc
}
step_smoke() {
    timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { echo smoke failed; tail -5 "$O/smoke.log"; return 1; }
    echo smoke ok
}
step_bench() {  # NAME ARGS...
    local n=$1; shift
    timeout -k 10 400 python -u bench.py "$@" > "$O/bench_$n.log" 2>&1 \
        || { echo "bench $n failed"; tail -5 "$O/bench_$n.log"; return 1; }
    grep '^{' "$O/bench_$n.log" | tail -1 > "$O/bench_$n.json"
    echo "bench $n: $(python -c "import json,sys; j=json.load(open('$O/bench_$n.json')); print(j['ms_per_step'], 'ms/step', j.get('kernels_ms'))")"
}
step_prof() {  # NAME ARGS...
    local n=$1; shift
    ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_$n" -o run \
        -- python "$R/bench.py" --no-cpu "$@" > "$R/$O/prof_$n.log" 2>&1 ) || { echo "prof $n failed"; return 1; }
    grep '^{' "$O/prof_$n.log" | tail -1 > "$O/bench_under_rocprof_$n.json"
    echo "prof $n ok"
}
step_pmc() {  # NAME ARGS...
    local n=$1; shift
    PMC_ARGS="--steps 2 --warmup 1 --no-cpu $*" bash tools/pmc_passes.sh "$R/$O/pmc_$n" FETCH_SIZE WRITE_SIZE \
        || { echo "pmc $n failed"; return 1; }
    python tools/pmc_summary.py "$O/pmc_$n" > "$O/pmc_${n}_summary.txt" 2>&1
    echo "pmc $n ok"
}
step_sq() {  # NAME ARGS...
    local n=$1; shift
    local P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
    local P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
    PMC_ARGS="--steps 2 --warmup 1 --no-cpu $*" bash tools/pmc_passes.sh "$R/$O/sq_$n" "$P1" "$P2" \
        || { echo "sq $n failed"; return 1; }
    python tools/pmc_summary.py "$O/sq_$n" > "$O/sq_${n}_summary.txt" 2>&1
    echo "sq $n ok"
}
step_ab() {
    timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 20 --warmup 10" base "$@" \
        > "$O/ab_head.log" 2>&1 || { echo ab failed; tail -5 "$O/ab_head.log"; return 1; }
    grep MEDIAN "$O/ab_head.log"
    timeout -k 10 400 python -u tools/ab.py --rounds 3 --kbench-args "--steps 10 --warmup 5 --aniso 25" base "$@" \
        > "$O/ab_thin.log" 2>&1 || { echo ab failed; tail -5 "$O/ab_thin.log"; return 1; }
    grep MEDIAN "$O/ab_thin.log"
}
step_graph() {
    for sc in torch_recipe dgs_recipe torch_eager_then_capture dgs_eager_then_capture dgs_after_history; do
        timeout -k 10 120 python -u tools/graph_probe2.py $sc > "$O/$sc.log" 2>&1
        local rc=$?
        echo "$sc rc=$rc: $(tail -1 "$O/$sc.log")"
        case $rc in 0|1) ;; *) echo "stopping after rc=$rc"; return 3;; esac
    done
}

case $CMD in
    tests) step_tests ;;
    smoke) step_smoke ;;
    bench) step_bench main "$@" ;;
    prof) step_prof main "$@" ;;
    pmc) step_pmc main "$@" ;;
    sq) step_sq main "$@" ;;
    ab) step_ab "$@" ;;
    graph) step_graph ;;
    final)  # (two gpurun calls: each stays within gpurun's 20-minute limit)
        { step_tests; [ $? -le 1 ]; } && step_smoke && echo ALLDONE ;;
    lines)
        step_bench head --pigs-graph \
        && step_prof head \
        && step_bench thin --aniso 25 \
        && step_prof thin --aniso 25 \
        && step_bench config2 --P 100000 --N 256000 --C 16 \
        && step_bench calltime --calltime --steps 5 --warmup 1 \
        && step_pmc head && step_pmc thin --aniso 25 && step_pmc config2 --P 100000 --N 256000 --C 16 \
        && step_sq head \
        && { DGS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 \
                 > "$O/bench2.log" 2>&1 && grep '^{' "$O/bench2.log" | tail -1 > "$O/bench2_rehearsal.json"; } \
        && echo ALLDONE ;;
    *) echo "unknown step $CMD"; exit 2 ;;
esac
