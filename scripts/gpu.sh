#!/bin/bash
# The one driver of GPU-box work (replaces the per-round drivers of rounds 3-4):
#
#   bash scripts/gpu.sh <tag> <step> [<step> ...]          outputs: gpurun_out/$R/<tag>/ (R: round, default r06)
#
# Steps run in order, each under its own time limit; the first failing step
# ends the call (no GPU work after a fault, an abort or a time limit).
#   tests           the GPU suite in one process ($TESTS: a subset)    (tests.log)
#   smoke           __graft_entry__.smoke()                            (smoke.log)
#   bench           the default bench line; extra flags: $BENCH_ARGS   (bench.json)
#   benches         cfg3, cfg4, cfg5, cfg5 --grad-on-light, eval lines (bench_<cfg>.json)
#   stats           rocprofv3 --kernel-trace --stats of a short bench run (stats/)
#   sq              two SQ counter passes over bench's step (sq_a/, sq_b/; scripts/sq_report.py)
#   traffic         FETCH_SIZE and WRITE_SIZE passes, separate runs (fetch/, write/; scripts/traffic.py)
#   abalt:<n>:<v,v> alternating same-box A/B bench lines, n rounds; variant base |
#                   lib:<name> (ablibs/libnerf_pl_amd_<name>.so) | env:<VAR=value>
#   dist            bench.py's distributed path: 4 gloo ranks x cfg4, 2 x cfg2, 4 x cfg5
#                   --grad-on-light --light-shard, RCCL at one rank
#   gaps:<bench args, _ for spaces>   a kernel trace of 10 steps (scripts/gaps.py)
#   trained         2000 training steps that save their weights, then the step on them
#                   (dev/trained_step.py)
#   defer_sweep     the deferral crossover on weights after 100 / 300 / 1000 / 2000 steps
#   randperm        VERDICT r4 item 6: the pre-fix sampler's 64M device randperm, kernel trace
#   emptylist       VERDICT r4 item 5: listed launches with 0 / 20% / all samples listed (dev/empty_list_probe.py)
# Every profiling pass is its own rocprofv3 run with --kernel-trace only besides --pmc.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${R:-r06}
tag=$1; shift
out=gpurun_out/$R/$tag
mkdir -p "$out"

run() {  # run <name> <timeout> <cmd...>: stdout to <name>.log, stops the call on failure
    local name=$1 to=$2; shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(grep -h '^{' "$out/$name.log" 2>/dev/null | head -c 200)"
    if [ $rc -ne 0 ]; then tail -15 "$out/$name.log"; exit $rc; fi
}
json() { grep -h '^{' "$out/$1.log" > "$out/$1.json"; }
# a short bench run to profile: both arithmetics (main region f16x3, the exact-fp32 leg)
B="bench.py --steps 3 --warmup 2 --fp32-leg-steps 3 --cpu-baseline-seconds 0 --no-kernel-timing ${BENCH_ARGS:-}"
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"

for step in "$@"; do
  case "$step" in
  tests)
    run tests 1000 python -u -m pytest ${TESTS:-tests} -m gpu -q -x -rA --timeout 200 --timeout-method thread \
      -p no:cacheprovider ;;
  smoke)
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    run bench 400 python bench.py ${BENCH_ARGS:-}; json bench ;;
  benches)
    for c in cfg3 cfg4 cfg5 cfg5gol eval; do
      a="--config $c"; [ $c = cfg5gol ] && a="--config cfg5 --grad-on-light"
      run bench_$c 300 python bench.py $a --cpu-baseline-seconds 0; json bench_$c
    done ;;
  stats)
    run stats 300 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 --no-kernel-timing ${BENCH_ARGS:-} ;;
  sq)
    run sq_a 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU \
      GRBM_GUI_ACTIVE -d "$out/sq_a" -o run --output-format csv -- python $B
    run sq_b 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
      -d "$out/sq_b" -o run --output-format csv -- python $B ;;
  traffic)
    run fetch 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/fetch" -o run --output-format csv -- python $B
    run write 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$out/write" -o run --output-format csv -- python $B ;;
  abalt:*)
    IFS=: read -r _ rounds vs <<< "$step"
    for ((i = 1; i <= rounds; i++)); do
      for v in ${vs//,/ }; do
        envs=()
        case "$v" in
          base) ;;
          lib:*) envs=(NERF_PL_AMD_LIB=$PWD/ablibs/libnerf_pl_amd_${v#lib:}.so) ;;
          env:*) envs=("${v#env:}") ;;
        esac
        name=ab_$(echo "$v" | tr ':=/' '___')_$i
        run "$name" 200 env "${envs[@]}" python bench.py --fp32-leg-steps 0 --cpu-baseline-seconds 0 ${BENCH_ARGS:-}
        grep -h '^{' "$out/$name.log" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); r=j["rooflines"]; f=j.get("fp32_leg") or {}; print(j["value"], j["ms_per_step"], *[(k, r[k]["avg_launch_ms"]) for k in r], "| fp32 leg", f.get("value"), *[(k, v["avg_launch_ms"]) for k, v in (f.get("rooflines") or {}).items()])' || true
      done
    done ;;
  dist)
    NR_BENCH_DIST_BACKEND=gloo run cfg4_gloo4 500 $TR --nproc-per-node 4 --master-port 29621 \
      bench.py --gpus 4 --config cfg4
    NR_BENCH_DIST_BACKEND=gloo run cfg2_gloo2 300 $TR --nproc-per-node 2 --master-port 29622 bench.py --gpus 2
    NR_BENCH_DIST_BACKEND=gloo run cfg5_gol_shard_gloo4 500 $TR --nproc-per-node 4 --master-port 29623 \
      bench.py --gpus 4 --config cfg5 --grad-on-light --light-shard --light-importance -1
    NR_BENCH_FORCE_DIST=1 run cfg2_rccl1 300 $TR --nproc-per-node 1 --master-port 29624 \
      bench.py --cpu-baseline-seconds 0 ;;
  gaps:*)
    a=${step#gaps:}; a=${a//_/ }
    n=gaps_$(ls -d "$out"/gaps_* 2>/dev/null | wc -l)
    echo "$a" > "$out/$n.args"
    run "$n" 240 rocprofv3 --kernel-trace -d "$out/$n" -o run --output-format csv -- \
      python bench.py $a --steps 10 --warmup 3 --fp32-leg-steps 0 --cpu-baseline-seconds 0 --no-kernel-timing ;;
  trained)
    run train 300 python scripts/psnr_compare.py --impl ours --steps 2000 --eval-every 500 --draw-seed 7 \
      --save-weights "$out/w7.safetensors" --out "$out/train_s7.json"
    run trained_step 300 python dev/trained_step.py "$out/w7.safetensors" --steps 40 --out "$out/trained_step.json" ;;
  defer_sweep)
    for st in 100 300 1000 2000; do
      run train_$st 200 python scripts/psnr_compare.py --impl ours --steps $st --eval-every $st --draw-seed 7 \
        --save-weights "$out/w_$st.safetensors" --out "$out/train_$st.json"
      run step_$st 200 python dev/trained_step.py "$out/w_$st.safetensors" --steps 40 --modes all,none,auto \
        --out "$out/step_$st.json"
    done ;;
  emptylist)
    for f in 0 0.2 1; do
      run empty_$f 200 rocprofv3 --kernel-trace --stats -d "$out/empty_$f" -o run --output-format csv -- \
        python dev/empty_list_probe.py --frac $f
    done ;;
  randperm)
    run randperm 300 rocprofv3 --kernel-trace --stats -d "$out/randperm" -o probe --output-format csv -- \
      python -u dev/randperm_probe.py --out "$out/randperm_probe.json" ;;
  *)
    echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo done
