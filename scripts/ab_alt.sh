#!/bin/bash
# Alternating same-box A/B of library variants / environment settings (bench
# lines only): bash scripts/ab_alt.sh <tag> <rounds> <variant>...
# variant: base | lib:<name> (ablibs/libnerf_pl_amd_<name>.so) | env:<VAR=value>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
tag=$1; rounds=$2; shift 2
out=gpurun_out/r04/abalt_$tag
mkdir -p "$out"
for ((i = 1; i <= rounds; i++)); do
  for v in "$@"; do
    envs=()
    case "$v" in
      base) ;;
      lib:*) envs=(NERF_PL_AMD_LIB=$PWD/ablibs/libnerf_pl_amd_${v#lib:}.so) ;;
      env:*) envs=("${v#env:}") ;;
    esac
    name=$(echo "$v" | tr ':=/' '___')_$i
    env "${envs[@]}" timeout -k 10 200 python bench.py --fp32-leg-steps 0 --cpu-baseline-seconds 0 ${BENCH_ARGS:-} > "$out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(grep -h '^{' "$out/$name.log" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); r=j["rooflines"]; print(j["value"], j["ms_per_step"], *[(k, r[k]["avg_launch_ms"]) for k in r])' 2>/dev/null)"
    if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; exit $rc; fi
  done
done
