#!/bin/bash
# The one gpurun driver: every GPU step is a subcommand, run under its own time
# limit, chained with && so the first failure (fault, abort, timeout) ends the call.
#
#   gpurun --timeout 900 -- bash tools/gpu.sh NAME STEP [STEP ...]
#
# Outputs go to gpurun_out/NAME/.  A STEP is one shell word (quote it when it
# has arguments); the arguments after ':' are split on spaces:
#   tests[:K]           pytest -m gpu (-k K when given)
#   smoke               __graft_entry__.smoke()
#   'bench:ARGS'        bench.py --gpus 1 --steps 20 --warmup 5 (ARGS replace the defaults)
#   'probe:SCRIPT ARGS' python tools/SCRIPT ARGS      (stdout -> NAME/probe_SCRIPT.log)
#   'prof:SCRIPT ARGS'  rocprofv3 --kernel-trace --stats of python tools/SCRIPT ARGS,
#                       summarised by tools/prof_summary.py (-> NAME/prof_SCRIPT.md)
#   'pmc:CTRS SCRIPT ARGS'  one rocprofv3 --pmc pass (CTRS joined by '+') over tools/SCRIPT
#   step                prof of the GPT-2-medium training step (tools/train_probe.py)
#   'stepab:C1 C2 ..'   in-process GPT-2-medium step under each env config Ci (K=V[;K=V..]),
#                       ROUNDS (default 3) interleaved rounds of STEPS (default 20) steps
#   'resab:C1 C2 ..'    the same for the ResNet-50 step (tools/bench_resnet.py)
#   'soab:SCRIPT ARGS'  A/B built extensions: every ab/*.so (env:AB_GLOB=ab/x_*.so to pick) in turn
#                       over the tree's _pdo_hip.so, python tools/SCRIPT ARGS with each, 2 rounds; restored after
#   env:K=V             export K=V for the following steps
set -o pipefail
NAME=${1:?name}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$NAME; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
PMC_PASS=0
BENCH_PASS=0
PROF_PASS=0
say() { echo "[gpu.sh $(date +%H:%M:%S)] $*"; }

run_step() {
  local step=$1 kind=${1%%:*} arg=""
  [[ $step == *:* ]] && arg=${step#*:}
  read -r -a A <<< "$arg"
  case $kind in
    env) export "$arg"; say "env $arg" ;;
    tests)
      local k=(); [[ -n $arg ]] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/pytest_gpu.log" 2>&1 || { tail -60 "$O/pytest_gpu.log"; return 1; }
      tail -3 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { tail -40 "$O/smoke.log"; return 1; }
      tail -2 "$O/smoke.log" ;;
    bench)
      BENCH_PASS=$((BENCH_PASS + 1))
      local b=(--gpus 1 --steps 20 --warmup 5); [[ -n $arg ]] && b=("${A[@]}")
      local bj=$O/bench.json be=$O/bench.err
      (( BENCH_PASS > 1 )) && { bj=$O/bench$BENCH_PASS.json; be=$O/bench$BENCH_PASS.err; }
      timeout -k 10 600 python bench.py "${b[@]}" > "$bj" 2> "$be" \
        || { tail -60 "$be"; return 1; }
      cat "$bj" ;;
    probe)
      local s=${A[0]}
      timeout -k 10 600 python -u "tools/$s" "${A[@]:1}" > "$O/probe_${s%.py}.log" 2>&1 \
        || { tail -40 "$O/probe_${s%.py}.log"; return 1; }
      cat "$O/probe_${s%.py}.log" ;;
    prof|step)
      PROF_PASS=$((PROF_PASS + 1))
      local s=${A[0]:-train_probe.py} rest=("${A[@]:1}")
      [[ $kind == step ]] && { s=train_probe.py; rest=(--dist --steps 7 --warmup 2); }
      local tag=prof${PROF_PASS}_${s%.py}   # numbered: several passes in one call keep their tables
      local d=$O/$tag
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$d" -o run -- python3 "$R/tools/$s" "${rest[@]}" ) \
        > "$O/$tag.log" 2>&1 || { tail -30 "$O/$tag.log"; return 1; }
      local db; db=$(find "$d" -name '*.db' | head -1)
      local steps=0; [[ $kind == step ]] && steps=9  # 2 warmup + 7 timed steps are all traced; 0 = count AdamW dispatches
      python3 tools/prof_summary.py "$db" --steps $steps --top 40 > "$O/$tag.md" &&
        { [[ $kind != step ]] || python3 tools/prof_sequence.py "$db" --last 800 --list > "$O/$tag.seq.md"; } && rm -rf "$d"
      tail -5 "$O/$tag.log"; head -45 "$O/$tag.md" ;;
    pmc)
      PMC_PASS=$((PMC_PASS + 1))
      local ctr=${A[0]//+/ } s=${A[1]} p=$O/pmc${PMC_PASS}_${A[1]%.py}
      ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d "$p" -o run -- python3 "$R/tools/$s" "${A[@]:2}" ) \
        > "$p.log" 2>&1 || { tail -30 "$p.log"; return 1; }
      python3 tools/pmc_summary.py $(find "$p" -name "*.db") > "$p.md" 2>&1 && rm -rf "$p"; head -60 "$p.md" ;;
    stepab)
      local round cfg
      for round in $(seq 1 "${ROUNDS:-3}"); do
        for cfg in "${A[@]}"; do
          ( IFS=';'; for kv in $cfg; do export "$kv"; done
            timeout -k 10 300 python tools/train_probe.py --dist --steps "${STEPS:-20}" --warmup 3 ) \
            > "$O/stepab.json" 2> "$O/stepab.err" || { tail -30 "$O/stepab.err"; return 1; }
          echo "$round [$cfg] $(tail -1 "$O/stepab.json")"
        done
      done ;;
    resab)
      local round cfg
      for round in $(seq 1 "${ROUNDS:-3}"); do
        for cfg in "${A[@]}"; do
          ( IFS=';'; for kv in $cfg; do export "$kv"; done
            timeout -k 10 300 python tools/bench_resnet.py --steps 20 --warmup 5 ) \
            > "$O/resab.json" 2> "$O/resab.err" || { tail -30 "$O/resab.err"; return 1; }
          echo "$round [$cfg] $(tail -1 "$O/resab.json")"
        done
      done ;;
    soab)
      local so=paddle_operator_amd/_pdo_hip.so round v out rc=0
      cp "$so" "$O/.tree_hip.so"
      for round in 1 2; do
        for v in ${AB_GLOB:-ab/*.so}; do
          cp "$v" "$so"
          out=$(timeout -k 10 300 python "tools/${A[0]}" "${A[@]:1}" 2> "$O/soab.err") || { rc=1; tail -20 "$O/soab.err"; break 2; }
          echo "$round $(basename "$v" .so) $out"
        done
      done
      cp "$O/.tree_hip.so" "$so"; rm -f "$O/.tree_hip.so"
      return $rc ;;
    *) say "unknown step $step"; return 2 ;;
  esac
}

for st in "$@"; do
  say "step $st"
  run_step "$st" || { say "step $st failed"; exit 1; }
done
say "done"
