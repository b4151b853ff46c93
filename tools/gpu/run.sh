# One GPU call's steps, read from stdin, one per line (round 6: replaces the
# per-experiment r0*_*.sh scripts; tools/gpu/README.md maps the old names).
#
#   bash tools/gpu/run.sh OUTDIR <<'EOF'
#   tests                        # every -m gpu test (pytest.log)
#   tests  NAME  -k EXPR ...     # a subset; extra pytest args after the name
#   smoke                        # __graft_entry__.smoke()
#   bench  NAME  ARGS...         # python bench.py ARGS > NAME.json (one summary line printed)
#   prof   NAME  ARGS...         # rocprofv3 --kernel-trace --stats of bench.py ARGS -> NAME/,
#                                #   summaries of the timed window (tools/kernel_window.py)
#   pmc    NAME  CFG ARGS...     # PMC passes of bench.py --config CFG ARGS (tools/gpu/pmc.sh),
#                                #   summarised to NAME.traffic.json (tools/pmc_report.py)
#   ab     NAME  ROUNDS  LIB...  -- ARGS...
#                                # interleaved A/B: for each round, each library variant
#                                #   (cur = the in-tree library, X = noise-c_amd/ab/libnoise_aead_hip_X.so)
#                                #   runs bench.py ARGS -> NAME.jsonl
#   abargs NAME  ROUNDS  -- ARGS_A  ::  ARGS_B  [:: ARGS_C ...]
#                                # interleaved A/B of bench argument sets on the in-tree library
#                                #   (a set may start with VAR=value words: its environment)
#   cmd    NAME  SECONDS  COMMAND...   # any command, its own time limit, output NAME.log
#   EOF
#
# Every step runs under its own `timeout -k 10`; a step that times out,
# aborts or crashes (exit >= 124) ends the call — nothing more touches the
# GPU after it.  A failing test or a bench error (exit 1/2) is reported and
# the next step runs.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
O=$R/gpurun_out/${1:?usage: run.sh OUTDIR < steps}
mkdir -p "$O"
export TMPDIR=/tmp
FAILED=0

fatal() {  # rc: a timeout / kill / abort / crash ends the call
  [ "$1" -ge 124 ]
}

summ() {  # one line per bench JSON
  python3 - "$1" "$2" <<'PY'
import json, sys
n, p = sys.argv[1], sys.argv[2]
try:
    d = json.loads(open(p).read().strip().splitlines()[-1])
except Exception as e:
    print(n, "no line", e); sys.exit(0)
r = d.get("roofline") or {}
c = d.get("config") or {}
print(n, d.get("value"), d.get("unit"), "ms/step", d.get("ms_per_step"), "kernel", r.get("kernel"),
      "launch_ms", r.get("avg_launch_ms"), "frac", r.get("frac"), "seal", d.get("seal_gibs"),
      "open", d.get("open_gibs"), "verified", d.get("verified"), "order", (c.get("open_order") or "")[:14],
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
}

step() {  # kind name args...
  local kind=$1; shift
  local rc=0
  case $kind in
  tests)
    local name=${1:-pytest}; [ $# -gt 0 ] && shift
    timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -x --durations=15 --timeout 300 \
      --timeout-method thread -p no:cacheprovider "$@" > "$O/$name.log" 2>&1 || rc=$?
    echo "tests $name rc=$rc: $(tail -1 "$O/$name.log")"
    [ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)|Error" "$O/$name.log" | head -20 ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || rc=$?
    echo "smoke rc=$rc: $(tail -1 "$O/smoke.log")" ;;
  bench)
    local name=$1; shift
    timeout -k 10 400 python bench.py "$@" > "$O/$name.json" 2> "$O/$name.err" || rc=$?
    if [ $rc -eq 0 ]; then summ "$name" "$O/$name.json"; else echo "bench $name rc=$rc"; tail -5 "$O/$name.err"; fi ;;
  prof)
    local name=$1; shift
    ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- \
        python3 "$R/bench.py" "$@" > "$O/$name.json" 2> "$O/$name.err" ) || rc=$?
    if [ $rc -eq 0 ]; then
      summ "$name" "$O/$name.json"
      # the timed window: the last --steps dispatches of the line's kernel
      python3 - "$O/$name" "$O/$name.json" > "$O/$name.window.txt" 2>&1 <<'PY' || true
import json, subprocess, sys
d, j = sys.argv[1], sys.argv[2]
line = json.loads(open(j).read().strip().splitlines()[-1])
k = (line.get("roofline") or {}).get("kernel")
if k:
    subprocess.run([sys.executable, "tools/kernel_window.py", d, k, str(line["steps"]), d + "/kernel_stats_timed.csv"])
    print(open(d + "/kernel_stats_timed.csv").read())
PY
      head -8 "$O/$name.window.txt"
    else echo "prof $name rc=$rc"; tail -5 "$O/$name.err"; fi ;;
  pmc)
    local name=$1 cfg=$2; shift 2
    bash tools/gpu/pmc.sh "$cfg" "$O/pmc_$name" "$@" > "$O/pmc_$name.log" 2>&1 || rc=$?
    if [ $rc -eq 0 ]; then
      python3 tools/pmc_report.py "$O/pmc_$name" "$cfg" "$O/$name.traffic.json" > "$O/$name.pmc.txt" 2>&1 || true
      head -20 "$O/$name.pmc.txt"
    else echo "pmc $name rc=$rc"; tail -5 "$O/pmc_$name.log"; fi ;;
  ab)
    local name=$1 rounds=$2; shift 2
    local libs=""
    while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs="$libs $1"; shift; done
    [ "${1:-}" = "--" ] && shift
    local i v
    for i in $(seq "$rounds"); do
      for v in $libs; do
        if [ "$v" = cur ]; then unset NOISE_AEAD_LIB; else export NOISE_AEAD_LIB=$R/noise-c_amd/ab/libnoise_aead_hip_$v.so; fi
        timeout -k 10 400 python bench.py "$@" > "$O/$name.$v.$i.json" 2> "$O/$name.$v.$i.err" || rc=$?
        unset NOISE_AEAD_LIB
        if [ $rc -ne 0 ]; then echo "ab $name $v rc=$rc"; tail -5 "$O/$name.$v.$i.err"; fatal $rc && return $rc; rc=0; continue; fi
        python3 -c "import json,sys;d=json.loads(open('$O/$name.$v.$i.json').read().strip().splitlines()[-1]);d['ab']={'variant':'$v','round':$i};print(json.dumps(d))" >> "$O/$name.jsonl"
        summ "$name $v r$i" "$O/$name.$v.$i.json"
      done
    done ;;
  abargs)
    local name=$1 rounds=$2; shift 2; [ "${1:-}" = "--" ] && shift
    local sets=() cur="" a i k
    for a in "$@"; do
      if [ "$a" = "::" ]; then sets+=("$cur"); cur=""; else cur="$cur $a"; fi
    done
    sets+=("$cur")
    for i in $(seq "$rounds"); do
      for k in "${!sets[@]}"; do
        # leading VAR=value words of a set are its environment
        local envs=() args=() w
        for w in ${sets[$k]}; do
          if [ ${#args[@]} -eq 0 ] && [[ "$w" == [A-Z]*=* ]]; then envs+=("$w"); else args+=("$w"); fi
        done
        timeout -k 10 400 env "${envs[@]}" python bench.py "${args[@]}" > "$O/$name.$k.$i.json" 2> "$O/$name.$k.$i.err" || rc=$?
        if [ $rc -ne 0 ]; then echo "abargs $name $k rc=$rc"; tail -5 "$O/$name.$k.$i.err"; fatal $rc && return $rc; rc=0; continue; fi
        python3 -c "import json;d=json.loads(open('$O/$name.$k.$i.json').read().strip().splitlines()[-1]);d['ab']={'args':'''${sets[$k]}''','round':$i};print(json.dumps(d))" >> "$O/$name.jsonl"
        summ "$name [${sets[$k]} ] r$i" "$O/$name.$k.$i.json"
      done
    done ;;
  cmd)
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1 || rc=$?
    echo "cmd $name rc=$rc: $(tail -1 "$O/$name.log")" ;;
  *) echo "unknown step $kind"; rc=2 ;;
  esac
  return $rc
}

while read -r line; do
  case "$line" in ''|'#'*) continue;; esac
  # the line's words, shell quoting honoured ("-k 'a or b'")
  eval "set -- $line"
  step "$@" < /dev/null
  rc=$?
  if [ $rc -ne 0 ]; then
    FAILED=1
    if fatal $rc; then echo "step '$line' ended with rc=$rc: stopping (no further GPU work in this call)"; exit $rc; fi
  fi
done
echo "run.sh done (failures: $FAILED)"
