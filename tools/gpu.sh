#!/bin/bash
# The one GPU-box driver (repo root, on the box, via gpurun).  Every GPU step runs under its own
# time limit; the first failing step ends the call (no retries).
#
#   bash tools/gpu.sh OUT tests [pytest args...]     pytest -m gpu (default: the whole suite)
#   bash tools/gpu.sh OUT bench [bench.py args...]   one bench line -> OUT/bench.json
#   bash tools/gpu.sh OUT prof [bench.py args...]    rocprofv3 kernel trace + stats of a short
#                                                    bench -> OUT/kernel_stats.csv, timed_avg.json
#   bash tools/gpu.sh OUT pmc                        the HBM / VALU counter passes of
#                                                    tools/pmc_run.sh -> OUT/N.pmc_summary.txt and
#                                                    OUT/N.pmc_traffic.json (bench.py --pmc input;
#                                                    copy it to profiles/pmc_traffic.json)
#   bash tools/gpu.sh OUT ab VAR "v1 v2" [reps]      env-knob A/B of the bench step (other legs
#                                                    off unless $AB_LEGS says otherwise, 300
#                                                    steps), one line per value and rep
#   bash tools/gpu.sh OUT lib VARIANT_DIR bench ...  any of the above with another build of the
#                                                    library (WALRUS_RS2_LIB=VARIANT_DIR/libwalrus_rs2.so)
#   bash tools/gpu.sh OUT micro BIN [args...]        a tools/micro binary -> OUT/micro_BIN.txt
#   bash tools/gpu.sh OUT with VAR=VAL step ...      any step with an environment variable set
# Several steps chain with '+':  bash tools/gpu.sh OUT tests -k dist + bench --subsets fixed
set -u
OUT=${1:?usage: tools/gpu.sh OUT step [args] [+ step [args]]...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
SHORT_LEGS="--cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --node off"
SHORT="--steps 30 --warmup 5 $SHORT_LEGS"
n=0
run_step() {
  local step=$1
  shift
  n=$((n + 1))
  local tag="$OUT/$n.$step"
  case "$step" in
    tests)
      [ $# -eq 0 ] && set -- tests
      timeout -k 10 900 python3 -u -m pytest -m gpu -x -v --timeout 300 \
        --timeout-method thread "$@" > "$tag.log" 2>&1
      local rc=$?
      grep -E "FAILED|ERROR|passed|failed" "$tag.log" | tail -8
      return $rc ;;
    bench)
      timeout -k 10 500 python3 bench.py "$@" > "$tag.json" 2> "$tag.err"
      local rc=$?
      cat "$tag.json"
      [ $rc -ne 0 ] && tail -20 "$tag.err"
      return $rc ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$tag.d" -o run \
        -- python3 bench.py $SHORT "$@" > "$tag.json" 2> "$tag.err"
      local rc=$?
      [ $rc -ne 0 ] && { tail -20 "$tag.err"; return $rc; }
      find "$tag.d" -name '*kernel_stats.csv' -exec cp {} "$tag.kernel_stats.csv" \;
      find "$tag.d" -name '*kernel_trace.csv' -exec cp {} "$tag.kernel_trace.csv" \;
      python3 tools/trace_timed_avg.py "$tag.kernel_trace.csv" --warmup 5 --steps 30 \
        > "$tag.timed_avg.json" && cat "$tag.timed_avg.json"
      cut -c1-160 "$tag.kernel_stats.csv" | head -14
      return 0 ;;
    pmc)
      bash tools/pmc_run.sh "$tag.pmc" || return $?
      python3 tools/pmc_summary.py "$tag.pmc" > "$tag.pmc_summary.txt" || return $?
      python3 tools/pmc_traffic.py "$tag.pmc" "$tag.pmc_traffic.json" > /dev/null || return $?
      cat "$tag.pmc_traffic.json"
      return 0 ;;
    ab)
      local var=$1 vals=$2 reps=${3:-2}
      for rep in $(seq 1 "$reps"); do
        for v in $vals; do
          env "$var=$v" timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 ${AB_LEGS:-$SHORT_LEGS} \
            > "$tag.$v.$rep.json" 2> "$tag.$v.$rep.err"
          local rc=$?
          echo "$var=$v rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('$tag.$v.$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'])" 2>/dev/null)"
          [ $rc -ne 0 ] && { tail -3 "$tag.$v.$rep.err"; return $rc; }
        done
      done
      return 0 ;;
    micro)
      local bin=$1
      shift
      timeout -k 10 120 "tools/micro/bin/$bin" "$@" > "$tag.$bin.txt" 2>&1
      local rc=$?
      cat "$tag.$bin.txt"
      return $rc ;;
    with)
      local kv=$1
      shift
      ( export "$kv"; run_step "$@" )
      local rc=$?
      n=$((n + 1))  # the subshell's step took tag n+1
      return $rc ;;
    lib)
      local dir=$1
      shift
      WALRUS_RS2_LIB="$dir/libwalrus_rs2.so" run_step "$@"
      return $? ;;
    *)
      echo "unknown step $step"
      return 2 ;;
  esac
}
args=()
for a in "$@" "+"; do
  if [ "$a" = "+" ]; then
    [ ${#args[@]} -eq 0 ] && continue
    echo "== step ${args[*]}"
    run_step "${args[@]}" || { echo "step failed: ${args[*]}"; exit 1; }
    args=()
  else
    args+=("$a")
  fi
done
exit 0
