#!/bin/bash
# rocprofv3 kernel stats + PMC passes of the bench workload alone (no CPU / host-IO / C3 legs).
# usage (repo root, on the box): bash tools/profile_clean.sh gpurun_out/TAG
set -u
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --cpu-baseline off --host-io off --c3 off > "$OUT/trace_bench.json" 2> "$OUT/trace.err" \
  || { echo "trace rc=$?"; tail -5 "$OUT/trace.err"; exit 1; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
bash tools/pmc_run.sh "$OUT/pmc" || exit $?
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.txt" || exit $?
python3 tools/pmc_traffic.py "$OUT/pmc" "$OUT/pmc_traffic.json" > /dev/null || exit $?
echo "profile ok"
