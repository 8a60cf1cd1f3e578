#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel stats of the bench + PMC passes.
# usage (repo root, on the box): bash tools/profile_round.sh gpurun_out/prof_rNN
set -u
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --host-io off --c3 off > "$OUT/trace.log" 2>&1 || { echo "trace rc=$?"; tail -5 "$OUT/trace.log"; exit 1; }
echo "trace ok"
bash tools/pmc_run.sh "$OUT/pmc"
