#!/bin/bash
# Round evidence on the GPU box: parity tests + bench + rocprofv3 kernel stats (gpu_round.sh),
# then the PMC passes and the per-stage HBM traffic table bench.py reads.
# usage (repo root, on the box): bash tools/gpu_full.sh gpurun_out/TAG
set -u
OUT=${1:-gpurun_out/full}
bash tools/gpu_round.sh "$OUT" || exit $?
bash tools/pmc_run.sh "$OUT/pmc" || exit $?
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.txt" || exit $?
python3 tools/pmc_traffic.py "$OUT/pmc" "$OUT/pmc_traffic.json" > /dev/null || exit $?
echo "pmc ok"
