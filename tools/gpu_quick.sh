#!/bin/bash
# Quick GPU iteration: gpu parity tests, then the bench line without the CPU / host-IO legs.
# usage (repo root, on the box): bash tools/gpu_quick.sh gpurun_out/TAG
set -u
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --cpu-baseline off --host-io off > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
[ $rc -ne 0 ] && { tail -20 "$OUT/bench.err"; exit $rc; }
exit 0
