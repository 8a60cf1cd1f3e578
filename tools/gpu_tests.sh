#!/bin/bash
# GPU tests only (optionally a -k selection): bash tools/gpu_tests.sh gpurun_out/TAG [pytest -k expr]
set -u
OUT=${1:-gpurun_out/tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${2:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$2" > "$OUT/pytest_gpu.log" 2>&1
else
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; exit $rc
