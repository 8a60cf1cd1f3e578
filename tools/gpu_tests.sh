#!/bin/bash
# Full GPU test suite into OUTDIR/pytest.log (repo root, on the box).  usage: tools/gpu_tests.sh OUTDIR [-k EXPR]
OUT=${1:-gpurun_out/tests}; shift
mkdir -p "$OUT" && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -8; exit $rc
