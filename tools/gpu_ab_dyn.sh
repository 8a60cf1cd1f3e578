#!/bin/bash
# Dynamic-tile pipelined encode: GPU suite, then the step A/B over RS2_PIPE_DYN x decode priority.
OUT=${1:-gpurun_out/dyn}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for pr in 0 -1; do
  RS2_DEC_PRIORITY=$pr bash tools/ab_env.sh "$OUT/ab_pr$pr" RS2_PIPE_DYN "0 1" 2 || exit $?
done
