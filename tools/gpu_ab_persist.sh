#!/bin/bash
# Persistent-decode A/B: variant parity test, then the bench step with RS2_DEC_PERSIST unset / 1.
OUT=${1:-gpurun_out/persist}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/variants.log" 2>&1
rc=$?; tail -2 "$OUT/variants.log"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh "$OUT/ab" RS2_DEC_PERSIST "0 1" 2
