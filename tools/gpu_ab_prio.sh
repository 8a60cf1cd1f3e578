#!/bin/bash
# Encode-stream priority A/B: RS2_MAIN_PRIORITY (bench main stream) x RS2_SIDE_PRIORITY (the split
# encode's side stream).  usage: bash tools/gpu_ab_prio.sh OUTDIR
OUT=${1:-gpurun_out/prio}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for mp in 0 -1; do for sp in 0 1; do
  tag=m${mp}_s$sp.$rep
  RS2_MAIN_PRIORITY=$mp RS2_SIDE_PRIORITY=$sp timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 \
    --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  rc=$?
  echo "$tag rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['decode_roundtrip_ok'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 "$OUT/$tag.err"; exit $rc; }
done; done; done
exit 0
