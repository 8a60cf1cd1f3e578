#!/bin/bash
# Stream / hardware-queue A/B of the bench step: RS2_BENCH_MAIN (stream | perset) x
# GPU_MAX_HW_QUEUES (HIP's default 4, 8, 16).  usage: bash tools/gpu_ab_queues.sh OUTDIR
OUT=${1:-gpurun_out/queues}; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for m in stream perset; do for q in 4 8 16; do
  tag=${m}_q$q.$rep
  RS2_BENCH_MAIN=$m GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 \
    --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  rc=$?
  echo "$tag rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/$tag.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['decode_roundtrip_ok'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 "$OUT/$tag.err"; exit $rc; }
done; done; done
exit 0
