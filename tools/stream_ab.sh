#!/bin/bash
# A/B of the bench's stream layout (RS2_BENCH_MAIN / RS2_BENCH_DEC / --overlap); one line each.
set -u
OUT=${1:-gpurun_out/stream_ab}
mkdir -p "$OUT"
for cfg in "null 2 on" "stream 2 on" "null 1 on" "stream 1 on" "null 2 off"; do
  set -- $cfg
  RS2_BENCH_MAIN=$1 RS2_BENCH_DEC=$2 timeout -k 10 120 python3 bench.py --steps 300 --warmup 10 \
    --overlap $3 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off \
    > "$OUT/$1_$2_$3.json" 2> "$OUT/$1_$2_$3.err" || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/$1_$2_$3.json')); print('$cfg', d['value'], d['ms_per_step'], d['decode_roundtrip_ok'])"
done
