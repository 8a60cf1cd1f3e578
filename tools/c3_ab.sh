#!/bin/bash
# C3 leg A/B over engine knobs: one bench line each (short main step, C3 leg only)
OUT=gpurun_out/c3ab; mkdir -p $OUT; export TMPDIR=/tmp
for spec in "all:" "noaux:RS2_TAIL_AUX=0" "nosplit:RS2_SPLIT_LEAF=0" "none:RS2_TAIL_AUX=0 RS2_SPLIT_LEAF=0"; do
  label=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 200 env $envs python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > $OUT/$label.json 2> $OUT/$label.err || { echo "$label failed"; tail -5 $OUT/$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$label.json'))['c3_small_blobs']; print('$label', d['encode_gibs'], d['encode_gibs_streams'])"
done
