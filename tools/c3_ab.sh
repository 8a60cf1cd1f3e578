#!/bin/bash
# C3 leg A/B over engine knobs / library variants: one bench line each (short main step, C3 leg
# only).  usage: tools/c3_ab.sh OUTDIR "label:ENV=.." ...
OUT=${1:-gpurun_out/c3ab}; shift; mkdir -p $OUT; export TMPDIR=/tmp
[ $# -eq 0 ] && set -- "all:" "noaux:RS2_TAIL_AUX=0" "nosplit:RS2_SPLIT_LEAF=0" "none:RS2_TAIL_AUX=0 RS2_SPLIT_LEAF=0"
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 200 env $envs python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > $OUT/$label.json 2> $OUT/$label.err || { echo "$label failed"; tail -5 $OUT/$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$label.json')); c=d['c3_small_blobs']; print('$label', c['encode_gibs'], c['encode_gibs_streams'], d['value'], d['stages_ms_per_step'].get('enc_merkle_trees'))"
done
