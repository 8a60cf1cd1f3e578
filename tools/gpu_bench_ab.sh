#!/bin/bash
# Bench A/B lines only (no tests): bash tools/gpu_bench_ab.sh OUTDIR "label:ENV=.. ARGS" ...
set -u
OUT=${1:-gpurun_out/ab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}
  envs=""; args=""
  for w in $rest; do case $w in *=*) envs="$envs $w";; *) args="$args $w";; esac; done
  timeout -k 10 150 env $envs python3 bench.py $args --steps 300 --warmup 10 --cpu-baseline off \
    --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "$label failed"; tail -5 "$OUT/$label.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$label.json')); s=d['stages_ms_solo'] or d['stages_ms_per_step']; print('$label', d['value'], d['ms_per_step'], d['decode_roundtrip_ok'], 'cols_sys', s['enc_cols_sys_codec'], 'rows', s['enc_rows_codec'], 'cols_rep', s['enc_cols_rep_codec'], 'dec', s['dec_codec'])"
done
