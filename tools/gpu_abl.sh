#!/bin/bash
# Ablation A/B: sequential per-stage times (--overlap off) of library variants.
# usage (repo root, on the box): bash tools/gpu_abl.sh OUTDIR lib1.so lib2.so ...
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
for lib in "$@"; do
  name=$(basename "$lib" .so)
  WALRUS_RS2_LIB=$lib timeout -k 10 200 python3 bench.py --steps 60 --warmup 5 --overlap off \
    --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off \
    > "$OUT/$name.$rep.json" 2> "$OUT/$name.$rep.err"
  rc=$?
  echo "$name rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/$name.$rep.json')); s=d['stages_ms_per_step']; print(d['value'], {k: s[k] for k in s if 'codec' in k or 'hash' in k or 'tree' in k})" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 "$OUT/$name.$rep.err"; exit $rc; }
done; done
exit 0
