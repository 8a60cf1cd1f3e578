#!/bin/bash
# A/B the bench over library variants: tools/ab_variants.sh OUT lib1.so lib2.so ...
OUT=$1; shift
mkdir -p "$OUT"
for rep in 1 2; do
for lib in "$@"; do
  name=$(basename "$lib" .so)
  WALRUS_RS2_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --host-io off --c3 off > "$OUT/$name.$rep.json" 2> "$OUT/$name.$rep.err"
  rc=$?
  echo "$name rep=$rep rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.$rep.json')); print(d['value'], d['stages_ms_per_step'])" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -3 "$OUT/$name.$rep.err"; exit $rc; fi
done; done
