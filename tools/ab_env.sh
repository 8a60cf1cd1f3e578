#!/bin/bash
# Env-knob A/B of the bench step: bash tools/ab_env.sh OUTDIR VAR "v1 v2 ..." [reps]
# (runs bench.py --steps 300 with the other legs off, once per value per rep)
OUT=$1; VAR=$2; VALS=$3; REPS=${4:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in $(seq 1 $REPS); do
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --cpu-baseline off \
    --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/$v.$rep.json" 2> "$OUT/$v.$rep.err"
  rc=$?
  echo "$VAR=$v rep=$rep rc=$rc $(python3 -c "import json; d=json.load(open('$OUT/$v.$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'])" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -3 "$OUT/$v.$rep.err"; exit $rc; }
done; done
exit 0
