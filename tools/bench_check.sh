#!/bin/bash
# One bench run into OUTDIR (repo root, on the box); prints value, cpu baseline and null fields.
OUT=${1:-gpurun_out/bench}; shift
mkdir -p "$OUT"
timeout -k 10 600 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; tail -3 "$OUT/bench.err"
[ $rc -ne 0 ] && exit $rc
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"], json.dumps(d["cpu_baseline"]))
print("null:", sorted(k for k, v in d.items() if v is None))
PY
