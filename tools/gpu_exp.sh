#!/bin/bash
# One experiment session: quick parity subset, bench variants (one line each), phase stamps.
# usage: bash tools/gpu_exp.sh OUTDIR "label:ENV=.. ARGS" ...
set -u
OUT=${1:-gpurun_out/exp}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fixture or smoke or blocks or c1_device or checks or partition" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}
  envs=""; args=""
  for w in $rest; do case $w in *=*) envs="$envs $w";; *) args="$args $w";; esac; done
  timeout -k 10 150 env $envs python3 bench.py $args --steps 300 --warmup 10 --cpu-baseline off \
    --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "$label failed"; tail -5 "$OUT/$label.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$label.json')); print('$label', d['value'], d['ms_per_step'], d['decode_roundtrip_ok'], json.dumps(d['stages_ms_solo'] or d['stages_ms_per_step']))"
done
if [ -f walrus_amd/libwalrus_rs2_stamps.so ]; then
  rm -f "$OUT/stamps.bin"
  RS2_STAMP_FILE="$OUT/stamps.bin" timeout -k 10 120 python3 tools/stamps_run.py > "$OUT/stamps_run.log" 2>&1 && \
    python3 tools/stamps_summary.py "$OUT/stamps.bin" > "$OUT/stamps.txt"
  grep -E "^==|decode ok" "$OUT/stamps.txt" "$OUT/stamps_run.log"
fi
exit 0
