#!/bin/bash
# FETCH_SIZE per stage for env variants (one rocprofv3 pass each): tools/pmc_fetch_ab.sh OUT "label:ENV=.." ...
set -u
OUT=${1:-gpurun_out/fetch_ab}; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}
  for cnt in FETCH_SIZE WRITE_SIZE; do
    mkdir -p "$OUT/$label/$cnt"
    timeout -k 10 120 env $rest rocprofv3 --pmc $cnt --output-format csv -d "$OUT/$label/$cnt/p1" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --overlap off > "$OUT/$label/$cnt.log" 2>&1 || { echo "$label $cnt failed"; tail -5 "$OUT/$label/$cnt.log"; exit 1; }
  done
  mkdir -p "$OUT/$label/all"; cp -r "$OUT/$label/FETCH_SIZE/p1" "$OUT/$label/all/p1"; cp -r "$OUT/$label/WRITE_SIZE/p1" "$OUT/$label/all/p2"
  python3 tools/pmc_traffic.py "$OUT/$label/all" "$OUT/$label/traffic.json" > /dev/null
  python3 -c "
import json; d=json.load(open('$OUT/$label/traffic.json'))
print('$label', ' '.join('%s r%.0f w%.0f' % (k, d[k]['read_bytes_per_launch']/1e6, d[k]['write_bytes_per_launch']/1e6) for k in ('dec_codec','enc_cols_sys_codec','enc_rows_codec','enc_cols_rep_codec') if k in d))"
done
