#!/bin/bash
# Instruction-cache counters for the bench workload (two passes, one counter group each).
# usage: tools/pmc_icache.sh OUTDIR
set -u
OUT=${1:-gpurun_out/pmc_ic}; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for grp in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --overlap off > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"; grep -A5 -E "^(rs2_decode|rs2_encode_shared|rs2_encode_mixed|leaf_hash)" "$OUT/summary.txt"
