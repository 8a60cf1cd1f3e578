#!/bin/bash
# Read-request sizes at the L2's memory side (is the leaf kernels' 1.4-1.6x
# FETCH_SIZE over-fetch real or an artefact of the x2 correction?).  FETCH_SIZE tallies every
# TCC_EA0_RDREQ at 64 B; here the requests are split by size (32 / 64 / 128 B), on the
# calibration kernels of tools/micro/fetchbench (known byte counts) and on the bench workload.
# usage (repo root, on the box): bash tools/pmc_reqsize.sh OUTDIR
set -u
OUT=${1:-gpurun_out/reqsize}
mkdir -p "$OUT"
export TMPDIR=/tmp
A="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_BUBBLE_sum"
B="TCC_EA0_RDREQ_128B_sum FETCH_SIZE"
i=0
for grp in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d "$OUT/fb/p$i" -o run -- \
    ./tools/micro/fetchbench > "$OUT/fb_p$i.log" 2>&1
  rc=$?; echo "fetchbench pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/fb_p$i.log"; exit $rc; }
done
i=0
for grp in "$A" "$B"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/bench/p$i" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --overlap off > "$OUT/bench_p$i.log" 2>&1
  rc=$?; echo "bench pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_p$i.log"; exit $rc; }
done
python3 tools/pmc_summary.py "$OUT/fb" > "$OUT/fb_summary.txt"
python3 tools/pmc_summary.py "$OUT/bench" > "$OUT/bench_summary.txt"
exit 0
