#!/bin/bash
# Round evidence on the GPU box, in the order the bench line needs it: parity tests, the PMC
# passes (per-stage HBM traffic and VALU counts, written to profiles/pmc_traffic.json, which
# bench.py reads for its roofline), the default bench line, then a rocprofv3 kernel trace of
# the bench command.  usage (repo root, on the box): bash tools/gpu_final.sh gpurun_out/TAG
set -u
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_run.sh "$OUT/pmc" || exit $?
python3 tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.txt" || exit $?
python3 tools/pmc_traffic.py "$OUT/pmc" "$OUT/pmc_traffic.json" > /dev/null || exit $?
cp "$OUT/pmc_traffic.json" profiles/pmc_traffic.json
echo "pmc ok"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
[ $rc -ne 0 ] && { tail -20 "$OUT/bench.err"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 30 --warmup 5 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "rocprof rc=$rc"
[ $rc -ne 0 ] && { tail -20 "$OUT/trace.err"; exit $rc; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/trace" -name '*kernel_trace.csv' -exec cp {} "$OUT/kernel_trace.csv" \;
python3 tools/trace_timed_avg.py "$OUT/kernel_trace.csv" --warmup 5 --steps 30 > "$OUT/timed_avg.json" && cat "$OUT/timed_avg.json"
cut -c1-160 "$OUT/kernel_stats.csv" | head -14
exit 0
