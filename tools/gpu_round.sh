#!/bin/bash
# One GPU-box session: gpu parity tests, the bench line, a rocprofv3 kernel-trace summary of
# the same bench command.  Every GPU step has its own time limit; the first failure ends it.
# usage (repo root, on the box): bash tools/gpu_round.sh gpurun_out/TAG [skip-tests]
set -u
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && exit $rc
fi
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
cut -c1-160 "$OUT/kernel_stats.csv" | head -12
exit 0
