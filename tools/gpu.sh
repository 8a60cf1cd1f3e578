#!/bin/bash
# Run a command on the GPU box via gpurun; re-request the box (never re-run a started command)
# only when gpurun reports the infrastructure failed before the command ran (status=transient).
# usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpu.sh] attempt $attempt: infrastructure not ready, waiting" >&2
    sleep 75
    continue
  fi
  echo "$out"
  exit 0
done
echo "[gpu.sh] gave up after repeated infrastructure failures" >&2
echo "$out"
exit 3
