#!/bin/bash
# GPU tests, then the C3 leg with the register-only small-symbol leaf kernel vs the LDS-window
# kernel (RS2_SMALL_LEAF=0).
set -u
OUT=${1:-gpurun_out/smallleaf}; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_tests.sh $OUT || exit $?
for v in "small:RS2_X=1" "lds:RS2_SMALL_LEAF=0" "small2:RS2_X=1" "lds2:RS2_SMALL_LEAF=0"; do
  label=${v%%:*}; envs=${v#*:}
  timeout -k 10 200 env $envs python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > $OUT/c3_$label.json 2> $OUT/c3_$label.err || { echo "c3 $label failed"; tail -5 $OUT/c3_$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$label.json')); c=d['c3_small_blobs']; print('c3 $label', c['encode_gibs'], c['ms_per_batch'], c['serial_reencode_matches'], c['batched_matches_streams'], 'main', d['value'])"
done
