#!/bin/bash
# GPU tests, then A/B of the in-tree library against walrus_amd/libwalrus_rs2_head.so (the last
# commit's build): main bench lines and the C3 batch leg.  usage: tools/gpu_lib_ab.sh OUTDIR
set -u
OUT=${1:-gpurun_out/libab}; mkdir -p $OUT; export TMPDIR=/tmp
HEAD=/root/repo/walrus_amd/libwalrus_rs2_head.so
bash tools/gpu_tests.sh $OUT || exit $?
bash tools/gpu_bench_ab.sh $OUT/ab "new:RS2_X=1" "head:WALRUS_RS2_LIB=$HEAD" "new_seq:--overlap off" "head_seq:WALRUS_RS2_LIB=$HEAD --overlap off" || exit $?
for v in "new:RS2_X=1" "head:WALRUS_RS2_LIB=$HEAD" "new2:RS2_X=1" "head2:WALRUS_RS2_LIB=$HEAD"; do
  label=${v%%:*}; envs=${v#*:}
  timeout -k 10 200 env $envs python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > $OUT/c3_$label.json 2> $OUT/c3_$label.err || { echo "c3 $label failed"; tail -5 $OUT/c3_$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$label.json')); c=d['c3_small_blobs']; print('c3 $label', c['encode_gibs'], c['ms_per_batch'], c['serial_reencode_matches'], c['batched_matches_streams'])"
done
