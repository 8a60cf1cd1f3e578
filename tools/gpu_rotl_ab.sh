#!/bin/bash
# GPU tests, then Blake2b's rotate-left-by-one as one v_lshl_add_u64 + one shift (default)
# against two v_alignbit_b32 (RS2_ROTL1_ADD=0 build): main bench overlapped / sequential and C3.
# usage: bash tools/gpu_rotl_ab.sh OUTDIR
set -u
OUT=${1:-gpurun_out/rotl}; mkdir -p $OUT; export TMPDIR=/tmp
R0=WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_rot0.so
bash tools/gpu_tests.sh $OUT || exit $?
bash tools/gpu_bench_ab.sh $OUT/ab "new_seq:--overlap off" "rot0_seq:$R0 --overlap off" "new:RS2_X=1" "rot0:$R0" "new2_seq:--overlap off" "rot02_seq:$R0 --overlap off" || exit $?
for f in $OUT/ab/*_seq.json; do python3 -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('$f', 'leaf_a', s['enc_leaf_hash_a'], 'leaf', s['enc_leaf_hash'], 'trees', s['enc_merkle_trees'])"; done
for v in "new:RS2_X=1" "rot0:$R0" "new2:RS2_X=1" "rot02:$R0"; do
  label=${v%%:*}; envs=${v#*:}
  timeout -k 10 200 env $envs python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > $OUT/c3_$label.json 2> $OUT/c3_$label.err || { echo "c3 $label failed"; tail -5 $OUT/c3_$label.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/c3_$label.json')); c=d['c3_small_blobs']; print('c3 $label', c['encode_gibs'], c['ms_per_batch'], c['serial_reencode_matches'], c['batched_matches_streams'])"
done
