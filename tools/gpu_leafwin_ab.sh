#!/bin/bash
# GPU tests, then the one-window-per-block leaf staging (default: 4 waves per SIMD, w3: 3)
# against the last commit's two half-block windows (v_head): bench lines overlapped and
# sequential, and a FETCH_SIZE pass per library.  usage: bash tools/gpu_leafwin_ab.sh OUTDIR
set -u
OUT=${1:-gpurun_out/leafwin}; mkdir -p $OUT; export TMPDIR=/tmp
H=WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_head.so
W3=WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_w3.so
bash tools/gpu_tests.sh $OUT || exit $?
for lib in "new:RS2_X=1" "head:$H" "w3:$W3"; do
  label=${lib%%:*}; envs=${lib#*:}
  timeout -k 10 120 env $envs rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$label/p1" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --overlap off > "$OUT/pmc_$label.log" 2>&1 || { echo "pmc $label failed"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$label" | grep -A1 leaf_hash_kernel
done
bash tools/gpu_bench_ab.sh $OUT/ab "new:RS2_X=1" "head:$H" "w3:$W3" "new_seq:--overlap off" "head_seq:$H --overlap off" "w3_seq:$W3 --overlap off" "new2:RS2_X=1" "head2:$H" || exit $?
for f in $OUT/ab/*_seq.json; do python3 -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('$f', 'leaf_a', s['enc_leaf_hash_a'], 'leaf', s['enc_leaf_hash'])"; done
