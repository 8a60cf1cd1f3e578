#!/bin/bash
# Leaf kernel occupancy vs its memory-side reads (is the 1.44x an L2-footprint effect?): the
# default (3 workgroups per CU, VGPR-bound) against LDS-padded builds with 2 and 1 workgroups
# per CU; FETCH_SIZE pass and sequential bench line each.  usage: bash tools/gpu_leafocc_ab.sh OUT
set -u
OUT=${1:-gpurun_out/leafocc}; mkdir -p $OUT; export TMPDIR=/tmp
for lib in "occ3:RS2_X=1" "occ2:WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_occ2.so" "occ1:WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_occ1.so"; do
  label=${lib%%:*}; envs=${lib#*:}
  timeout -k 10 120 env $envs rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$label/p1" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --overlap off > "$OUT/pmc_$label.log" 2>&1 || { echo "pmc $label failed"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$label" | grep -A1 leaf_hash_kernel
done
bash tools/gpu_bench_ab.sh $OUT/ab "occ3_seq:--overlap off" "occ2_seq:WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_occ2.so --overlap off" "occ1_seq:WALRUS_RS2_LIB=/root/repo/walrus_amd/libwalrus_rs2_v_occ1.so --overlap off" || exit $?
for f in $OUT/ab/*_seq.json; do python3 -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('$f', 'leaf_a', s['enc_leaf_hash_a'], 'leaf', s['enc_leaf_hash'])"; done
