# round-6 probe: the leaf kernel with and without its L2 re-fetch
# (RS2_ABL_LEAF_LINE variant: line-aligned windows, same instruction stream), timing + FETCH_SIZE
set -u
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
SL="--cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --node off"
for rep in 1 2; do
for v in default leafline; do
  if [ $v = default ]; then L=walrus_amd/libwalrus_rs2.so; else L=walrus_amd/libwalrus_rs2_v_leafline.so; fi
  WALRUS_RS2_LIB=$L timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 $SL > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -5 $O/$v.$rep.err; exit 1; }
  python3 -c "
import json
p=json.load(open('$O/$v.$rep.json'))
s=p['stages_ms_solo']
print('$v rep $rep value', p['value'], 'leaf_a solo', s.get('enc_leaf_hash_a'), 'leaf_c solo', s.get('enc_leaf_hash'), 'step leaf_a', p['stages_ms_per_step'].get('enc_leaf_hash_a'))
"
done
done
for v in default leafline; do
  if [ $v = default ]; then L=walrus_amd/libwalrus_rs2.so; else L=walrus_amd/libwalrus_rs2_v_leafline.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    WALRUS_RS2_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$v/p_$c -o run -- python3 bench.py --steps 2 --warmup 1 $SL --overlap off > $O/pmc_$v.$c.log 2>&1 || { tail -5 $O/pmc_$v.$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $O/pmc_$v $O/pmc_$v.traffic.json > /dev/null && python3 -c "
import json
d=json.load(open('$O/pmc_$v.traffic.json'))
for k in ('enc_leaf_hash_a','enc_leaf_hash'): print('$v', k, d.get(k))
"
done
