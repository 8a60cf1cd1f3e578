# round-6 probe: hash x2 parity tests + C3 A/B (RS2_HASH_X2=1 default vs 0)
set -u
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_variants.py tests/test_gpu_smoke_parity.py tests/test_gpu_recovery.py tests/test_gpu_metadata.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SL="--cpu-baseline off --host-io off --c4 off --host-abi off --quilt off --node off"
for rep in 1 2; do
for v in 1 0; do
RS2_HASH_X2=$v timeout -k 10 300 python3 bench.py --steps 300 --warmup 10 $SL > $O/x2_$v.$rep.json 2> $O/x2_$v.$rep.err || { tail -5 $O/x2_$v.$rep.err; exit 1; }
python3 -c "
import json
p=json.load(open('$O/x2_$v.$rep.json'))
print('X2=$v rep $rep value', p['value'], 'c3', p['c3_small_blobs']['encode_gibs'], p['c3_small_blobs']['ms_per_batch'], 'trees', p['stages_ms_solo'].get('enc_merkle_trees'), 'leaf', p['stages_ms_solo'].get('enc_leaf_hash'))
"
done
done
