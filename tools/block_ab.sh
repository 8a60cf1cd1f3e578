set -u
mkdir -p gpurun_out/blk
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline off --host-io off --c3 off"
run() { timeout -k 10 120 env $2 $B > gpurun_out/blk/$1.json 2>gpurun_out/blk/$1.err && python3 -c "import json;d=json.load(open('gpurun_out/blk/$1.json'));print('$1',d['value'],d['ms_per_step'],d['decode_roundtrip_ok'],d['stages_ms_solo'])"; }
run b512 X=0 && run b256 RS2_BLOCK_MAX=256 && run b128 RS2_BLOCK_MAX=128
