set -u
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline off --host-io off --c3 off"
run() { timeout -k 10 120 $B $2 > gpurun_out/pipe/$1.json 2>gpurun_out/pipe/$1.err && python3 -c "import json;d=json.load(open('gpurun_out/pipe/$1.json'));print('$1',d['value'],d['ms_per_step'],d['decode_roundtrip_ok'],d['roofline']['ms_per_launch'])"; }
run p1 "--pipeline 1" && run p2 "--pipeline 2" && run p1b "--pipeline 1" && run p2b "--pipeline 2"
rc=$?; [ $rc -ne 0 ] && tail -5 gpurun_out/pipe/*.err; exit $rc
