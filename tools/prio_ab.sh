set -u
mkdir -p gpurun_out/prio
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline off --host-io off --c3 off --steps 30"
run() { timeout -k 10 120 env $2 $B > gpurun_out/prio/$1.json 2>/dev/null && python3 -c "import json;d=json.load(open('gpurun_out/prio/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
run base1 X=0 && run side1 RS2_SIDE_PRIORITY=1 && run dec1 RS2_DEC_PRIORITY=-1 && run both1 "RS2_SIDE_PRIORITY=1 RS2_DEC_PRIORITY=-1" && \
run base2 X=0 && run side2 RS2_SIDE_PRIORITY=1 && run dec2 RS2_DEC_PRIORITY=-1 && run both2 "RS2_SIDE_PRIORITY=1 RS2_DEC_PRIORITY=-1"
