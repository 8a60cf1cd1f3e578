# needs the RS2_MAIN_PRIORITY knob (main stream = torch.cuda.Stream(priority)) from the experiment, since removed from bench.py
set -u
mkdir -p gpurun_out/prio3
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline off --host-io off --c3 off --quilt off"
run() { timeout -k 10 120 env $2 $B > gpurun_out/prio3/$1.json 2>gpurun_out/prio3/$1.err && python3 -c "import json;d=json.load(open('gpurun_out/prio3/$1.json'));print('$1',d['value'],d['ms_per_step'],d['decode_roundtrip_ok'])" || { tail -5 gpurun_out/prio3/$1.err; exit 1; }; }
run base X=0 && run main_lo RS2_MAIN_PRIORITY=1 && run main_0 RS2_MAIN_PRIORITY=0 && run main_lo_dec_hi "RS2_MAIN_PRIORITY=1 RS2_DEC_PRIORITY=-1" && run base2 X=0 && run main_lo2 RS2_MAIN_PRIORITY=1
