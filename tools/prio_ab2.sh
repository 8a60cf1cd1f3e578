set -u
mkdir -p gpurun_out/prio2
export TMPDIR=/tmp
python3 -c "
import torch, ctypes
lib = ctypes.CDLL('libamdhip64.so')
lo, hi = ctypes.c_int(), ctypes.c_int()
lib.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
print('priority range least', lo.value, 'greatest', hi.value)
"
B="python3 bench.py --cpu-baseline off --host-io off --c3 off"
run() { timeout -k 10 120 env $2 $B > gpurun_out/prio2/$1.json 2>gpurun_out/prio2/$1.err && python3 -c "import json;d=json.load(open('gpurun_out/prio2/$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
run base X=0 && run decp1 RS2_DEC_PRIORITY=1 && run decm1 RS2_DEC_PRIORITY=-1 && run base2 X=0 && run decp1b RS2_DEC_PRIORITY=1
