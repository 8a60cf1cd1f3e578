# round-6 probe: upload completion without fences (single-workgroup copy, relaxed store) vs the
# fenced multi-workgroup version; GPU tests of the upload paths first
set -u
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_uploads.py tests/test_gpu_checks.py tests/test_gpu_recovery.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SL="--cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --node off"
for rep in 1 2 3; do
for v in relaxed fenced; do
  if [ $v = relaxed ]; then L=walrus_amd/libwalrus_rs2.so; else L=walrus_amd/libwalrus_rs2_v_fenced.so; fi
  WALRUS_RS2_LIB=$L timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 $SL > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -5 $O/$v.$rep.err; exit 1; }
  WALRUS_RS2_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $SL > $O/$v.$rep.s20.json 2> $O/$v.$rep.s20.err || { tail -5 $O/$v.$rep.s20.err; exit 1; }
  python3 -c "
import json
p=json.load(open('$O/$v.$rep.json')); q=json.load(open('$O/$v.$rep.s20.json'))
print('$v rep $rep value300', p['value'], 'value20', q['value'], 'dec_setup', p['stages_ms_per_step'].get('dec_setup'), 'ok', p['decode_roundtrip_ok'], q['decode_roundtrip_ok'])
"
done
done
