# round-6 probe: non-temporal stores per kernel (decode blob stores, row codec outputs), A/B
set -u
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
SL="--cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --node off"
for rep in 1 2; do
for v in default ntdec ntrows ntboth; do
  if [ $v = default ]; then L=walrus_amd/libwalrus_rs2.so; else L=walrus_amd/libwalrus_rs2_v_$v.so; fi
  WALRUS_RS2_LIB=$L timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 $SL > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -5 $O/$v.$rep.err; exit 1; }
  python3 -c "
import json
p=json.load(open('$O/$v.$rep.json'))
s=p['stages_ms_solo']
print('$v rep $rep value', p['value'], 'dec solo', s.get('dec_codec'), 'rows solo', s.get('enc_rows_codec'), 'cols_sys', s.get('enc_cols_sys_codec'), 'ok', p['decode_roundtrip_ok'])
"
done
done
