set -u
mkdir -p gpurun_out/sched
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline off --host-io off --c3 off --quilt off"
for rep in 1 2; do for v in default max-ilp iterative-ilp; do
  WALRUS_RS2_LIB=walrus_amd/abvar/lib_$v.so timeout -k 10 120 $B > gpurun_out/sched/$v.$rep.json 2> gpurun_out/sched/$v.$rep.err || { tail -3 gpurun_out/sched/$v.$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sched/$v.$rep.json'));print('$v',d['value'],d['ms_per_step'],d['decode_roundtrip_ok'],d['stages_ms_solo'])"
done; done
