set -u
mkdir -p gpurun_out/copy
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/copy/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/copy/pytest.log; [ $rc -ne 0 ] && exit $rc
B="python3 bench.py --cpu-baseline off --host-io off --c3 off"
run() { timeout -k 10 120 env $2 $B > gpurun_out/copy/$1.json 2>gpurun_out/copy/$1.err && python3 -c "import json;d=json.load(open('gpurun_out/copy/$1.json'));print('$1',d['value'],d['ms_per_step'],d['stages_ms_solo']['enc_blob_copy'],d['c1_c2_split'] if 'c1_c2_split' in d else '')"; }
run blit RS2_BLIT_COPY=1 && run kern X=0 && run blit2 RS2_BLIT_COPY=1 && run kern2 X=0
