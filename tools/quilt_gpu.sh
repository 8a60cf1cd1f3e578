set -u
mkdir -p gpurun_out/quilt2
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_quilt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quilt2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/quilt2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --cpu-baseline off --host-io off --c3 off --steps 10 > gpurun_out/quilt2/bench.json 2> gpurun_out/quilt2/bench.err; rc=$?
python3 -c "import json;d=json.load(open('gpurun_out/quilt2/bench.json'));print(d['value'], d['quilt'])" || tail -20 gpurun_out/quilt2/bench.err
exit $rc
