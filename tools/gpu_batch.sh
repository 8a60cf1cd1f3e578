mkdir -p gpurun_out/batch1 && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py -x -v --timeout 300 --timeout-method thread > gpurun_out/batch1/pytest.log 2>&1; rc=$?; tail -12 gpurun_out/batch1/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --host-io off --c4 off --host-abi off --quilt off > gpurun_out/batch1/bench.json 2> gpurun_out/batch1/bench.err; rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/batch1/bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/batch1/bench.json')); print(d['value'], json.dumps(d['c3_small_blobs']))"
