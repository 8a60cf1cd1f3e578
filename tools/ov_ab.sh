set -u
mkdir -p gpurun_out/ov
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --cpu-baseline off --host-io off --c3 off --overlap off > gpurun_out/ov/off.json 2> gpurun_out/ov/off.err && \
timeout -k 10 300 python3 bench.py --cpu-baseline off --host-io off --c3 off --overlap on > gpurun_out/ov/on.json 2> gpurun_out/ov/on.err
rc=$?; cat gpurun_out/ov/*.json; tail -5 gpurun_out/ov/on.err; exit $rc
