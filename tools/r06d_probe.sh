# round-6 probe: Blake2b mix floor micro, the driver's bench command with clock samples, rocprof
set -u
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/micro/bin/b2mix > $O/b2mix.txt 2>&1 || { cat $O/b2mix.txt; exit 1; }
cat $O/b2mix.txt
RS2_BENCH_CLOCKS=1 timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -5 $O/bench20.err; exit 1; }
python3 -c "
import json
p=json.load(open('$O/bench20.json'))
print('value', p['value'], 'solo', p['roofline']['solo'], 'c2', p['c1_c2_split']['c2_decode_random_ms'])
print(json.dumps(p.get('gpu_clocks')))
"
bash tools/gpu.sh $O prof --steps 30 --warmup 5
