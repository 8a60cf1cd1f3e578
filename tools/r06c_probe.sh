set -u
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/micro/bin/xwave > $O/xwave.txt 2>&1 || { cat $O/xwave.txt; exit 1; }
cat $O/xwave.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/xw_pmc -o run -- tools/micro/bin/xwave > $O/xw_pmc.log 2>&1 || { tail -5 $O/xw_pmc.log; exit 1; }
SL="--cpu-baseline off --host-io off --c3 off --c4 off --host-abi off --quilt off --node off"
RS2_BENCH_CLOCKS=1 timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 $SL > $O/clk0.json 2> $O/clk0.err || { tail -5 $O/clk0.err; exit 1; }
RS2_BENCH_CLOCKS=1 RS2_BENCH_SOLO_PAUSE=0.5 timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 $SL > $O/clk5.json 2> $O/clk5.err || { tail -5 $O/clk5.err; exit 1; }
RS2_BENCH_CLOCKS=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 $SL > $O/clk20.json 2> $O/clk20.err || { tail -5 $O/clk20.err; exit 1; }
for f in clk0 clk5 clk20; do python3 -c "
import json,sys
p=json.load(open('$O/$f.json'))
print('$f', p['value'], p['roofline']['solo']['ms_each'])
print(json.dumps(p.get('gpu_clocks')))
"; done
