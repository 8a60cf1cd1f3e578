#!/bin/bash
# GPU tests, then the bench A/B of the tile-pipelined shared-input kernel (RS2_PIPE=0 = off).
set -u
OUT=${1:-gpurun_out/pipe1}; mkdir -p $OUT
bash tools/gpu_tests.sh $OUT && \
bash tools/gpu_bench_ab.sh $OUT/ab "pipe:" "nopipe:RS2_PIPE=0" "pipe_seq:--overlap off" "nopipe_seq:RS2_PIPE=0 --overlap off"
