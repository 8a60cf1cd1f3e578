set -u
OUT=gpurun_out/pair1; mkdir -p $OUT
bash tools/gpu_tests.sh $OUT && \
bash tools/gpu_exp.sh $OUT/ab "pair:" "nopair:RS2_PAIR=0" "pair_seq:--overlap off" "nopair_seq:RS2_PAIR=0 --overlap off"
