set -u
HEAD=/root/repo/walrus_amd/libwalrus_rs2_head.so
bash tools/gpu_tests.sh ${OUT:-gpurun_out/txab} -k "fixture or blocks or decode or fullsize or variants" && \
bash tools/gpu_bench_ab.sh ${OUT:-gpurun_out/txab}/ab "new:RS2_X=1" "head:WALRUS_RS2_LIB=$HEAD" "new2:RS2_X=1" "head2:WALRUS_RS2_LIB=$HEAD" "new_seq:--overlap off" "head_seq:WALRUS_RS2_LIB=$HEAD --overlap off" && \
bash tools/pmc_fetch_ab.sh ${OUT:-gpurun_out/txab}/fetch "new:RS2_X=1"
