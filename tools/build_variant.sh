#!/bin/bash
# Build an experiment variant of the engine: walrus_amd/libwalrus_rs2_v_NAME.so with extra
# compile flags (load it with WALRUS_RS2_LIB).  usage: tools/build_variant.sh NAME "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/../walrus_amd/csrc"
make -j16 LIB=../libwalrus_rs2_v_$1.so BUILD=build_v_$1 EXTRA="$2" > /dev/null
echo "walrus_amd/libwalrus_rs2_v_$1.so"
