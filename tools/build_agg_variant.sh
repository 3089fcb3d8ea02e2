#!/bin/bash
# Builds a host-side variant of the engine library with extra compile flags
# for aggregator.cpp (the other objects from the normal build):
#   tools/build_agg_variant.sh NAME "-DSRTP_AGG_PIPE=3 ..."
#     ->  libjitsi_amd/variants/agg_NAME/libsrtp_mi355x.so
# The tools link the library by RUNPATH, so LD_LIBRARY_PATH=libjitsi_amd/variants/agg_NAME
# swaps it in (tools/gpurun.sh sync with AGG_VARIANTS).
set -e
cd "$(dirname "$0")/../libjitsi_amd/csrc"
make -s -j8
NAME=$1; FLAGS=$2
mkdir -p build_agg_$NAME ../variants/agg_$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $FLAGS -x c++ -c aggregator.cpp -o build_agg_$NAME/aggregator.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/agg_$NAME/libsrtp_mi355x.so build/srtp_kernels.o build/engine.o build/host_crypto.o build/dispatch.o build/dtls_keys.o build_agg_$NAME/aggregator.o build/rawpacket.o
echo "built libjitsi_amd/variants/agg_$NAME/libsrtp_mi355x.so"
