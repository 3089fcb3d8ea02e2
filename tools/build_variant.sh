#!/bin/bash
# Builds a diagnostic / candidate variant of the engine library with extra
# compile flags for srtp_kernels.hip (the other objects from the normal build):
#   tools/build_variant.sh NAME "-DFLAG=1 ..." [--lean R]  ->  libjitsi_amd/variants/libsrtp_NAME.so
# --lean R: the AES rounds generated with R lookup registers (tools/gen_aes_asm.py --lean)
# Load it with SRTP_MI355X_LIB=libjitsi_amd/variants/libsrtp_NAME.so (bench.py, tests).
set -e
cd "$(dirname "$0")/../libjitsi_amd/csrc"
make -s -j8
NAME=$1; FLAGS=$2
mkdir -p build_$NAME ../variants
if [ "$3" = "--lean" ]; then
  python3 ../../tools/gen_aes_asm.py --lean "$4" --out build_$NAME/aes_rounds_asm.inc
  FLAGS="$FLAGS -DSRTP_AES_ROUNDS=\"build_$NAME/aes_rounds_asm.inc\""
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds -Rpass-analysis=kernel-resource-usage $FLAGS -c srtp_kernels.hip -o build_$NAME/srtp_kernels.o 2> build_$NAME/resource_usage.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/libsrtp_$NAME.so build_$NAME/srtp_kernels.o build/engine.o build/host_crypto.o build/dispatch.o build/dtls_keys.o build/aggregator.o build/rawpacket.o
echo "built libjitsi_amd/variants/libsrtp_$NAME.so"
