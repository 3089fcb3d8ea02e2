#!/bin/bash
# Builds the SRTP_STAMPS diagnostic library that tools/stamps.py loads
# (tools/stamps/libsrtp_stamps.so): srtp_kernels.hip and engine.cpp with
# -DSRTP_STAMPS (per-wave clock stamps at kernel entry, after the T-table fill
# and at the end), the other objects from the normal build.
set -e
cd "$(dirname "$0")/../libjitsi_amd/csrc"
make -s -j8
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -DSRTP_STAMPS"
mkdir -p build_stamps ../../tools/stamps
$H $F --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds -c srtp_kernels.hip -o build_stamps/srtp_kernels.o
$H $F -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c engine.cpp -o build_stamps/engine.o
$H --offload-arch=gfx950 -shared -fPIC -o ../../tools/stamps/libsrtp_stamps.so build_stamps/srtp_kernels.o \
    build_stamps/engine.o build/host_crypto.o build/dispatch.o build/dtls_keys.o build/aggregator.o build/rawpacket.o
echo "built tools/stamps/libsrtp_stamps.so"
