#!/bin/bash
# Build kernel-timing experiment variants of libtd3hip.so into tools/exp/ (not product code).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/exp
for e in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -ffp-contract=off -DTD3_EXP=$e $EXP_FLAGS \
    td3_amd/csrc/replay.hip td3_amd/csrc/kernels.hip td3_amd/csrc/encoder.hip td3_amd/csrc/td3.hip -o tools/exp/libtd3hip_exp$e.so -lrccl &
done
wait
ls -la tools/exp
