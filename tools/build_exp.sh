#!/bin/bash
# Build an experiment variant of libtd3hip.so into tools/exp/ (not product code).
#   tools/build_exp.sh NAME "-DSOME_KNOB=1 ..."   ->  tools/exp/libtd3hip_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/exp
name=$1; flags=${2:-}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=6 $flags \
  td3_amd/csrc/replay.hip td3_amd/csrc/kernels.hip td3_amd/csrc/encoder.hip td3_amd/csrc/td3.hip \
  -o tools/exp/libtd3hip_$name.so -lrccl
ls -la tools/exp/libtd3hip_$name.so
