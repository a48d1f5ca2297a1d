#!/bin/bash
# Build library variants for A/B runs on the GPU (tools/gpu_check.sh STEPS=exp):
#   tools/build_exp.sh name:-DFLAG=1+-DOTHER=2 name2:...
# Each variant recompiles verify_kernels.hip and bdls_hip.cpp (which sizes
# device buffers from verify.h) with its flags and links them with the other
# default host objects into exp/libbdlship_<name>.so (git-ignored, shipped to
# the GPU box; objects stay in build/exp). Parallel.
set -eu
cd "$(dirname "$0")/.."
make -s bdls_amd/lib/bdls_hip.o bdls_amd/lib/bdls_msg.o bdls_amd/lib/fabric.o
mkdir -p build/exp exp  # variants accumulate; rm exp/*.so to start over
HIPCC=/opt/rocm/bin/hipcc
one() {
  n=${1%%:*}; f=$(echo "${1#*:}" | tr '+' ' ')
  $HIPCC -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $f \
    -c bdls_amd/csrc/verify_kernels.hip -o build/exp/vk_$n.o &&
  # the host side sizes device buffers from verify.h's constants: same flags
  $HIPCC -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function $f \
    -c bdls_amd/csrc/bdls_hip.cpp -o build/exp/bh_$n.o &&
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o exp/libbdlship_$n.so build/exp/vk_$n.o \
    build/exp/bh_$n.o bdls_amd/lib/bdls_msg.o bdls_amd/lib/fabric.o -lpthread &&
  echo "built $n"
}
export -f one; export HIPCC
printf '%s\n' "$@" | xargs -P 4 -I{} bash -c 'one "$@"' _ {}
