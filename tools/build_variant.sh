#!/bin/bash
# Dev builds of libspx.so with extra -D flags into tools/bin/libspx_<name>.so
# (timing splits / A-B variants for tools/km_step_once.py); never the product build.
#   tools/build_variant.sh NAME [-DFLAG ...]
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$here/tools/bin"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 -mllvm -amdgpu-promote-alloca-to-vector-limit=1024 "$@" \
  -o "$here/tools/bin/libspx_$name.so" "$here/spartan_amd/csrc/spx.hip" \
  "$here/spartan_amd/csrc/tiling.cpp" "$here/spartan_amd/csrc/comm.cpp" -ldl
