#!/bin/bash
# Test infrastructure: compile the reference's own C++ for the tiling solver
#  into oracle/_ref/ -- only where /root/reference
# exists (this container); the GPU box never builds or reads it.
#   bash oracle/build_ref.sh
# Lines 1-92 of spartan/expr/tiling.cc (the search) are compiled as they lie
# in the reference tree, against the system Python.h the file includes (it
# uses no Python API in those lines); lines 94-143 are the Python-2 module
# binding, which this image cannot build, and are replaced by
# oracle/ref_tiling_harness.cpp (a plain C entry point).  Nothing is copied
# into the repository: the selected lines go to the compiler on stdin.
set -euo pipefail
here=$(cd "$(dirname "$0")" && pwd)
ref=${SPARTAN_REFERENCE:-/root/reference}/spartan/expr/tiling.cc
[ -f "$ref" ] || { echo "build_ref: $ref not found; nothing built"; exit 0; }
out=$here/_ref
mkdir -p "$out"
pyinc=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
sed -n '1,92p' "$ref" | g++ -std=c++14 -O2 -fPIC -w -I"$pyinc" -x c++ -c - -o "$out/tiling_core.o"
g++ -std=c++14 -O2 -fPIC -shared "$here/ref_tiling_harness.cpp" "$out/tiling_core.o" -o "$out/libreftiling.so.tmp"
mv "$out/libreftiling.so.tmp" "$out/libreftiling.so"
echo "build_ref: $out/libreftiling.so"
