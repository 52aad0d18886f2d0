#!/bin/bash
# Dev builds: libspx with ONE text substitution applied to a copy of spx.hip
# (the product source carries no switches) -> tools/bin/libspx_NAME.so
#   tools/build_sub.sh NAME 'old text' 'new text'
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
name=$1
mkdir -p "$here/tools/bin"
src=$here/tools/bin/spx_$name.hip
python3 - "$here/spartan_amd/csrc/spx.hip" "$src" "$2" "$3" <<'PY'
import sys
s = open(sys.argv[1]).read()
a, b = sys.argv[3], sys.argv[4]
assert s.count(a) == 1, ('substitution target found %d times' % s.count(a), a)
s = s.replace(a, b)
root = sys.argv[2].rsplit('/tools/', 1)[0]
s = s.replace('#include "../../include/spx.h"', '#include "%s/include/spx.h"' % root)
s = s.replace('#include "gemm_kernels.h"', '#include "%s/spartan_amd/csrc/gemm_kernels.h"' % root)
open(sys.argv[2], 'w').write(s)
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 \
  -mllvm -amdgpu-promote-alloca-to-vector-limit=1024 -o "$here/tools/bin/libspx_$name.so" "$src" \
  "$here/spartan_amd/csrc/tiling.cpp" "$here/spartan_amd/csrc/comm.cpp" -ldl
rm -f "$src"
echo "built tools/bin/libspx_$name.so"
