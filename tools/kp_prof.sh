#!/bin/bash
# Dev build: k_kmeans_pp with per-wave s_memtime cycle counters per loop
# segment -> tools/bin/libspx_kpprof.so (read by tools/kp_prof.py).  The
# product source carries no instrumentation: this script inserts it into a
# copy of spx.hip at fixed code lines (it fails loudly if a line moved).
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$here/tools/bin"
src=$here/tools/bin/spx_kpprof.hip
python3 - "$here/spartan_amd/csrc/spx.hip" "$src" <<'PY'
import sys
s = open(sys.argv[1]).read()
def ins(anchor, text, after=True, count=1):
    global s
    n = s.count(anchor)
    assert n == count, 'anchor %r found %d times' % (anchor[:50], n)
    s = s.replace(anchor, anchor + text if after else text + anchor)
prof = '''
__device__ unsigned long long g_kp_prof[1024 * 8 * 8];
extern "C" int spx_dev_kp_prof(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_kp_prof), sizeof(g_kp_prof)) == hipSuccess ? 0 : 1;
}
#define KPT(k) { const unsigned long long now_ = __builtin_amdgcn_s_memtime(); pacc_[k] += now_ - plast_; plast_ = now_; }
'''
ins('template <int KS, int NCT>\nstruct KpStep {', prof, after=False)
ins('  const int col0 = CPW * s + CPL * hr;\n',
    '  unsigned long long pacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, plast_ = __builtin_amdgcn_s_memtime();\n')
ins('    __syncthreads();\n    if constexpr (c == 0)\n', '    KPT(7)\n', after=False)
ins('    __syncthreads();\n    if constexpr (c == 0)\n', '') 
s = s.replace('    KPT(7)\n    __syncthreads();\n    if constexpr (c == 0)\n', '    KPT(7)\n    __syncthreads();\n    KPT(0)\n    if constexpr (c == 0)\n')
ins('    if (mf && scr1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cc1, ones, acc1, 0, 0, 0);\n', '    KPT(1)\n')
ins('    // labels (-1 for an undecided row', '    KPT(2)\n', after=False)
ins('    load(r, tt + KP_AHEAD);\n', '    KPT(3)\n')
if '    // (4) each decided row' in s:  # decision in the vector role (round-4 v3 / v4)
    ins('    // (4) each decided row', '    KPT(4)\n', after=False)
    ins('    // (6) stage of unit t + 1\n', '    KPT(5)\n', after=False)
    ins('    if (s == 0 && h == 0) dres[', '    KPT(6)\n', after=False)
else:  # decision in the matrix role: vector = fold + exv (4), stage (6)
    ins('    __builtin_amdgcn_sched_barrier(0);\n    if (us < nit) {\n', '    KPT(4)\n', after=False)
    ins('      stage(rs, mu4, us);\n    }\n', '    KPT(6)\n')
ins('  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];\n}\n',
    '', after=True)
s = s.replace('  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];\n}\n\ntemplate <int KS, int NCT>\nstatic void kp_launch',
              '  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];\n  if (lane == 0 && KS == 8 && NCT == 8)\n'
              '    for (int k = 0; k < 8; ++k) g_kp_prof[(blockIdx.x * 8 + w) * 8 + k] = pacc_[k];\n}\n\n'
              'template <int KS, int NCT>\nstatic void kp_launch')
assert 'g_kp_prof[(blockIdx.x' in s
s = s.replace('#include "../../include/spx.h"', '#include "%s/include/spx.h"' % sys.argv[2].rsplit('/tools/', 1)[0])
s = s.replace('#include "gemm_kernels.h"', '#include "%s/spartan_amd/csrc/gemm_kernels.h"' % sys.argv[2].rsplit('/tools/', 1)[0])
open(sys.argv[2], 'w').write(s)
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 \
  -mllvm -amdgpu-promote-alloca-to-vector-limit=1024 -o "$here/tools/bin/libspx_kpprof.so.tmp" "$src" \
  "$here/spartan_amd/csrc/tiling.cpp" "$here/spartan_amd/csrc/comm.cpp" -ldl
mv "$here/tools/bin/libspx_kpprof.so.tmp" "$here/tools/bin/libspx_kpprof.so"
echo "built tools/bin/libspx_kpprof.so"
