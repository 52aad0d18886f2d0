#!/bin/bash
# Dev build: k_kmeans_pp with two s_memtime stamps per slot per wave -- at the
# role's start (after the slot barrier) and at its end (before the next) --
# summed per role into a device array read by tools/kp_roles.py.  The product
# source carries no instrumentation (text substitution on a copy).
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$here/tools/bin"
name=${1:-kproles}
src=$here/tools/bin/spx_$name.hip
python3 - "$here/spartan_amd/csrc/spx.hip" "$src" "$name" <<'PY'
import sys
s = open(sys.argv[1]).read()
variant = sys.argv[3]
def sub(a, b):
    global s
    assert s.count(a) == 1, a[:60]
    s = s.replace(a, b)
sub('template <int KS, int NCT>\nstruct KpStep {', '''__device__ unsigned long long g_kp_roles[1024 * 8 * 4];
extern "C" int spx_dev_kp_roles(unsigned long long* host_out) {
  return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_kp_roles), sizeof(g_kp_roles)) == hipSuccess ? 0 : 1;
}
template <int KS, int NCT>
struct KpStep {''')
sub('  const int col0 = CPW * s + CPL * hr;\n',
    '  const int col0 = CPW * s + CPL * hr;\n  unsigned long long rs_[4] = {0, 0, 0, 0}, r_t0 = 0, r_first = 0;\n')
sub('''    if constexpr ((c & 1) == GR)
      matrix_role(tt, ring[((c + KP_UNR - KP_LAG) >> 1) % NR]);
    else
      vector_role(tt, ring[((c + 1) >> 1) % NR]);
  };''', '''    r_t0 = __builtin_amdgcn_s_memtime();
    if (r_first == 0) r_first = r_t0;
    if constexpr ((c & 1) == GR)
      matrix_role(tt, ring[((c + KP_UNR - KP_LAG) >> 1) % NR]);
    else
      vector_role(tt, ring[((c + 1) >> 1) % NR]);
    {
      const unsigned long long r_t1 = __builtin_amdgcn_s_memtime();
      rs_[((c & 1) == GR) ? 0 : 1] += r_t1 - r_t0;
      rs_[2] = r_t1 - r_first;
      rs_[3] += 1;
    }
  };''')
sub('  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];\n}\n\ntemplate <int KS, int NCT>\nstatic void kp_launch',
    '  if (t < K) pcnt[(i64)bk * K + t] = cnts[t];\n  if (lane == 0 && KS == 8 && NCT == 8)\n'
    '    for (int k = 0; k < 4; ++k) g_kp_roles[(blockIdx.x * 8 + w) * 4 + k] = rs_[k];\n}\n\n'
    'template <int KS, int NCT>\nstatic void kp_launch')
NR = ('const int rnd = av ? (int)((unsigned int)dr >> 16) : 0xffff;', 'const int rnd = 0xffff;')
extra = {
  'kproles': [],
  'kproles_nr': [NR],
  # on top of no adds: the vector role without its fold / its decision
  'kproles_nofold': [NR, ('    if (scr0) fold16(acc0, 2 * s, lo0, sec0, il0);  // (unused when !fv: exv is written only if fv)\n',
                          '    lo0 = acc0[0]; sec0 = acc0[1]; il0 = __builtin_bit_cast(int, acc0[2]);\n'),
                     ('    if (scr1) fold16(acc1, 2 * s + 1, lo1, sec1, il1);\n',
                      '    lo1 = acc1[0]; sec1 = acc1[1]; il1 = __builtin_bit_cast(int, acc1[2]);\n')],
  'kproles_nodec': [NR, ('      const bool dec = fin && B1 - B2 > 1.0001f * e;\n      const bool add = rlive && fin && IB < (int)K;',
                         '      const bool dec = IB >= 0;\n      const bool add = false;')],
  'kproles_nostage': [NR, ('      stage(rs, mu4, us);\n', '      p2p[t] = rs[0][0];\n')],
}[variant]
for a, b in extra:
  assert s.count(a) == 1, (variant, a[:60], s.count(a))
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
