#!/bin/bash
# Dev builds (round 5): k_kmeans_pp ablations on the woven matrix role (work
# removed by text substitution on a copy of spx.hip -- the product source
# carries no switches) -> tools/bin/libspx_NAME.so, built in parallel, timed by
# tools/gpu_session.sh kab (results wrong by design; only the time is read).
#   tools/kp_ablate2.sh name...
#   names: norounds nofold nomfma r_noload r_novector r_nomatrix r_nostage
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$here/tools/bin"
build() {
  local name=$1 src=$here/tools/bin/spx_$1.hip
  python3 - "$here/spartan_amd/csrc/spx.hip" "$src" "$name" <<'PY'
import sys
s = open(sys.argv[1]).read()
name = sys.argv[3]
NR = ('const int rnd = av ? (int)((unsigned int)dr >> 16) : 0xffff;', 'const int rnd = 0xffff;')
M0 = '      if (mf && scr0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[0][ks], bq[ks % NB], acc0, 0, 0, 0);\n'
M1 = '      if (mf && scr1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[1][ks], bq[ks % NB], acc1, 0, 0, 0);\n'
VR = '  auto vector_role = [&](int tt, const kb_f4 (&rs)[NQ]) __attribute__((always_inline)) {\n'
MR = '  auto matrix_role = [&](int tt, kb_f4 (&r)[NQ]) __attribute__((always_inline)) {\n'
subs = {
  'norounds': [NR],
  'nofold': [('    if (fv && scr0) fold16(acc0, 2 * s, lo0, sec0, il0);\n', '    lo0 = acc0[0]; sec0 = acc0[1];\n'),
             ('    if (fv && scr1) fold16(acc1, 2 * s + 1, lo1, sec1, il1);\n', '    lo1 = acc1[0]; sec1 = acc1[1];\n')],
  'nomfma': [(M0, '      acc0[ks] += (float)bq[ks % NB][0];\n'), (M1, '      acc1[ks] += (float)bq[ks % NB][1];\n')],
  'r_nostage': [NR, ('      stage(rs, mu4, us);\n', '')],
  'r_nofold': [NR, ('    if (fv && scr0) fold16(acc0, 2 * s, lo0, sec0, il0);\n',
                    '    lo0 = acc0[0]; sec0 = acc0[1]; il0 = __builtin_bit_cast(int, acc0[2]);\n'),
               ('    if (fv && scr1) fold16(acc1, 2 * s + 1, lo1, sec1, il1);\n',
                '    lo1 = acc1[0]; sec1 = acc1[1]; il1 = __builtin_bit_cast(int, acc1[2]);\n')],
  'r_nomfma': [NR, (M0, '      acc0[ks] += (float)bq[ks % NB][0];\n'), (M1, '      acc1[ks] += (float)bq[ks % NB][1];\n')],
  # loads kept but served from L2 (each block re-reads its first 64 rows): HBM latency / traffic vs issue cost
  'r_l2load': [NR, ('    i64 row = un * U + jr;\n    row = row < N ? row : N - 1;\n',
                    '    i64 row = (bk * U + jr + (u & 1) * 32) % N;\n')],
  # no label / undecided-mask stores
  'r_nostore': [NR, ('      *la = (i64)dlab;\n', ''), ('      *ma = m;\n', '')],
  # (A/B) the product without the provisional-add limit
  'nopadd': [(' && (dec || pn <= padd_lim);', ';')],
  # no -cc/2 MFMAs (the per-centre constant): what those 2 of 18 MFMAs cost
  'r_nocc': [NR, ('    if (mf && scr0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cc0, ones, acc0, 0, 0, 0);\n', ''),
             ('    if (mf && scr1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cc1, ones, acc1, 0, 0, 0);\n', '')],
  # the ring loads non-temporal (global_load ... nt)
  'ntload': [('    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 4 * qof(q));\n',
              '    for (int q = 0; q < NQ; ++q) r[q] = __builtin_nontemporal_load((const kb_f4*)(p + 4 * qof(q)));\n')],
  # rows of rank >= NRU (3) not added: what the rare-round loop costs
  'noloop3': [('    for (int k = NRU; k < U && __ballot(rnd >= k && rnd != 0xffff) != 0ull; ++k)\n',
               '    for (int k = NRU; k < U && nit < 0 && __ballot(rnd >= k && rnd != 0xffff) != 0ull; ++k)\n')],
  # wave priority: none, or on the vector role instead of the matrix role
  'noprio': [('    __builtin_amdgcn_s_setprio(1);\n    const int ua = tt - KP_LAG;', '    const int ua = tt - KP_LAG;')],
  'prio_vec': [('    __builtin_amdgcn_s_setprio(1);\n    const int ua = tt - KP_LAG;', '    const int ua = tt - KP_LAG;'),
               (VR, VR + '    __builtin_amdgcn_s_setprio(1);\n'),
               ('    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (dl & 0xffff) | (rnd << 16);\n  };',
                '    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (dl & 0xffff) | (rnd << 16);\n    __builtin_amdgcn_s_setprio(0);\n  };')],
  'r_nobarrier': [NR, ('    __syncthreads();\n    if constexpr (c == 0)\n', '    if constexpr (c == 0)\n')],
  # the decision's rank / count atomics and their round trip (ranks all 0)
  'r_noatomic': [NR, ('    if (s == 0 && h == 0 && act) {\n      rk = __hip_atomic_fetch_add', '    if (s == 0 && h == 0 && act && nit < 0) {\n      rk = __hip_atomic_fetch_add')],
  'r_noload': [NR, ('    load(r, tt + KP_AHEAD);\n    __builtin_amdgcn_sched_barrier(0);\n', '    __builtin_amdgcn_sched_barrier(0);\n')],
  # one role only (the other returns at once): what each role costs alone
  'r_novector': [NR, (VR, VR + '    if (nit >= 0) return;\n')],
  'r_nomatrix': [NR, (MR, MR + '    if (nit >= 0) { load(r, tt + KP_AHEAD); return; }\n')],
}[name]
for a, b in subs:
  assert s.count(a) == 1, (name, a[:60], s.count(a))
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
}
for n in "$@"; do build $n & done
wait
