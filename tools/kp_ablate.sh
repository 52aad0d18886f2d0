#!/bin/bash
# Dev builds: k_kmeans_pp ablations (work removed by text substitution on a
# copy of spx.hip -- the product source carries no switches) ->
# tools/bin/libspx_abl_<name>.so, timed by tools/km_step_once.py under a
# kernel trace (the results are wrong by design; only the time is read).
#   tools/kp_ablate.sh name...   (names: base norounds noloop nostage noatomic nobarrier)
set -e
here=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$here/tools/bin"
build() {
  local name=$1 src=$here/tools/bin/spx_abl_$1.hip
  python3 - "$here/spartan_amd/csrc/spx.hip" "$src" "$name" <<'PY'
import sys
s = open(sys.argv[1]).read()
name = sys.argv[3]
NR = ('const int rnd = av ? (int)((unsigned int)dr >> 16) : 0xffff;', 'const int rnd = 0xffff;')
subs = {
  'base': [],
  # on top of norounds (no adds): what the rest of the slot costs
  'r_nofold': [NR, ('    if (fv && scr0) fold16(acc0, 2 * s, lo0, sec0, il0);\n', '    lo0 = acc0[0]; sec0 = acc0[1];\n'),
               ('    if (fv && scr1) fold16(acc1, 2 * s + 1, lo1, sec1, il1);\n', '    lo1 = acc1[0]; sec1 = acc1[1];\n')],
  'r_nomfma': [NR, ('      if (mf && scr0) acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[0][ks], bq[ks & 3], acc0, 0, 0, 0);\n', '      acc0[ks] += (float)bq[ks & 3][0];\n'),
               ('      if (mf && scr1) acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ca[1][ks], bq[ks & 3], acc1, 0, 0, 0);\n', '      acc1[ks] += (float)bq[ks & 3][1];\n')],
  'r_nostage': [NR, ('if (us < nit) stage(', 'if (us < 0) stage(')],
  'r_noload': [NR, ('    load(r, tt + KP_AHEAD);\n  };', '  };')],
  # every load instruction reads whole 128-B row segments (8 lanes per row; wrong data, same bytes)
  'coal': [('    const float* p = P + row * ldp + col0;\n#pragma unroll\n    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 4 * qof(q));\n',
            '    const float* p = P + (un * U + (lane >> 3)) * ldp + CPW * s + 4 * (lane & 7);\n#pragma unroll\n    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 8 * q * ldp);\n')],
  'r_coal': [NR, ('    const float* p = P + row * ldp + col0;\n#pragma unroll\n    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 4 * qof(q));\n',
            '    const float* p = P + (un * U + (lane >> 3)) * ldp + CPW * s + 4 * (lane & 7);\n#pragma unroll\n    for (int q = 0; q < NQ; ++q) r[q] = *(const kb_f4*)(p + 8 * q * ldp);\n')],
  # wave priority by role (s_setprio 1 while in the role)
  'prio_mat': [('  auto matrix_role = [&](int tt, kb_f4 (&r)[NQ]) __attribute__((always_inline)) {\n',
                '  auto matrix_role = [&](int tt, kb_f4 (&r)[NQ]) __attribute__((always_inline)) {\n    __builtin_amdgcn_s_setprio(1);\n'),
               ('    load(r, tt + KP_AHEAD);\n  };', '    load(r, tt + KP_AHEAD);\n    __builtin_amdgcn_s_setprio(0);\n  };')],
  'prio_vec': [('  auto vector_role = [&](int tt, const kb_f4 (&rs)[NQ]) __attribute__((always_inline)) {\n',
                '  auto vector_role = [&](int tt, const kb_f4 (&rs)[NQ]) __attribute__((always_inline)) {\n    __builtin_amdgcn_s_setprio(1);\n'),
               ('    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (d & 0xffff) | (rnd << 16);\n  };',
                '    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (d & 0xffff) | (rnd << 16);\n    __builtin_amdgcn_s_setprio(0);\n  };')],
  # the staging of unit t + 1 first in the vector role (its LDS writes drain
  # under the fold and the decision instead of in front of the barrier)
  'stagefirst': [('    const kb_f4 p4 = *(const kb_f4*)(pr + 16 * h);\n',
                  '    const kb_f4 p4 = *(const kb_f4*)(pr + 16 * h);\n    {\n      kb_f4 mu4s[NQ];\n      mu_load(mu4s);\n      if (us < nit) stage(rs, mu4s, us);\n    }\n'),
                 ('    kb_f4 mu4[NQ];\n    mu_load(mu4);\n    const float fb1', '    const float fb1'),
                 ('    if (us < nit) stage(rs, mu4, us);\n', '')],
  'sf_dres': [('    const kb_f4 p4 = *(const kb_f4*)(pr + 16 * h);\n',
                  '    const kb_f4 p4 = *(const kb_f4*)(pr + 16 * h);\n    {\n      kb_f4 mu4s[NQ];\n      mu_load(mu4s);\n      if (us < nit) stage(rs, mu4s, us);\n    }\n'),
                 ('    kb_f4 mu4[NQ];\n    mu_load(mu4);\n    const float fb1', '    const float fb1'),
                 ('    if (us < nit) stage(rs, mu4, us);\n', ''),
                 ('    if (s == 0 && h == 0 && act) __hip_atomic_store(rcnt + d, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n',
                  '    if (s == 0 && h == 0 && act) __hip_atomic_store(rcnt + d, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (d & 0xffff) | ((act ? (int)rk : 0xffff) << 16);\n'),
                 ('    const int rnd = act ? (int)rk : 0xffff;  // add round (0xffff: no add)\n    if (s == 0 && h == 0) dres[(u2 & 3) * U + j] = (d & 0xffff) | (rnd << 16);\n', '')],
  # register-ring depth of the gathered accumulation (list mode in the step)
  'ka4': [('constexpr int KA_STAGES = 3;', 'constexpr int KA_STAGES = 4;')],
  'ka2': [('constexpr int KA_STAGES = 3;', 'constexpr int KA_STAGES = 2;')],
  'r_nobarrier': [NR, ('    constexpr int GR = decltype(gc)::value, c = decltype(cc)::value;\n    __syncthreads();\n',
                 '    constexpr int GR = decltype(gc)::value, c = decltype(cc)::value;\n')],
  'norounds': [('const int rnd = av ? (int)((unsigned int)dr >> 16) : 0xffff;', 'const int rnd = 0xffff;')],
  'noloop': [('for (int k = 1; k < U && __ballot', 'for (int k = 1; k < 1 && __ballot')],
  'nostage': [('if (us < nit) stage(', 'if (us < 0) stage(')],
  'noatomic': [('rk = __hip_atomic_fetch_add(rcnt + d, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);', 'rk = 0;')],
  # k_kmeans_filter_as MODE 0 (the bf16x3 list pass): wave priority 1 over the
  # centre sweep (as_prio) or over the split / decision instead (as_prio_epi)
  'as_prio': [('      kb_acc a0, b0;\n      chain(0, a0);\n', '      kb_acc a0, b0;\n      __builtin_amdgcn_s_setprio(1);\n      chain(0, a0);\n'),
              ('        fold(NCT - 1, b0);\n      }\n    }\n    float lo0[16];', '        fold(NCT - 1, b0);\n      }\n      __builtin_amdgcn_s_setprio(0);\n    }\n    float lo0[16];')],
  'as_prio_epi': [('  for (; tile < ntiles; tile += stride) {\n    load(tile);', '  for (; tile < ntiles; tile += stride) {\n    __builtin_amdgcn_s_setprio(1);\n    load(tile);'),
                  ('      kb_acc a0, b0;\n      chain(0, a0);\n', '      kb_acc a0, b0;\n      __builtin_amdgcn_s_setprio(0);\n      chain(0, a0);\n'),
                  ('        fold(NCT - 1, b0);\n      }\n    }\n    float lo0[16];', '        fold(NCT - 1, b0);\n      }\n      __builtin_amdgcn_s_setprio(1);\n    }\n    float lo0[16];')],
  'nobarrier': [('    constexpr int GR = decltype(gc)::value, c = decltype(cc)::value;\n    __syncthreads();\n',
                 '    constexpr int GR = decltype(gc)::value, c = decltype(cc)::value;\n')],
}[name]
for a, b in subs:
    assert s.count(a) == 1, '%s: %r found %d times' % (name, a[:60], s.count(a))
    s = s.replace(a, b)
root = sys.argv[2].rsplit('/tools/', 1)[0]
s = s.replace('#include "../../include/spx.h"', '#include "%s/include/spx.h"' % root)
s = s.replace('#include "gemm_kernels.h"', '#include "%s/spartan_amd/csrc/gemm_kernels.h"' % root)
open(sys.argv[2], 'w').write(s)
PY
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -std=c++17 \
    -mllvm -amdgpu-promote-alloca-to-vector-limit=1024 -o "$here/tools/bin/libspx_abl_$name.so.tmp" "$src" \
    "$here/spartan_amd/csrc/tiling.cpp" "$here/spartan_amd/csrc/comm.cpp" -ldl
  mv "$here/tools/bin/libspx_abl_$name.so.tmp" "$here/tools/bin/libspx_abl_$name.so"
  echo "built tools/bin/libspx_abl_$name.so"
}
pids=()
for n in "$@"; do build "$n" & pids+=($!); done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
exit $rc
