#!/bin/bash
# Dev (GPU box): effective shader clock during the dot GEMMs
# (GRBM_GUI_ACTIVE / 8 XCDs / kernel time) and the GEMM rate against the MFMA
# peak AT that clock -- evidence independent of SQ_VALU_MFMA_BUSY_CYCLES.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/dotclk -o p --output-format csv -- python3 $R/tools/dot_prof.py 16384 > $R/gpurun_out/dotclk.log 2>&1 || exit 1
python3 - $R/gpurun_out/dotclk <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/*counter_collection.csv')[0]
acc = {}
for r in csv.DictReader(open(f)):
    if 'gemm' not in r['Kernel_Name']:
        continue
    k = r['Dispatch_Id']
    d = acc.setdefault(k, {'v': 0.0, 'ns': int(r['End_Timestamp']) - int(r['Start_Timestamp']), 'n': r['Kernel_Name']})
    d['v'] += float(r['Counter_Value'])
S = 16384
for k, d in acc.items():
    f32 = 'float' in d['n'].split('<')[1][:6]
    ghz = d['v'] / 8 / d['ns']
    tf = 2.0 * S ** 3 / (d['ns'] * 1e-9) / 1e12
    peak_clk = 1024 * (64 if f32 else 32) * ghz * 1e9 / 1e12   # flop/clk/SIMD: fp32 MFMA 64, fp64 MFMA 32
    print('%s %.2f ms  clock %.3f GHz  %.1f TF/s  = %.1f %% of the MFMA peak at that clock (%.1f TF/s), %.1f %% of nominal' %
          ('f32' if f32 else 'f64', d['ns'] / 1e6, ghz, tf, 100 * tf / peak_clk, peak_clk, 100 * tf / (157.3 if f32 else 78.6)))
PY
