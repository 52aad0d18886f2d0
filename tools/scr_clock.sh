#!/bin/bash
# Dev (GPU box): effective shader clock of the fp16 screen kernel
# (GRBM_GUI_ACTIVE / 8 XCDs / kernel time, MI355X_MICROARCH.md DVFS notes)
# for each given libspx.so.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lib in $R/spartan_amd/libspx.so "$@"; do
  n=$(basename $lib .so)
  KM_MODES=scr timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $R/gpurun_out/clk_$n -o p --output-format csv -- python3 $R/tools/km_modes.py $lib 100000000 100000 > $R/gpurun_out/clk_$n.log 2>&1 || exit 1
  python3 - $R/gpurun_out/clk_$n $n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/*counter_collection.csv')[0]
rows = list(csv.DictReader(open(f)))
acc = {}
for r in rows:
    if 'filter_as' not in r['Kernel_Name'] or 'Li1EE' not in r['Kernel_Name']:
        continue
    key = r.get('Dispatch_Id') or r.get('Correlation_Id')
    d = acc.setdefault(key, {'v': 0.0, 'ns': int(r['End_Timestamp']) - int(r['Start_Timestamp'])})
    d['v'] += float(r['Counter_Value'])
for k, d in list(acc.items())[-3:]:
    print(sys.argv[2], 'screen %.3f ms  clock %.3f GHz' % (d['ns'] / 1e6, d['v'] / 8 / d['ns']))
PY
done
