#!/bin/bash
# Dev (GPU box): rocprofv3 kernel stats of the cfg3 assignment for each
# given libspx.so (dev timing splits: KS_DEV_NOFOLD / NODEC / NOGLOBAL
# builds from tools/build_variant.sh); prints the fp16 screen kernel's mean.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lib in $R/spartan_amd/libspx.so "$@"; do
  n=$(basename $lib .so)
  KM_MODES=scr timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/split_$n -o p --output-format csv -- python3 $R/tools/km_modes.py $lib 100000000 100000 > $R/gpurun_out/split_$n.log 2>&1 || exit 1
  python3 - $R/gpurun_out/split_$n/p_kernel_stats.csv $n <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'filter_as' in r['Name'] or 'accum' in r['Name']:
        print(sys.argv[2], r['Name'][:40], r['Calls'], '%.3f ms' % (float(r['AverageNs']) / 1e6))
PY
done
