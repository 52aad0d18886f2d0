"""Dev: clock and wave-state summary of gpu_session.sh 'kclk' passes (the
fused k-means kernel, last dispatch): effective clock = GRBM_GUI_ACTIVE / 8
XCDs / kernel time (MI355X_MICROARCH.md DVFS note), wave-cycle shares.
  python tools/kclk_summary.py gpurun_out/TAG [kernel_ms_by_name.json]"""
import collections
import csv
import glob
import os
import sys


def main():
  d = sys.argv[1]
  for sub in sorted(glob.glob(os.path.join(d, 'kclk_*'))):
    if not os.path.isdir(sub):
      continue
    f = glob.glob(sub + '/*counter_collection.csv')
    if not f:
      continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = {}
    for r in csv.DictReader(open(f[0])):
      if 'k_kmeans_pp' not in r['Kernel_Name']:
        continue
      acc[r['Dispatch_Id']][r['Counter_Name']] += float(r['Counter_Value'])
      if 'End_Timestamp' in r and r.get('Start_Timestamp'):
        durs[r['Dispatch_Id']] = (float(r['End_Timestamp']) - float(r['Start_Timestamp'])) * 1e-9
    last = sorted(acc, key=int)[-1]
    c = acc[last]
    dur = durs.get(last)
    clk = c['GRBM_GUI_ACTIVE'] / 8 / dur / 1e9 if dur else float('nan')
    wc = c['SQ_WAVE_CYCLES']
    print('%-24s %6.2f ms  clk %.2f GHz  wait_any %.2f  wait_inst %.2f  active %.2f  valu/wave %.3g salu/wave %.3g' % (
        os.path.basename(sub), (dur or 0) * 1e3, clk, c['SQ_WAIT_ANY'] / wc, c['SQ_WAIT_INST_ANY'] / wc,
        c['SQ_ACTIVE_INST_ANY'] / wc, c['SQ_INSTS_VALU'] / c['SQ_WAVES'], c['SQ_INSTS_SALU'] / c['SQ_WAVES']))


if __name__ == '__main__':
  main()
