"""Dev: summarise a gpu_session.sh 'kab' A/B (fused k-means kernel and step
times per build).  python tools/kab_summary.py gpurun_out/TAG"""
import csv
import glob
import os
import re
import sys


def main():
  d = sys.argv[1]
  for sub in sorted(glob.glob(os.path.join(d, 'kab_*_[0-9]'))):
    name = os.path.basename(sub)
    f = glob.glob(sub + '/p_kernel_stats.csv')
    row = {}
    if f:
      for r in csv.DictReader(open(f[0])):
        if 'k_kmeans_pp' in r['Name']:
          row = r
    log = open(sub + '.log').read() if os.path.exists(sub + '.log') else ''
    m = re.search(r'(?:step|first): ([0-9.]+) ms per iteration', log)
    print('%-22s kernel avg %7.3f min %7.3f ms  step %s ms' % (
        name, float(row.get('AverageNs', 'nan')) / 1e6, float(row.get('MinNs', 'nan')) / 1e6,
        m.group(1) if m else '?'))


if __name__ == '__main__':
  main()
