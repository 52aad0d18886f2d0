"""Dev: per-dispatch SQ / LDS counters of the k-means step kernels from the
kfspmc / kfslds passes of tools/gpu_session.sh (one --pmc group per pass).
  python tools/kfs_summary.py gpurun_out/TAG
Per kernel: mean per dispatch of every counter, and the derived figures
  cycles      = GRBM_GUI_ACTIVE / 8 (one count per XCD)
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
  valu/wave   = SQ_INSTS_VALU / SQ_WAVES (MFMAs included), likewise mfma, lds
  wait_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict= SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"""
import collections
import csv
import glob
import os
import sys

KERNELS = (('k_kmeans_pp', 'fused screen + accumulate (k_kmeans_pp)'),
           ('k_kmeans_filter_asILi8ELi8ELi0E', 'bf16x3 list pass (filter_as MODE 0)'),
           ('k_kmeans_filter_b3', 'all-accumulator filter (filter_b3)'),
           ('k_kmeans_cand16', 'exact candidates (cand16)'))


def load(d):
  per = collections.defaultdict(lambda: collections.defaultdict(float))
  for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
      per[(f, r['Dispatch_Id'], r['Kernel_Name'])][r['Counter_Name']] += float(r['Counter_Value'])
  return per


def main():
  root = sys.argv[1]
  per = {}
  for sub in ('kfs_a', 'kfs_b', 'kfs_lds'):
    if os.path.isdir(os.path.join(root, sub)):
      per.update(load(os.path.join(root, sub)))
  for key, label in KERNELS:
    agg = collections.defaultdict(list)
    for (_, _, name), cs in per.items():
      if key in name:
        for c, v in cs.items():
          agg[c].append(v)
    if not agg:
      continue
    m = {c: sum(v) / len(v) for c, v in agg.items()}
    print('%s  (%d dispatch records)' % (label, max(len(v) for v in agg.values())))
    for c in sorted(m):
      print('  %-28s %.4g' % (c, m[c]))
    cyc = m.get('GRBM_GUI_ACTIVE', 0.0) / 8.0
    der = []
    if cyc and 'SQ_VALU_MFMA_BUSY_CYCLES' in m:
      der.append('mfma_busy %.3f' % (m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024.0 * cyc)))
    if m.get('SQ_WAVES'):
      for c, n in (('SQ_INSTS_VALU', 'valu'), ('SQ_INSTS_MFMA', 'mfma'), ('SQ_INSTS_LDS', 'lds'),
                   ('SQ_INSTS_SALU', 'salu')):
        if c in m:
          der.append('%s/wave %.4g' % (n, m[c] / m['SQ_WAVES']))
    if m.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_INST_ANY' in m:
      der.append('wait_frac %.3f' % (m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']))
    if m.get('SQ_LDS_IDX_ACTIVE') and 'SQ_LDS_BANK_CONFLICT' in m:
      der.append('lds_conflict %.3f' % (m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']))
    print('  derived: cycles %.4g  %s' % (cyc, '  '.join(der)))


if __name__ == '__main__':
  main()
