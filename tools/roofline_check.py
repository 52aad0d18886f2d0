"""Dev: every roofline fraction of a bench.py JSON line recomputed from the
rocprofv3 --kernel-trace --stats summary of the SAME run (gpu_session.sh
benchtrace), so each leg's fraction is reproducible from a committed trace.
  python tools/roofline_check.py BENCH.json KERNEL_STATS.csv"""
import csv
import json
import sys

HBM = 8000.0
PEAK = {'f32': 157.3, 'f64': 78.6}


def main():
  d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1])
  st = {r['Name']: (int(r['Calls']), float(r['AverageNs']) * 1e-6) for r in csv.DictReader(open(sys.argv[2]))}

  def avg(pred):
    hits = [(c, a) for n, (c, a) in st.items() if pred(n)]
    n = sum(c for c, _ in hits)
    return (sum(c * a for c, a in hits) / n if n else None), [(c, round(a, 4)) for c, a in hits]

  rows = []

  def row(leg, line_frac, kernel, ms, algo, unit):
    if ms is None:
      rows.append('%-16s line %-8s trace: no %s dispatch' % (leg, line_frac, kernel))
      return
    if unit == 'GB/s':
      frac = algo / (ms * 1e-3) / 1e9 / HBM
    else:
      frac = algo / (ms * 1e-3) / 1e12 / PEAK[unit]
    rel = (frac / line_frac - 1.0) * 100 if line_frac else float('nan')
    rows.append('%-16s line %.4f  trace %.4f  (%+.1f %%)  %s avg %.4f ms' % (leg, line_frac, frac, rel, kernel, ms))

  S = d['config']['shape'][1]
  b2 = d['roofline']['bytes_per_launch']
  c0, _ = avg(lambda n: n == 'spx_reduce_cols_8da20c40')
  c1, _ = avg(lambda n: n == 'spx_reduce_rows_ed017d42')
  row('cfg2 headline', d['roofline']['frac'], 'cols_8da20c40 / rows_ed017d42', (c0 + c1) / 2 if c0 and c1 else None,
      b2, 'GB/s')
  if 'cfg2_axis_none' in d:
    row('cfg2 axis=None', d['cfg2_axis_none']['roofline']['frac'], 'rows_ed017d42 (axis 1 and None)', c1,
        d['cfg2_axis_none']['roofline']['bytes_per_launch'], 'GB/s')
  if 'cfg2_map' in d:
    k = d['cfg2_map']['roofline']['kernel']
    m, _ = avg(lambda n: n == k)
    row('cfg2 map', d['cfg2_map']['roofline']['frac'], k, m, d['cfg2_map']['roofline']['bytes_per_launch'], 'GB/s')
  if 'lreg' in d and d['lreg'].get('kernel_ms'):
    # the fused gradient kernel: the spx_reduce_cols kernel whose time matches the leg's events
    cand = [(abs(a - d['lreg']['kernel_ms']), n) for n, (c, a) in st.items()
            if n.startswith('spx_reduce_cols') and c >= 10 and n != 'spx_reduce_cols_8da20c40']
    n = min(cand)[1] if cand else None
    row('lreg', d['lreg']['kernel_hbm_frac'], n, st[n][1] if n else None, 4.0 * 1e8 * 65, 'GB/s')
  if 'kmeans' in d and d['kmeans'].get('kernel_ms'):
    m, _ = avg(lambda n: 'k_kmeans_pp' in n)
    row('kmeans fused', d['kmeans']['kernel_hbm_frac'], 'k_kmeans_pp', m, 4.0 * 1e8 * 128, 'GB/s')
  # (round 6: the fp32 product runs gemm_f32_p3, the three-stage kernel)
  for t, tags in (('f32', ('gemm<float', 'gemm_f32_p3')), ('f64', ('gemm<double', 'gemm_f64_p3'))):
    v = d.get('dot', {}).get(t)
    tag = '/'.join(tags)
    if v and v.get('kernel_mfma_frac'):
      m, _ = avg(lambda n: any(g in n for g in tags) and 'spx_mfma' in n)
      row('dot ' + t, v['kernel_mfma_frac'], tag, m, 2.0 * 32768 ** 3, t)
  print('\n'.join(rows))


if __name__ == '__main__':
  main()
