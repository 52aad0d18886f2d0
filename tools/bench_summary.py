"""Dev: one-screen summary of a bench.py JSON line.  python tools/bench_summary.py FILE"""
import json
import sys


def main():
  d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith('{')][-1])
  r = d['roofline']
  print('cfg2 %.1f GB/s  %.4f ms/step  kernel %.4f ms  frac %.4f  checked %s' % (
      d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['checked']))
  if 'cold_start' in d:
    print('cold', {k: v for k, v in d['cold_start'].items() if k != 'note'})
  for k in ('cfg2_axis_none', 'cfg2_map'):
    if k in d:
      v = d[k]
      print('%-15s %.1f GB/s  %.4f ms  kernel %s ms  frac %s  %s' % (k, v['GBps'], v['ms_per_eval'], v['kernel_ms'],
                                                                    v['roofline']['frac'], v['checked']))
  if 'lreg' in d and 'ms_per_iter' in d['lreg']:
    l = d['lreg']
    print('lreg %.3f ms/iter  kernel %s ms (frac %s)  device %s ms  %s' % (
        l['ms_per_iter'], l.get('kernel_ms'), l.get('kernel_hbm_frac'), l.get('device_ms_per_iter'), l['checked']))
  for k in ('kmeans', 'kmeans_api'):
    if k in d and 'ms_per_iter' in d[k]:
      v = d[k]
      print('%s %.3f ms/iter  kernel %s  step %s  frac %s  %s' % (k, v['ms_per_iter'], v.get('kernel_ms'),
                                                                 v.get('step_ms'), v.get('kernel_hbm_frac'),
                                                                 v['checked']))
  if 'dot' in d:
    for t in ('f32', 'f64'):
      v = d['dot'].get(t)
      if v:
        print('dot %s %.1f TF  %.4f s  frac %.4f  kernel %s ms (%s)  %s' % (
            t, v['gflops'] / 1e3, v['seconds'], v['mfma_frac_per_gpu'], v.get('kernel_ms'), v.get('kernel_mfma_frac'),
            v['checked']))
  if 'cpu_baseline' in d:
    print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['unit'], d['cpu_baseline']['cores'])


if __name__ == '__main__':
  main()
