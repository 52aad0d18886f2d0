"""Dev: per-launch HBM bytes from a profile_round.sh directory.
FETCH_SIZE / WRITE_SIZE (KB) from separate --pmc passes, FETCH_SIZE x2 for the
gfx950 16-byte-per-lane streaming reads (MI355X_MICROARCH.md HBM section).
  python tools/pmc_summary.py gpurun_out/prof_TAG OUT_cfg2.json OUT_kmeans.json"""
import collections
import csv
import glob
import json
import sys


def per_dispatch(d, counter):
  f = glob.glob(d + '/*counter_collection.csv')[0]
  acc = collections.OrderedDict()
  for r in csv.DictReader(open(f)):
    if r['Counter_Name'] != counter:
      continue
    key = (r['Dispatch_Id'], r['Kernel_Name'])
    acc[key] = acc.get(key, 0.0) + float(r['Counter_Value']) * 1024.0
  return acc


def by_kernel(acc):
  out = collections.OrderedDict()
  for (_, name), v in acc.items():
    out.setdefault(name, []).append(v)
  return out


def main():
  d, out2, outk = sys.argv[1:4]
  f2, w2 = by_kernel(per_dispatch(d + '/c2f', 'FETCH_SIZE')), by_kernel(per_dispatch(d + '/c2w', 'WRITE_SIZE'))
  red = [k for k in f2 if k.startswith('spx_reduce')]
  fetch = [2.0 * v for k in red for v in f2[k]]
  write = [v for k in red for v in w2.get(k, [])]
  algo = 3 * 4 * 2 ** 30 + 4 * 32768
  c2 = {'command': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 bench.py --dot 0 '
                   '--workloads 0 --cpu-baseline 0 --steps 3 --warmup 1',
        'correction': 'KB; FETCH_SIZE x2 on gfx950', 'launches': len(fetch),
        'fetch_bytes_per_launch': sum(fetch) / max(len(fetch), 1),
        'write_bytes_per_launch': sum(write) / max(len(write), 1),
        'algorithmic_bytes_per_launch': algo}
  c2['traffic_bytes_per_launch'] = c2['fetch_bytes_per_launch'] + c2['write_bytes_per_launch']
  c2['traffic_over_algorithmic'] = c2['traffic_bytes_per_launch'] / algo
  c2['hbm_bytes_per_launch'] = c2['traffic_bytes_per_launch']  # the key bench.py reads
  json.dump(c2, open(out2, 'w'), indent=1)
  fk, wk = by_kernel(per_dispatch(d + '/kmf', 'FETCH_SIZE')), by_kernel(per_dispatch(d + '/kmw', 'WRITE_SIZE'))
  iters = 3  # tools/km_iter.py 100000000 2: one warm-up iteration + 2
  per = collections.OrderedDict()
  for k in fk:
    if 'kmeans' not in k and 'ks_compact' not in k:
      continue
    per[k] = {'calls': len(fk[k]), 'fetch_bytes': 2.0 * sum(fk[k]) / iters,
              'write_bytes': sum(wk.get(k, [])) / iters}
  km = {'command': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 tools/km_iter.py '
                   '100000000 2 (cfg3 shape; per iteration = over the 3 assign + accumulate rounds)',
        'correction': 'KB; FETCH_SIZE x2 on gfx950', 'per_kernel_per_iteration': per,
        'fetch_bytes_per_iteration': sum(v['fetch_bytes'] for v in per.values()),
        'write_bytes_per_iteration': sum(v['write_bytes'] for v in per.values()),
        'points_bytes': 100000000 * 128 * 4}
  km['fetch_over_one_pass'] = km['fetch_bytes_per_iteration'] / km['points_bytes']
  json.dump(km, open(outk, 'w'), indent=1)
  print(json.dumps(c2, indent=1))
  print(json.dumps({k: v for k, v in km.items() if k != 'per_kernel_per_iteration'}, indent=1))
  for k, v in per.items():
    print('%-60s %3d calls  fetch %.3f GB  write %.3f GB' % (k[:60], v['calls'], v['fetch_bytes'] / 1e9,
                                                           v['write_bytes'] / 1e9))


if __name__ == '__main__':
  main()
