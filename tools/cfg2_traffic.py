"""Dev: per-launch HBM bytes of the cfg2 kernels from two rocprofv3 counter
passes (FETCH_SIZE, WRITE_SIZE; gpurun_out/TAG/c2f, c2w, written by
tools/gpu_session.sh cfg2pmc) -> profiles/OUT.json, the file bench.py quotes
as roofline.traffic.  FETCH_SIZE x2: the gfx950 16-byte-per-lane correction
(MI355X_MICROARCH.md, HBM section).
  python tools/cfg2_traffic.py gpurun_out/TAG profiles/r03_cfg2_pmc_traffic.json"""
import collections
import csv
import glob
import json
import sys


HEADLINE = ('spx_reduce_cols_8da20c40', 'spx_reduce_rows_ed017d42')  # cfg2 axis 0 / axis 1 (codegen.named)


def per_launch(d, counter):
  f = glob.glob(d + '/*counter_collection.csv')[0]
  acc = collections.OrderedDict()
  for r in csv.DictReader(open(f)):
    # the headline's two kernels only (the bench's cold-start, axis=None and
    # map legs and its fp64 checks launch other spx_reduce kernels)
    if r['Counter_Name'] == counter and r['Kernel_Name'] in HEADLINE:
      key = (r['Dispatch_Id'], r['Kernel_Name'])
      acc[key] = acc.get(key, 0.0) + float(r['Counter_Value']) * 1024.0
  return list(acc.values())


def main():
  d, out = sys.argv[1], sys.argv[2]
  fetch = [2.0 * v for v in per_launch(d + '/c2f', 'FETCH_SIZE')]
  write = per_launch(d + '/c2w', 'WRITE_SIZE')
  algo = 3 * 4 * 2 ** 30 + 4 * 32768
  f = sum(fetch) / len(fetch)
  w = sum(write) / len(write)
  json.dump({'command': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 bench.py --dot 0 '
                        '--workloads 0 --cpu-baseline 0 --steps 3 --warmup 1',
             'correction': 'KB; FETCH_SIZE x2 on gfx950', 'launches': len(fetch),
             'fetch_bytes_per_launch': f, 'write_bytes_per_launch': w, 'algorithmic_bytes_per_launch': algo,
             'traffic_bytes_per_launch': f + w, 'traffic_over_algorithmic': (f + w) / algo,
             'hbm_bytes_per_launch': f + w}, open(out, 'w'), indent=1)
  print(out, (f + w) / algo)


if __name__ == '__main__':
  main()
