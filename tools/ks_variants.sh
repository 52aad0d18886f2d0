#!/bin/bash
# Dev: the cfg3 assignment (A-stationary filter path) of the product build and
# of every tools/bin/libspx_ks*.so variant, labels checked against the exact
# kernel on a prefix (tools/km_modes.py).
set -e
cd "$(dirname "$0")/.."
for lib in spartan_amd/libspx.so tools/bin/libspx_ks*.so; do
  echo "== $lib"
  KM_MODES=as timeout -k 10 120 python3 -u tools/km_modes.py "$lib" 100000000 1000000
  KM_MODES=as timeout -k 10 120 python3 -u tools/km_modes.py "$lib" 100000000 1000000
done
