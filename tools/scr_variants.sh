#!/bin/bash
# Dev: the cfg3 assignment (fp16 screen path) of the product build and of
# every tools/bin/libspx_*.so variant given, labels checked against the exact
# kernel on a prefix (tools/km_modes.py).
#   bash tools/scr_variants.sh tools/bin/libspx_a.so ...
set -e
cd "$(dirname "$0")/.."
for lib in spartan_amd/libspx.so "$@"; do
  echo "== $lib"
  KM_MODES=scr,scr timeout -k 10 120 python3 -u tools/km_modes.py "$lib" 100000000 1000000
done
