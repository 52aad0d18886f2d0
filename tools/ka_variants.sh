#!/bin/bash
# Dev: time the cfg3 accumulate of the product build and of every
# tools/bin/libspx_ka*.so variant (tools/build_variant.sh), assign once each.
set -e
cd "$(dirname "$0")/.."
for lib in spartan_amd/libspx.so tools/bin/libspx_ka*.so; do
  echo "== $lib"
  KM_MODES=as timeout -k 10 120 python3 -u tools/km_modes.py "$lib" 100000000 1000000
done
