#!/bin/bash
# Dev (GPU box): lreg ms/iter of the tree's package against a copy of an
# older package in old_spx/spartan_amd (A/B, interleaved).
cd "$(dirname "$0")/.."
R=$(pwd)
for i in 1 2 3; do
  echo -n "new "; GRAFT_REPO_ROOT=$R timeout -k 10 200 python3 tools/lreg_prof.py 100000000 50 2>&1 | grep -v amdgpu | tail -1
  echo -n "old "; GRAFT_REPO_ROOT=$R/old_spx timeout -k 10 200 python3 tools/lreg_prof.py 100000000 50 2>&1 | grep -v amdgpu | tail -1
done
