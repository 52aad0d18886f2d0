#!/bin/bash
# A/B of arg-reduction codegen: HEAD copy (tools/bin/codegen_head.py) vs working tree.
set -e
cp spartan_amd/codegen.py /tmp/codegen_new.py
cp tools/bin/codegen_head.py spartan_amd/codegen.py
echo "== head"; timeout -k 10 300 python -u tools/arg_ceiling.py
cp /tmp/codegen_new.py spartan_amd/codegen.py
echo "== new"; timeout -k 10 300 python -u tools/arg_ceiling.py
