#!/bin/bash
# scripts/dev/determinism_streams.py under several variant libraries / knobs (one process each);
# the settings one per line in $CONFIG_FILE (default: a built-in list)
if [ -n "${CONFIG_FILE:-}" ]; then mapfile -t CFG < "$CONFIG_FILE"; else
  CFG=("ERP_LIP2=0" "ERP_ZOOM_LEVELS=0" "ERP_LIP2=0 ERP_LIPG=0"); fi
for e in "${CFG[@]}"; do
  echo "== $e"
  env $e SAME=${SAME:-0} timeout -k 10 300 python scripts/dev/determinism_streams.py 2>&1 | grep -v amdgpu.ids | grep -E "identical|differs|unlike" | cut -c1-300 || exit 1
done
