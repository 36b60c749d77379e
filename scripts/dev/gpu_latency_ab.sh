#!/bin/bash
# round 5: single-pair latency A/B of the small-batch knobs (one process per variant)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
TAG=${TAG:-r05g}
: > gpurun_out/latency_ab_$TAG.txt
for v in "" "ERP_SMALL_ZOOM=0" "ERP_SAMPLER_ILP=1" "ERP_SMALL_ZOOM=0 ERP_SAMPLER_ILP=1" ""; do
  echo "== $v" | tee -a gpurun_out/latency_ab_$TAG.txt
  env $v timeout -k 10 120 python scripts/latency_probe.py --runs 30 2>/dev/null | tee -a gpurun_out/latency_ab_$TAG.txt || exit 1
done
