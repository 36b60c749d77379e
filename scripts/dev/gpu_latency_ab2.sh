#!/bin/bash
# round 5: single-pair latency, plain and HIP-graph replay, a few repeats (one process each)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
TAG=${TAG:-r05m}
: > gpurun_out/latency_ab_$TAG.txt
for v in "" "--graph" "" "--graph"; do
  echo "== $v" | tee -a gpurun_out/latency_ab_$TAG.txt
  timeout -k 10 120 python scripts/latency_probe.py --runs 50 $v 2>/dev/null | tee -a gpurun_out/latency_ab_$TAG.txt || exit 1
done
