#!/bin/bash
# split-kernel phase stamps of three library versions on one box (diagnostic builds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in st0 stamps; do
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 120 python scripts/latency_probe.py --runs 2 > gpurun_out/stamps_$v.log 2>&1 || exit 1
  echo "== $v"; grep -a "split wave" gpurun_out/stamps_$v.log | tail -4 | sort
  ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 120 python scripts/latency_probe.py --runs 30 > gpurun_out/lat_$v.json 2>/dev/null || exit 1
done
for g in "" "--graph"; do timeout -k 10 120 python scripts/latency_probe.py --runs 30 $g || exit 1; done
