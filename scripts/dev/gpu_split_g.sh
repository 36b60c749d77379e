#!/bin/bash
# split replay: segments per iteration group (variant libraries), single-pair latency + trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in g2 default g5 g7; do
  if [ $v = default ]; then L=erp_match_eightpoint_test_amd/lib/liberp_match.so; else L=scripts/dev/libs/$v/liberp_match.so; fi
  ERP_LIB_PATH=$L timeout -k 10 120 python scripts/latency_probe.py --runs 30 > gpurun_out/lat_$v.json || exit 1
  ERP_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/latg_$v -o run --output-format csv -- python3 scripts/latency_probe.py --runs 10 > gpurun_out/latg_$v.log 2>&1 || exit 1
  python scripts/latency_probe.py --report $(find gpurun_out/latg_$v -name "*kernel_trace.csv" | head -1) --runs 10 > gpurun_out/latg_$v.trace.json || exit 1
  echo "$v $(python -c "import json;a=json.load(open('gpurun_out/lat_$v.json'));d=json.load(open('gpurun_out/latg_$v.trace.json'));print(round(a['single_pair_ms_median'],4), d['span_us_median'], d['kernels_us_in_median_run'].get('sampler_split_kernel'))")"
done
ERP_LIB_PATH=scripts/dev/libs/g7/liberp_match.so ERP_SAMPLER_SPLIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sampler or sample or full or find or fixture" > gpurun_out/pytest_g7.log 2>&1 || { tail -30 gpurun_out/pytest_g7.log; exit 1; }
tail -1 gpurun_out/pytest_g7.log
