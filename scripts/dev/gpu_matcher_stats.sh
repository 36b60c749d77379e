#!/bin/bash
# matcher probe under rocprofv3 kernel stats + the correctness probe (dev)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ms}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof_${TAG} -o run --output-format csv -- ./scripts/dev/matcher_probe 128 4096 > gpurun_out/mprobe_${TAG}.txt 2>&1 || exit 1
grep -v "^[0-9]*:" gpurun_out/mprobe_${TAG}.txt | head -8
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/mprof_${TAG}/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
"
timeout -k 10 200 python scripts/dev/matcher_debug.py > gpurun_out/mdbg_${TAG}.txt 2>&1; tail -2 gpurun_out/mdbg_${TAG}.txt
