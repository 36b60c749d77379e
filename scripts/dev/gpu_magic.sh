#!/bin/bash
# sampler d < 256 steps by the magic quotient: GPU suite, split forced on for the sampler tests,
# bench A/B against the previous library (two rounds), single-pair latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
A=scripts/dev/libs/base/liberp_match.so
B=erp_match_eightpoint_test_amd/lib/liberp_match.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_magic.log 2>&1 || { tail -30 gpurun_out/pytest_magic.log; exit 1; }
tail -1 gpurun_out/pytest_magic.log
ERP_SAMPLER_SPLIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "sampler or sample or full or find or fixture" > gpurun_out/pytest_magic_split.log 2>&1 || { tail -30 gpurun_out/pytest_magic_split.log; exit 1; }
tail -1 gpurun_out/pytest_magic_split.log
for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  ERP_LIB_PATH=$L timeout -k 10 120 python scripts/latency_probe.py --runs 30 > gpurun_out/lat_magic_$v.json || exit 1
  echo "lat $v $(cat gpurun_out/lat_magic_$v.json)"
done
for r in 1 2; do for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  ERP_LIB_PATH=$L timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --hard-steps 0 --worst-steps 0 > gpurun_out/bench_magic_$v$r.json 2> gpurun_out/bench_magic_$v$r.err || { tail -20 gpurun_out/bench_magic_$v$r.err; exit 1; }
  echo "$v$r $(python -c "import json;d=json.load(open('gpurun_out/bench_magic_$v$r.json'));s=d['stages_ms_serial_step'];print(round(d['value']), round(d['ms_per_step'],2), s['sampler'], d['latency']['single_pair_ms'])")"
done; done
