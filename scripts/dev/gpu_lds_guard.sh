#!/bin/bash
# LDS-interference probe runs (scripts/dev/lds_guard_probe.py), one process per configuration
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
run() {  # name, env...
  local name=$1; shift
  echo "== $name" | tee -a gpurun_out/lds_guard.log
  env "$@" timeout -k 10 300 python -u scripts/dev/lds_guard_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/lds_guard.log
}
: > gpurun_out/lds_guard.log
run glibc SAMPLER=0 REPS=${REPS:-10} MASKS=${MASKS:-1,2,4,8,16,31} &&
run philox SAMPLER=1 REPS=${REPS:-10} MASKS=4,31 PAIRS=${PPAIRS:-1} &&
run glibc_clamp SAMPLER=0 REPS=${REPS:-10} MASKS=4,31 ERP_LIB_PATH=scripts/dev/libs/clamp/liberp_match.so
