#!/bin/bash
# round 5 bisection, second call: guard launched behind the stage; verify build of the pruning pass
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
run() {
  local name=$1; shift
  echo "== $name" | tee -a gpurun_out/lds_guard2.log
  env "$@" timeout -k 10 300 python -u scripts/dev/lds_guard_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/lds_guard2.log
}
: > gpurun_out/lds_guard2.log
run guard_after SAMPLER=0 REPS=20 MASKS=1,8,31 GUARD_AFTER=1 PAIRS=0 &&
run verify SAMPLER=0 REPS=10 MASKS=8,31 GUARD=0 ERP_LIB_PATH=scripts/dev/libs/verify/liberp_match.so
