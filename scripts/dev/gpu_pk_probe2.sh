#!/bin/bash
# round 5 bisection, fourth call: packed f32 beside synthetic instruction classes, and beside
# the Gram kernel / the eigen + estimate kernels separately
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
set -o pipefail
: > gpurun_out/pk_probe2.log
timeout -k 10 120 python -u scripts/dev/pk_synth.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/pk_probe2.log &&
env SAMPLER=0 REPS=10 MASKS=8,32 GUARD=0 PAIRS=1 PK=1 timeout -k 10 300 python -u scripts/dev/lds_guard_probe.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/pk_probe2.log
