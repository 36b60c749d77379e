#!/bin/bash
# same-box A/B of the hardware queue count under the 6-stream step (GPU_MAX_HW_QUEUES: HIP maps
# streams onto that many hardware queues; 4 by default, so two of the six sub-batch streams
# share a queue with another)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do for q in 4 6 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --no-cpu-baseline --steps 8 --warmup 2 --hard-steps 0 \
    --worst-steps 0 > gpurun_out/hwq_$q$r.json 2> gpurun_out/hwq_$q$r.err || { tail -20 gpurun_out/hwq_$q$r.err; exit 1; }
  echo "q$q r$r $(python -c "import json;d=json.load(open('gpurun_out/hwq_$q$r.json'));print(round(d['value']), round(d['ms_per_step'],2), d['exact'], d['overlap'])")"
done; done
