#!/bin/bash
# consensus GPU tests + binned-row counts of single-cluster sets (Lipschitz pre-pruning)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "consensus or batch or find" > gpurun_out/pytest_cons.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_cons.log; [ $rc -ne 0 ] && exit $rc
python - <<'PY'
import numpy as np, sys
sys.path.insert(0, ".")
import torch
torch.zeros(1, device='cuda')
from erp_match_eightpoint_test_amd import dist as D, Context
ctx = Context(0)
rng = np.random.default_rng(11)
for K in (2000, 6000, 20000):
    rv = (rng.standard_normal((K, 3)) * 6e-5 + 0.2).astype(np.float32)
    r = D.gpu_consensus(ctx, "cuda")(rv, np.zeros_like(rv))
    print(K, "binned", r["binned_rows"], "surv", r["survivors"])
PY
echo "== bench" && timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_dev.json 2> gpurun_out/bench_dev.err || { tail -20 gpurun_out/bench_dev.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_dev.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline_stages']['consensus_bounds'], d['stages_ms_serial_step']['consensus_bounds'])"
export TMPDIR=/tmp
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dev -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 0 --warmup 1 --pairs 128 --streams 1 > gpurun_out/prof_dev.log 2>&1 || { tail -20 gpurun_out/prof_dev.log; exit 1; }
find gpurun_out/prof_dev -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-5 {} | head -30'
