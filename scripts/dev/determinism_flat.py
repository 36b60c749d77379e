"""Run-to-run determinism and pruning counts of the consensus on two-cluster configs[1]-shaped
pairs (scripts/twin_seeds.json) under knob settings / variant libraries (a probe; one child
process per setting): (min_idx, survivors, binned_rows) per run and pair, the rows that
survive in some runs only, and the consensus stage times of the batch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import json, os, sys
import numpy as np, torch
torch.cuda.init()
ROOT = %r
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from erp_match_eightpoint_test_amd import Context, PairBatchRunner, results_to_numpy, synth, capi
from test_gpu_parity import _batch
seeds = json.load(open(os.path.join(ROOT, "scripts", "twin_seeds.json")))["seeds"]
args = _batch([synth.make_pair(seeds[i], n_kpts=4096, inlier_frac=0.98) for i in (0, 3, 4, 5)])
out, live = [], []
for it in range(3):
    ctx = Context(0)
    ctx.set_profiling(True)
    o = PairBatchRunner(ctx=ctx, iters=10000).run(*args, want=("dist",))
    torch.cuda.synchronize()
    r = results_to_numpy(o["results"])
    out.append([(int(x["min_idx"]), int(x["survivors"]), int(x["binned_rows"])) for x in r])
    d = o["dist"][0, :int(r[0]["K"])].cpu().numpy()
    live.append(set(np.nonzero(np.isfinite(d))[0].tolist()))
    st = ctx.stage_times()
u, i = set.union(*live), set.intersection(*live)
print(out[0], "same all runs:", all(x == out[0] for x in out), "| pair0 some-runs-only rows:",
      len(u - i), "| ms:", {k: round(v[0], 3) for k, v in st.items() if k.startswith("consensus") and v[1]})
'''
LIBS = os.path.join(ROOT, "devlibs")
for env in ({"ERP_LIB_PATH": os.path.join(LIBS, "liberp_old.so")}, {}, {"ERP_FLAT_REFS": "0"},
            {"ERP_REFINE_HINT": "0"}, {"ERP_FLAT_REFS": "0", "ERP_REFINE_HINT": "0"}):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=e, capture_output=True,
                       text=True, timeout=400)
    print({k: os.path.basename(v) for k, v in env.items()}, r.stdout.strip(),
          r.stderr.strip()[-1500:] if r.returncode else "", flush=True)
