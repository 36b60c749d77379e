"""Result records and hypothesis records of one seeded 48-pair batch (10k iterations) through the
library ERP_LIB_PATH names, saved to --out (.npz): two libraries' outputs compared byte for byte
(a change that claims identical results, e.g. a reformulated exact recombination)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--pairs", type=int, default=48)
    ap.add_argument("--worst", action="store_true")
    a = ap.parse_args()
    import torch
    from erp_match_eightpoint_test_amd import Context, PairBatchRunner
    pairs = (bench.make_worst_batch(0, a.pairs, 4096, 0.03) if a.worst
             else bench.make_batch(0, a.pairs, 4096, 20200423))
    b = bench.to_device(pairs, "cuda")
    run = PairBatchRunner(ctx=Context(0), iters=10000)
    o = run.run(b["desc_l"], b["desc_r"], b["kp_l"], b["kp_r"], b["off_l"], b["off_r"], b["width"],
                b["height"], b["max_nq"], b["max_nt"], want=("hyps", "rvec", "tvec"))
    torch.cuda.synchronize()
    np.savez(a.out, **{k: v.cpu().numpy() for k, v in o.items()})
    print(a.out, {k: tuple(v.shape) for k, v in o.items()})


if __name__ == "__main__":
    main()
