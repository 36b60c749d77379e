#!/bin/bash
# byte comparison of two libraries' records (scripts/dev/dump_records.py, a normal and a
# worst-case batch), then the A/B of scripts/dev/gpu_list_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in ${LIBS:-base join}; do
  for kind in normal worst; do
    W=""; [ $kind = worst ] && W=--worst
    ERP_LIB_PATH=scripts/dev/libs/$v/liberp_match.so timeout -k 10 300 python scripts/dev/dump_records.py \
      --out /tmp/rec_${TAG}_${v}_$kind.npz $W > gpurun_out/rec_${TAG}_${v}_$kind.log 2>&1 \
      || { tail -20 gpurun_out/rec_${TAG}_${v}_$kind.log; exit 1; }
  done
done
python - <<'PY'
import numpy as np, os
tag = os.environ["TAG"]; libs = os.environ.get("LIBS", "base join").split()
for kind in ("normal", "worst"):
    a = np.load(f"/tmp/rec_{tag}_{libs[0]}_{kind}.npz"); b = np.load(f"/tmp/rec_{tag}_{libs[1]}_{kind}.npz")
    print(kind, {k: bool(np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))) for k in a.files})
PY
bash scripts/dev/gpu_list_ab.sh
