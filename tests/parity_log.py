"""Measured parity deviations of the GPU tests (VERDICT r05 "next" 7).

The estimator tests compare float outputs with the oracle under fixed bars (tests/test_gpu_*.py);
record() keeps, per fixture, the LARGEST deviation each comparison actually saw, so the bars can
be judged against measurements.  With ERP_PARITY_OUT=<path> set, conftest.pytest_sessionfinish
writes the table as JSON (scripts/gpu_check.sh keeps it under profiles/).  Keys:
  R: the Euler angles (rad; {R1, R2} as a set for per-iteration records), T: the unit
  translation, E: the solved 9-vector up to sign, per iteration or final (the winner's).
"""
from __future__ import annotations

import json
import os

_TABLE: dict = {}


def record(fixture: str, **devs) -> None:
    """keep the max over every call of each named deviation of `fixture`"""
    d = _TABLE.setdefault(fixture, {})
    for k, v in devs.items():
        d[k] = max(d.get(k, 0.0), float(v))


def dump() -> None:
    path = os.environ.get("ERP_PARITY_OUT")
    if not path or not _TABLE:
        return
    out = {"note": "largest |GPU - oracle| seen per fixture and quantity (rad for R, unit "
                   "vector components for T, 9-vector components up to sign for E); bars: "
                   "R, T 1e-6 (SURVEY 8c), E 1e-6", "fixtures": _TABLE}
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
