#!/usr/bin/env python3
"""Regenerate tests/golden/vectors.json: the golden output vectors of SURVEY.md
§8(c), computed by the CPU oracle (oracle/, the SoftwareSpMV restatement that
tests/test_oracle.py pins to the reference's golden.bin files and KATs).

* every reference fixture (tests/golden/matrices) x {ones, 1..n, seeded
  vector} x beta {0, 1}: sha256 of the y bytes plus its first/last 8 words;
* synthetic configs from the numpy generators in synth_numpy.py (C3 at full
  size, a rank-1 shard of it, a small stripe matrix, R-MAT scale 14):
  sha256 + first/last 8 words.

Inputs are defined by splitmix64 (synth_numpy.py), not by numpy's RNG, so the
file is reproducible from this script alone:
    python tests/golden/make_vectors.py        # rewrites vectors.json
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import fixtures as fx  # noqa: E402
import oracle  # noqa: E402
import synth_numpy as sn  # noqa: E402

OUT = os.path.join(HERE, "vectors.json")


def x_inputs(name: str, cols: int) -> dict:
    if "uint64" in name:
        return {"ones": np.ones(cols, np.uint64), "iota": np.arange(1, cols + 1, dtype=np.uint64),
                "sm5": sn.vector_u64(cols, 5)}
    return {"ones": np.ones(cols), "iota": np.arange(1, cols + 1, dtype=np.float64), "sm3": sn.vector_f64(cols, 3)}


def x_input(kind: str, n: int, u64: bool) -> np.ndarray:
    if kind == "ones":
        return np.ones(n, np.uint64) if u64 else np.ones(n)
    if kind == "iota":
        return np.arange(1, n + 1, dtype=np.uint64 if u64 else np.float64)
    if kind == "sm5":
        return sn.vector_u64(n, 5)
    if kind == "sm3":
        return sn.vector_f64(n, 3)
    raise KeyError(kind)


def y0_input(rows: int, u64: bool) -> np.ndarray:
    """the y a beta=1 run accumulates into"""
    return sn.vector_u64(rows, 11) if u64 else sn.vector_f64(rows, 11)


def digest(y: np.ndarray) -> dict:
    w = np.ascontiguousarray(y).view(np.uint64)
    return {"sha256": hashlib.sha256(w.tobytes()).hexdigest(),
            "head": [f"{int(v):016x}" for v in w[:8]], "tail": [f"{int(v):016x}" for v in w[-8:]]}


SYNTHETIC = {
    # name: (generator kwargs, x kinds)
    "stripe_4096x4096_k32": (dict(kind="stripe", row0=0, rows=4096, cols=4096, k=32), ["sm3", "ones"]),
    "C3_1Mx1M_k32": (dict(kind="stripe", row0=0, rows=1 << 20, cols=1 << 20, k=32), ["sm3", "ones"]),
    "C3_rank1_shard_64Kx1M": (dict(kind="stripe", row0=1 << 20, rows=1 << 16, cols=1 << 20, k=32), ["sm3"]),
    "rmat_s14_ef16": (dict(kind="rmat", scale=14, edge_factor=16, seed=4), ["sm3"]),
}


def synth_csr(spec: dict):
    if spec["kind"] == "stripe":
        rowptr, colind, vals = sn.stripe_csr(spec["row0"], spec["rows"], spec["cols"], spec["k"])
        return spec["rows"], spec["cols"], rowptr, colind, vals
    rowptr, colind, vals = sn.rmat_csr(spec["scale"], spec["edge_factor"], spec["seed"])
    n = 1 << spec["scale"]
    return n, n, rowptr, colind, vals


def main() -> None:
    out = {"about": "y = A*x (beta 0) or y0 + A*x (beta 1) from the SoftwareSpMV oracle; "
                    "see tests/golden/make_vectors.py", "fixtures": {}, "synthetic": {}}
    for name in fx.ALL_FIXTURES:
        rows, cols, colptr, rowind, vals = fx.load(name)
        u64 = vals.dtype == np.uint64
        ent = {"rows": rows, "cols": cols, "nnz": int(rowind.size), "cases": {}}
        for xk, x in x_inputs(name, cols).items():
            for beta in (0, 1):
                y = y0_input(rows, u64).copy() if beta else None
                y = oracle.spmv_csc(colptr, rowind, vals, x, y=y, rows=rows)
                ent["cases"][f"{xk}/beta{beta}"] = digest(y)
        out["fixtures"][name] = ent
    for name, (spec, xkinds) in SYNTHETIC.items():
        rows, cols, rowptr, colind, vals = synth_csr(spec)
        colptr, rowind, cvals = oracle.csr2csc(rows, cols, rowptr, colind, vals)
        ent = {"spec": spec, "rows": rows, "cols": cols, "nnz": int(colind.size), "cases": {}}
        for xk in xkinds:
            y = oracle.spmv_csc(colptr, rowind, cvals, x_input(xk, cols, False), rows=rows)
            ent["cases"][f"{xk}/beta0"] = digest(y)
        out["synthetic"][name] = ent
        print(name, ent["nnz"], flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
