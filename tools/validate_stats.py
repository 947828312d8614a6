"""Statistical validation of a full-length sweep against the reference's shipped tables.

    python tools/validate_stats.py <collapsed.txt> <homo|maps|shuf> [out.json]

The reference's published runs are not seed-reproducible (numba RNG seeded
from os.urandom), so the check is per grid cell: the mean over
seeds of every metric column against the shipped per-cell mean
(tests/golden/shipped_cell_stats.npz), as a z-score with the two-sample
standard error sqrt(s1^2/n1 + s2^2/n2).  Reported per metric: the fraction of
cells with |z| < 3, the median |z|, and the mean difference relative to the
spread of the shipped cell means.
"""
import json
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))


def compare(path, kind):
    st = np.load(os.path.join(HERE, "..", "tests", "golden", "shipped_cell_stats.npz"))
    cols = list(st["columns"])
    df = pd.read_csv(path).drop_duplicates(subset=["seed", "delta_G", "delta_sigma"])
    g = df.drop(columns=["rank", "seed"]).groupby(["delta_G", "delta_sigma"])
    mean, std, cnt = g.mean(), g.std(), g.size()
    ref_cells = [tuple(c) for c in st[f"{kind}_cells"]]
    idx = {c: i for i, c in enumerate(ref_cells)}
    rows = [idx[(round(a, 4), round(b, 4))] for a, b in mean.index]
    rm, rs, rn = st[f"{kind}_mean"][rows], st[f"{kind}_std"][rows], st[f"{kind}_count"][rows]
    m, s, n = mean[cols].to_numpy(), std[cols].to_numpy(), cnt.to_numpy()[:, None]
    se = np.sqrt(s ** 2 / n + rs ** 2 / rn[:, None])
    z = (m - rm) / np.where(se > 0, se, np.inf)
    out = {"file": os.path.basename(path), "kind": kind, "cells": len(rows), "sims": int(n.sum()), "metrics": {}}
    for j, c in enumerate(cols):
        spread = rm[:, j].std()
        out["metrics"][c] = {"frac_cells_absz_lt3": float(np.mean(np.abs(z[:, j]) < 3)),
                             "median_absz": float(np.median(np.abs(z[:, j]))),
                             "mean_diff": float(np.mean(m[:, j] - rm[:, j])),
                             "mean_diff_over_cell_spread": float(np.mean(m[:, j] - rm[:, j]) / spread) if spread else None,
                             "corr_of_cell_means": float(np.corrcoef(m[:, j], rm[:, j])[0, 1]) if spread else None}
    return out


if __name__ == "__main__":
    res = compare(sys.argv[1], sys.argv[2])
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(txt)
    for c, v in res["metrics"].items():
        print(f"{c:9s} |z|<3: {v['frac_cells_absz_lt3']:.2f}  med|z| {v['median_absz']:.2f}  "
              f"diff {v['mean_diff']:+.4f}  r(cell means) {v['corr_of_cell_means']}")
