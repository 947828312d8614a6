"""The reference's own consumer of the sweep table, heatmaps.py, on this build's output.

heatmaps.py cannot be imported here (seaborn, matplotlib at module top), so its extract()
(heatmaps.py:30-72) is restated line for line below, without the plotting; the restatement
reproduces the optima run_many_seeds.py:34-38 quotes for the homogeneous model when applied to
the shipped table (tests/golden/shipped_heatmaps.npz, made by make_heatmap_golden.py).

Applied to this build's full homogeneous sweep (profiles/r02_homo_sweep.txt.gz: 20,000
simulations x 1001 s, read with pandas exactly as heatmaps.py reads output/*.txt) it must give
euccorr maps that track the shipped ones cell by cell, and the same W optimum.
"""
import os

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATES = ("W", "N1", "N2", "N3")
VAR_EX = {"euccorr": "min", "e": "min", "ssim": "max", "corr": "max"}  # heatmaps.py:23
THX, THY = (-0.08, 0.2), (-0.2, 0.08)                                  # heatmaps.py:26


def extract(data_pre, xv="delta_G", yv="delta_sigma", var2see="euccorr", C1=0, w=1, thx=THX, thy=THY):
    """heatmaps.py:30-72 without the violin padding's plotting use; returns the same dict."""
    nseed = 50
    data_pre = data_pre[(thx[0] <= data_pre[xv]) & (data_pre[xv] <= thx[1]) & (thy[0] <= data_pre[yv])
                        & (data_pre[yv] <= thy[1])].copy()
    for st in STATES:
        data_pre[f"euccorr{st}"] = data_pre[f"e{st}"] / (C1 + w * abs(data_pre[f"corr{st}"]))
    data = data_pre.groupby([xv, yv]).agg("mean").reset_index()  # agg(np.nanmean): no NaN in the tables
    x_vals = np.sort(data[xv].unique())
    y_vals = np.sort(data[yv].unique())
    plotmats, coors_o, vals_o, violins_o = [], [], [], []
    for var in [var2see + s for s in STATES] + ["mean", "sync", "meta"]:
        plotmat = np.zeros((len(y_vals), len(x_vals)))
        for i, d2 in enumerate(y_vals):
            plotmat[i, :] = data[data[yv] == d2].sort_values(xv)[var].values
        if VAR_EX[var2see] == "min":
            iy, ix = np.unravel_index(plotmat.argmin(), plotmat.shape)
        else:
            iy, ix = np.unravel_index(plotmat.argmax(), plotmat.shape)
        xo, yo, oval = x_vals[ix], y_vals[iy], plotmat[iy, ix]
        violin = data_pre[(data_pre[xv] == xo) & (data_pre[yv] == yo)][var].values
        violin = np.array(list(violin) + (nseed - len(violin)) * [violin.mean()])
        plotmats.append(plotmat)
        coors_o.append((ix, iy))
        vals_o.append((xo, yo, oval))
        violins_o.append(violin)
    return {"x_vals": x_vals, "y_vals": y_vals, "plotmats": plotmats, "coors_o": coors_o, "vals_o": vals_o,
            "violins_o": violins_o}


def test_restated_consumer_gives_the_reference_optima():
    g = np.load(os.path.join(ROOT, "tests", "golden", "shipped_heatmaps.npz"))
    # run_many_seeds.py:34-38, homogeneous: W (0, 0), N1 (0.04, 0), N2 (0, 0), N3 (-0.04, 0.04)
    want = [(0.0, 0.0), (0.04, 0.0), (0.0, 0.0), (-0.04, 0.04)]
    assert [tuple(np.round(v[:2], 4)) for v in g["vals_o"][:4]] == want


def test_heatmaps_on_this_builds_full_sweep():
    ours = extract(pd.read_csv(os.path.join(ROOT, "profiles", "r02_homo_sweep.txt.gz")))
    g = np.load(os.path.join(ROOT, "tests", "golden", "shipped_heatmaps.npz"))
    np.testing.assert_allclose(ours["x_vals"], g["x_vals"])
    np.testing.assert_allclose(ours["y_vals"], g["y_vals"])
    for k, st in enumerate(STATES + ("mean", "sync", "meta")):
        a, b = g["plotmats"][k], ours["plotmats"][k]
        r = np.corrcoef(a.ravel(), b.ravel())[0, 1]
        rel = np.abs(b - a).max() / np.abs(a).max()
        print(f"{st}: cell maps r = {r:.4f}, max relative cell difference {rel:.3f}")
        assert r > 0.99 and rel < 0.08, (st, r, rel)
    assert tuple(np.round(ours["vals_o"][0][:2], 4)) == (0.0, 0.0)  # the W optimum of the model
    # the other states' optima sit on a flat valley: each of ours is within 0.05 of the shipped
    # one's euccorr value at the shipped optimum
    for k in range(1, 4):
        xo, yo, oval = g["vals_o"][k]
        assert ours["vals_o"][k][2] <= oval * 1.05
