"""The reference's own consumers of the sweep outputs, on this build's outputs.

heatmaps.py, analyze_many_seeds.py and figures/Fig5/fig5.py cannot be imported here (seaborn,
matplotlib, statsmodels and data paths at module top level), and /root/reference does not travel
to the GPU box.  tests/golden/make_consumer_golden.py therefore ran the REFERENCE's own functions --
heatmaps.py:30-72 ``extract``, Figure 3's ``extract`` and statistics loop (new_figure3.py:81-123,
155-164) and the pickle loaders analyze_many_seeds.py:69-81 / fig5.py:117-129
``load``, taken out of the sources with ``ast`` and executed unmodified -- on

  * the shipped homogeneous, map and shuffled tables (tests/golden/shipped_{homo,maps,shuf}_table.csv.gz),
  * this build's full C3 sweep (profiles/r06_homo_sweep.txt.gz: 20,000 simulations x 1001 s on one
    MI355X, `python -m nremmodfc_amd.sweep homo`) and the C4 job's two tables (r06_{maps,shuf}_sweep),
  * this build's C2 pickles (`sweep many --modality homo|map|shuf`, 200 simulations each, device HMA),
    read by those loaders and by Fig4's module-level loop (figures/Fig4/new_figure4.py:103-117),

and committed their outputs (tests/golden/consumer_golden.npz).  The restatements below must give
those outputs EXACTLY on the same inputs; the -m gpu tests regenerate the C2 pickles with the engine
(deterministic) and checks their contents against the digests of the ones the reference's code read.
Fig5's ``corr_HMA`` / ``load_dfs`` (fig5.py:134-198) compare against the shipped empirical pickle
(output/emp_15inds_output_16dic.pickle): a pickle shipped inside the reference, which no safe loader
reads, so they are not run; their per-model part is ``load``, pinned above.
"""
import os

import numpy as np
import pandas as pd
import pytest

from tests.golden.make_consumer_golden import array_digest, pickle_digest, sha256

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "consumer_golden.npz")
SHIPPED = os.path.join(ROOT, "tests", "golden", "shipped_homo_table.csv.gz")
SHIPPED_MAPS = os.path.join(ROOT, "tests", "golden", "shipped_maps_table.csv.gz")
SHIPPED_SHUF = os.path.join(ROOT, "tests", "golden", "shipped_shuf_table.csv.gz")
PRODUCT = os.path.join(ROOT, "profiles", "r06_homo_sweep.txt.gz")
PRODUCT_MAPS = os.path.join(ROOT, "profiles", "r06_maps_sweep.txt.gz")   # the C4 job's two tables
PRODUCT_SHUF = os.path.join(ROOT, "profiles", "r06_shuf_sweep.txt.gz")
STATES = ("W", "N1", "N2", "N3")
VAR_EX = {"euccorr": "min", "e": "min", "ssim": "max", "corr": "max"}  # heatmaps.py:23
THX, THY = (-0.08, 0.2), (-0.2, 0.08)                                  # heatmaps.py:28


def extract(data_pre, xv="delta_G", yv="delta_sigma", var2see="euccorr", C1=0, w=1, thx=THX, thy=THY):
    """heatmaps.py:30-72 restated (takes the DataFrame instead of the path); the same dict."""
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


def extract_fig3(data_pre, xv="delta_G", yv="delta_sigma", var2see="euccorr", C1=0, w=1, thx=THX, thy=THY):
    """figures/Fig3/new_figure3.py:81-123 restated: heatmaps' extract with the grid values rounded
    to two decimals first (:83-84)."""
    data_pre = data_pre.copy()
    data_pre[xv] = np.round(data_pre[xv].values, decimals=2)
    data_pre[yv] = np.round(data_pre[yv].values, decimals=2)
    return extract(data_pre, xv, yv, var2see, C1, w, thx, thy)


def fig3_stats(out_homo, out_map, out_shuf):
    """new_figure3.py:155-164 restated: per state, the two-sample t-test p-value and Cohen's d
    (utils.py:18-22) of homo vs map and shuffled vs map, over the optima's seed distributions."""
    from scipy.stats import ttest_ind
    from nremmodfc_amd.utils import cohen_d
    p, d = [], []
    for s in range(len(STATES)):
        h, m, sh = (o["violins_o"][s] for o in (out_homo, out_map, out_shuf))
        p += [ttest_ind(h, m)[1], ttest_ind(sh, m)[1]]
        d += [cohen_d(h, m), cohen_d(sh, m)]
    return np.array(p), np.array(d)


def fdr_bh(p):
    """Benjamini-Hochberg adjusted p-values (statsmodels' multipletests(method='fdr_bh'), which
    new_figure3.py:165 applies; statsmodels is not installed here, so this step is restated only:
    parity unpinned)."""
    p = np.asarray(p, dtype=float)
    order = np.argsort(p)
    adj = p[order] * len(p) / np.arange(1, len(p) + 1)
    adj = np.minimum.accumulate(adj[::-1])[::-1]
    out = np.empty_like(adj)
    out[order] = np.minimum(adj, 1.0)
    return out


def load_many_seeds(dic, nseeds=None):
    """analyze_many_seeds.py:69-81 (nseeds from "metainfo") / fig5.py:117-129 (nseeds=50) restated:
    per-state seed-mean FC, and the per-seed nodal integration / segregation."""
    n = {st: (dic["metainfo"][st] if nseeds is None else nseeds) for st in STATES}
    matts = {st: np.zeros((n[st], 90, 90)) for st in STATES}
    hin = {st: np.zeros((n[st], 90)) for st in STATES}
    hse = {st: np.zeros((n[st], 90)) for st in STATES}
    for key, v in dic.items():
        if key != "metainfo":
            s, state = key
            matts[state][s] = v["sFC"]
            hin[state][s] = v["Hin_node_sim"]
            hse[state][s] = v["Hse_node_sim"]
    return {st: matts[st].mean(axis=0) for st in STATES}, hin, hse


def _check_extract_equals_reference(path, prefix, fn=extract):
    g = np.load(GOLD)
    assert sha256(path) == str(g[f"{prefix}__sha256"]), f"{path} is not the input the reference's extract() read"
    ours = fn(pd.read_csv(path))
    np.testing.assert_array_equal(ours["x_vals"], g[f"{prefix}__x_vals"])
    np.testing.assert_array_equal(ours["y_vals"], g[f"{prefix}__y_vals"])
    np.testing.assert_array_equal(np.stack(ours["plotmats"]), g[f"{prefix}__plotmats"])
    np.testing.assert_array_equal(np.array(ours["coors_o"]), g[f"{prefix}__coors_o"])
    np.testing.assert_array_equal(np.array(ours["vals_o"]), g[f"{prefix}__vals_o"])
    np.testing.assert_array_equal(np.stack(ours["violins_o"]), g[f"{prefix}__violins_o"])
    return ours


def test_restated_extract_equals_reference_on_shipped_table():
    ours = _check_extract_equals_reference(SHIPPED, "shipped_homo")
    # and the reference's own code gives the optima run_many_seeds.py:34-38 quotes for the
    # homogeneous model: W (0, 0), N1 (0.04, 0), N2 (0, 0), N3 (-0.04, 0.04)
    want = [(0.0, 0.0), (0.04, 0.0), (0.0, 0.0), (-0.04, 0.04)]
    assert [tuple(np.round(v[:2], 4)) for v in ours["vals_o"][:4]] == want


def test_restated_extract_equals_reference_on_this_builds_sweep():
    _check_extract_equals_reference(PRODUCT, "product_homo")


def test_restated_extract_equals_reference_on_the_c4_tables():
    """The C4 job (`sweep maps --map-ids 1 1 2 2 --seeds 50 --seed0 0`) writes the map and the
    shuffled-map tables; the reference's extract() read both.  On the shuffled table it finds exactly
    the optima run_many_seeds.py:44-47 quotes, on the map table those of N1 and N2 (:39-42; W and N3
    sit one or two grid steps away on the flat valley of the published, seed-irreproducible runs)."""
    maps = _check_extract_equals_reference(PRODUCT_MAPS, "product_maps")
    shuf = _check_extract_equals_reference(PRODUCT_SHUF, "product_shuf")
    opt = lambda r: [tuple(float(x) for x in np.round(v[:2], 4)) for v in r["vals_o"][:4]]  # noqa: E731
    assert opt(shuf) == [(0.0, 0.0), (0.0, 0.04), (0.0, 0.0), (0.0, -0.04)]
    assert opt(maps)[1:3] == [(0.18, -0.02), (0.02, -0.04)]


def test_fig3_extract_and_statistics_equal_reference():
    """Figure 3 (new_figure3.py:138-165) on the shipped homo, map and shuffled tables and on this
    build's three: the restated extract and t-test / Cohen's d loop equal the reference's code on
    the same inputs exactly.  On the build's tables, as on the shipped ones, every homo-vs-map and
    shuffled-vs-map difference of the optima's seed distributions is significant after the FDR step
    (restated, statsmodels absent) with the same sign of Cohen's d."""
    g = np.load(GOLD)
    adj = {}
    for which, paths in (("shipped", (SHIPPED, SHIPPED_MAPS, SHIPPED_SHUF)),
                         ("product", (PRODUCT, PRODUCT_MAPS, PRODUCT_SHUF))):
        res = [_check_extract_equals_reference(pth, f"fig3_{which}_{mod}", extract_fig3)
               for mod, pth in zip(("homo", "maps", "shuf"), paths)]
        p, d = fig3_stats(*res)
        np.testing.assert_array_equal(p, g[f"fig3_{which}__p_vals"])
        np.testing.assert_array_equal(d, g[f"fig3_{which}__cohen_ds"])
        adj[which] = (fdr_bh(p), d)
        print(which, "FDR p", np.round(adj[which][0], 6), "d", np.round(d, 3))
    assert (adj["shipped"][0] < 0.05).all() and (adj["product"][0] < 0.05).all()
    np.testing.assert_array_equal(np.sign(adj["product"][1]), np.sign(adj["shipped"][1]))


def test_heatmaps_of_this_builds_sweep_track_the_shipped_ones():
    """The reference's extract() output on the build's table against its output on the shipped
    table (both from consumer_golden.npz): the same axes, cell maps correlated > 0.99, the same W
    optimum; the sleep states' optima lie on a flat valley (within 5% of the shipped optimum's value)."""
    g = np.load(GOLD)
    np.testing.assert_array_equal(g["product_homo__x_vals"], g["shipped_homo__x_vals"])
    np.testing.assert_array_equal(g["product_homo__y_vals"], g["shipped_homo__y_vals"])
    for k, st in enumerate(STATES + ("mean", "sync", "meta")):
        a, b = g["shipped_homo__plotmats"][k], g["product_homo__plotmats"][k]
        r = np.corrcoef(a.ravel(), b.ravel())[0, 1]
        rel = np.abs(b - a).max() / np.abs(a).max()
        print(f"{st}: cell maps r = {r:.4f}, max relative cell difference {rel:.3f}")
        assert r > 0.99 and rel < 0.08, (st, r, rel)
    ours, ship = g["product_homo__vals_o"], g["shipped_homo__vals_o"]
    assert tuple(np.round(ours[0][:2], 4)) == (0.0, 0.0)
    for k in range(1, 4):
        assert ours[k][2] <= ship[k][2] * 1.05


def fig4_matts(dic_homo, dic_map, dic_shuf):
    """figures/Fig4/new_figure4.py:103-117 restated: the three C2 pickles read together under the
    homo pickle's keys; per modality and state the mean over the 50 seeds of sFC."""
    out = {}
    for mod, dic in (("homo", dic_homo), ("map", dic_map), ("shuf", dic_shuf)):
        m = {st: np.zeros((50, 90, 90)) for st in STATES}
        for key in dic_homo:
            if key != "metainfo":
                s, state = key
                m[state][s] = dic[key]["sFC"]
        out[mod] = np.stack([m[st].mean(axis=0) for st in STATES])
    return out


@pytest.fixture(scope="module")
def c2_pickles(tmp_path_factory, cuda):
    """run_many_seeds.py (C2) through the product on this GPU for the three modalities."""
    import pickle
    from nremmodfc_amd import sweep
    out = str(tmp_path_factory.mktemp("c2"))
    dics = {}
    for mod in ("homo", "map", "shuf"):
        sweep.main(["many", "--modality", mod, "--out", out, "--tag", f"c2{mod}"])
        with open(os.path.join(out, f"c2{mod}.pickle"), "rb") as f:  # our own file
            dics[mod] = pickle.load(f)
    return dics


@pytest.mark.gpu
def test_c2_pickle_regenerates_and_loads_like_the_reference(c2_pickles):
    """run_many_seeds.py (C2, homogeneous optima) through the product on this GPU: the pickle's
    contents equal the pickle the reference's loaders read when the fixture was made (sha256 of
    every array), and the restated loaders give the reference's matts / Hin_nodes / Hse_nodes."""
    d = c2_pickles["homo"]
    g = np.load(GOLD)
    assert pickle_digest(d) == str(g["c2_homo__digest"])
    for tag, nseeds in (("asm", None), ("fig5", 50)):
        matts, hin, hse = load_many_seeds(d, nseeds)
        np.testing.assert_array_equal(np.stack([matts[s] for s in STATES]), g[f"c2_homo__{tag}_matts"])
        np.testing.assert_array_equal(np.stack([hin[s] for s in STATES]), g[f"c2_homo__{tag}_Hin_nodes"])
        np.testing.assert_array_equal(np.stack([hse[s] for s in STATES]), g[f"c2_homo__{tag}_Hse_nodes"])


@pytest.mark.gpu
def test_c2_map_and_shuffled_pickles_load_like_fig4(c2_pickles):
    """Fig4 (new_figure4.py:94-117) reads the homo, map and shuffled C2 pickles together, indexing
    the map and shuffled ones with the homo pickle's keys: the regenerated map and shuffled pickles
    equal the ones the reference's Fig4 statements read (digests), share the homo pickle's keys, and
    the restated loop gives the reference's seed-mean FCs exactly."""
    g = np.load(GOLD)
    for mod in ("map", "shuf"):
        assert pickle_digest(c2_pickles[mod]) == str(g[f"c2_{mod}__digest"])
        assert set(c2_pickles[mod]) == set(c2_pickles["homo"])
    got = fig4_matts(c2_pickles["homo"], c2_pickles["map"], c2_pickles["shuf"])
    assert array_digest(got["homo"]) == str(g["c2_homo__fig4_matts_sha256"])
    for mod in ("map", "shuf"):
        np.testing.assert_array_equal(got[mod], g[f"c2_{mod}__fig4_matts"])
