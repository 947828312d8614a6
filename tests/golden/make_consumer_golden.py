#!/usr/bin/env python3
"""consumer_golden.npz: the reference's OWN consumers run on this build's outputs (build container only).

SURVEY.md 8(f) rank 2: heatmaps.py and the pickle loaders of analyze_many_seeds.py / Fig5 must run
unchanged on what the sweep drivers write.  Those scripts cannot be imported here (seaborn,
matplotlib, statsmodels and data paths at module top level), but the consumer functions themselves
need only numpy and pandas.  This generator reads the reference sources at generation time, takes
out with `ast` exactly

  * heatmaps.py:30-72          ``extract(filepath, ...)`` plus the module constants it closes over
                               (``states``, ``var_ex``, ``thx``, ``thy``, heatmaps.py:22-28),
  * analyze_many_seeds.py:69-81 ``load(dic)``          (+ ``states``, :19),
  * figures/Fig5/fig5.py:117-129 ``load(dic, nseeds=50)`` (+ ``states``, :24),
  * figures/Fig3/new_figure3.py:81-123 ``extract`` (+ ``states``, ``var_ex``, :46-47) on the homo, map
    and shuffled tables, and its statistics loop :155-164 (Welch-free two-sample t-tests and
    utils.py:18-22 ``cohen_d`` between the optima's seed distributions; the statsmodels FDR step
    :165 is left out, statsmodels is not installed),
  * figures/Fig4/new_figure4.py:103-117, the module-level loop that reads the homo, map and shuffled
    C2 pickles together (+ ``states``, :43) -- top-level statements, not a function, so they are
    taken out by what they assign,

executes those definitions unmodified in a namespace holding numpy and pandas, and applies them to

  (i)  the reference's shipped homogeneous table (output/sweep_delta_homoW_..._9dic24_50iter.txt),
       committed gz'd as tests/golden/shipped_homo_table.csv.gz so the CPU test has the same input;
  (ii) this build's full C3 sweep table (profiles/r06_homo_sweep.txt.gz: 20,000 simulations x the
       full 1001 s schedule, written by `python -m nremmodfc_amd.sweep homo` on one MI355X), and the
       C4 job's map and shuffled-map tables (profiles/r06_{maps,shuf}_sweep.txt.gz, 2 x 20,000);
  (iii) this build's C2 pickles (`python -m nremmodfc_amd.sweep many --modality homo|map|shuf`,
       200 simulations each with device HMA; our own files, loaded with pickle).

Only OUTPUTS are committed (plot matrices, optima, violins; matts, Hin_nodes, Hse_nodes) together
with the sha256 of each input, so tests/test_consumers.py can show that its restatement of these
functions equals the reference's code on the same inputs, and the -m gpu C2 test can show that
the engine regenerates the pickle's contents exactly.  No reference source is copied.

  python tests/golden/make_consumer_golden.py --pickle gpurun_out/r06a/many/run_50seeds_output_homo.pickle \
      --pickle-map gpurun_out/r06n/many/run_50seeds_output_map.pickle \
      --pickle-shuf gpurun_out/r06n/many/run_50seeds_output_shuf.pickle
"""
import argparse
import ast
import gzip
import hashlib
import os
import pickle
import shutil
import sys
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
SHIPPED_HOMO = os.path.join(REF, "output", "sweep_delta_homoW_fromG0.16_sigma7.68_maps_0_0_9dic24_50iter.txt")
SHIPPED_COPY = os.path.join(HERE, "shipped_homo_table.csv.gz")
# the shipped map and shuffled tables (Fig3 reads all three)
SHIPPED_MAPS = os.path.join(REF, "output", "sweep_deltamaps_from_homoW_fromG0.16_sigma7.68_maps_1_1_9dic24_50iter.txt")
SHIPPED_SHUF = os.path.join(REF, "output", "sweep_deltaSHUFFLED_from_homoW_fromG0.16_sigma7.68_maps_2_2_9dic24_50iter.txt")
SHIPPED_MAPS_COPY = os.path.join(HERE, "shipped_maps_table.csv.gz")
SHIPPED_SHUF_COPY = os.path.join(HERE, "shipped_shuf_table.csv.gz")
PRODUCT_TABLE = os.path.join(ROOT, "profiles", "r06_homo_sweep.txt.gz")
# the C4 job's two tables (`sweep maps --map-ids 1 1 2 2 --seeds 50 --seed0 0`, one round-robin job)
PRODUCT_MAPS = os.path.join(ROOT, "profiles", "r06_maps_sweep.txt.gz")
PRODUCT_SHUF = os.path.join(ROOT, "profiles", "r06_shuf_sweep.txt.gz")
STATES = ("W", "N1", "N2", "N3")


def reference_defs(relpath, funcs, consts):
    """The named top-level functions and the FIRST top-level assignment of each named constant of
    a reference source file, executed (unchanged) in a fresh namespace with np and pd."""
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    keep, seen = [], set()
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in funcs:
            keep.append(node)
        elif isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name in consts and name not in seen:
                seen.add(name)
                keep.append(node)
    missing = (set(funcs) | set(consts)) - {getattr(n, "name", None) for n in keep} - seen
    assert not missing, (relpath, missing)
    ns = {"np": np, "pd": pd, "__name__": "ref_" + os.path.basename(relpath)[:-3]}
    exec(compile(ast.Module(body=keep, type_ignores=[]), os.path.join(REF, relpath), "exec"), ns)
    return ns


def shipped_copy(src, dst):
    if not os.path.exists(dst) or pd.read_csv(dst).shape != pd.read_csv(src).shape:
        with open(src, "rb") as fi, gzip.GzipFile(dst, "wb", mtime=0) as fo:
            shutil.copyfileobj(fi, fo)
    assert pd.read_csv(dst).equals(pd.read_csv(src))


def reference_stmts(relpath, names, loop_over, first_only=False, body_has=""):
    """The top-level statements of a reference script that assign one of `names` (every such
    assignment in source order, or only the first of each with first_only) or loop over
    `loop_over` (the first such loop), plus its first ``states`` assignment, compiled unchanged, to
    be executed in a namespace holding what they read: for figure scripts whose loaders and
    statistics are module code, not functions."""
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    keep, seen, have_loop = [], set(), False
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name == "states" and name not in seen:
                seen.add(name)
                keep.append(node)
            elif name in names and not (first_only and name in seen):
                seen.add(name)
                keep.append(node)
        elif (isinstance(node, ast.For) and not have_loop and loop_over in ast.get_source_segment(src, node.iter)
              and body_has in ast.get_source_segment(src, node)):
            have_loop = True
            keep.append(node)
    assert "states" in seen and have_loop and set(names) <= seen, relpath
    code = compile(ast.Module(body=keep, type_ignores=[]), os.path.join(REF, relpath), "exec")
    return code, [ast.get_source_segment(src, n).splitlines()[0] for n in keep]


def array_digest(a):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, dtype=np.float64)).tobytes()).hexdigest()


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def pickle_digest(d):
    """sha256 over the pickle's contents in a fixed order (key order, then each array's bytes):
    independent of how the dict was pickled."""
    h = hashlib.sha256()
    h.update(repr(sorted((k, v) for k, v in d["metainfo"].items())).encode())
    for key in sorted(k for k in d if k != "metainfo"):
        h.update(repr(key).encode())
        v = d[key]
        for name in ("Hin_sim", "Hse_sim", "Hin_node_sim", "Hse_node_sim", "sFC"):
            h.update(name.encode())
            h.update(np.ascontiguousarray(np.asarray(v[name], dtype=np.float64)).tobytes())
    return h.hexdigest()


def heatmap_fields(prefix, out):
    return {f"{prefix}__x_vals": out["x_vals"], f"{prefix}__y_vals": out["y_vals"],
            f"{prefix}__plotmats": np.stack(out["plotmats"]), f"{prefix}__coors_o": np.array(out["coors_o"]),
            f"{prefix}__vals_o": np.array(out["vals_o"]), f"{prefix}__violins_o": np.stack(out["violins_o"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pickle", required=True, help="the C2 pickle written by `sweep many --modality homo`")
    ap.add_argument("--pickle-map", required=True, help="... `--modality map`")
    ap.add_argument("--pickle-shuf", required=True, help="... `--modality shuf`")
    args = ap.parse_args()
    warnings.filterwarnings("ignore")  # heatmaps.py:18-19 does the same (pandas chained-assignment notes)

    hm = reference_defs("heatmaps.py", ["extract"], ["states", "var_ex", "thx", "thy"])
    asm = reference_defs("analyze_many_seeds.py", ["load"], ["states"])
    f5 = reference_defs(os.path.join("figures", "Fig5", "fig5.py"), ["load"], ["states"])

    for src, dst in ((SHIPPED_HOMO, SHIPPED_COPY), (SHIPPED_MAPS, SHIPPED_MAPS_COPY), (SHIPPED_SHUF, SHIPPED_SHUF_COPY)):
        shipped_copy(src, dst)

    out = {}
    # extract() reads the file itself (pd.read_csv(filepath), heatmaps.py:31): give it the paths
    for prefix, path in (("shipped_homo", SHIPPED_COPY), ("product_homo", PRODUCT_TABLE),
                         ("product_maps", PRODUCT_MAPS), ("product_shuf", PRODUCT_SHUF)):
        res = hm["extract"](path)
        out.update(heatmap_fields(prefix, res))
        out[f"{prefix}__sha256"] = np.array(sha256(path))
        print(prefix, [tuple(np.round(v, 4)) for v in res["vals_o"][:4]])

    # Fig3 (new_figure3.py:142-164): its own extract() on the homo, map and shuffled tables, then the
    # t-tests and Cohen's d between the optima's seed distributions, state by state
    from scipy.stats import ttest_ind
    f3 = reference_defs(os.path.join("figures", "Fig3", "new_figure3.py"), ["extract"], ["states", "var_ex"])
    ut = reference_defs("utils.py", ["cohen_d"], [])
    stats_code, stats_lines = reference_stmts(os.path.join("figures", "Fig3", "new_figure3.py"),
                                              {"p_vals", "cohen_ds"}, "enumerate(states)", first_only=True,
                                              body_has="ttest(")
    print("fig3 statements:", stats_lines)
    for which, paths in (("shipped", (SHIPPED_COPY, SHIPPED_MAPS_COPY, SHIPPED_SHUF_COPY)),
                         ("product", (PRODUCT_TABLE, PRODUCT_MAPS, PRODUCT_SHUF))):
        res = [f3["extract"](pth) for pth in paths]
        for mod, r, pth in zip(("homo", "maps", "shuf"), res, paths):
            out.update(heatmap_fields(f"fig3_{which}_{mod}", r))
            out[f"fig3_{which}_{mod}__sha256"] = np.array(sha256(pth))
        ns = {"np": np, "states": STATES, "ttest": ttest_ind, "utils": argparse.Namespace(cohen_d=ut["cohen_d"]),
              "output_homo": res[0], "output_map": res[1], "output_shuf": res[2]}
        exec(stats_code, ns)
        out[f"fig3_{which}__p_vals"] = np.array(ns["p_vals"])
        out[f"fig3_{which}__cohen_ds"] = np.array(ns["cohen_ds"])
        print(which, "fig3 optima", [[tuple(np.round(v[:2], 4)) for v in r["vals_o"][:4]] for r in res])
        print(which, "fig3 p", np.round(ns["p_vals"], 6), "d", np.round(ns["cohen_ds"], 3))

    with open(args.pickle, "rb") as f:  # our own file (written by nremmodfc_amd.sweep)
        d = pickle.load(f)
    out["c2_homo__digest"] = np.array(pickle_digest(d))
    for tag, ns in (("asm", asm), ("fig5", f5)):
        matts, hin, hse = ns["load"]({k: dict(v) if k != "metainfo" else v for k, v in d.items()})
        out[f"c2_homo__{tag}_matts"] = np.stack([matts[s] for s in STATES])
        out[f"c2_homo__{tag}_Hin_nodes"] = np.stack([hin[s] for s in STATES])
        out[f"c2_homo__{tag}_Hse_nodes"] = np.stack([hse[s] for s in STATES])

    # Fig4 (new_figure4.py:94-117): the three pickles read together, keyed by the homo pickle's keys
    fig4, lines = reference_stmts(os.path.join("figures", "Fig4", "new_figure4.py"),
                                  {"homo_matts", "map_matts", "shuf_matts"}, "dic_homo")
    print("fig4 statements:", lines)
    dics = {}
    for mod, path in (("map", args.pickle_map), ("shuf", args.pickle_shuf)):
        with open(path, "rb") as f:  # our own files
            dics[mod] = pickle.load(f)
        out[f"c2_{mod}__digest"] = np.array(pickle_digest(dics[mod]))
    ns = {"np": np, "dic_homo": d, "dic_map": dics["map"], "dic_shuf": dics["shuf"]}
    exec(fig4, ns)
    for mod in ("homo", "map", "shuf"):
        m = np.stack([ns[f"{mod}_matts"][s] for s in STATES])
        if mod == "homo":  # the same seed means as the loaders above: kept as a digest only
            assert np.array_equal(m, out["c2_homo__fig5_matts"])
            out["c2_homo__fig4_matts_sha256"] = np.array(array_digest(m))
        else:
            out[f"c2_{mod}__fig4_matts"] = m
    np.savez_compressed(os.path.join(HERE, "consumer_golden.npz"), **out)
    print("c2 digests", out["c2_homo__digest"], out["c2_map__digest"], out["c2_shuf__digest"])


if __name__ == "__main__":
    main()
