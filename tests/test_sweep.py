"""Sweep drivers (nremmodfc_amd/sweep.py) against the reference drivers' lists,
formats and the shipped output tables (tests/golden/shipped_*_head.csv are the
first rows of /root/reference/output/*.txt, copied by make_golden.py)."""
import itertools
import json
import os

import numpy as np
import pytest

from nremmodfc_amd import datasets, sweep

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_homo_list_matches_reference_product():
    sims = sweep.homogeneous(n_iterations=3, n_init=5)
    dG = np.linspace(-0.1, 0.3, 20, endpoint=False)
    dS = np.linspace(-0.2, 0.2, 20, endpoint=False)
    ref = list(itertools.product(np.arange(5, 8), dG, dS))  # whole_sweep_both_maps.py:92-96
    assert len(sims) == len(ref) == 1200
    for s, (seed, g, d) in zip(sims, ref):
        assert (s.seed, s.dG, s.dsigma) == (seed, g, d)
        np.testing.assert_array_equal(s.G, 0.16 + g * np.ones(90))
        np.testing.assert_array_equal(s.sigma, 7.68 + d * np.ones(90))
    assert len({(s.seed, s.stream) for s in sims}) == len(sims)  # distinct noise streams


def test_script_grid():
    sims = sweep.homogeneous(1, 0, grid="script")
    assert sims[21].dG == np.linspace(-0.1, 0.5, 20, endpoint=False)[1]
    assert sims[21].dsigma == np.linspace(-1, 1, 20, endpoint=False)[1]


def test_maps_list():
    sims = sweep.maps(1, 1, n_iterations=1, n_init=25)
    ach = np.load(os.path.join(datasets.DATA, "DIST_VAChT_feobv_hc18_aghourian.npy"))
    na = np.load(os.path.join(datasets.DATA, "DIST_LC_proj.npy"))
    ach, na = ach / ach.mean(), na / na.mean()  # in the file dtype (float32 for VAChT), :57/:65
    s = sims[47]
    np.testing.assert_array_equal(s.G, 0.16 + s.dG * ach)  # whole_sweep_both_maps.py:103-106
    np.testing.assert_array_equal(s.sigma, 7.68 + s.dsigma * na)
    assert s.seed == 25


def test_many_seeds_list():
    sims = sweep.many_seeds("map", n_iterations=2)
    assert [(s.seed, s.state) for s in sims] == list(itertools.product(range(2), datasets.STATES))
    n1 = sims[1]
    ach = datasets.load_map(datasets.MAPNAMES_ACH[1])
    np.testing.assert_allclose(n1.G, 0.16 + ach * 0.18)
    assert sweep.many_seeds("homo", 1)[3].dG == -0.04


def test_shard_is_reference_round_robin():
    sims = sweep.homogeneous(2)
    parts = [sweep.shard(sims, r, 7) for r in range(7)]
    assert sorted(s.index for p in parts for s in p) == list(range(len(sims)))
    assert all(s.index % 7 == r for r, p in enumerate(parts) for s in p)


def test_c4_job_round_robin_over_both_tables():
    """BASELINE config 4 as one job: `maps --map-ids 1 1 2 2 --seeds 50 --seed0 0` lists the real-map
    and the shuffled sweeps (2 x 20,000, whole_sweep_both_maps.py:27-28,92-108) and deals their
    concatenation round robin, so each of 8 ranks holds 5,000 simulations, half of each table;
    one table alone is the reference's `sim % threads == rank`."""
    args = sweep.argparse.Namespace(kind="maps", map_ids=[1, 1, 2, 2], seeds=50, seed0=0, grid="shipped", nodes=90,
                                    tag=None, limit=None)
    jobs = sweep._jobs(args)
    assert [len(j[0]) for j in jobs] == [20000, 20000]
    assert [t for _, t in jobs] == ["sweep_deltamaps_from_homoW_fromG0.16_sigma7.68_maps_1_1",
                                    "sweep_deltaSHUFFLED_from_homoW_fromG0.16_sigma7.68_maps_2_2"]
    for world in (1, 2, 4, 8, 3):
        shards = [sweep.job_shards(jobs, r, world) for r in range(world)]
        sizes = [sum(len(p) for p in sh) for sh in shards]
        assert max(sizes) - min(sizes) <= 1 and sum(sizes) == 40000
        for k in (0, 1):
            assert sorted(s.index for sh in shards for s in sh[k]) == list(range(20000))
        if world == 8:
            assert sizes == [5000] * 8 and all(len(sh[0]) == len(sh[1]) == 2500 for sh in shards)
    one = sweep._jobs(sweep.argparse.Namespace(**dict(vars(args), map_ids=[2, 2])))
    assert [s.index for s in sweep.job_shards(one, 3, 7)[0]] == [s.index for s in sweep.shard(one[0][0], 3, 7)]


def _shipped(kind):
    import pandas as pd
    return pd.read_csv(os.path.join(GOLD, f"shipped_{kind}_head.csv"))


@pytest.mark.parametrize("kind", ["homo", "maps", "shuf"])
def test_rank_files_collapse_to_shipped_format(tmp_path, kind):
    """TSV lines written like whole_sweep_both.py:116, collapsed, reproduce the
    shipped comma-separated table byte for byte."""
    df = _shipped(kind)
    paths = {}
    for rank, g in df.groupby("rank", sort=False):
        sims = [sweep.Sim(0, int(r.seed), r.delta_G, r.delta_sigma, None, None, 0) for r in g.itertuples()]
        rows = [{c: getattr(r, c) for c in sweep.METRIC_COLS} for r in g.itertuples()]
        p = str(tmp_path / f"r{rank}")
        sweep.append_rows(p, rank, sims, rows)
        paths[rank] = p
    out = tmp_path / "collapsed.txt"
    sweep.collapse([paths[r] for r in dict.fromkeys(df["rank"])], out)
    with open(os.path.join(GOLD, f"shipped_{kind}_head.csv")) as f:
        want = f.read()
    assert out.read_text() == want


def test_resume_skips_done(tmp_path):
    sims = sweep.homogeneous(1)[:5]
    rows = [{c: 0.5 for c in sweep.METRIC_COLS} for _ in sims]
    p = str(tmp_path / "rank0")
    sweep.append_rows(p, 0, sims[:3], rows[:3])
    have = sweep.done_keys(p)
    todo = [s for s in sims if (s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}") not in have]
    assert [s.index for s in todo] == [3, 4]
    sweep.append_rows(p, 0, todo, rows[3:])
    with open(p) as f:
        lines = f.readlines()
    assert lines[0].rstrip("\n").split("\t") == sweep.HEADER and len(lines) == 6


def _gather_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sims = sweep.shard(sweep.homogeneous(1)[:11], rank, world)
    rows = [{c: s.index + 0.01 * j for j, c in enumerate(sweep.METRIC_COLS)} for s in sims]
    t = sweep.gather_table(sweep.rows_table(rank, sims, rows), dist, torch.device("cpu"))
    q.put((rank, t))
    dist.destroy_process_group()


def test_gather_gloo_world2():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in (0, 1):
        t = got[r]
        assert t.shape == (11, 20)
        np.testing.assert_array_equal(t[:, 1], np.arange(11))
        np.testing.assert_array_equal(t[:, 0], np.arange(11) % 2)
        np.testing.assert_allclose(t[:, 4], np.arange(11))


def _gathered_path_worker(rank, world, port, out, q):
    """A torchrun job's end of run: rank 1 resumes (a previous run left part of its shard in its
    rank file), every rank gathers its whole shard, rank 0 writes the table from the gathered rows."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sims = sweep.homogeneous(1)[:13]
    mine = sweep.shard(sims, rank, world)
    rng = np.random.default_rng(rank)
    rows = [{c: (float(rng.normal()) if j % 5 else float("nan")) for j, c in enumerate(sweep.METRIC_COLS)}
            for _ in mine]
    path = os.path.join(out, "temp", f"g_rank{rank}")
    done = 3 if rank == 1 else 0  # rows of an earlier run of this rank
    if done:
        sweep.append_rows(path, rank, mine[:done], rows[:done])
    have = sweep.done_keys(path)
    todo = [s for s in mine if (s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}") not in have]
    sweep.append_rows(path, rank, todo, rows[done:])
    table = sweep.gather_table(sweep.shard_table(rank, mine, todo, rows[done:], path), dist, torch.device("cpu"))
    if rank == 0:
        os.makedirs(os.path.join(out, "g"), exist_ok=True)
        sweep.write_gathered(sims, os.path.join(out, "g"), "g", table)
    q.put(rank)
    dist.destroy_process_group()


def test_gathered_path_equals_file_path_gloo_world2(tmp_path):
    """With a process group the collapsed CSV and rows.npy come from the all-gathered rows, not
    from other ranks' files; they equal the rank-file path's output byte for byte (resumed rows
    and NaN columns included)."""
    import socket
    import torch.multiprocessing as mp
    out = str(tmp_path)
    os.makedirs(os.path.join(out, "temp"))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gathered_path_worker, args=(r, 2, port, out, q)) for r in range(2)]
    for p in ps:
        p.start()
    assert sorted(q.get(timeout=120) for _ in ps) == [0, 1]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    sims = sweep.homogeneous(1)[:13]
    sweep.collapse_sweep(sims, out, "g", 2)  # the file path over the same rank files
    with open(os.path.join(out, "g", "g.txt"), "rb") as a, open(os.path.join(out, "g.txt"), "rb") as b:
        ga, fb = a.read(), b.read()
    assert ga == fb and ga.count(b"\n") == 14
    np.testing.assert_array_equal(np.load(os.path.join(out, "g", "g_rows.npy")), np.load(os.path.join(out, "g_rows.npy")))


@pytest.mark.gpu
def test_sweep_main_short(tmp_path, cuda):
    """End to end: a short-schedule homogeneous sweep of 6 simulations writes
    the rank TSV and the collapsed table; a second invocation resumes (no new rows)."""
    import pandas as pd
    out = str(tmp_path)
    sweep.main(["homo", "--seeds", "1", "--short", "--limit", "6", "--out", out, "--tag", "t"])
    df = pd.read_csv(os.path.join(out, "t.txt"))
    assert len(df) == 6 and list(df.columns) == sweep.HEADER
    assert np.isfinite(df[sweep.METRIC_COLS].to_numpy()).all()
    assert (df["corrW"].abs() <= 1).all() and (df["peakfreq"] > 0).all()
    sweep.main(["homo", "--seeds", "1", "--short", "--limit", "6", "--out", out, "--tag", "t"])
    assert len(pd.read_csv(os.path.join(out, "t.txt"))) == 6
    with open(os.path.join(out, "temp", "t_rank0_perf.jsonl")) as f:  # one perf line per invocation
        perf = [json.loads(line) for line in f]
    assert [p["sims"] for p in perf] == [6, 0] and perf[0]["node_steps_per_s"] > 0


@pytest.mark.gpu
def test_c4_one_job_equals_the_two_sweeps(tmp_path, cuda):
    """The C4 job (both map-id pairs in one run, one batch holding simulations of both tables) writes
    the same two tables, byte for byte, as the two sweeps run one after the other."""
    a, b = str(tmp_path / "job"), str(tmp_path / "sep")
    sweep.main(["maps", "--map-ids", "1", "1", "2", "2", "--seeds", "1", "--seed0", "0", "--short", "--limit", "10",
                "--out", a])
    for ids in (["1", "1"], ["2", "2"]):
        sweep.main(["maps", "--map-ids", *ids, "--seeds", "1", "--seed0", "0", "--short", "--limit", "10", "--out", b])
    for t in ("sweep_deltamaps_from_homoW_fromG0.16_sigma7.68_maps_1_1",
              "sweep_deltaSHUFFLED_from_homoW_fromG0.16_sigma7.68_maps_2_2"):
        with open(os.path.join(a, t + ".txt"), "rb") as f, open(os.path.join(b, t + ".txt"), "rb") as g:
            x, y = f.read(), g.read()
        assert x == y and x.count(b"\n") == 11


@pytest.mark.gpu
def test_many_seeds_main_short(tmp_path, cuda):
    """run_many_seeds.py drop-in: (seed, state) keys, the reference's HMA dict per
    simulation and the "metainfo" counts (run_many_seeds.py:130-146)."""
    import pickle
    out = str(tmp_path)
    sweep.main(["many", "--modality", "homo", "--seeds", "2", "--short", "--out", out, "--tag", "m"])
    with open(os.path.join(out, "m.pickle"), "rb") as f:  # our own file
        d = pickle.load(f)
    assert d["metainfo"] == {s: 2 for s in datasets.STATES}
    keys = [k for k in d if k != "metainfo"]
    assert sorted(keys) == sorted(itertools.product(range(2), datasets.STATES))
    v = d[(0, "W")]
    assert set(v) == {"Hin_sim", "Hse_sim", "Hin_node_sim", "Hse_node_sim", "sFC"}
    assert v["sFC"].shape == (90, 90) and (v["sFC"] >= 0).all()  # clipped in place like the reference
    assert v["Hin_node_sim"].shape == (90,) and np.isfinite(v["Hin_sim"])
    # the device-batched HMA (wc_hma) agrees with the host facade on the saved (clipped) sFC
    from nremmodfc_amd import HMA
    for k in keys:
        h = HMA.integration_segregation(d[k]["sFC"].copy())
        np.testing.assert_allclose(d[k]["Hin_sim"], h["Hin_sim"], rtol=1e-12)
        np.testing.assert_allclose(d[k]["Hse_sim"], h["Hse_sim"], rtol=1e-11)
        np.testing.assert_allclose(d[k]["Hse_node_sim"], h["Hse_node_sim"], rtol=1e-9, atol=1e-15)


def _write_rank_files(out, tag, sims, world, ranks):
    os.makedirs(os.path.join(out, "temp"), exist_ok=True)
    for r in ranks:
        mine = sweep.shard(sims, r, world)
        rows = [{c: s.index + 0.001 * j for j, c in enumerate(sweep.METRIC_COLS)} for s in mine]
        sweep.append_rows(os.path.join(out, "temp", f"{tag}_rank{r}"), r, mine, rows)


def test_collapse_waits_for_every_rank_file(tmp_path):
    """SLURM-array runs (no process group): the table is assembled only once every
    rank file holds its whole shard; rows.npy comes from the rank files (resumed rows included)."""
    out = str(tmp_path)
    sims = sweep.homogeneous(1)[:7]
    _write_rank_files(out, "c", sims, 2, [0])
    argv = ["collapse", "--of", "homo", "--seeds", "1", "--limit", "7", "--world", "2", "--out", out, "--tag", "c"]
    with pytest.raises(SystemExit):
        sweep.main(argv)
    assert not os.path.exists(os.path.join(out, "c.txt"))
    _write_rank_files(out, "c", sims, 2, [1])
    sweep.main(argv)
    import pandas as pd
    df = pd.read_csv(os.path.join(out, "c.txt"))
    assert len(df) == 7 and list(df.columns) == sweep.HEADER
    rows = np.load(os.path.join(out, "c_rows.npy"))
    np.testing.assert_array_equal(rows[:, 1], np.arange(7))
    np.testing.assert_array_equal(rows[:, 0], np.arange(7) % 2)
    np.testing.assert_allclose(rows[:, 4], np.round(np.arange(7), 4))


def test_collapse_orders_rows_like_the_gathered_path(tmp_path):
    """A resumed run can append a shard's rows out of shard order; the file path sorts by (rank,
    index), as write_gathered does, so both paths give the same bytes for any append order."""
    out = str(tmp_path)
    sims = sweep.homogeneous(1)[:9]
    os.makedirs(os.path.join(out, "temp"), exist_ok=True)
    for r in range(2):
        mine = sweep.shard(sims, r, 2)
        rows = [{c: s.index + 0.001 * j for j, c in enumerate(sweep.METRIC_COLS)} for s in mine]
        path = os.path.join(out, "temp", f"o_rank{r}")
        # the second half first, then the first (a non-prefix resume)
        h = len(mine) // 2
        sweep.append_rows(path, r, mine[h:], rows[h:])
        sweep.append_rows(path, r, mine[:h], rows[:h])
    sweep.collapse_sweep(sims, out, "o", 2)
    import pandas as pd
    df = pd.read_csv(os.path.join(out, "o.txt"))
    order = [s.index for r in range(2) for s in sweep.shard(sims, r, 2)]
    np.testing.assert_allclose(df[sweep.METRIC_COLS[0]].to_numpy(), np.array(order, dtype=float), atol=1e-9)
    table = np.array([[r, s.index, 0, 0] + [s.index + 0.001 * j for j in range(len(sweep.METRIC_COLS))]
                      for r in range(2) for s in sweep.shard(sims, r, 2)], dtype=float)
    os.makedirs(os.path.join(out, "g"), exist_ok=True)
    sweep.write_gathered(sims, os.path.join(out, "g"), "o", table[::-1].copy())
    with open(os.path.join(out, "g", "o.txt"), "rb") as a, open(os.path.join(out, "o.txt"), "rb") as b:
        assert a.read() == b.read()


def test_c4_job_collapse_waits_for_both_tables_rank_files(tmp_path):
    """A SLURM-array C4 job (`maps --map-ids 1 1 2 2`, no process group): each task writes its share of
    BOTH tables (the round robin over the concatenated lists, so the shuffled table's shard of rank r
    starts at global position len(maps list)); `collapse` assembles each table only when every rank
    file of it holds that shard, and the rank column follows the global round robin."""
    import pandas as pd
    out = str(tmp_path)
    args = sweep.argparse.Namespace(kind="maps", map_ids=[1, 1, 2, 2], seeds=1, seed0=0, grid="shipped", nodes=90,
                                    tag=None, limit=5)
    jobs = sweep._jobs(args)
    os.makedirs(os.path.join(out, "temp"), exist_ok=True)

    def write(rank):
        for (sims, tag), mine in zip(jobs, sweep.job_shards(jobs, rank, 2)):
            rows = [{c: s.index + 0.001 * j for j, c in enumerate(sweep.METRIC_COLS)} for s in mine]
            sweep.append_rows(os.path.join(out, "temp", f"{tag}_rank{rank}"), rank, mine, rows)

    argv = ["collapse", "--of", "maps", "--map-ids", "1", "1", "2", "2", "--seeds", "1", "--seed0", "0",
            "--limit", "5", "--world", "2", "--out", out]
    write(0)
    with pytest.raises(SystemExit):
        sweep.main(argv)
    write(1)
    sweep.main(argv)
    for k, (sims, tag) in enumerate(jobs):
        df = pd.read_csv(os.path.join(out, tag + ".txt"))
        assert len(df) == 5 and list(df.columns) == sweep.HEADER
        rows = np.load(os.path.join(out, tag + "_rows.npy"))
        np.testing.assert_array_equal(rows[:, 1], np.arange(5))
        np.testing.assert_array_equal(rows[:, 0], (np.arange(5) + 5 * k) % 2)  # global position % world


def test_slurm_rank_world(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("SLURM_ARRAY_TASK_ID", "3")
    monkeypatch.setenv("SLURM_ARRAY_TASK_MAX", "7")
    monkeypatch.setenv("SLURM_LOCALID", "1")
    assert sweep._rank_world() == (3, 8, 1, "slurm")


def test_n1000_sim_lists_use_synthetic_maps():
    sims = sweep.maps(1, 1, n_iterations=1, n_init=0, n=1000)
    assert sims[0].G.shape == (1000,) and abs(sims[0].G.mean() - (0.16 + sims[0].dG)) < 1e-12
    shuf = sweep.maps(2, 2, n_iterations=1, n_init=0, n=1000)
    assert sorted(shuf[5].G) == pytest.approx(sorted(sims[5].G))
    assert not np.array_equal(shuf[5].G, sims[5].G)


@pytest.mark.gpu
def test_slurm_array_two_tasks(tmp_path, cuda, monkeypatch):
    """Two SLURM-array tasks run one after the other: the first writes only its rank
    file, the second (finding every rank file complete) assembles the table."""
    import pandas as pd
    out = str(tmp_path)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("SLURM_ARRAY_TASK_MAX", "1")
    argv = ["homo", "--seeds", "1", "--short", "--limit", "5", "--out", out, "--tag", "s"]
    monkeypatch.setenv("SLURM_ARRAY_TASK_ID", "1")
    sweep.main(argv)
    assert os.path.exists(os.path.join(out, "temp", "s_rank1")) and not os.path.exists(os.path.join(out, "s.txt"))
    monkeypatch.setenv("SLURM_ARRAY_TASK_ID", "0")
    sweep.main(argv)
    df = pd.read_csv(os.path.join(out, "s.txt"))
    assert sorted(df["rank"]) == [0, 0, 0, 1, 1] and np.isfinite(df[sweep.METRIC_COLS].to_numpy()).all()


@pytest.mark.gpu
def test_sweep_main_n1000_short(tmp_path, cuda):
    """Config 5 through the driver: the synthetic 1000-node connectome, no empirical FC
    (gof columns NaN), FC-derived columns and the Welch peak written."""
    import pandas as pd
    out = str(tmp_path)
    sweep.main(["homo", "--seeds", "1", "--short", "--limit", "3", "--nodes", "1000", "--out", out, "--tag", "n"])
    df = pd.read_csv(os.path.join(out, "n.txt"))
    assert len(df) == 3 and list(df.columns) == sweep.HEADER
    assert df[[c for c in sweep.METRIC_COLS if c[:4] in ("ssim", "corr") or c[0] == "e"]].isna().all().all()
    good = df[["sync", "meta", "mean", "peakfreq"]].to_numpy()
    assert np.isfinite(good).all() and (df["peakfreq"] > 0).all()


@pytest.mark.gpu
def test_many_seeds_main_n1000_short(tmp_path, cuda):
    """run_many_seeds.py at N = 1000 (HMA.py has no N cap): the driver integrates, then the
    N > 96 HMA path (device eigensolver + wc_hma_modes) produces every pickle entry."""
    import pickle
    out = str(tmp_path)
    sweep.main(["many", "--modality", "homo", "--seeds", "1", "--short", "--nodes", "1000", "--out", out,
                "--tag", "m1k"])
    with open(os.path.join(out, "m1k.pickle"), "rb") as f:  # our own file
        d = pickle.load(f)
    assert d["metainfo"] == {s: 1 for s in datasets.STATES}
    v = d[(0, "N2")]
    assert v["sFC"].shape == (1000, 1000) and (v["sFC"] >= 0).all()
    assert v["Hse_node_sim"].shape == (1000,) and np.isfinite(v["Hin_sim"]) and np.isfinite(v["Hse_sim"])
    from nremmodfc_amd import HMA
    h = HMA.integration_segregation(d[(0, "W")]["sFC"].copy())
    np.testing.assert_allclose(d[(0, "W")]["Hin_sim"], h["Hin_sim"], rtol=1e-10)
    np.testing.assert_allclose(d[(0, "W")]["Hse_sim"], h["Hse_sim"], rtol=1e-9)


@pytest.mark.gpu
def test_many_seeds_full_size(tmp_path, cuda):
    """Config 2 at full size: run_many_seeds.py's 50 seeds x 4 states at the map optima over
    the full 1001 s schedule (run_many_seeds.py:105-146) -> the collapsed pickle, read the way
    the figure scripts read it (figures/Fig5/fig5.py:117-129, load(dic, nseeds=50)); the
    device-batched HMA equals the host facade (the reference's algorithm) on every saved sFC."""
    import pickle
    import time
    from nremmodfc_amd import HMA
    out = str(tmp_path)
    t0 = time.perf_counter()
    sweep.main(["many", "--modality", "map", "--out", out, "--tag", "c2"])
    print(f"C2 full size: 200 simulations x 1001 s in {time.perf_counter() - t0:.1f} s")
    with open(os.path.join(out, "c2.pickle"), "rb") as f:  # our own file
        d = pickle.load(f)
    assert d["metainfo"] == {s: 50 for s in datasets.STATES}
    from tests.test_consumers import load_many_seeds  # fig5.py:117-129's load(dic, nseeds=50)
    matts, hin, hse = load_many_seeds(d, 50)
    for key in d:
        if key != "metainfo":
            assert np.isscalar(d[key]["Hin_sim"]) or np.ndim(d[key]["Hin_sim"]) == 0
    matts = {st: np.stack([d[(s, st)]["sFC"] for s in range(50)]) for st in datasets.STATES}
    for st in datasets.STATES:
        assert np.isfinite(matts[st]).all() and (matts[st] >= 0).all()
        assert np.isfinite(hin[st]).all() and np.isfinite(hse[st]).all()
        assert np.allclose(np.diagonal(matts[st], axis1=1, axis2=2), 1.0)
    for key in [k for k in d if k != "metainfo"]:
        h = HMA.integration_segregation(d[key]["sFC"].copy())
        np.testing.assert_allclose(d[key]["Hin_sim"], h["Hin_sim"], rtol=1e-12)
        np.testing.assert_allclose(d[key]["Hse_sim"], h["Hse_sim"], rtol=1e-11)
        np.testing.assert_allclose(d[key]["Hin_node_sim"], h["Hin_node_sim"], rtol=1e-9, atol=1e-15)
        np.testing.assert_allclose(d[key]["Hse_node_sim"], h["Hse_node_sim"], rtol=1e-9, atol=1e-15)
