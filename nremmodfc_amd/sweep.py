"""Sweep drivers: whole_sweep_both.py, whole_sweep_both_maps.py, run_many_seeds.py.

The reference runs each driver as a 64-task SLURM array of single-threaded
processes (`sim % threads == rank`, whole_sweep_both.py:63-64) that append one
TSV line per simulation (:112-116); a human then concatenates the per-rank
files into the comma-separated `output/*.txt` that heatmaps.py reads.  Here one
process per GPU (torchrun / the same SLURM variables) takes its shard of the
same `itertools.product` list, runs it through the streamed GPU pipeline in
large batches, appends the same TSV lines (resumable: simulations already in
the rank's file are skipped), and rank 0 gathers every rank's shard over RCCL
(one all-gather of a float64 table) and writes the collapsed CSV from the
gathered rows (the rank files stay for resume; SLURM-array tasks, which have no
process group, assemble the table from the rank files instead).

  python -m nremmodfc_amd.sweep homo      [--seeds 50 --seed0 0] [--grid shipped|script]
  python -m nremmodfc_amd.sweep maps      --map-ids 1 1  [--seeds 25 --seed0 25]
  python -m nremmodfc_amd.sweep maps      --map-ids 1 1 2 2 --seeds 50 --seed0 0   (C4: both tables, one job)
  python -m nremmodfc_amd.sweep many      --modality homo|map|shuf
  torchrun --nproc-per-node 8 -m nremmodfc_amd.sweep homo ...
"""
from __future__ import annotations

import argparse
import dataclasses
import itertools
import json
import os
import time
import pickle
from typing import List, Optional

import numpy as np

from . import datasets

STATES = datasets.STATES
METRIC_COLS = (["ssim" + s for s in STATES] + ["corr" + s for s in STATES] + ["e" + s for s in STATES]
               + ["sync", "meta", "mean", "peakfreq"])
HEADER = ["rank", "seed", "delta_G", "delta_sigma"] + METRIC_COLS  # whole_sweep_both.py:115
BASE_G, BASE_SIGMA = 0.16, 7.68  # whole_sweep_both.py:30 ("W optimal")

# run_many_seeds.py:34-47 -- (G, delta_G, sigmaE, delta_sigmaE) per state, from heatmaps.py
OPTIMALS = {
    "homo": {"W": (0.16, 0.0, 7.68, 0.0), "N1": (0.16, 0.04, 7.68, 0.0), "N2": (0.16, 0.0, 7.68, 0.0),
             "N3": (0.16, -0.04, 7.68, 0.04)},
    "map": {"W": (0.16, -0.02, 7.68, -0.02), "N1": (0.16, 0.18, 7.68, -0.02), "N2": (0.16, 0.02, 7.68, -0.04),
            "N3": (0.16, 0.02, 7.68, -0.12)},
    "shuf": {"W": (0.16, 0.0, 7.68, 0.0), "N1": (0.16, 0.0, 7.68, 0.04), "N2": (0.16, 0.0, 7.68, 0.0),
             "N3": (0.16, 0.0, 7.68, -0.04)},
}
MODALITY_MAPS = {"homo": (0, 0), "map": (1, 1), "shuf": (2, 2)}


@dataclasses.dataclass
class Sim:
    index: int              # position in the reference's product list
    seed: int
    dG: float
    dsigma: float
    G: np.ndarray           # (N,)
    sigma: np.ndarray       # (N,)
    stream: int             # Philox stream id (grid cell / state index): key = (seed, stream)
    state: Optional[str] = None


def _grids(kind):
    if kind == "script":   # the values written in whole_sweep_both.py:57-58
        return np.linspace(-0.1, 0.5, 20, endpoint=False), np.linspace(-1, 1, 20, endpoint=False)
    # the grid the shipped outputs were produced on (whole_sweep_both_maps.py:92-93; SURVEY.md 0, gotcha 5)
    return np.linspace(-0.1, 0.3, 20, endpoint=False), np.linspace(-0.2, 0.2, 20, endpoint=False)


def homogeneous(n_iterations=50, n_init=0, grid="shipped", n=90) -> List[Sim]:
    """whole_sweep_both.py:57-72: G = 0.16 + dG, sigmaE = 7.68 + dsigma on every node."""
    return maps(0, 0, n_iterations, n_init, grid, n)


def maps(map_id1=1, map_id2=1, n_iterations=25, n_init=25, grid="shipped", n=90) -> List[Sim]:
    """whole_sweep_both_maps.py:92-108: G_i = 0.16 + dG*ach_i, sigmaE_i = 7.68 + dsigma*na_i
    (maps normalised to mean 1; id 0 homogeneous, 1 real, 2 hemisphere-symmetric shuffle)."""
    ach = datasets.load_map(datasets.MAPNAMES_ACH[map_id1], n)
    na = datasets.load_map(datasets.MAPNAMES_NA[map_id2], n)
    dGs, dSs = _grids(grid)
    seeds = range(n_init, n_init + n_iterations)
    out = []
    for i, (seed, a, b) in enumerate(itertools.product(seeds, range(len(dGs)), range(len(dSs)))):
        dG, dS = dGs[a], dSs[b]
        out.append(Sim(i, seed, dG, dS, BASE_G + dG * ach, BASE_SIGMA + dS * na, a * len(dSs) + b))
    return out


def many_seeds(modality="map", n_iterations=50, n_init=0, n=90) -> List[Sim]:
    """run_many_seeds.py:105-117: product(seeds, states) at each state's optimum."""
    m1, m2 = MODALITY_MAPS[modality]
    ach = datasets.load_map(datasets.MAPNAMES_ACH[m1], n)
    na = datasets.load_map(datasets.MAPNAMES_NA[m2], n)
    out = []
    seeds = range(n_init, n_init + n_iterations)
    for i, (seed, state) in enumerate(itertools.product(seeds, STATES)):
        G, dG, s, dS = OPTIMALS[modality][state]
        out.append(Sim(i, seed, dG, dS, G + ach * dG, s + na * dS, 1000 + STATES.index(state), state))
    return out


def shard(sims: List[Sim], rank: int, world: int) -> List[Sim]:
    """The reference's round-robin: simulation i belongs to rank i % world."""
    return [s for s in sims if s.index % world == rank]


def format_row(rank, sim: Sim, vals: dict) -> str:
    """One TSV line exactly as whole_sweep_both.py:116 writes it."""
    parts = [str(rank), str(sim.seed), f"{sim.dG:.4f}", f"{sim.dsigma:.4f}"] + [f"{vals[c]:.4f}" for c in METRIC_COLS]
    return "\t".join(parts) + "\n"


def done_keys(path):
    """(seed, delta_G, delta_sigma) already in a rank file (resume after a crash)."""
    if not os.path.exists(path):
        return set()
    keys = set()
    with open(path) as f:
        next(f, None)
        for line in f:
            p = line.rstrip("\n").split("\t")
            if len(p) == len(HEADER):
                keys.add((int(p[1]), p[2], p[3]))
    return keys


def read_rank_rows(path):
    """{(seed, delta_G, delta_sigma): metric dict} of the rows already in a rank file (as written, %.4f)."""
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        next(f, None)
        for line in f:
            p = line.rstrip("\n").split("\t")
            if len(p) == len(HEADER):
                out[(int(p[1]), p[2], p[3])] = {c: float(v) for c, v in zip(METRIC_COLS, p[4:])}
    return out


def append_rows(path, rank, sims, results):
    new = not os.path.isfile(path)
    with open(path, "a") as f:
        if new:
            f.write("\t".join(HEADER) + "\n")
        for s, r in zip(sims, results):
            f.write(format_row(rank, s, r))


def collapse(paths, out_csv, sims=None):
    """Concatenate per-rank TSV files into the comma-separated table heatmaps.py reads.

    With `sims` (the product list) the rows are ordered by (rank, the simulation's index in the
    list), the order write_gathered uses, whatever order resumed runs appended them in."""
    import pandas as pd
    df = pd.concat([pd.read_csv(p, sep="\t") for p in paths if os.path.exists(p)], ignore_index=True)
    if sims is not None and len(df):
        index = {(s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}"): s.index for s in sims}
        idx = np.array([index.get((int(r.seed), f"{r.delta_G:.4f}", f"{r.delta_sigma:.4f}"), -1)
                        for r in df.itertuples(index=False)])
        df = df.iloc[np.lexsort((idx, df["rank"].to_numpy()))].reset_index(drop=True)
    df.to_csv(out_csv, index=False)
    return df


def run_sims(sims: List[Sim], sc, empfcs, schedule=None, precision="f32", batch=20_000, device="cuda",
             want_fc=False, progress=None, on_batch=None):
    """Run simulations through the GPU pipeline in batches -> (list of metric dicts, FCs or None).

    on_batch(part, rows) is called after every batch (the drivers append and flush
    the batch's rows there, so a crash loses at most the running batch).  Without
    empirical FCs (e.g. the 1000-node synthetic connectome) the goodness-of-fit
    columns are NaN."""
    from .model import sim_keys
    from .pipeline import run_sweep
    rows, fcs = [], []
    timings = []
    if sims:  # at most ~2.5 M node-columns per batch (N = 1000: 2,500 sims, ~80 GB of ring + BOLD state)
        batch = max(1, min(batch, 2_500_000 // len(sims[0].G)))
    for b0 in range(0, len(sims), batch):
        part = sims[b0:b0 + batch]
        G = np.stack([s.G for s in part])
        S = np.stack([s.sigma for s in part])
        keys = sim_keys([s.seed for s in part], [s.stream for s in part])
        res = run_sweep(sc, G, S, keys, empfcs, schedule, precision=precision, want_fc=want_fc, device=device,
                        progress=progress)
        cols = res.columns()
        timings.append(dict(res.timings, sims=len(part)))
        nan = np.full(len(part), np.nan)
        new = [{c: float(cols.get(c, nan)[i]) for c in METRIC_COLS} for i in range(len(part))]
        if on_batch is not None:
            on_batch(part, new)
        rows += new
        if want_fc:
            fcs += list(res.fc)
    run_sims.last_timings = timings
    return rows, (fcs if want_fc else None)


class Progress:
    """Progress lines about once a minute.  Every call (one per launch: <= 500k Euler steps, a
    recorded chunk) synchronises the device, so the host never queues more than one launch
    ahead and the line reflects finished work: a persistent launch integrates its whole range
    in one kernel, so without the wait the host would queue the sweep in milliseconds and stay
    silent until the end."""

    def __init__(self, rank, every_s=60.0):
        import time
        self.t0 = self.last = time.perf_counter()
        self.rank, self.every = rank, every_s

    def __call__(self, phase, step, total):
        import time
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        now = time.perf_counter()
        if now - self.last >= self.every:
            print(f"[rank {self.rank}] {phase}: step {step}/{total} ({100 * step / total:.1f}%), "
                  f"{now - self.t0:.0f} s", flush=True)
            self.last = now


def rows_table(rank, sims, rows):
    """float64 table [n][4 + 16]: rank, index, seed, stream, metrics."""
    t = np.zeros((len(sims), 4 + len(METRIC_COLS)))
    for i, (s, r) in enumerate(zip(sims, rows)):
        t[i, :4] = (rank, s.index, s.seed, s.stream)
        t[i, 4:] = [r[c] for c in METRIC_COLS]
    return t


def gather_table(table, dist, device):
    """All ranks' row tables on every rank (one all-gather over RCCL/gloo), sorted by index."""
    import torch
    n = torch.tensor([table.shape[0]], device=device)
    world = dist.get_world_size()
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = int(max(x.item() for x in ns))
    buf = torch.full((m, table.shape[1]), float("nan"), dtype=torch.float64, device=device)
    buf[:table.shape[0]] = torch.as_tensor(table, dtype=torch.float64, device=device)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    full = torch.cat([o[:int(k.item())] for o, k in zip(out, ns)]).cpu().numpy()
    return full[np.argsort(full[:, 1], kind="stable")]


def _rank_world():
    """(rank, world, local rank, launcher).  torchrun: one process group over RCCL.
    SLURM array (the reference's launcher, whole_sweep_both.py:23-24): independent
    tasks with no process group; each writes only its own rank file and the table is
    collapsed once every rank file is complete (`sweep collapse`, or the last task)."""
    if "WORLD_SIZE" in os.environ:
        return (int(os.environ.get("RANK", 0)), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0)),
                "torch")
    if "SLURM_ARRAY_TASK_ID" in os.environ:
        return (int(os.environ["SLURM_ARRAY_TASK_ID"]), int(os.environ["SLURM_ARRAY_TASK_MAX"]) + 1,
                int(os.environ.get("SLURM_LOCALID", 0)), "slurm")
    return 0, 1, 0, "single"


def _sim_list(args):
    """The driver's simulation list and output tag (whole_sweep_both.py, _maps.py, run_many_seeds.py)."""
    jobs = _jobs(args)
    if len(jobs) != 1:
        raise SystemExit("this command takes one map-id pair")
    return jobs[0]


def _jobs(args):
    """[(simulation list, output tag)]: one table per map-id pair.  `maps --map-ids 1 1 2 2` is the
    C4 job (BASELINE config 4): the real-map and the shuffled-map sweeps as ONE round-robin job over
    their concatenated lists (whole_sweep_both_maps.py:27-28,92-153 run once per pair), so every rank
    holds a share of both; each pair is still written to its own table under the reference's name."""
    n = args.nodes
    if args.kind == "homo":
        sims = homogeneous(args.seeds or 50, args.seed0 or 0, args.grid, n)
        tag = args.tag or f"sweep_delta_homoW_fromG{BASE_G}_sigma{BASE_SIGMA}_maps_0_0" + (f"_N{n}" if n != 90 else "")
        jobs = [(sims, tag)]
    elif args.kind == "maps":
        ids = list(args.map_ids)
        if len(ids) % 2 or not ids:
            raise SystemExit("--map-ids takes pairs: m1 m2 [m1 m2 ...]")
        pairs = [(ids[i], ids[i + 1]) for i in range(0, len(ids), 2)]
        if len(set(pairs)) != len(pairs):
            raise SystemExit("--map-ids: each pair once")
        if args.tag and len(pairs) > 1:
            raise SystemExit("--tag names one table: give one map-id pair")
        jobs = []
        for m1, m2 in pairs:
            sims = maps(m1, m2, args.seeds or 25, 25 if args.seed0 is None else args.seed0, args.grid, n)
            name = "deltaSHUFFLED" if (m1, m2) == (2, 2) else "deltamaps"
            tag = args.tag or (f"sweep_{name}_from_homoW_fromG{BASE_G}_sigma{BASE_SIGMA}_maps_{m1}_{m2}"
                               + (f"_N{n}" if n != 90 else ""))
            jobs.append((sims, tag))
    else:
        sims = many_seeds(args.modality, args.seeds or 50, args.seed0 or 0, n)
        tag = args.tag or f"run_50seeds_output_{args.modality}" + (f"_N{n}" if n != 90 else "")
        jobs = [(sims, tag)]
    if args.limit:
        jobs = [(sims[:args.limit], tag) for sims, tag in jobs]
    return jobs


def job_shards(jobs, rank, world):
    """The round robin over the jobs' concatenated lists: position g (job j's simulation i sits at
    g = sum of the earlier lists' lengths + i) belongs to rank g % world; for one job, g = i and this
    is whole_sweep_both.py:63-64's `sim % threads == rank`.  -> [this rank's simulations of job j]."""
    out, g0 = [], 0
    for sims, _ in jobs:
        out.append([s for s in sims if (g0 + s.index) % world == rank])
        g0 += len(sims)
    return out


def rank_files_complete(sims, out, tag, world, g0=0):
    """True when every rank's TSV file holds its whole round-robin shard (g0: the list's offset in a
    multi-table job, job_shards)."""
    for r in range(world):
        want = {(s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}") for s in sims if (g0 + s.index) % world == r}
        if not want <= done_keys(os.path.join(out, "temp", f"{tag}_rank{r}")):
            return False
    return True


def collapse_sweep(sims, out, tag, world):
    """{tag}.txt (the comma-separated table heatmaps.py reads) and {tag}_rows.npy, both
    built from the rank files (so rows restored by a resumed run are included).  The path
    of SLURM-array runs, which have no process group; torchrun runs use write_gathered."""
    paths = [os.path.join(out, "temp", f"{tag}_rank{r}") for r in range(world)]
    tmp = os.path.join(out, f".{tag}.txt.{os.getpid()}")
    df = collapse(paths, tmp, sims)
    os.replace(tmp, os.path.join(out, f"{tag}.txt"))
    return _save_rows(sims, out, tag, df)


def shard_table(rank, mine, todo, rows, path):
    """This rank's whole shard as a rows_table: this run's rows for `todo`, the rows a
    previous (resumed) run left in the rank's own file for the rest, in shard order."""
    new = {s.index: r for s, r in zip(todo, rows)}
    old = read_rank_rows(path) if len(new) < len(mine) else {}
    have, vals = [], []
    for s in mine:
        r = new.get(s.index)
        if r is None:
            r = old.get((s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}"))
        if r is not None:
            have.append(s)
            vals.append(r)
    return rows_table(rank, have, vals)


def write_gathered(sims, out, tag, table):
    """{tag}.txt and {tag}_rows.npy from the gathered rows (rank 0 of a torchrun job): the
    rows go through the same text the rank files hold (format_row, %.4f) and the same
    pandas read/write as collapse_sweep, rank-major in shard order, so the two paths write
    the same bytes; no rank file is read."""
    import io
    import pandas as pd
    by_index = {s.index: s for s in sims}
    order = np.lexsort((table[:, 1], table[:, 0]))
    text = ["\t".join(HEADER) + "\n"]
    for i in order:
        t = table[i]
        text.append(format_row(int(t[0]), by_index[int(t[1])], dict(zip(METRIC_COLS, t[4:]))))
    df = pd.read_csv(io.StringIO("".join(text)), sep="\t")
    tmp = os.path.join(out, f".{tag}.txt.{os.getpid()}")
    df.to_csv(tmp, index=False)
    os.replace(tmp, os.path.join(out, f"{tag}.txt"))
    return _save_rows(sims, out, tag, df)


def _save_rows(sims, out, tag, df):
    """{tag}_rows.npy: the collapsed table as float64 [n][4 + 16] (rank, index, seed, stream,
    metrics as printed), sorted by the simulation's index in the reference's product list."""
    index = {(s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}"): s for s in sims}
    table = np.full((len(df), 4 + len(METRIC_COLS)), np.nan)
    for i, r in enumerate(df.itertuples(index=False)):
        s = index.get((int(r.seed), f"{r.delta_G:.4f}", f"{r.delta_sigma:.4f}"))
        table[i, :4] = (r.rank, s.index if s else -1, r.seed, s.stream if s else -1)
        table[i, 4:] = [getattr(r, c) for c in METRIC_COLS]
    table = table[np.argsort(table[:, 1], kind="stable")]
    np.save(os.path.join(out, f"{tag}_rows.npy"), table)
    return table


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("kind", choices=("homo", "maps", "many", "collapse"))
    ap.add_argument("--seeds", type=int, default=None)
    ap.add_argument("--seed0", type=int, default=None)
    ap.add_argument("--grid", default="shipped", choices=("shipped", "script"))
    ap.add_argument("--map-ids", type=int, nargs="+", default=(1, 1),
                    help="m1 m2 (whole_sweep_both_maps.py:33); several pairs, e.g. 1 1 2 2 with --seeds 50 "
                         "--seed0 0 (BASELINE config 4), run as one round-robin job writing one table per pair")
    ap.add_argument("--modality", default="map", choices=("homo", "map", "shuf"))
    ap.add_argument("--nodes", type=int, default=90,
                    help="90: the AAL connectome (SC_opti_25julio); other N: the synthetic connectome of "
                         "BASELINE config 5 (datasets.synthetic_sc), no empirical FC so the gof columns are NaN")
    ap.add_argument("--out", default="output")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--precision", default="f32", choices=("f32", "f64"))
    ap.add_argument("--batch", type=int, default=20_000)
    ap.add_argument("--short", action="store_true", help="short schedule (smoke runs): 0.02/0.2/20 s")
    ap.add_argument("--limit", type=int, default=None, help="only the first LIMIT simulations of the list")
    ap.add_argument("--of", default="homo", choices=("homo", "maps"), help="collapse: which sweep's list")
    ap.add_argument("--world", type=int, default=None, help="collapse: number of rank files")
    args = ap.parse_args(argv)

    if args.kind == "collapse":  # SLURM-array runs: assemble the table once every rank file is complete
        args.kind = args.of
        world = args.world or _rank_world()[1]
        g0 = 0
        for sims, tag in _jobs(args):
            if not rank_files_complete(sims, args.out, tag, world, g0):
                raise SystemExit(f"collapse: the {world} rank files of {tag} are not complete yet")
            collapse_sweep(sims, args.out, tag, world)
            g0 += len(sims)
        return

    import torch
    from .model import Schedule
    rank, world, local, launcher = _rank_world()
    dist = None
    if launcher == "slurm":
        local %= max(1, torch.cuda.device_count())
    device = f"cuda:{local}"
    # every launcher: the library launches on torch's current stream and queries the current
    # HIP device (CU count, occupancy), so the current device must be this rank's GPU
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if launcher == "torch" and world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    os.makedirs(os.path.join(args.out, "temp"), exist_ok=True)
    jobs = _jobs(args)
    sims, tag = jobs[0]
    sched = Schedule(n_trans1=200, n_trans2=2000, n_sim=200_000) if args.short else Schedule()
    if args.nodes == 90:
        empfcs = {s: datasets.load_empfc(s) for s in STATES}
        sc = datasets.load_sc()
    else:
        empfcs = {}
        sc = datasets.synthetic_sc(args.nodes)
    from .pipeline import check_supported
    check_supported(sc.shape[0], sched)  # fail before integrating, not in the epilogue
    shards = job_shards(jobs, rank, world)
    mine = shards[0]

    if args.kind == "many":
        from . import HMA
        t0 = time.perf_counter()
        rows, fcs = run_sims(mine, sc, empfcs, sched, args.precision, args.batch, device, want_fc=True)
        hma = HMA.integration_segregation_batch(fcs, device) if fcs else []
        wall = time.perf_counter() - t0
        n_steps = len(mine) * sc.shape[0] * sched.n_total
        perf = json.dumps({"rank": rank, "sims": len(mine), "nodes": sc.shape[0], "wall_s": wall,
                           "node_steps": n_steps, "node_steps_per_s": n_steps / wall if wall else None,
                           "includes": "integration, BOLD, FC, metrics, Welch, device HMA",
                           "batches": getattr(run_sims, "last_timings", None)})
        print(perf, flush=True)
        with open(os.path.join(args.out, "temp", f"{tag}_rank{rank}_perf.jsonl"), "a") as f:
            f.write(perf + "\n")
        save = {(s.seed, s.state): d for s, d in zip(mine, hma)}
        part_path = os.path.join(args.out, "temp", f"{tag}_rank{rank}.pickle")
        with open(part_path + ".tmp", "wb") as f:
            pickle.dump(save, f)
        os.replace(part_path + ".tmp", part_path)
        if dist:
            parts = [None] * world
            dist.all_gather_object(parts, save)
        elif launcher == "slurm":  # merge only once every task's part exists (our own files)
            paths = [os.path.join(args.out, "temp", f"{tag}_rank{r}.pickle") for r in range(world)]
            parts = None
            if all(os.path.exists(p) for p in paths):
                parts = []
                for p in paths:
                    with open(p, "rb") as f:
                        parts.append(pickle.load(f))
        else:
            parts = [save]
        if parts is not None and (rank == 0 or launcher == "slurm"):
            merged = {k: v for p in parts for k, v in p.items()}
            merged["metainfo"] = {st: sum(1 for k in merged if k != "metainfo" and k[1] == st) for st in STATES}
            final = os.path.join(args.out, f"{tag}.pickle")
            with open(final + f".{os.getpid()}", "wb") as f:
                pickle.dump(merged, f)
            os.replace(final + f".{os.getpid()}", final)
    else:
        # every table of the job in one run: this rank's share of each list, integrated together
        paths = [os.path.join(args.out, "temp", f"{t}_rank{rank}") for _, t in jobs]
        todos = []
        for m, path in zip(shards, paths):
            have = done_keys(path)
            todos.append([s for s in m if (s.seed, f"{s.dG:.4f}", f"{s.dsigma:.4f}") not in have])
        flat = [(k, s) for k, todo in enumerate(todos) for s in todo]

        def on_batch(part, new):
            for k in range(len(jobs)):
                sel = [i for i, s in enumerate(part) if owner[id(s)] == k]
                if sel:
                    append_rows(paths[k], rank, [part[i] for i in sel], [new[i] for i in sel])
        owner = {id(s): k for k, s in flat}
        t0 = time.perf_counter()
        rows_all, _ = run_sims([s for _, s in flat], sc, empfcs, sched, args.precision, args.batch, device,
                               progress=Progress(rank), on_batch=on_batch)
        wall = time.perf_counter() - t0
        n_steps = len(flat) * sc.shape[0] * sched.n_total
        perf = json.dumps({"rank": rank, "sims": len(flat), "nodes": sc.shape[0], "wall_s": wall,
                           "node_steps": n_steps, "node_steps_per_s": n_steps / wall if wall else None,
                           "tables": [t for _, t in jobs], "batches": getattr(run_sims, "last_timings", None)})
        print(perf, flush=True)
        for path in paths:  # one line per run
            with open(path + "_perf.jsonl", "a") as f:
                f.write(perf + "\n")
        done, g0 = 0, 0
        for (sims, tag), mine, todo, path in zip(jobs, shards, todos, paths):
            rows = rows_all[done:done + len(todo)]
            done += len(todo)
            if dist:  # the data path: every rank's whole shard reaches rank 0 in one all-gather over RCCL
                gathered = gather_table(shard_table(rank, mine, todo, rows, path), dist, torch.device(device))
                # every rank holds the whole gathered table: all ranks check it, so they raise together
                # (a rank-0-only raise would leave the others blocked in the final barrier)
                if len(gathered) != len(sims):
                    raise RuntimeError(f"gathered {len(gathered)} rows for {len(sims)} simulations")
                if rank == 0:
                    write_gathered(sims, args.out, tag, gathered)
            elif launcher == "slurm":
                if rank_files_complete(sims, args.out, tag, world, g0):  # the last task to finish assembles
                    collapse_sweep(sims, args.out, tag, world)
            elif rank == 0:
                collapse_sweep(sims, args.out, tag, world)
            g0 += len(sims)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
