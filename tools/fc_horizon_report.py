#!/usr/bin/env python3
"""Fixed-seed FC parity at the full 1001 s horizon: the report (run here, on the CPU).

Inputs: tests/golden/ref_replay_full.npz (tools/fc_horizon_ref.py: the reference's own run()
and the C oracle, fp64, identical Philox noise, 32 keys of cell (0, 0)) and the GPU run of
tools/fc_horizon_gpu.py (fp64, fp64 with the initial E of node 0 scaled by 1 + eps, fp32).

For every variant X: per-seed FC SSIM (utils.py:48, data_range = 1) against the reference's
run() at the same seed, against the oracle, the between-seed floor, the seed-averaged FC against
the reference's split-half floor, and the 16 metric columns (pathwise |diff|, column means).

  python tools/fc_horizon_report.py GPU.npz [OUT.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle.sigchain as osg  # noqa: E402

N = 90


def full(flat):
    fc = np.eye(N)
    iu = np.triu_indices(N, 1)
    fc[iu] = flat
    fc[iu[1], iu[0]] = flat
    return fc


def ssims(A, B):
    return np.array([osg.ssim(full(a), full(b), 1.0) for a, b in zip(A, B)])


def stats(x):
    return {"mean": float(np.mean(x)), "min": float(np.min(x)), "max": float(np.max(x))}


def main():
    fx = np.load(os.path.join(ROOT, "tests", "golden", "ref_replay_full.npz"))
    g = np.load(sys.argv[1])
    out_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r03_fc_horizon.json")
    assert np.array_equal(fx["keys"], g["keys"])
    ref, orc = fx["fc_ref"], fx["fc_orc"]
    K = len(ref)
    cols = [str(c) for c in fx["columns"]]
    variants = {"oracle (C, fp64)": (orc, fx["m_orc"]), "gpu f64": (g["fc_f64"], g["m_f64"]),
                "gpu f32 (product)": (g["fc_f32"], g["m_f32"])}
    for e in g["eps"]:
        variants[f"gpu f64, E0 x (1 + {e:.0e})"] = (g[f"fc_f64_eps{e:.0e}"], g[f"m_f64_eps{e:.0e}"])
    shift = np.roll(np.arange(K), 1)
    rep = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "K": K,
           "between_seed_floor_ref": stats(ssims(ref, ref[shift])),
           "split_half_floor_ref": float(osg.ssim(full(ref[:K // 2].mean(0)), full(ref[K // 2:].mean(0)), 1.0)),
           "variants": {}}
    for name, (fc, m) in variants.items():
        d = np.abs(m - fx["m_ref"])
        rep["variants"][name] = {
            "ssim_vs_reference_same_seed": stats(ssims(fc, ref)),
            "ssim_vs_oracle_same_seed": stats(ssims(fc, orc)),
            "ssim_vs_gpu_f64_same_seed": stats(ssims(fc, g["fc_f64"])),
            "seed_mean_fc_ssim_vs_reference": float(osg.ssim(full(fc.mean(0)), full(ref.mean(0)), 1.0)),
            "columns_mean_abs_diff_vs_reference": dict(zip(cols, d.mean(0).round(5).tolist())),
            "columns_mean": dict(zip(cols, m.mean(0).round(5).tolist())),
        }
    rep["columns_mean_reference"] = dict(zip(cols, fx["m_ref"].mean(0).round(5).tolist()))
    rep["columns_sd_reference"] = dict(zip(cols, fx["m_ref"].std(0, ddof=1).round(5).tolist()))
    rep["divergence_ref_vs_oracle_max_abs_E_first_recorded_second"] = stats(fx["div"][:, 0])
    with open(out_path, "w") as f:
        json.dump(rep, f, indent=1)
    for name, v in rep["variants"].items():
        print(f"{name:34s} same-seed SSIM vs ref {v['ssim_vs_reference_same_seed']['mean']:.4f} "
              f"vs oracle {v['ssim_vs_oracle_same_seed']['mean']:.4f}  seed-mean {v['seed_mean_fc_ssim_vs_reference']:.4f}")
    print(f"between-seed floor {rep['between_seed_floor_ref']['mean']:.4f}, split-half floor "
          f"{rep['split_half_floor_ref']:.4f}")


if __name__ == "__main__":
    main()
