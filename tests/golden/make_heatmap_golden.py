#!/usr/bin/env python3
"""shipped_heatmaps.npz: heatmaps.py's extract() (heatmaps.py:30-72, var2see="euccorr", C1=0, w=1,
the thresholds of :26) applied to the reference's shipped homogeneous table
output/sweep_delta_homoW_fromG0.16_sigma7.68_maps_0_0_9dic24_50iter.txt (run here, where
/root/reference exists; only the resulting 15 x 15 cell maps and their optima are committed).

  python tests/golden/make_heatmap_golden.py
"""
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.test_consumers import extract  # noqa: E402

SHIPPED = "/root/reference/output/sweep_delta_homoW_fromG0.16_sigma7.68_maps_0_0_9dic24_50iter.txt"


def main():
    out = extract(pd.read_csv(SHIPPED))
    np.savez(os.path.join(HERE, "shipped_heatmaps.npz"), x_vals=out["x_vals"], y_vals=out["y_vals"],
             plotmats=np.stack(out["plotmats"]), vals_o=np.array(out["vals_o"]))
    print({st: v for st, v in zip(("W", "N1", "N2", "N3"), out["vals_o"])})


if __name__ == "__main__":
    main()
