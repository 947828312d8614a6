"""Long run of the SC optimiser (optimize_SC_Hopf.py with its two optional steps off, the
setting that matches the shipped SC_opti_25julio.txt): how the homotopic
weights approach the shipped ones with the iteration count, which the reference does not
record.  Prints one JSON line every --every iterations: homotopic mean, Pearson r and RMS
difference against the shipped homotopic weights, and the four fitting measures.
python tools/sc_converge.py [iters] [every]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    from nremmodfc_amd import datasets, optimize_sc
    shipped = datasets.load_sc()
    h0, h1 = optimize_sc.HOMOTOPIC[:, 0], optimize_sc.HOMOTOPIC[:, 1]
    ref = shipped[h0, h1]
    deco = datasets.load_deco_sc()
    print(json.dumps({"iter": -1, "shipped_homotopic_mean": float(ref.mean()),
                      "deco_homotopic_mean": float(deco[h0, h1].mean()),
                      "deco_r": float(np.corrcoef(deco[h0, h1], ref)[0, 1])}), flush=True)
    t0 = time.perf_counter()
    state = {}

    def log(d):
        state["last"] = d

    # run in blocks so the current C is visible between them (optimize() returns C)
    C = deco
    done = 0
    while done < iters:
        n = min(every, iters - done)
        C, _, fit = optimize_sc.optimize(n, 10, 0.03, sc=C, log=log, threshold=0, lock_sum=False)
        done += n
        hv = C[h0, h1]
        print(json.dumps({"iter": done, "homotopic_mean": float(hv.mean()),
                          "r_vs_shipped": float(np.corrcoef(hv, ref)[0, 1]),
                          "rms_vs_shipped": float(np.sqrt(np.mean((hv - ref) ** 2))),
                          "fitting": fit[:, -1].tolist(), "wall_s": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
