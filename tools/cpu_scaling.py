"""CPU baseline against core count on the GPU box's host, up to one GPU's share (bench.CPU_SHARE = 16):
the compiled port (oracle/wc_oracle.c, OpenMP over simulations, 2 simulations per thread) and the
interpreted NumPy loop (oracle/numpy_run.py, one process per core), at 1, 2, 4, 8 and 16 cores.
The box's operator rules cap a job's worker pools at that share, so the all-core figure stays an
extrapolation; this log shows how the rate scales up to the cap.

  PYTHONPATH=. python tools/cpu_scaling.py [seconds per point]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import oracle  # noqa: E402
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import driver_params  # noqa: E402


def compiled(sc, nthreads, seconds, steps=2000):
    G, S, keys = bench.sweep_batch(0)
    B = 2 * nthreads
    ob = oracle.OracleBatch(sc, G[:B], S[:B], keys[:B], driver_params())
    ob.integrate(200, 2.0, 20, nthreads=nthreads)
    t0, n = time.perf_counter(), 0
    while True:
        ob.integrate(steps, 2.0, 20, nthreads=nthreads)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return B * sc.shape[0] * steps * n / (time.perf_counter() - t0)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    sc = datasets.synthetic_sc(90) if os.environ.get("SYNTH") else datasets.load_sc()
    avail, cap = bench._cores()
    print(f"affinity mask: {avail} cores; cap (one GPU's share): {cap}", flush=True)
    for t in (1, 2, 4, 8, 16):
        if t > cap:
            break
        r = compiled(sc, t, seconds)
        print(f"compiled port, {t:2d} threads: {r:.3e} node-steps/s ({r / t:.3e} per core)", flush=True)
    for t in (1, 4, 16):
        if t > cap:
            break
        bench.CPU_SHARE = t
        r = bench.cpu_baseline_numpy(steps=40_000)
        print(f"numpy loop, {t:2d} processes: {r['value']:.3e} node-steps/s ({r['per_core']['mean']:.3e} per core)",
              flush=True)


if __name__ == "__main__":
    main()
