"""bench.py keeps the driver's JSON contract (task spec).

CPU: the cpu_baseline legs (the compiled C port, the cost of the reference's numba-compiled loop,
as the value; the interpreted NumPy loop, oracle/numpy_run.py, one process per core, beside it)
on a short sample.
GPU: one short bench run as a child process; its single JSON line carries every
contract key, the roofline and issued-MFMA objects, and consistent arithmetic.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_leg():
    sys.path.insert(0, ROOT)
    import bench
    from nremmodfc_amd import datasets
    cb = bench.cpu_baseline(datasets.load_sc(), seconds=0.3, steps=200)
    assert cb["kind"] == "port" and cb["unit"] == "node-timesteps/sec"
    assert cb["value"] > 0 and 1 <= cb["cores"] <= 16 and "oracle/wc_oracle.c" in cb["sample"]
    assert cb["cores"] == min(cb["cores_available"], cb["cores_cap"])
    npy = cb["numpy_interpreted"]
    assert npy["kind"] == "interpreted" and npy["value"] > 0 and "oracle/numpy_run.py" in npy["sample"]
    assert npy["cores"] == cb["cores"]


def test_cpu_baseline_leg_n1000():
    """C5's CPU baseline: the reference's NumPy loop at N = 1000 (np.dot(CM, E) a
    BLAS gemv, wc:81) and the compiled C port, the faster as the value, the other beside it."""
    sys.path.insert(0, ROOT)
    import bench
    from nremmodfc_amd import datasets
    cb = bench.cpu_baseline(datasets.synthetic_sc(1000), seconds=0.2, steps=200)
    other = cb.get("compiled_port") or cb.get("numpy_interpreted")
    assert cb["value"] >= other["value"] > 0 and "N=1000" in cb["sample"] and "N=1000" in other["sample"]
    assert cb["cores"] == other["cores"] == min(cb["cores_available"], cb["cores_cap"])


def test_pmc_stamp_is_the_loaded_library():
    sys.path.insert(0, ROOT)
    import hashlib

    import bench
    from nremmodfc_amd import _build
    _build.build()
    assert bench.loaded_lib_sha256() == hashlib.sha256(open(_build.LIB_LOAD, "rb").read()).hexdigest()


@pytest.mark.gpu
def test_bench_json_contract(cuda):
    out = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--cpu-seconds", "1",
                          "--secondary-steps", "2"], cwd=ROOT, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"].startswith("node-timesteps/sec") and d["unit"] == "node-timesteps/sec"
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "strong" and d["vs_baseline"] is None and d["weak_scaling"] is None and d["dtype"].startswith("f32")
    assert "workload" in d["config"] and d["config"]["sims_per_gpu"] == 20000
    # value = node-steps of the timed steps / wall time
    ns = d["config"]["sims_per_gpu"] * d["config"]["nodes"] * d["config"]["euler_steps_per_step"] * d["steps"]
    assert abs(ns / (d["ms_per_step"] * 1e-3 * d["steps"]) / d["value"] - 1) < 1e-6
    r = d["roofline"]
    assert r["bound"] == "valu" and r["unit"] == "TFLOP/s" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
    assert "frac" not in r["state_streaming_equiv"]
    assert 0 < r["frac"] < 1.2 and r["issued_mfma"]["dtype"] == "f16"
    assert d["cpu_baseline"]["kind"] == "port" and d["cpu_baseline"]["value"] > 0
    # the 1000-node and reference-precision lines of the same run, each with its own roofline,
    # kernel times and CPU baseline
    c5, f64 = d["secondary"]["c5"], d["secondary"]["f64"]
    assert c5["config"]["nodes"] == 1000 and c5["roofline"]["bound"] == "mfma" and c5["kernel_ms"]["sde"] > 0
    assert "N=1000" in c5["cpu_baseline"]["sample"] and c5["value"] > 0
    assert f64["dtype"] == "f64" and f64["config"]["nodes"] == 90 and 0 < f64["roofline"]["frac"] < 1
    assert f64["cpu_baseline"]["kind"] == "port" and f64["value"] > 0 and f64["kernel_ms"]["welch"] > 0


@pytest.mark.gpu
def test_bench_c5_line_priced_on_mfma(cuda):
    out = subprocess.run([sys.executable, "bench.py", "--config", "c5", "--steps", "1", "--warmup", "0",
                          "--sde-only", "--cpu-seconds", "1"], cwd=ROOT, capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1 and r["peak"] == 2500.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12 and r["operand_stream"]["GBps"] > 0
    o = r["operand_stream"]
    assert abs(o["x_ic_gather_peak"] - o["GBps"] / o["ic_gather_peak_GBps"]) < 1e-12
    if "frac" in o:  # the L2-hit / IC-miss split ceiling, from counters stamped on this library
        assert 0 < o["l2_hit_rate"] < 1 and abs(o["frac"] - o["GBps"] / o["split_peak_GBps"]) < 1e-12
    assert d["config"]["nodes"] == 1000 and d["config"]["sims_per_gpu"] == 2500
    # the CPU baseline at N = 1000 in the same run (north_star)
    assert d["cpu_baseline"]["value"] > 0 and "N=1000" in d["cpu_baseline"]["sample"]
    # counters are attached only when taken on the library this run loaded
    assert r["pmc"] is None or r["pmc_lib_sha256"] is not None
