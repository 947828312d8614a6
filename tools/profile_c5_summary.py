#!/usr/bin/env python3
"""Summaries of the four C5 PMC passes (tools/profile_c5_pass.sh fetch|write|sqa|sqb, one gpurun call
each, merged back under gpurun_out/prof_c5/), run on the CPU from the repo root:
  profiles/pmc_sde_c5.json  HBM bytes per persist_kernel step, scaled to bench.py's 20,000-step launch
  profiles/pmc_c5_sq.json   instruction mix, MFMA / VALU busy and the wave-cycle split per wave-step"""
def _dump(d, name):
    """profiles/<name>, and a copy under gpurun_out/prof_c5/ (the only directory a GPU call returns)."""
    import json, os
    json.dump(d, open(os.path.join("profiles", name), "w"), indent=1)
    os.makedirs("gpurun_out/prof_c5", exist_ok=True)
    json.dump(d, open(os.path.join("gpurun_out/prof_c5", name), "w"), indent=1)


def hbm():
    import json, os, sys
    sys.path.insert(0, "tools")
    from pmc_summary import summary
    from pmc_summary import lib_stamp
    stamp = lib_stamp("gpurun_out/prof_c5/fetch", "gpurun_out/prof_c5/write")
    (kf, vf), = summary("gpurun_out/prof_c5/fetch", "persist_kernel").items()
    (kw, vw), = summary("gpurun_out/prof_c5/write", "persist_kernel").items()
    B, N, STEPS = 2500, 1000, 20000
    RUN = int(os.environ.get("C5STEPS", "400"))  # one persist_kernel launch integrates RUN steps
    fetch = 2 * vf["FETCH_SIZE"] * 1024.0 / RUN
    write = vw["WRITE_SIZE"] * 1024.0 / RUN
    Np, Bp = 1024, 2560
    img = Np * Bp * 4           # the fp16 hi/lo E image every node block publishes each step
    recs = B * N * 4 / 20       # one fp32 E record per node every 20 steps
    d = {"kernel": kf, "lib_sha256": stamp, "B": B, "N": N, "euler_steps": STEPS, "precision": "f32",
         "fetch_bytes_per_step": fetch, "write_bytes_per_step": write,
         "write_bytes_per_step_algorithmic": img + recs,
         "write_excess": write / (img + recs),
         "fetch_bytes_per_launch": fetch * STEPS, "write_bytes_per_launch": write * STEPS,
         "hbm_bytes_per_launch": (fetch + write) * STEPS, "dispatches": vf["dispatches"],
         "state_bytes_per_step": B * N * 36, "connectome_bytes_per_step": 1024 * 1024 * 2 * 2,
         "algorithmic_bytes_per_launch": B * N * (STEPS // 20 * 4 + 2 * 3 * 8 + 2 * 8),
         "note": "rocprofv3 --pmc passes of `python3 tools/c5_pmc_run.py 400` (tools/profile_c5_pass.sh fetch / write): one persist_kernel "
                 "dispatch of 400 Euler steps, divided by 400 and scaled by 20,000 to bench.py's per-chunk 'launch'. FETCH_SIZE x2 (gfx950), KB -> B; the "
                 "counters include Infinity-Cache (MALL) hits; the state stays in registers, so the bytes are the "
                 "per-step operand stream (connectome rows and the E image)."}
    if os.path.isdir("gpurun_out/prof_c5/writering"):
        (_, vr), = summary("gpurun_out/prof_c5/writering", "persist_kernel").items()
        d["write_bytes_per_step_ring_records"] = vr["WRITE_SIZE"] * 1024.0 / RUN
        d["note_ring"] = ("the round-5 harness recorded into a node-major ring with ld = 20 (4-B stores at an 80-B "
                          "stride: partial-line writes); bench.py and the fp32 pipeline record time-major, as "
                          "write_bytes_per_step is measured")
    _dump(d, "pmc_sde_c5.json")
    print(json.dumps(d))


def sq():
    import json, sys
    sys.path.insert(0, "tools")
    from pmc_summary import summary
    from pmc_summary import lib_stamp
    stamp = lib_stamp("gpurun_out/prof_c5/sqa", "gpurun_out/prof_c5/sqb")
    (ka, a), = summary("gpurun_out/prof_c5/sqa", "persist_kernel").items()
    (_, b), = summary("gpurun_out/prof_c5/sqb", "persist_kernel").items()
    STEPS, WAVES = 400, 256 * 8
    act = a["GRBM_GUI_ACTIVE"] / 8 * 1024
    d = {"kernel": ka, "lib_sha256": stamp, "steps": STEPS, "waves": WAVES,
         "per_wave_step": {k: a[k] / (WAVES * STEPS) for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD")},
         "salu_per_wave_step": b["SQ_INSTS_SALU"] / (WAVES * STEPS),
         "mfma_busy_frac": a["SQ_VALU_MFMA_BUSY_CYCLES"] / act,
         "valu_issue_busy_frac": 4 * a["SQ_ACTIVE_INST_VALU"] / act,
         "lds_bank_conflict_frac": b["SQ_LDS_BANK_CONFLICT"] / max(1.0, b["SQ_LDS_IDX_ACTIVE"]),
         "wave_cycle_split": {k: b[k] / b["SQ_WAVE_CYCLES"] for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")},
         "note": "rocprofv3 --pmc passes of tools/c5_pmc_run.py 400 (one persist_kernel dispatch of 400 Euler steps at the "
                 "C5 shard, 2,500 x 1000, 8 waves per CU on 256 CUs). Busy fractions over GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs."}
    _dump(d, "pmc_c5_sq.json")
    print(json.dumps(d))


def tcc():
    """L2 (TCC) hit rate of the operand stream: where the connectome rows and the E image come from."""
    import json, sys
    sys.path.insert(0, "tools")
    from pmc_summary import summary
    from pmc_summary import lib_stamp
    stamp = lib_stamp("gpurun_out/prof_c5/tcc")
    (k, t), = summary("gpurun_out/prof_c5/tcc", "persist_kernel").items()
    STEPS = 400
    req = t["TCC_HIT_sum"] + t["TCC_MISS_sum"]
    d = {"kernel": k, "lib_sha256": stamp, "steps": STEPS,
         "tcc_requests_per_step": req / STEPS, "tcc_hits_per_step": t["TCC_HIT_sum"] / STEPS,
         "tcc_misses_per_step": t["TCC_MISS_sum"] / STEPS, "l2_hit_rate": t["TCC_HIT_sum"] / req,
         "ea_read_requests_per_step": t["TCC_EA0_RDREQ_sum"] / STEPS,
         "unique_operand_bytes_per_step": 8 * (4 * 128 * 25 * 32 * 4 + 8 * 80 * 1024 * 4),
         "note": "rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum over tools/c5_pmc_run.py 400 (one persist_kernel "
                 "dispatch, 400 steps; tools/profile_c5_pass.sh tcc). unique_operand_bytes_per_step: per XCD the streamed "
                 "connectome rows of its 4 node blocks (25 of 32 K chunks; 7 stay in LDS) plus the E image of its 8 "
                 "simulation blocks, summed over the 8 XCDs (4.2 MB per XCD against a 4 MB L2)."}
    _dump(d, "pmc_c5_tcc.json")
    print(json.dumps(d))


if __name__ == "__main__":
    import sys as _s
    for f in (_s.argv[1:] or ["hbm", "sq", "tcc"]):
        {"hbm": hbm, "sq": sq, "tcc": tcc}[f]()
