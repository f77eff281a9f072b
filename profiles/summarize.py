#!/usr/bin/env python3
"""Condense a profiles/run_profiles.sh output directory into a committed per-round summary.

    python profiles/summarize.py gpurun_out/prof r01 [tag]

writes profiles/<round>[_<tag>]_kernel_stats.csv (rocprofv3 --kernel-trace --stats, as produced) and
profiles/<round>[_<tag>]_summary.json with, per kernel (tag: the bench workload, e.g. decent_n10_N5,
which bench.py looks up for its roofline):
  avg_ms                 average duration from the kernel-trace pass
  fetch_kb, write_kb     FETCH_SIZE / WRITE_SIZE per launch (separate PMC passes)
  hbm_bytes              2 * FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, HBM section: on gfx950
                         FETCH_SIZE tallies half the bytes of wide reads; WRITE_SIZE is exact)
  f64_wave_instrs        SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64 per launch (wave instructions)
  f64_flop               64 lanes * (2 FMA + MUL + ADD + TRANS): an upper bound (masked lanes count)
  lane_util              SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU): active lanes per VALU issue
  f64_flop_active        f64_flop * lane_util (masked lanes removed, assuming the F64 share is uniform)
  valu_issue_frac        SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave lifetime issuing VALU)
  wait_frac, stall_frac  SQ_WAIT_ANY, SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (parked on waitcnt / issue-stalled)
  waves_per_cu           mean resident waves per CU: 4 SQ_WAVE_CYCLES (quad-cycles) / (GRBM_GUI_ACTIVE / 8 XCDs) / 256 CUs
  SQ_INSTS_VMEM_RD/_WR   vector memory instructions (scratch included) per launch, SQ_INSTS_SMEM scalar loads;
  TCC_EA0_WRREQ_sum      L2-to-fabric write requests, TCC_EA0_WRREQ_64B_sum those that are whole 64-byte
                         transactions (the rest 32 B: partial lines), "mem" pass (round 6)
bench.py reads hbm_bytes of its dominant kernel from here as roofline.traffic.
"""

from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys


def per_kernel(path: str) -> dict:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def short(name: str) -> str:
    for k in ("k_qp_gi", "k_qp_ipm", "k_enum", "k_cost", "k_select", "k_inst_prep", "k_bnb_root_coop", "k_bnb_root",
              "k_bnb_expand", "k_bnb_bound_refill", "k_bnb_bound_coop", "k_bnb_bound",
              "k_bnb_key", "k_bnb_write", "k_bnb_finish", "k_gadmm_qp_coop", "k_gadmm_qp", "k_gadmm_update",
              "k_gadmm_rollout", "k_gadmm_switch", "k_admm_update", "k_l1_root", "k_l1_bound", "k_qp_l1", "k_lp_root_init", "k_lp_dive_prep", "k_lp_bound_refill",
              "k_lp_root", "k_lp_bound", "k_qp_lp", "k_bnb_dive_prep",
              "k_cent_bnb", "k_cent_tasks", "k_cent_final", "k_cent_init", "k_env_step", "k_decent_params"):
        if k in name:
            return k
    return name[:48]


def main() -> None:
    src, rnd = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else None
    if tag:
        rnd = f"{rnd}_{tag}"
    here = os.path.dirname(os.path.abspath(__file__))
    out = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            k = short(r["Name"])
            out.setdefault(k, {})["avg_ms"] = float(r["AverageNs"]) / 1e6
            out[k]["calls"] = int(r["Calls"])
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(here, f"{rnd}_kernel_stats.csv"))
    # extra workloads traced on their own (e.g. gadmm/): kernel stats kept as <round>_<name>_kernel_stats.csv
    extra = {}
    for name in sorted(os.listdir(src)):
        p = os.path.join(src, name, "trace", "run_kernel_stats.csv")
        if name == "trace" or not os.path.exists(p):
            continue
        shutil.copy(p, os.path.join(here, f"{rnd}_{name}_kernel_stats.csv"))
        with open(p) as f:
            extra[name] = {short(r["Name"]): {"avg_ms": float(r["AverageNs"]) / 1e6, "calls": int(r["Calls"])}
                           for r in csv.DictReader(f)}
    for sub in ("fetch", "write", "f64", "occ", "mem"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for name, ctr in per_kernel(p).items():
            k = short(name)
            d = out.setdefault(k, {})
            for c, vals in ctr.items():
                d[c] = sum(vals) / len(vals)
    for k, d in out.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["fetch_kb"] = d.pop("FETCH_SIZE")
            d["write_kb"] = d.pop("WRITE_SIZE")
            d["hbm_bytes"] = (2.0 * d["fetch_kb"] + d["write_kb"]) * 1024.0
        f64 = [d.get(f"SQ_INSTS_VALU_{t}_F64") for t in ("FMA", "MUL", "ADD", "TRANS")]
        if all(v is not None for v in f64):
            d["f64_wave_instrs"] = sum(f64)
            d["f64_flop"] = 64.0 * (2 * f64[0] + f64[1] + f64[2] + f64[3])
            if d.get("avg_ms"):
                d["f64_tflops"] = d["f64_flop"] / (d["avg_ms"] * 1e-3) / 1e12
        if d.get("SQ_ACTIVE_INST_VALU") and d.get("SQ_THREAD_CYCLES_VALU") is not None:
            d["lane_util"] = d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"])
            if "f64_flop" in d:
                d["f64_flop_active"] = d["f64_flop"] * d["lane_util"]
                if d.get("avg_ms"):
                    d["f64_tflops_active"] = d["f64_flop_active"] / (d["avg_ms"] * 1e-3) / 1e12
        wc = d.get("SQ_WAVE_CYCLES")
        if wc:
            for key, c in (("valu_issue_frac", "SQ_ACTIVE_INST_VALU"), ("wait_frac", "SQ_WAIT_ANY"),
                           ("stall_frac", "SQ_WAIT_INST_ANY"), ("active_frac", "SQ_ACTIVE_INST_ANY")):
                if d.get(c) is not None:
                    d[key] = d[c] / wc
            if d.get("GRBM_GUI_ACTIVE"):
                d["waves_per_cu"] = 4.0 * wc / (d["GRBM_GUI_ACTIVE"] / 8.0) / 256.0
    sha_path = os.path.join(src, "lib_sha256.txt")
    meta = {"round": rnd, "tag": tag, "source": "profiles/run_profiles.sh (rocprofv3 kernel trace + separate PMC passes)",
            "lib_sha256": open(sha_path).read().strip() if os.path.exists(sha_path) else None,
            "workload": open(os.path.join(src, "cmd.txt")).read().strip() if os.path.exists(os.path.join(src, "cmd.txt")) else None,
            "kernels": out, "workloads": extra}
    with open(os.path.join(here, f"{rnd}_summary.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
