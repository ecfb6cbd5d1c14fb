"""Per-step HBM traffic, matrix-core busy fraction and effective clock of the update kernels from
the rocprofv3 PMC passes of tools/profile_r06.sh (earlier rounds: profile_r02.sh - r04.sh).

    python tools/pmc_summary.py gpurun_out/prof6 > profiles/r06/pmc_summary.json

Traffic: FETCH_SIZE and WRITE_SIZE come from separate passes (kB per dispatch); FETCH_SIZE is
doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B).  Per workload the
bytes of every update-kernel dispatch are summed and divided by the minibatch steps they cover:
  local: one fused k_update_ffn launch = 10 epochs x 6400 steps x 4 policies (4096 envs)
  c4:    one fused launch = 10 x 25600 steps x 1 policy (SharedDecentral, 4096 envs)
  c5:    k_gnn<2, 2> per step (round 4: one launch, the reduction and Adam in its tail),
         + k_gnn_gather per 1024 steps, one epoch of 12,800 steps (2048 envs)
  c5_3launch: the same with DDRL_GNN_TAIL=0 (+ k_gnn_reduce + k_gnn_adam per step)

Matrix cores and clock (pass "MFMA": SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES,
GRBM_GUI_ACTIVE with --kernel-trace), per kernel summed over its dispatches:
  * kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the counter over the 8 XCDs,
    MI355X_MICROARCH.md "DVFS give-back");
  * clock_ghz = kernel cycles / the dispatches' kernel-trace duration (the guide: within 3 % of
    the in-kernel clock for dispatches of >= 10 ms, reads high below ~0.3 ms);
  * SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over the SIMDs
    (= 32 per v_mfma_f32_16x16x4_f32, 2048 FLOP at 64 FLOP / cycle / SIMD);
    mfma_busy_frac_chip = busy / (kernel cycles x 1024 SIMDs);
    mfma_busy_frac_of_active_simds = busy / (kernel cycles x the SIMDs the launch occupies:
    one wave per SIMD, 4 per workgroup, the workgroups that have work);
  * mfma_flop_per_busy_cycle_per_simd = the kernel's algorithmic FLOP / busy: 64 when every
    busy cycle does useful f32 work, lower when MFMAs run on zero padding.
"""
import csv
import json
import os
import sys

GFX950_FETCH_CORRECTION = 2.0
N_SIMD = 1024
LONG_CLOCK_GHZ = 2.39   # set from the local / c4 update dispatches in main()
WORKLOADS = {
    "local": {"kernels": ["void k_update_ffn<2, 9"], "steps": 10 * 6400 * 4,
              "workload": "QuantrupedMultiEnv_Local, 4096 envs, T=200 (one fused launch: 10 x 6400 steps x 4 policies)",
              # the dominant kernel, its occupied SIMDs (16 workgroups x 4 waves) and algorithmic
              # FLOP per step (bench.py ffn_flops_per_row(35, 2) x 128 rows)
              "mfma": {"kernel": "void k_update_ffn<2, 9", "active_simds": 64, "flop_per_step": 68992 * 128},
              "also": ["void k_act_ffn<2, 9"]},
    "c4": {"kernels": ["void k_update_ffn<2, 5"], "steps": 10 * 25600,
           "workload": "QuantrupedMultiEnv_SharedDecentral, 4096 envs, T=200 (one fused launch: 10 x 25600 steps)",
           "mfma": {"kernel": "void k_update_ffn<2, 5", "active_simds": 16, "flop_per_step": 2 * (2 * (19 * 64 + 64 * 64 + 64 * 4 + 19 * 64 + 64 * 64 + 64) + (64 * 64 + 64 * 4) + (64 * 64 + 64)) * 128},
           "also": ["void k_act_ffn<2, 5"]},
    # round 5: the C5 passes run the bench configuration itself (2048 envs, T = 200: 680 MB of
    # records, so the per-step record gathers read HBM, not the Infinity Cache), one epoch
    # (bench.py --sgd-iter 1: 12,800 steps; the per-step figures do not depend on the epochs)
    "c5": {"kernels": ["void k_gnn<2, 2", "k_gnn_reduce", "k_gnn_adam", "k_gnn_gather"], "steps": 12800,
           "workload": "QuantrupedMultiEnv_DecentralShared_Graph, 2048 envs, T=200 (one epoch: 12,800 one-launch "
                       "steps, plus one record gather per 1024 steps)",
           # gradient launch: 32 tiles x 2 nets x 4 backward shares x 4 waves; FLOP: bench.py
           # gnn_flops_per_row(2) x 128 rows (the forward counted once, not once per share)
           "mfma": {"kernel": "void k_gnn<2, 2", "active_simds": 1024, "flop_per_step": 764800 * 128},
           "also": ["void k_gnn<2, 0"]},
    "c5_3launch": {"kernels": ["void k_gnn<2, 2", "k_gnn_reduce", "k_gnn_adam", "k_gnn_gather"], "steps": 12800,
                   "workload": "the same with DDRL_GNN_TAIL=0: k_gnn<GRAD> + k_gnn_reduce + k_gnn_adam per step",
                   "mfma": {"kernel": "void k_gnn<2, 2", "active_simds": 1024, "flop_per_step": 764800 * 128},
                   "also": ["k_gnn_reduce", "k_gnn_adam"]},
}
# LDS / issue counters (tools/profile_r06.sh "lds" passes), summed per kernel over its dispatches
DETAIL = {"local": "void k_update_ffn<2, 9", "c5": "void k_gnn<2, 2"}
DETAIL_COUNTERS = ["SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_LDS", "SQ_LDS_ADDR_CONFLICT",
                   "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"]


def detail(d):
    """Per-workload sums of the LDS / issue counters, and the bank-conflict cycles per LDS
    instruction and per active LDS cycle."""
    out = {}
    for name, k in DETAIL.items():
        pdir = os.path.join(d, f"lds_{name}")
        path = os.path.join(pdir, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        res = {"kernel": k}
        for c in DETAIL_COUNTERS:
            v, n = counter(path, c, k)
            if n:
                res[c] = v
                res["dispatches"] = n
        if res.get("SQ_INSTS_LDS"):
            res["bank_conflict_cycles_per_lds_inst"] = res.get("SQ_LDS_BANK_CONFLICT", 0.0) / res["SQ_INSTS_LDS"]
        if res.get("SQ_ACTIVE_INST_LDS"):
            res["bank_conflict_over_active_lds"] = res.get("SQ_LDS_BANK_CONFLICT", 0.0) / res["SQ_ACTIVE_INST_LDS"]
        out[name] = res
    return out


def _rows(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            r["Kernel_Name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            yield r


def counter(path, name, prefix):
    tot, n = 0.0, 0
    for r in _rows(path):
        if r["Counter_Name"] == name and r["Kernel_Name"].startswith(prefix):
            tot += float(r["Counter_Value"])
            n += 1
    return tot, n


def mfma_stats(d, prefix, active_simds, flop_total=None):
    """Matrix-core busy and clock of the dispatches of one kernel in pass directory d."""
    cpath = os.path.join(d, "run_counter_collection.csv")
    tpath = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(cpath):
        return None
    per = {}
    for r in _rows(cpath):
        if not r["Kernel_Name"].startswith(prefix):
            continue
        k = r.get("Dispatch_Id") or r.get("Correlation_Id")
        e = per.setdefault(k, {})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            e["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    if not per:
        return None
    if os.path.exists(tpath) and any("ns" not in e for e in per.values()):
        for r in _rows(tpath):
            k = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if k in per:
                per[k]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    tot = {}
    for e in per.values():
        for k, v in e.items():
            tot[k] = tot.get(k, 0.0) + v
    cyc = tot.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    busy = tot.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    ns = tot.get("ns", 0.0)
    # GRBM_GUI_ACTIVE / duration reads high on dispatches shorter than ~0.3 ms (the guide); for
    # those the kernel cycles are the trace duration at the clock of the long update dispatches
    # (LONG_CLOCK_GHZ, measured on the 0.7-2.7 s fcnet update launches of the same run)
    short = len(per) and ns / len(per) < 1e6
    if short and ns > 0:
        cyc = ns * LONG_CLOCK_GHZ
    out = {"kernel": prefix, "dispatches": len(per), "duration_ns": ns, "kernel_cycles": cyc,
           "cycles_source": ("trace duration x %.3f GHz (dispatches < 1 ms: GRBM_GUI_ACTIVE reads high)" % LONG_CLOCK_GHZ
                             if short else "GRBM_GUI_ACTIVE / 8"),
           "SQ_VALU_MFMA_BUSY_CYCLES": busy, "SQ_BUSY_CYCLES": tot.get("SQ_BUSY_CYCLES"),
           "SQ_WAVE_CYCLES": tot.get("SQ_WAVE_CYCLES"), "GRBM_GUI_ACTIVE": tot.get("GRBM_GUI_ACTIVE"),
           "clock_ghz": (tot.get("GRBM_GUI_ACTIVE", 0.0) / 8.0) / ns if ns > 0 and not short else None,
           "mfma_busy_frac_chip": busy / (cyc * N_SIMD) if cyc > 0 else None,
           "active_simds": active_simds,
           "mfma_busy_frac_of_active_simds": busy / (cyc * active_simds) if cyc > 0 and active_simds else None}
    if flop_total and busy > 0:
        out["mfma_flop_per_busy_cycle_per_simd"] = flop_total / busy
    return out


def main(d):
    global LONG_CLOCK_GHZ
    for name in ("local", "c4"):   # the clock the chip holds under the long update launches
        st = mfma_stats(os.path.join(d, f"pmc_{name}_MFMA"), WORKLOADS[name]["mfma"]["kernel"], 1)
        if st and st.get("clock_ghz"):
            LONG_CLOCK_GHZ = st["clock_ghz"]
            break
    out = {"command": "tools/profile_r06.sh: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | "
                      "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE (separate passes, "
                      "--kernel-trace) -- python3 bench.py --steps 1 --warmup 0 ...",
           "gfx950_fetch_correction": GFX950_FETCH_CORRECTION, "workloads": {}}
    for name, w in WORKLOADS.items():
        per = {}
        total = 0.0
        if not os.path.isdir(os.path.join(d, f"pmc_{name}_FETCH_SIZE")):
            continue
        for k in w["kernels"]:
            f_kb, nf = counter(os.path.join(d, f"pmc_{name}_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE", k)
            w_kb, nw = counter(os.path.join(d, f"pmc_{name}_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE", k)
            if not nf or not nw:
                if k == w["kernels"][0]:
                    raise SystemExit(f"{name}: no {k} dispatch in the PMC passes under {d}")
                continue   # e.g. k_gnn_reduce / k_gnn_adam: absent when the GNN step is one launch
            b = (f_kb * GFX950_FETCH_CORRECTION + w_kb) * 1024.0
            per[k] = {"dispatches": nf, "fetch_kb": f_kb, "write_kb": w_kb,
                      "hbm_bytes_per_step": round(b / w["steps"], 1)}
            total += b
        res = {"workload": w["workload"], "steps": w["steps"], "kernels": per,
               "hbm_bytes_per_step": round(total / w["steps"], 1)}
        m = w["mfma"]
        mdir = os.path.join(d, f"pmc_{name}_MFMA")
        flop = m["flop_per_step"] * w["steps"] if m["flop_per_step"] else None
        st = mfma_stats(mdir, m["kernel"], m["active_simds"], flop)
        if st is not None:
            res["mfma"] = st
            res["mfma_other"] = [x for x in (mfma_stats(mdir, k, None) for k in w.get("also", [])) if x]
        out["workloads"][name] = res
    out["lds_detail"] = detail(d)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof4")
