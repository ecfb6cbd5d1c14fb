"""HBM traffic per launch of the fused update kernel from the rocprofv3 PMC passes of
tools/profile_r01.sh (FETCH_SIZE and WRITE_SIZE in separate runs, kB per dispatch).

    python tools/pmc_summary.py gpurun_out/prof > profiles/r01/pmc_update.json

FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B).
The per-step figure divides by the (policy, minibatch) steps of the profiled launch
(Local, 4096 envs, T = 200: 10 epochs x 6400 minibatches x 4 policies)."""
import csv, json, os, sys

GFX950_FETCH_CORRECTION = 2.0


def counter(path, name, kernel_prefix):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == name and r["Kernel_Name"].startswith(kernel_prefix):
                vals.append((r["Kernel_Name"], float(r["Counter_Value"])))
    return vals


def main(d, kernel_prefix="void k_update_ffn<2, 9", policy_steps=10 * 6400 * 4):
    fetch = counter(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE", kernel_prefix)
    write = counter(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE", kernel_prefix)
    if not fetch or not write:
        raise SystemExit(f"no {kernel_prefix} dispatch in the PMC passes under {d}")
    kname = fetch[-1][0]
    f_kb = sum(v for _, v in fetch) / len(fetch)
    w_kb = sum(v for _, v in write) / len(write)
    hbm = (f_kb * GFX950_FETCH_CORRECTION + w_kb) * 1024.0
    out = {
        "kernel": kname,
        "command": "tools/profile_r01.sh: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- "
                   "python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline",
        "workload": "QuantrupedMultiEnv_Local, 4096 envs, T=200: 10 epochs x 6400 minibatch steps x 4 policies per launch",
        "dispatches": len(fetch),
        "fetch_size_kb": f_kb,
        "write_size_kb": w_kb,
        "gfx950_fetch_correction": GFX950_FETCH_CORRECTION,
        "hbm_bytes_per_launch": hbm,
        "policy_steps_per_launch": policy_steps,
        "hbm_bytes_per_policy_step": round(hbm / policy_steps, 3),
        "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md; includes the partner-exchange polls of the "
                "row split (sc1 loads of the partner's granules)",
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
