"""HBM traffic per minibatch step of the update kernels from the rocprofv3 PMC passes of
tools/profile_r02.sh / profile_r03.sh (FETCH_SIZE and WRITE_SIZE in separate runs, kB per dispatch).

    python tools/pmc_summary.py gpurun_out/prof > profiles/r02/pmc_summary.json

FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B).
Per workload the bytes of every update-kernel dispatch are summed and divided by the
minibatch steps they cover:
  local: one fused k_update_ffn launch = 10 epochs x 6400 steps x 4 policies (4096 envs)
  c4:    one fused launch = 10 x 25600 steps x 1 policy (SharedDecentral, 4096 envs)
  c5:    k_gnn<2, 2> + k_gnn_reduce + k_gnn_adam per step (+ k_gnn_gather per 1024 steps),
         10 x 800 steps (128 envs)
"""
import csv, json, os, sys

GFX950_FETCH_CORRECTION = 2.0
WORKLOADS = {
    "local": {"kernels": ["void k_update_ffn<2, 9"], "steps": 10 * 6400 * 4,
              "workload": "QuantrupedMultiEnv_Local, 4096 envs, T=200 (one fused launch: 10 x 6400 steps x 4 policies)"},
    "c4": {"kernels": ["void k_update_ffn<2, 5"], "steps": 10 * 25600,
           "workload": "QuantrupedMultiEnv_SharedDecentral, 4096 envs, T=200 (one fused launch: 10 x 25600 steps)"},
    "c5": {"kernels": ["void k_gnn<2, 2", "k_gnn_reduce", "k_gnn_adam", "k_gnn_gather"], "steps": 10 * 800,
           "workload": "QuantrupedMultiEnv_DecentralShared_Graph, 128 envs, T=200 (10 x 800 steps, 3 launches "
                       "each, plus one record gather per 1024 steps)"},
}


def counter(path, name, prefix):
    tot, n = 0.0, 0
    with open(path) as f:
        for r in csv.DictReader(f):
            kn = r["Kernel_Name"].replace("(anonymous namespace)::", "")   # r03: kernels in an unnamed namespace
            if r["Counter_Name"] == name and kn.startswith(prefix):
                tot += float(r["Counter_Value"])
                n += 1
    return tot, n


def main(d):
    out = {"command": "tools/profile_r0N.sh: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- "
                      "python3 bench.py --steps 1 --warmup 0 ...",
           "gfx950_fetch_correction": GFX950_FETCH_CORRECTION, "workloads": {}}
    for name, w in WORKLOADS.items():
        per = {}
        total = 0.0
        for k in w["kernels"]:
            f_kb, nf = counter(os.path.join(d, f"pmc_{name}_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE", k)
            w_kb, nw = counter(os.path.join(d, f"pmc_{name}_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE", k)
            if not nf or not nw:
                raise SystemExit(f"{name}: no {k} dispatch in the PMC passes under {d}")
            b = (f_kb * GFX950_FETCH_CORRECTION + w_kb) * 1024.0
            per[k] = {"dispatches": nf, "fetch_kb": f_kb, "write_kb": w_kb,
                      "hbm_bytes_per_step": round(b / w["steps"], 1)}
            total += b
        out["workloads"][name] = {"workload": w["workload"], "steps": w["steps"], "kernels": per,
                                  "hbm_bytes_per_step": round(total / w["steps"], 1)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
