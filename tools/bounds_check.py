"""Bounds-checked run of the fused update (GPU box): loads libddrl_hip_bounds.so (built with
-DDDRL_BOUNDS by `python -m ddrl_amd.build --bounds`, see ppo_ffn.hip) in place of the
production library, runs the update parity cases of tests/test_gpu_parity.py -- every fcnet
shape, the Centralized A = 8 kernels (C1: one env x 160 rows, d = 43; TVel d = 44) -- with the
row split (KSP = 2, default) and without it (DDRL_UPDATE_SPLIT=1: the 4-wave, spilling A = 8
instance), plus data-parallel gradient launches of <= 64 rows, and prints one JSON line with
the violation counters of the staging / record / schedule / LDS / parameter indices.
Exit status 0 only if every case passed its parity check and every counter is zero.

    python tools/bounds_check.py
"""
import ctypes as C
import json
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from ddrl_amd import native as N  # noqa: E402

LIB = os.path.join(os.path.dirname(N.LIB_PATH), os.environ.get("DDRL_BOUNDS_LIB", "libddrl_hip_bounds.so"))
KINDS = ["staging_row", "record_row", "schedule_index", "lds_dma_dst", "staged_read", "param_index"]


def counters(lib, reset=False):
    buf = (C.c_uint * len(KINDS))()
    if lib.ddrl_diag_bounds(buf, 1 if reset else 0) != 0:
        raise RuntimeError("ddrl_diag_bounds failed")
    return dict(zip(KINDS, list(buf)))


def main():
    lib = N.load(LIB)           # every later N.load() returns this library
    lib.ddrl_diag_bounds.argtypes = [C.POINTER(C.c_uint), C.c_int]
    import test_gpu_parity as T
    cases = []
    for split in ("2", "1"):
        os.environ["DDRL_UPDATE_SPLIT"] = split
        for args in T.UPDATE_CASES:
            cases.append((f"update{args[:4]} split={split}", lambda a=args: T.test_ppo_update_parity(*a)))
        cases.append((f"ddp grad/apply split={split}", T.test_ddp_grad_and_apply_match_fused_step))
    results, ok = [], True
    counters(lib, reset=True)
    for name, fn in cases:
        os.environ["DDRL_UPDATE_SPLIT"] = name.rsplit("=", 1)[1]
        try:
            fn()
            status = "pass"
        except Exception as e:   # parity failure: report, keep checking the others
            status = f"FAIL {type(e).__name__}: {e}"
            traceback.print_exc()
            ok = False
        c = counters(lib, reset=True)
        ok = ok and not any(c.values())
        results.append({"case": name, "status": status, "violations": c})
        print(json.dumps(results[-1]), flush=True)
    print(json.dumps({"bounds_check": "ok" if ok else "FAILED", "cases": len(results)}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
