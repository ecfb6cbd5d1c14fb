"""Build libddrl_hip.so in-tree with hipcc for gfx950 (no torch extension machinery).

    python -m ddrl_amd.build            # incremental
    python -m ddrl_amd.build --force    # rebuild everything
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libddrl_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("DDRL_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE,
         "-Wno-unused-result"]


# per-source extra flags of the production build:
#  * the fused row-split update kernels are scheduled with LLVM's iterative ILP strategy (Local
#    10.66 -> 10.57 us per step, C4 10.01 -> 9.89; it crashes the compiler on gnn.hip and makes
#    the KSP = 1 kernels spill twice as much, so those stay in ppo_ffn_k1.hip without it);
#  * MFMA results in VGPRs rather than AGPRs (no v_accvgpr_read before every use): Local 10.59
#    -> 10.41, C4 9.93 -> 9.69, C5 (gnn.hip) 17.2 -> 16.9.  The state is the same bit for bit.
_ILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
_VGPR_MFMA = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
#  * the atomic-protocol fallback likewise (its fused step 12.64 -> 12.25 us)
SRC_FLAGS = {"ppo_ffn.hip": _ILP + _VGPR_MFMA, "ppo_ffn_peer.hip": _ILP + _VGPR_MFMA, "gnn.hip": _VGPR_MFMA,
             "ppo_ffn_atomic.hip": _VGPR_MFMA}


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, extra_flags=(), lib=None, build_dir=None) -> str:
    """extra_flags / lib / build_dir: diagnostic variants (e.g. -DDDRL_STAMPS into
    libddrl_hip_diag.so); the default builds the production library."""
    global BUILD, LIB
    BUILD_, LIB_ = BUILD, LIB
    if lib:
        BUILD, LIB = build_dir or BUILD + "_diag", lib
    try:
        return _build(force, verbose, list(extra_flags))
    finally:
        BUILD, LIB = BUILD_, LIB_


def _build(force, verbose, extra_flags):
    os.makedirs(BUILD, exist_ok=True)
    headers = _headers()
    jobs = []
    objs = []
    for src in _sources():
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src, os.path.abspath(__file__)] + headers):
            jobs.append([HIPCC, *FLAGS, *SRC_FLAGS.get(os.path.basename(src), []), *extra_flags, "-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {cmd[-3]}:\n{r.stderr}")
        return r

    n = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8))
    with ThreadPoolExecutor(max_workers=n) as ex:
        list(ex.map(run, jobs))
    if jobs or force or _stale(LIB, objs):
        run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs, "-L/opt/rocm/lib", "-lrccl", "-lpthread"])
    return LIB


BOUNDS_LIB = os.path.join(HERE, "libddrl_hip_bounds.so")


def build_bounds(force: bool = False, verbose: bool = False) -> str:
    """The bounds-checked diagnostic library (-DDDRL_BOUNDS: run-time index checks in the
    update kernel, counted instead of faulting; tools/bounds_check.py), with the exchange
    granules as relaxed agent-scope atomics (-DDDRL_XCHG_ATOMIC, the formally defined protocol)."""
    return build(force, verbose, extra_flags=["-DDDRL_BOUNDS", "-DDDRL_XCHG_ATOMIC"], lib=BOUNDS_LIB,
                 build_dir=os.path.join(HERE, "_build_bounds"))


ATOMIC_LIB = os.path.join(HERE, "libddrl_hip_atomic.so")


def build_atomic(force: bool = False, verbose: bool = False) -> str:
    """The production kernels with the exchange granules as relaxed agent-scope atomics
    (-DDDRL_XCHG_ATOMIC: valid for any workgroup placement, 1.1 us per step slower); load it
    with DDRL_LIB=libddrl_hip_atomic.so."""
    return build(force, verbose, extra_flags=["-DDDRL_XCHG_ATOMIC"], lib=ATOMIC_LIB,
                 build_dir=os.path.join(HERE, "_build_atomic"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--bounds", action="store_true", help="also build libddrl_hip_bounds.so")
    ap.add_argument("--atomic", action="store_true", help="also build libddrl_hip_atomic.so")
    a = ap.parse_args(argv)
    print(build(a.force, a.verbose))
    if a.bounds:
        print(build_bounds(a.force, a.verbose))
    if a.atomic:
        print(build_atomic(a.force, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
