"""r06: compiler-flag variants of the production library (scheduler knobs of the AMDGPU backend),
timed like tools/ablate.py (Local and C4 update us/step at 4096 envs; the state digest shows
bit-identity).

    python tools/r06_flags_ab.py build            # in the container (hipcc)
    python tools/r06_flags_ab.py time [rounds]    # on the GPU box
"""
import os, subprocess, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VARIANTS = {
    "trackers": ["-mllvm", "-amdgpu-use-amdgpu-trackers"],
    "noclusterrp": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"],
    "maxilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    # no SLP auto-packing of scalar f32 code into v_pk_* (MI355X_MICROARCH.md: packed f32 VALU
    # beside MFMAs is an anti-lever); Adam's explicit float2 ops stay packed
    "noslp": ["-fno-slp-vectorize"],
}


def paths(tag):
    from ddrl_amd import native as N
    d = os.path.dirname(N.LIB_PATH)
    return os.path.join(d, f"libddrl_hip_flags_{tag}.so"), os.path.join(d, f"_build_flags_{tag}")


def build(tags):
    from ddrl_amd import build as B
    for t in tags:
        lib, bd = paths(t)
        flags = VARIANTS[t]
        saved = dict(B.SRC_FLAGS)
        try:
            # the variant's flags replace the production flags of the fused update's sources only
            # (a later option of the same name wins on the hipcc line)
            for src in ("ppo_ffn.hip",):
                B.SRC_FLAGS[src] = saved.get(src, []) + flags
            print(B.build(lib=lib, build_dir=bd), flush=True)
        finally:
            B.SRC_FLAGS.clear()
            B.SRC_FLAGS.update(saved)


def time_all(rounds):
    from ddrl_amd import native as N
    libs = [("default", N.LIB_PATH)] + [(t, paths(t)[0]) for t in VARIANTS if os.path.exists(paths(t)[0])]
    for i in range(rounds):
        for tag, lib in libs:
            for env in ("QuantrupedMultiEnv_Local", "QuantrupedMultiEnv_SharedDecentral"):
                out = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "tools/ablate.py", "one", lib, "4096",
                                      env], capture_output=True, text=True)
                if out.returncode:
                    print(f"{tag} {env} failed: {out.stderr[-400:]}", flush=True)
                    sys.exit(out.returncode)
                print(f"run {i} {tag:12s} {env.split('_')[1]:16s} {out.stdout.strip()}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:] or list(VARIANTS))
    else:
        time_all(int(sys.argv[2]) if len(sys.argv) > 2 else 2)
