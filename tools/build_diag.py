"""Prebuild the stamp-diagnostic library (tools/diag_stamps.py) in the container."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddrl_amd import build, native as N
extra = os.environ.get("DDRL_EXTRA_FLAGS", "").split()
tag = "".join(ch for ch in "".join(extra) if ch.isalnum())[:24]
d = os.path.dirname(N.LIB_PATH)
print(build.build(extra_flags=["-DDDRL_STAMPS"] + extra, lib=os.path.join(d, f"libddrl_hip_diag{tag}.so"),
                  build_dir=os.path.join(d, f"_build_diag{tag}")))
