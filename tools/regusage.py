"""Register / spill / occupancy summary of the kernels in one HIP source (gfx950 flags).

    python tools/regusage.py [ddrl_amd/csrc/ppo_ffn.hip] [-Dextra ...]
"""
import os, re, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else "ddrl_amd/csrc/ppo_ffn.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
       "-Wno-unused-result", "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(ROOT, src),
       "-o", "/tmp/_regusage.o", *sys.argv[2:]]
err = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur, rows = None, {}
for line in err.splitlines():
    m = re.search(r"remark: (.*) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for f, r in rows.items():
    print(f"{f[:52]:52s} V={r.get('VGPRs')} A={r.get('AGPRs')} Vspill={r.get('VGPRs Spill')} "
          f"Sspill={r.get('SGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')}")
