"""Bounds-checked update kernel (the A = 8 illegal-address report).

tools/bounds_check.py loads libddrl_hip_bounds.so (-DDDRL_BOUNDS) in a child process and runs
every update parity case of test_gpu_parity.py -- the Centralized A = 8 kernels at the C1
shape (one env x 160 / 200 rows, d = 43 and TVel d = 44) among them -- with and without the
row split, plus the data-parallel gradient launches of <= 64 rows.  Every index the kernel
derives at run time (staging row of each LDS-DMA chunk, record row, perm / shuffle index,
LDS-DMA destination, staged-record read, Adam-state index) is checked; the test requires
parity green in every case and zero violations."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_update_kernel_indices_in_bounds():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "bounds_check.py")],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines and lines[-1].get("bounds_check") == "ok", r.stdout[-4000:] + r.stderr[-4000:]
    cases = lines[:-1]
    assert len(cases) == lines[-1]["cases"] >= 20
    assert any("Centralized" in c["case"] and "split=1" in c["case"] for c in cases)
    for c in cases:
        assert c["status"] == "pass" and not any(c["violations"].values()), c
    assert r.returncode == 0
