"""CPU checks of the C-ABI boundary: the library loads, exports every symbol the header
declares, and the ctypes mirror of ddrl_cfg matches the C struct byte for byte."""
import ctypes
import os
import subprocess
import tempfile

import pytest

from ddrl_amd import build, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    build.build()
    return native.load()


def test_exports_every_header_symbol(lib):
    syms = native.header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(native._SIGS), set(syms) ^ set(native._SIGS)
    assert lib.ddrl_abi_version() == native.ABI_VERSION == 4


def test_cfg_struct_layout_matches_header():
    fields = [f for f, _ in native.DdrlCfg._fields_]
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/ddrl_hip.h"',
           'int main(void){', 'printf("%zu\\n", sizeof(ddrl_cfg));']
    src += [f'printf("%zu\\n", offsetof(ddrl_cfg, {f}));' for f in fields]
    src += ['return 0;}']
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-std=c11", c, "-o", exe])
        out = [int(x) for x in subprocess.check_output([exe]).split()]
    assert out[0] == ctypes.sizeof(native.DdrlCfg)
    for f, off in zip(fields, out[1:]):
        assert getattr(native.DdrlCfg, f).offset == off, f


def test_errors_are_reported_without_gpu(lib):
    # A bad configuration is rejected on the host before any device call.
    from ddrl_amd.spec import make_cfg
    cfg, _ = make_cfg("QuantrupedMultiEnv_Local", 4, 2, {"sgd_minibatch_size": 64})
    h = ctypes.c_void_p()
    rc = lib.ddrl_ctx_create(ctypes.byref(cfg), 0, ctypes.byref(h))
    assert rc != 0
    assert b"sgd_minibatch_size" in lib.ddrl_last_error()
    assert lib.ddrl_observe(None, None) != 0
    assert b"null context" in lib.ddrl_last_error()


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(native, "_lib", None)
    with pytest.raises(native.DdrlError, match="missing"):
        native.load(str(tmp_path / "nope.so"))
