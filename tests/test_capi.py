"""The C-ABI from a C caller (tests/capi/capi_smoke.c, built by
__graft_entry__.build()): plan + execute and the stream API through
include/lfdas.h only, on inputs with closed-form zero-phase low-pass results."""
import os
import subprocess

import pytest

EXE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "capi", "capi_smoke")


def test_capi_smoke_built():
    assert os.path.exists(EXE), "build() compiles tests/capi/capi_smoke"


@pytest.mark.gpu
def test_capi_smoke_runs_on_gpu():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "capi smoke ok" in r.stdout
