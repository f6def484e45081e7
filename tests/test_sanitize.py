"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run (SURVEY §5:
the reference has no native code; this is the build's own hygiene).

tools/sanitize.sh compiles lfd_capi.cpp, lfd_stream.cpp and lfd_h5.cpp with
-fsanitize=address,undefined (host only) into two C-ABI drivers:
tests/capi/host_sanitize.cpp (host-only plans of every geometry the GPU
tests use — cfg1, cfg3, off-sample head skip, sub-blocks, 3 kHz lattice,
8th order — their debug accessors and error paths, the LFProc schedule, and
LFD_STREAM_DRY_RUN edge / continuous streams with gaps) and
tests/capi/h5_sanitize.cpp (the DASDAE round trip).  Any sanitizer report
aborts the driver with a non-zero status."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "sanitize")


@pytest.fixture(scope="module")
def built():
    if not shutil.which("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), OUT], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return OUT


def _run(exe, *args):
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env=env)


def test_host_code_clean_under_asan_ubsan(built):
    r = _run(os.path.join(built, "host_sanitize"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "host sanitize driver: ok" in out, out[-2000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out


def test_h5_clean_under_asan_ubsan(built, tmp_path):
    exe = os.path.join(built, "h5_sanitize")
    if not os.path.exists(exe):
        pytest.skip("libhdf5 headers not present: no DASDAE writer to check")
    r = _run(exe, str(tmp_path))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "h5 sanitize driver: ok" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out
