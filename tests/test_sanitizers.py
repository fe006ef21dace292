"""Host-code sanitizers: the Direct-Access reader, pglz and
the Criteo featuriser built with ASan+UBSan and fuzzed with corrupted pages /
streams / lines, and with TSan over their thread pools (csrc/da/da_fuzz.cpp).
CPU only; skipped when the toolchain has no sanitizer runtimes."""

import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "da", f) for f in ("da_fuzz.cpp", "pages.cpp", "pglz.cpp",
                                                       "criteo.cpp")]
CXX = shutil.which("g++")


def _build(tmp, name, flags):
    exe = os.path.join(tmp, name)
    cmd = [CXX, "-O1", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "csrc", "da")] + flags + \
        SRC + ["-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-400:])
    return exe


def _run(exe, tmp, iters, seed, env=None):
    d = tempfile.mkdtemp(dir=tmp)
    r = subprocess.run([exe, d, str(iters), str(seed)], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok:"), r.stdout
    return r.stdout


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_da_reader_fuzz_asan_ubsan(tmp_path):
    exe = _build(str(tmp_path), "da_fuzz_asan",
                 ["-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                  "-fno-omit-frame-pointer"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    for seed in (1, 2, 3):
        out = _run(exe, str(tmp_path), 1500, seed, env)
        assert "rejected cleanly" in out


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_da_reader_threads_tsan(tmp_path):
    exe = _build(str(tmp_path), "da_fuzz_tsan", ["-fsanitize=thread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    _run(exe, str(tmp_path), 100, 7, env)
