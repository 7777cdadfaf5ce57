"""SURVEY §5.2 race/memory checking of the host runtime: build the host C++
(csrc/{cpu,io,tokenize}) with -fsanitize=address,undefined into a standalone
harness (csrc/tests/host_sanitize_main.cpp: BPE on arbitrary/invalid UTF-8,
packer, .tensors range reader, HTTP response parser fed malformed responses,
host AdamW tails) and require a clean run."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_runtime_clean_under_asan_ubsan():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_ext
    exe = build_ext.build_sanitize()
    syms = subprocess.run(["nm", exe], capture_output=True, text=True).stdout
    assert "__asan_report" in syms and "__ubsan_handle" in syms  # really instrumented
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "harness: OK" in r.stdout
