"""Sanitizer runs on host code (run the CPU path under -fsanitize=address,undefined).

* The oracle (the parity checker): oracle/sanitize_main.c drives every entry point of
  oracle/fmskf_oracle.c on random and adversarial inputs (garbage WT901 streams, CAN extremes,
  NaN / huge KF inputs, validity masks, control events, empty ensemble ranges).
* The library's host code (csrc/api_*.cpp built with -Xarch_host sanitizers):
  tests/native/api_sanitize.cpp exercises the entry points that need no GPU and fmskf_create's
  clean failure without a device.
Any sanitizer report aborts the program (halt / abort on error)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def test_oracle_clean_under_asan_ubsan():
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", odir, "sanitize"], check=True)
    out = subprocess.run([os.path.join(odir, "_san", "orc_san")], capture_output=True, text=True,
                         timeout=300, env=ENV)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "sanitize ok" in out.stdout


def test_host_api_clean_under_asan_ubsan():
    import torch
    if torch.cuda.is_available():
        pytest.skip("checks fmskf_create's no-device failure path: CPU-only host")
    pkg = os.path.join(ROOT, "roboken-fmskf-robot-controller_amd")
    subprocess.run(["make", "-s", "-C", pkg, "sanitize"], check=True, stdout=subprocess.DEVNULL)
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0")
    out = subprocess.run([os.path.join(pkg, "build", "san", "api_sanitize")], capture_output=True,
                         text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "api sanitize ok" in out.stdout
