"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
section 5: host-code sanitizers are the only ones this pool runs; GPU ASan and
XNACK are unavailable).  oracle/sanitize_driver.c drives every oracle entry
point the tests use -- empty and one-particle systems, crowded boxes,
several species, walls, non-periodic boxes, 2-D and 3-D, cell-list vs
all-pairs runs -- and any memory error, leak or undefined behaviour aborts
it (-fno-sanitize-recover=all)."""

import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(ROOT / "oracle" / "_build" / "sanitize_driver")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize: ok" in r.stdout
    assert "runtime error" not in r.stderr
