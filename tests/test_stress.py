"""MRSW / MRMW stress benches (reference ctest configs, CMakeLists.txt:310-329), shortened."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "libsplinter_amd", "bin")


def run(tool, *args):
    exe = os.path.join(BIN, tool)
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", ROOT, "tools"], check=True, capture_output=True)
    r = subprocess.run([exe, "--quiet", *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("scrub", [[], ["--scrub"]])
def test_mrsw(uniq, scrub):
    res = run("splinter_stress", "--duration-ms", "1500", "--threads", "6", "--keys", "2000", "--slots", "5000",
              "--store", uniq, *scrub)
    assert res["integrity_failures"] == 0 and res["sets"] > 0 and res["gets"] > 0


def test_mrmw_lanes_with_incr(uniq):
    res = run("splinter_chi_sao", "--duration-ms", "1500", "--threads", "8", "--writers", "4", "--incr", "2",
              "--keys", "4000", "--slots", "10000", "--max-value", "512", "--store", uniq)
    assert res["integrity_failures"] == 0 and res["incr_exact"] and res["incrs"] > 0


def test_file_backend(tmp_path):
    res = run("splinter_stress", "--duration-ms", "800", "--threads", "4", "--keys", "500", "--slots", "2000",
              "--max-value", "256", "--store", str(tmp_path / "stress.spl"))
    assert res["integrity_failures"] == 0
