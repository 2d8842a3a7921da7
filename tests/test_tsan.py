"""ThreadSanitizer runs of the host store: the TAP suite (includes the
racing-inserter test that exposed the insert-protocol race fixed in round 1), MRSW
and MRMW stress with integer ops.  Any TSAN report fails the test."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TB = os.path.join(ROOT, "libsplinter_amd", "bin", "tsan")
ENV = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")


def _build():
    subprocess.run(["make", "-C", ROOT, "-j8", "tsan"], check=True, capture_output=True)


def _run(args, timeout=300):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=ENV)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return r


def test_tsan_tap_suite():
    _build()
    r = _run([os.path.join(TB, "splinter_test")])
    assert "not ok" not in r.stdout


def test_tsan_stress(uniq):
    _build()
    _run([os.path.join(TB, "splinter_stress"), "--quiet", "--duration-ms", "1000", "--threads", "4", "--keys", "300",
          "--slots", "1000", "--max-value", "256", "--store", uniq + "a"])
    _run([os.path.join(TB, "splinter_chi_sao"), "--quiet", "--duration-ms", "1000", "--threads", "6", "--writers",
          "3", "--incr", "1", "--keys", "300", "--slots", "1000", "--max-value", "256", "--store", uniq + "b"])
