"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host code (the reference runs
valgrind memcheck ctests, CMakeLists.txt:316-329): the TAP suite, MRSW / MRMW stress, the CLI
regression script, and the hand-written Lua and WASM interpreters (including malformed WASM
modules) under `make asan` builds.  Any sanitizer report fails the test."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB = os.path.join(ROOT, "libsplinter_amd", "bin", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=77",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=78")


def _build():
    subprocess.run(["make", "-C", ROOT, "-j8", "asan"], check=True, capture_output=True)


def _run(args, timeout=300, ok_codes=(0,), stdin=None):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=ENV, input=stdin)
    bad = ("AddressSanitizer" in r.stderr or "runtime error:" in r.stderr or "LeakSanitizer" in r.stderr)
    assert not bad, r.stderr[-4000:]
    assert r.returncode in ok_codes, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return r


def test_asan_tap_suite():
    _build()
    r = _run([os.path.join(AB, "splinter_test")])
    assert "not ok" not in r.stdout and "ok " in r.stdout


def test_asan_stress(uniq):
    _build()
    _run([os.path.join(AB, "splinter_stress"), "--quiet", "--duration-ms", "800", "--threads", "4", "--keys", "300",
          "--slots", "1000", "--max-value", "256", "--store", uniq + "a"])
    _run([os.path.join(AB, "splinter_chi_sao"), "--quiet", "--duration-ms", "800", "--threads", "6", "--writers",
          "3", "--incr", "1", "--keys", "300", "--slots", "1000", "--max-value", "256", "--store", uniq + "b"])
    _run([os.path.join(AB, "splinter_hostapi_bench"), "--store", uniq + "c", "--threads", "4", "--seconds", "0.3",
          "--keys", "2000", "--append-check", "8"])


def test_asan_cli_regression():
    _build()
    r = subprocess.run(["bash", os.path.join(ROOT, "tests", "cli_regression.sh"), AB], capture_output=True, text=True,
                       timeout=600, env=ENV)
    assert "AddressSanitizer" not in r.stdout + r.stderr and "runtime error:" not in r.stdout + r.stderr, \
        (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0 and "not ok" not in r.stdout, r.stdout[-3000:]


def test_asan_lua_and_wasm_interpreters(uniq, tmp_path):
    _build()
    ctl = os.path.join(AB, "splinterctl")
    st = f"asan_{uniq}"
    _run([ctl, "init", st])
    try:
        _run([ctl, "-u", st, "set", "src", "copied-value"])
        _run([ctl, "-u", st, "lua", os.path.join(ROOT, "tests", "data", "bus_check.lua"), "x", "y"])
        _run([ctl, "-u", st, "wasm", os.path.join(ROOT, "tests", "data", "wasm_suite.wat"), "run"])
        _run([ctl, "-u", st, "wasm", os.path.join(ROOT, "tests", "data", "wasm_suite.wat"), "trap"], ok_codes=(1,))
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from test_cli import _wasm_single_func
        for name, ops in {"store1": b"\x41\x05\x36\x02\x00\x0b", "tee": b"\x22\x00\x1a\x0b",
                          "br": b"\x02\x7f\x0c\x00\x0b\x1a\x0b", "select": b"\x41\x01\x1b\x1a\x0b"}.items():
            p = tmp_path / f"{name}.wasm"
            p.write_bytes(_wasm_single_func(ops))
            _run([ctl, "-u", st, "wasm", str(p)], ok_codes=(1,))
        # Lua: string library, tables, closures and errors through the interpreter
        lua = tmp_path / "t.lua"
        lua.write_text('local s = require("splinter")\nlocal t = {}\nfor i = 1, 200 do t[i] = string.rep("x", i) end\n'
                       's.set("big", t[200])\nassert(#s.get("big") == 200)\n'
                       'local ok, err = pcall(function() error("boom") end)\nassert(not ok)\n')
        _run([ctl, "-u", st, "lua", str(lua)])
        # patterns, metatables and coroutines (one thread per coroutine; a suspended one is unwound
        # and joined at interpreter teardown)
        for script in ("lua_patterns_meta.lua", "lua_coroutines.lua", "lua_stdlib.lua", "lua_more.lua"):
            _run([ctl, "-u", st, "lua", os.path.join(ROOT, "tests", "data", script)])
    finally:
        subprocess.run([ctl, "-u", st, "unset", "src"], capture_output=True, env=ENV)
        subprocess.run(["rm", "-f", f"/dev/shm/{st}"])
