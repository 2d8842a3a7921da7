"""splinterctl one-shot + REPL regression (reference CLI verbs, splinter_cli_cmd_*.c)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "libsplinter_amd", "bin")


def ctl(store, *args, stdin=None, name="splinterctl"):
    r = subprocess.run([os.path.join(BIN, name), "-u", store, *args], capture_output=True, text=True,
                       input=stdin, timeout=60)
    return r.returncode, r.stdout, r.stderr


@pytest.fixture
def store(uniq):
    if not os.path.exists(os.path.join(BIN, "splinterctl")):
        subprocess.run(["make", "-C", ROOT, "tools"], check=True, capture_output=True)
    rc, out, _ = ctl(uniq, "init", "--slots", "128", "--length", "512", uniq)
    assert rc == 0 and "Initializing store" in out
    yield uniq
    from libsplinter_amd import unlink
    unlink(uniq)


def test_kv_verbs(store):
    assert ctl(store, "set", "foo", "bar")[0] == 0
    assert ctl(store, "get", "foo")[1].startswith("bar\n")
    assert ctl(store, "getfoo_prefix_match_is_get", "foo")[1].startswith("bar\n")  # reference prefix dispatch
    assert ctl(store, "append", "foo", "baz")[0] == 0
    assert ctl(store, "get", "foo")[1].startswith("barbaz")
    head = ctl(store, "head", "foo")[1]
    assert "epoch:" in head and "key:        foo" in head and "DIM=768" in head
    assert ctl(store, "unset", "foo")[1].strip() == "6 bytes deleted."
    assert ctl(store, "get", "foo")[0] != 0


def test_types_math_labels(store):
    ctl(store, "set", "n", "10")
    assert ctl(store, "type", "n", "biguint")[0] == 0
    assert ctl(store, "type", "n")[1].startswith("SPL_SLOT_TYPE_BIGUINT:n")
    assert "successfully" in ctl(store, "math", "n", "inc", "5")[1]
    assert ctl(store, "get", "n")[1].split()[0] == "15"
    ctl(store, "math", "n", "and", "0x7")
    assert ctl(store, "get", "n")[1].split()[0] == "7"
    assert "applied to 'n'" in ctl(store, "label", "n", "0x40")[1]
    assert "0b1000000" in ctl(store, "head", "n")[1]
    assert "removed from" in ctl(store, "label", "n", "-0x40")[1]
    assert "Signal Group 3" in ctl(store, "bind", "0x40", "3")[1]


def test_list_export_orders_ingest(store, tmp_path):
    for k in ("alpha", "beta", "gamma"):
        ctl(store, "set", k, k.upper())
    out = ctl(store, "list", "^(alpha|beta)$")[1]
    assert "alpha" in out and "beta" in out and "gamma" not in out
    ex = json.loads(ctl(store, "export")[1])
    assert ex["store"]["active_keys"] == 3 and {k["key"] for k in ex["keys"]} == {"alpha", "beta", "gamma"}
    assert "OK" in ctl(store, "orders", "set", "t", "3")[1]
    assert ctl(store, "get", "t.2")[0] == 0
    assert ctl(store, "unset", "-r", "t")[0] == 0
    assert ctl(store, "get", "t.1")[0] != 0
    f = tmp_path / "doc.txt"
    f.write_text("x" * 1000)
    out = ctl(store, "ingest", str(f), "--key", "doc")[1]
    assert "3 chunk(s), 1000 bytes" in out  # chunk = max_val - 64 = 448
    meta = json.loads(ctl(store, "get", "doc")[1].splitlines()[0])
    assert meta["chunks"] == 3 and meta["bytes"] == 1000
    assert ctl(store, "type", "doc.2")[1].startswith("SPL_SLOT_TYPE_VARTEXT")


def test_config_caps_shard_uuid(store):
    cfg = ctl(store, "config")[1]
    assert "version:     4" in cfg and "slots:       128" in cfg
    # mode 2 does not clear HYBRID (reference splinter.c:276-299 quirk, kept): go through 0 first
    assert ctl(store, "config", "av", "0")[0] == 0 and "mop:         0" in ctl(store, "config")[1]
    assert ctl(store, "config", "av", "2")[0] == 0 and "mop:         2" in ctl(store, "config")[1]
    assert "lua=yes" in ctl(store, "caps")[1]
    assert "OK" in ctl(store, "shard", "claim", "0x77", "random", "5", "100000000000")[1]
    assert "0x77" in ctl(store, "shard", "table")[1]
    assert ctl(store, "shard", "who")[1].startswith("sovereign=0x77")
    assert ctl(store, "shard", "release", "0x77")[0] == 0
    u = ctl(store, "uuid")[1].strip()
    assert len(u) == 36 and u[14] == "4"


def test_search_regex_without_sidecar(store):
    ctl(store, "set", "findme", "v")
    rc, out, err = ctl(store, "search", "--regex", "find", "--timeout", "50", "--json", "q")
    assert rc == 0 and "timed out" in err
    res = json.loads(out)
    assert [r["key"] for r in res["results"]] == ["findme"] and res["results"][0]["similarity"] is None


def test_repl_and_namespace(store):
    script = f"use {store}\nset a 1\nget a\nhist\nquit\n"
    rc, out, _ = ctl(store, stdin=script, name="splinter_cli")
    assert rc == 0 and "1\n" in out and "set a 1" in out
    r = subprocess.run([os.path.join(BIN, "splinterctl"), "-u", store, "--prefix", "ns_", "set", "k", "v"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and ctl(store, "get", "ns_k")[1].startswith("v")


def test_sidecar_once_shows_debug_labelled_keys(store, tmp_path):
    ctl(store, "set", "dbgkey", "debug chatter")
    ctl(store, "label", "dbgkey", "0x0800000000000000")  # reference sidecar debug bloom (bit 59)
    r = subprocess.run([os.path.join(BIN, "sidecar"), f"spl:{store}", "--once"], capture_output=True, text=True,
                       timeout=30)
    assert r.returncode == 0, r.stderr
    assert "debug chatter" in r.stdout and "History (CPU" in r.stdout
    log = tmp_path / "app.log"
    log.write_text("line one\nline two\n")
    r = subprocess.run([os.path.join(BIN, "sidecar"), str(log), "--once"], capture_output=True, text=True, timeout=30)
    assert "line two" in r.stdout


def test_export_import_roundtrip(store, uniq, tmp_path):
    ctl(store, "set", "doc", "line one\nline \"two\"")
    ctl(store, "type", "doc", "vartext")
    dump = tmp_path / "dump.json"
    dump.write_text(ctl(store, "export")[1])
    other = uniq + "_imp"
    assert ctl(other, "init", "--slots", "64", "--length", "512", other)[0] == 0
    try:
        rc, out, err = ctl(other, "import", str(dump))
        assert rc == 0 and "imported 1 key(s)" in out, err
        assert ctl(other, "get", "doc")[1].startswith('line one\nline "two"')
        assert ctl(other, "type", "doc")[1].startswith("SPL_SLOT_TYPE_VARTEXT")
    finally:
        from libsplinter_amd import unlink
        unlink(other)


def test_lua_verb_splinter_module(store):
    ctl(store, "set", "test_key", "test_value")
    rc, out, err = ctl(store, "lua", os.path.join(ROOT, "tests", "data", "bus_check.lua"), "x", "y")
    assert rc == 0, err
    assert "args=2" in out and "test_key=test_value" in out and "ok 42" in out
    assert ctl(store, "get", "lua_t.2")[1].startswith("c")
    rc, _, err = ctl(store, "lua", os.devnull + "_missing.lua")
    assert rc != 0


@pytest.mark.parametrize("script", ["lua_patterns_meta.lua", "lua_coroutines.lua", "lua_stdlib.lua", "lua_more.lua"])
def test_lua_patterns_metatables_coroutines(store, script):
    """Lua 5.4 semantics the reference gets from liblua5.4: string patterns (find / match / gmatch /
    gsub), metatables and metamethods, coroutines, string.pack, load's env / _ENV, to-be-closed
    variables, __gc finalizers, the debug library -- each script asserts its expected values."""
    rc, out, err = ctl(store, "lua", os.path.join(ROOT, "tests", "data", script))
    assert rc == 0 and "ALL OK" in out, out + err
    if script == "lua_more.lua":  # the finalizers still pending run when the state closes
        assert out.index("FINALIZED AT CLOSE") > out.index("ALL OK"), out


def _pty_repl(store, keys, timeout=20.0):
    """Run the REPL on a pseudo-terminal, type `keys` (bytes, in chunks with small pauses so
    escape sequences arrive whole) and return everything it printed."""
    import pty
    import select
    import time
    pid, fd = pty.fork()
    if pid == 0:  # child: the REPL (any argv[0] other than splinterctl starts it)
        os.environ["TERM"] = "xterm"
        os.execv(os.path.join(BIN, "splinterctl"), ["splinter_cli", "-u", store])
    out = b""
    deadline = time.time() + timeout

    def drain(t=0.15):
        nonlocal out
        end = time.time() + t
        while time.time() < end:
            r, _, _ = select.select([fd], [], [], 0.05)
            if r:
                try:
                    out += os.read(fd, 65536)
                except OSError:
                    return
    drain(0.5)
    for chunk in keys:
        os.write(fd, chunk)
        drain()
    while time.time() < deadline:
        done, _ = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        drain(0.1)
    else:
        os.kill(pid, 9)
        os.waitpid(pid, 0)
    drain(0.2)
    os.close(fd)
    return out.decode(errors="replace")


def test_repl_line_editing_history_completion(store):
    """The REPL edits lines on a terminal (reference: linenoise, splinter_cli_main.c:832-872):
    backspace, Ctrl-A / Ctrl-K / Ctrl-U / Ctrl-W, arrow keys, history recall with Up, Tab completion
    of the command word, Ctrl-D to quit."""
    keys = [b"sett", b"\x7f", b" k1 hello\r",            # backspace fixes the verb
            b"get k1\r",
            b"\x1b[A", b"\x1b[A", b"\x15", b"ge", b"\t", b" k1\r",  # Up x2, Ctrl-U, "ge"+Tab -> "get"
            b"set k2 wrld", b"\x1b[D\x1b[D\x1b[D", b"o", b"\r",   # left arrows, insert 'o' -> "world"
            b"get k2\r",
            b"xyz get k1", b"\x01", b"\x0b", b"unset k2\r",   # Ctrl-A, Ctrl-K kills the line, retype
            b"get k2 junk words", b"\x17\x17", b"\r",          # Ctrl-W twice -> "get k2"
            b"\x04"]                                            # Ctrl-D on an empty line: exit
    out = _pty_repl(store, keys)
    assert "hello" in out, out[-2000:]
    assert out.count("hello") >= 2, out[-2000:]          # "get k1" twice (typed, then recalled/completed)
    assert "world" in out, out[-2000:]
    assert ctl(store, "get", "k1")[1].startswith("hello")
    assert ctl(store, "get", "k2")[0] != 0                # unset ran after Ctrl-A/Ctrl-K


def test_cli_regression_script():
    r = subprocess.run(["bash", os.path.join(ROOT, "tests", "cli_regression.sh"), BIN], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "not ok" not in r.stdout, r.stdout[-3000:]


def _wasm_binary_start_module() -> bytes:
    """Hand-assembled binary twin of the reference's test.wasm (WAT text):
    imports splinter.set, exports memory, _start() sets __debug = 'Hello from WASM!'."""
    def uleb(n):
        out = bytearray()
        while True:
            b = n & 0x7F
            n >>= 7
            out.append(b | (0x80 if n else 0))
            if not n:
                return bytes(out)

    def sec(i, body):
        return bytes([i]) + uleb(len(body)) + body

    def name(s):
        return uleb(len(s)) + s.encode()

    types = uleb(2) + b"\x60\x04\x7f\x7f\x7f\x7f\x01\x7f" + b"\x60\x00\x01\x7f"
    imports = uleb(1) + name("splinter") + name("set") + b"\x00" + uleb(0)
    funcs = uleb(1) + uleb(1)
    memory = uleb(1) + b"\x00" + uleb(1)
    exports = uleb(2) + name("memory") + b"\x02" + uleb(0) + name("_start") + b"\x00" + uleb(1)
    body = b"\x00" + b"\x41\x00\x41\x08\x41\x10\x41\x10\x10\x00\x0b"  # no locals; i32.const x4; call 0; end
    code = uleb(1) + uleb(len(body)) + body
    data = uleb(2) + b"\x00\x41\x00\x0b" + name("__debug") + b"\x00\x41\x10\x0b" + name("Hello from WASM!")
    return (b"\x00asm\x01\x00\x00\x00" + sec(1, types) + sec(2, imports) + sec(3, funcs) + sec(5, memory) +
            sec(7, exports) + sec(10, code) + sec(11, data))


def test_wasm_verb_reference_module_text_and_binary(store, tmp_path):
    """The reference's own test.wasm (WAT text) and its binary twin through the built-in interpreter
    (reference splinter_cli_cmd_wasm.c:85-143 on WasmEdge)."""
    ref = "/root/reference/test.wasm"
    if os.path.exists(ref):
        rc, _, err = ctl(store, "wasm", ref)
        assert rc == 0, err
        assert ctl(store, "get", "__debug")[1].startswith("Hello from WASM!")
        ctl(store, "unset", "__debug")
    p = tmp_path / "start.wasm"
    p.write_bytes(_wasm_binary_start_module())
    rc, _, err = ctl(store, "wasm", str(p))
    assert rc == 0, err
    assert ctl(store, "get", "__debug")[1].startswith("Hello from WASM!")
    assert "wasm=yes" in ctl(store, "caps")[1]


def test_wasm_suite_semantics(store):
    """Control flow, recursion, br_table, i64/f32/f64 ops, call_indirect, globals, memory.grow,
    host get/set, and a trap: results checked against Python."""
    import math
    import struct
    from libsplinter_amd import Store
    ctl(store, "set", "src", "copied-value")
    rc, _, err = ctl(store, "wasm", os.path.join(ROOT, "tests", "data", "wasm_suite.wat"), "run")
    assert rc == 0, err
    s = Store.open(store)
    try:
        g = s.get
        assert struct.unpack("<q", g("fact"))[0] == math.factorial(20)
        assert struct.unpack("<i", g("fib"))[0] == 832040
        assert struct.unpack("<i", g("tbl"))[0] == 100 + 200 * 1000 + 300 * 1000000
        exp = (-9 >> 1) - (1 << 63) + (2 ** 64 - 1) // 3
        assert struct.unpack("<q", g("i64"))[0] == (exp + 2 ** 63) % 2 ** 64 - 2 ** 63
        assert struct.unpack("<i", g("flt"))[0] == int(math.sqrt(2) * 1e6) + 2  # nearest(2.5) == 2
        assert struct.unpack("<i", g("ind"))[0] == 13 * 42
        assert struct.unpack("<i", g("cnt"))[0] == 5 * 100 + 3 - 1
        assert g("echo") == b"copied-value"
    finally:
        s.close()
    rc, _, err = ctl(store, "wasm", os.path.join(ROOT, "tests", "data", "wasm_suite.wat"), "trap")
    assert rc == 1 and "integer divide by zero" in err


def _wasm_single_func(body_ops: bytes, results: bytes = b"\x00") -> bytes:
    """A binary module exporting _start() with the given body (no locals) and 1 page of memory."""
    def uleb(n):
        out = bytearray()
        while True:
            b = n & 0x7F
            n >>= 7
            out.append(b | (0x80 if n else 0))
            if not n:
                return bytes(out)

    def sec(i, body):
        return bytes([i]) + uleb(len(body)) + body

    types = uleb(1) + b"\x60\x00" + results
    funcs = uleb(1) + uleb(0)
    memory = uleb(1) + b"\x00" + uleb(1)
    exports = uleb(1) + uleb(6) + b"_start" + b"\x00" + uleb(0)
    body = b"\x01\x01\x7f" + body_ops  # one i32 local
    code = uleb(1) + uleb(len(body)) + body
    return b"\x00asm\x01\x00\x00\x00" + sec(1, types) + sec(3, funcs) + sec(5, memory) + sec(7, exports) + sec(10, code)


def test_wasm_malformed_modules_fail_cleanly(store, tmp_path):
    """Unvalidated malformed modules must raise an interpreter error (exit 1), never touch memory
    outside the operand stack: a store with one operand, a local.tee on an empty stack, a branch
    whose label expects more values than the stack holds, a function missing its result."""
    cases = {
        "store1": b"\x41\x05\x36\x02\x00\x0b",         # i32.const 5; i32.store -- one operand
        "tee": b"\x22\x00\x1a\x0b",                     # local.tee 0 on an empty stack; drop
        "br": b"\x02\x7f\x0c\x00\x0b\x1a\x0b",         # block (result i32) br 0 (nothing) end drop
        "select": b"\x41\x01\x1b\x1a\x0b",              # i32.const 1; select -- needs three
    }
    for name, ops in cases.items():
        p = tmp_path / f"{name}.wasm"
        p.write_bytes(_wasm_single_func(ops))
        rc, _, err = ctl(store, "wasm", str(p))
        assert rc == 1 and "underflow" in err.lower(), (name, rc, err)
    p = tmp_path / "noresult.wasm"
    p.write_bytes(_wasm_single_func(b"\x0b", results=b"\x01\x7f"))
    rc, _, err = ctl(store, "wasm", str(p))
    assert rc == 1, (rc, err)
