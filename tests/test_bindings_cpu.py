"""Binding surfaces stay in step with the C ABI (splinter.h): every prototype is
exported by libsplinter.so / libsplinter_p.so, declared by the Rust -sys crate,
and every symbol the TypeScript binding dlopens exists.  (No Rust toolchain,
Deno or Bun in the build image: the bindings are checked structurally here.)"""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "libsplinter_amd/csrc/include/splinter.h")


def _header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"^[A-Za-z_][\w \*]*?\b(splinter_\w+)\s*\(", txt, flags=re.M))
    names.discard("splinter_now")  # static inline wrapper of splinter_now_ticks
    return names


def _exports(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "libsplinter_amd/lib", lib)],
                         capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_header_has_the_reference_surface():
    names = _header_functions()
    assert len(names) == 60, sorted(names)


def test_every_prototype_is_exported():
    names = _header_functions()
    for lib in ("libsplinter.so", "libsplinter_p.so"):
        missing = names - _exports(lib)
        assert not missing, (lib, sorted(missing))


def test_rust_sys_crate_declares_every_function():
    src = open(os.path.join(ROOT, "bindings/rust/libsplinter-amd-sys/src/lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    declared = set(re.findall(r"pub fn (splinter_\w+)\s*\(", block))
    assert declared == _header_functions(), (sorted(_header_functions() - declared),
                                             sorted(declared - _header_functions()))


def test_typescript_symbols_exist():
    src = open(os.path.join(ROOT, "bindings/ts/splinter.ts")).read()
    syms = set(re.findall(r"^\s+(spl\w+|splinter_\w+):\s*\{\s*parameters", src, flags=re.M))
    assert syms, "no FFI symbol table found"
    missing = syms - _exports("libsplinter.so")
    assert not missing, sorted(missing)
