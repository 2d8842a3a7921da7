"""Binding surfaces stay in step with the C ABI (splinter.h): every prototype is
exported by libsplinter.so / libsplinter_p.so, declared by the Rust -sys crate,
and every symbol the TypeScript binding dlopens exists.  (No Rust toolchain,
Deno or Bun in the build image: the bindings are checked at the ABI level here instead -- the Rust
extern block rewritten as C prototypes and compiled against splinter.h, the repr(C) struct layouts
computed from the Rust field lists against the C compiler's sizeof/offsetof, and the TypeScript FFI
table's arity and parameter widths against the C prototypes.)"""
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


# ---- ABI-level checks: the Rust declarations, compiled as C against splinter.h --------------------
_RS_SCALAR = {"u8": ("uint8_t", 1), "i8": ("int8_t", 1), "u16": ("uint16_t", 2), "i16": ("int16_t", 2),
              "u32": ("uint32_t", 4), "i32": ("int32_t", 4), "u64": ("uint64_t", 8), "i64": ("int64_t", 8),
              "usize": ("size_t", 8), "f32": ("float", 4), "f64": ("double", 8), "c_int": ("int", 4),
              "c_uint": ("unsigned int", 4), "c_ushort": ("unsigned short", 2), "c_char": ("char", 1),
              "c_void": ("void", 0), "splinter_integer_op_t": ("splinter_integer_op_t", 4),
              "splinter_enum_cb": ("splinter_enum_cb_t", 8)}


def _rs_type_to_c(t):
    """Rust FFI type -> C type (pointers keep their const-ness level by level)."""
    t = t.strip()
    if t.startswith("*const ") or t.startswith("*mut "):
        const = t.startswith("*const ")
        inner = _rs_type_to_c(t.split(" ", 1)[1])
        return f"{'const ' if const else ''}{inner}*" if "*" not in inner else \
            (f"{inner} const*" if const else f"{inner}*")
    if t in _RS_SCALAR:
        return _RS_SCALAR[t][0]
    if t in ("splinter_header", "splinter_slot", "splinter_shard_bid_snapshot"):
        return "struct " + t  # tagged structs of splinter.h (no typedef)
    return t  # a typedef of splinter.h


def _rs_functions():
    src = open(os.path.join(ROOT, "bindings/rust/libsplinter-amd-sys/src/lib.rs")).read()
    block = src[src.index('extern "C" {'):]
    block = block[: block.index("\n}\n")]
    block = re.sub(r"//[^\n]*", "", block)
    out = []
    for m in re.finditer(r"pub fn (splinter_\w+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", block, flags=re.S):
        name, params, ret = m.group(1), m.group(2), m.group(4)
        ps = [p.split(":", 1)[1] for p in re.split(r",\s*(?![^()]*\))", " ".join(params.split())) if p.strip()]
        out.append((name, [_rs_type_to_c(p) for p in ps], _rs_type_to_c(ret) if ret else "void"))
    return out


def test_rust_signatures_compile_against_the_c_header(tmp_path):
    """Every Rust extern declaration, rewritten as a C prototype, is redeclared after splinter.h:
    any parameter/return type that disagrees with the header (width, signedness, pointer const-ness)
    is a 'conflicting types' compile error."""
    fns = _rs_functions()
    assert len(fns) == len(_header_functions())
    lines = ['#include "splinter.h"', "typedef void (*splinter_enum_cb_t)(const char*, uint64_t, void*);"]
    for name, ps, ret in fns:
        lines.append(f"{ret} {name}({', '.join(ps) if ps else 'void'});")
    src = tmp_path / "rs_abi.c"
    src.write_text("\n".join(lines) + "\n")
    r = subprocess.run(["gcc", "-std=gnu11", "-fsyntax-only", "-Werror", "-I",
                        os.path.dirname(HDR), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def _rs_structs():
    src = open(os.path.join(ROOT, "bindings/rust/libsplinter-amd-sys/src/lib.rs")).read()
    consts = {m.group(1): m.group(2) for m in re.finditer(r"pub const (\w+): \w+ = ([^;]+);", src)}
    out = {}
    for m in re.finditer(r"#\[repr\(C(?:, align\((\d+)\))?\)\]\s*(?:#\[[^\]]*\]\s*)*pub struct (\w+)\s*\{(.*?)\n\}",
                         src, flags=re.S):
        fields = re.findall(r"pub (\w+): ([^,\n]+),", m.group(3))
        out[m.group(2)] = (int(m.group(1) or 0), fields)
    return out, consts


def test_rust_struct_layouts_match_c(tmp_path):
    """repr(C) layout of every Rust struct the ABI passes (computed here from the field list) equals
    sizeof/offsetof of the C struct of the same name, compiled and run on this host."""
    structs, consts = _rs_structs()

    def ev(expr):
        e = expr
        for _ in range(8):  # constants defined in terms of other constants
            for k, v in consts.items():
                e = re.sub(rf"\b{k}\b", f"({v})", e)
        e = re.sub(r"([0-9A-Fa-f])_(?=[0-9A-Fa-f])", r"\1", e)  # 0x534C_4E54
        return int(eval(e))  # integer constant expressions (a // b, 1 << n)

    def layout(t):
        t = t.strip()
        m = re.fullmatch(r"\[(.+);\s*(.+)\]", t)
        if m:
            sz, al = layout(m.group(1))
            return sz * ev(m.group(2).replace("/", "//")), al
        m = re.fullmatch(r"Aligned64<(.+)>", t)
        if m:
            sz, al = layout(m.group(1))
            al = max(al, 64)
            return (sz + al - 1) // al * al, al
        if t in _RS_SCALAR:
            return _RS_SCALAR[t][1], _RS_SCALAR[t][1]
        if t in structs:
            return struct_layout(t)[0:2]
        raise AssertionError(f"unknown Rust type {t}")

    def struct_layout(name):
        align, fields = structs[name]
        off, al, offs = 0, max(align, 1), {}
        for f, t in fields:
            sz, a = layout(t)
            off = (off + a - 1) // a * a
            offs[f] = off
            off += sz
            al = max(al, a)
        return (off + al - 1) // al * al, al, offs

    abi = ["splinter_header", "splinter_slot", "splinter_header_snapshot_t", "splinter_slot_snapshot_t",
           "splinter_shard_bid_snapshot"]
    prog = ['#include <stdio.h>', '#include <stddef.h>', '#include "splinter.h"', "int main(void) {"]
    want = []
    for s in abi:
        size, _, offs = struct_layout(s)
        ctype = s if s.endswith("_t") else "struct " + s
        prog.append(f'printf("%zu\\n", sizeof({ctype}));')
        want.append(size)
        for f, o in offs.items():
            if f.startswith("_pad"):
                continue
            prog.append(f'printf("%zu\\n", offsetof({ctype}, {f}));')
            want.append(o)
    prog.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(prog) + "\n")
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=gnu11", "-I", os.path.dirname(HDR), str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == want


_TS_SIZE = {"pointer": 8, "buffer": 8, "usize": 8, "isize": 8, "u64": 8, "i64": 8, "u32": 4, "i32": 4, "u16": 2,
            "i16": 2, "u8": 1, "i8": 1, "f32": 4, "f64": 8, "function": 8}


def test_typescript_ffi_arity_and_widths(tmp_path):
    """Every TypeScript FFI entry declares as many parameters as the C prototype, each of the C
    parameter's width (sizeof of the prototype's parameter types, taken from the compiler)."""
    src = open(os.path.join(ROOT, "bindings/ts/splinter.ts")).read()
    entries = re.findall(r"^\s+(splinter_\w+):\s*\{\s*parameters:\s*\[([^\]]*)\]", src, flags=re.M)
    assert entries
    rs = {n: ps for n, ps, _ in _rs_functions()}
    prog = ['#include <stdio.h>', '#include "splinter.h"',
            "typedef void (*splinter_enum_cb_t)(const char*, uint64_t, void*);", "int main(void) {"]
    want = []
    for name, params in entries:
        ts = [p.strip().strip('"') for p in params.split(",") if p.strip()]
        assert name in rs, name
        assert len(ts) == len(rs[name]), (name, ts, rs[name])
        for t, c in zip(ts, rs[name]):
            assert t in _TS_SIZE, (name, t)
            prog.append(f'printf("%zu\\n", sizeof({c}));')
            want.append(_TS_SIZE[t])
    prog.append("return 0; }")
    csrc = tmp_path / "ts.c"
    csrc.write_text("\n".join(prog) + "\n")
    exe = tmp_path / "ts"
    r = subprocess.run(["gcc", "-std=gnu11", "-I", os.path.dirname(HDR), str(csrc), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == want
