"""GGUF v2/v3 reader and writer (no external deps; numpy memmap, zero copy).

The reference daemon loads its Nomic model through llama.cpp
(/root/reference/splinference.cpp:423-446).  Here the file is parsed directly:
metadata + tensor table in Python, tensor bytes memory-mapped, and quantised
blocks expanded to bf16 on the GPU by ``nomic_dequant`` (HIP).  The writer
exists so tests and benchmarks can produce real GGUF files (random-init
nomic-bert weights, F16/Q8_0/Q4_0 payloads) without network access.
"""
from __future__ import annotations

import io
import struct
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

GGUF_MAGIC = b"GGUF"

# ggml tensor types: (id, block elements, block bytes)
GGML_TYPES = {
    "F32": (0, 1, 4), "F16": (1, 1, 2), "Q4_0": (2, 32, 18), "Q4_1": (3, 32, 20),
    "Q5_0": (6, 32, 22), "Q5_1": (7, 32, 24), "Q8_0": (8, 32, 34), "Q8_1": (9, 32, 36),
    "Q2_K": (10, 256, 84), "Q3_K": (11, 256, 110), "Q4_K": (12, 256, 144), "Q5_K": (13, 256, 176),
    "Q6_K": (14, 256, 210), "Q8_K": (15, 256, 292), "BF16": (30, 1, 2),
}
TYPE_BY_ID = {v[0]: (k, v[1], v[2]) for k, v in GGML_TYPES.items()}
DEVICE_DEQUANT = {0, 1, 2, 3, 8, 12, 14, 30}  # implemented by nomic_dequant

# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f",
           _BOOL: "<?", _U64: "<Q", _I64: "<q", _F64: "<d"}


@dataclass
class TensorInfo:
    name: str
    shape: Tuple[int, ...]      # numpy order (slowest first) = reversed ggml ne
    ggml_type: int
    offset: int                 # absolute file offset of the data
    nbytes: int

    @property
    def type_name(self) -> str:
        return TYPE_BY_ID[self.ggml_type][0]

    @property
    def nelems(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n


class GGUFFile:
    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        self.kv: Dict[str, Any] = {}
        self.tensors: Dict[str, TensorInfo] = {}
        self._parse()

    # ---------------------------------------------------------------- parse --
    def _parse(self):
        buf = self.mm
        pos = 0

        def take(n):
            nonlocal pos
            b = bytes(buf[pos: pos + n])
            pos += n
            return b

        def scalar(t):
            fmt = _SCALAR[t]
            return struct.unpack(fmt, take(struct.calcsize(fmt)))[0]

        def string():
            (n,) = struct.unpack("<Q", take(8))
            return take(n).decode("utf-8", "replace")

        def value(t):
            if t == _STR:
                return string()
            if t == _ARR:
                (et,) = struct.unpack("<I", take(4))
                (n,) = struct.unpack("<Q", take(8))
                if et == _STR:
                    return [string() for _ in range(n)]
                if et in _SCALAR:
                    fmt = _SCALAR[et]
                    sz = struct.calcsize(fmt)
                    arr = np.frombuffer(take(sz * n), dtype=np.dtype(fmt))
                    return arr.tolist()
                return [value(et) for _ in range(n)]
            return scalar(t)

        if take(4) != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file")
        (self.version,) = struct.unpack("<I", take(4))
        if self.version not in (2, 3):
            raise ValueError(f"unsupported GGUF version {self.version}")
        n_tensors, n_kv = struct.unpack("<QQ", take(16))
        for _ in range(n_kv):
            k = string()
            (t,) = struct.unpack("<I", take(4))
            self.kv[k] = value(t)
        infos = []
        for _ in range(n_tensors):
            name = string()
            (nd,) = struct.unpack("<I", take(4))
            ne = struct.unpack(f"<{nd}Q", take(8 * nd))
            (tt,) = struct.unpack("<I", take(4))
            (off,) = struct.unpack("<Q", take(8))
            infos.append((name, ne, tt, off))
        align = int(self.kv.get("general.alignment", 32))
        data0 = (pos + align - 1) // align * align
        for name, ne, tt, off in infos:
            if tt not in TYPE_BY_ID:
                raise ValueError(f"tensor {name}: unsupported ggml type {tt}")
            _, be, bb = TYPE_BY_ID[tt]
            n = 1
            for d in ne:
                n *= d
            self.tensors[name] = TensorInfo(name, tuple(reversed(ne)), tt, data0 + off, n // be * bb)

    # -------------------------------------------------------------- access --
    def raw(self, name: str) -> np.ndarray:
        t = self.tensors[name]
        return self.mm[t.offset: t.offset + t.nbytes]

    def get(self, key: str, default=None):
        return self.kv.get(key, default)

    def arch(self) -> str:
        return self.kv.get("general.architecture", "")

    def to_numpy_f32(self, name: str) -> np.ndarray:
        """Host dequantisation (F32/F16/BF16/Q8_0/Q4_0) — reference path for tests."""
        t = self.tensors[name]
        raw = self.raw(name)
        return dequant_host(raw, t.ggml_type, t.nelems).reshape(t.shape)


# ------------------------------------------------------------ host codecs --
def dequant_host(raw: np.ndarray, ggml_type: int, n: int) -> np.ndarray:
    raw = np.asarray(raw, dtype=np.uint8)
    if ggml_type == 0:
        return raw.view(np.float32)[:n].copy()
    if ggml_type == 1:
        return raw.view(np.float16)[:n].astype(np.float32)
    if ggml_type == 30:
        return (raw.view(np.uint16)[:n].astype(np.uint32) << 16).view(np.float32)
    if ggml_type == 8:
        b = raw.reshape(-1, 34)
        d = b[:, :2].copy().view(np.float16).astype(np.float32)
        q = b[:, 2:].view(np.int8).astype(np.float32)
        return (q * d).reshape(-1)[:n]
    if ggml_type == 2:
        b = raw.reshape(-1, 18)
        d = b[:, :2].copy().view(np.float16).astype(np.float32)
        qs = b[:, 2:]
        lo = (qs & 15).astype(np.float32) - 8
        hi = (qs >> 4).astype(np.float32) - 8
        return (np.concatenate([lo, hi], axis=1) * d).reshape(-1)[:n]
    if ggml_type == 3:
        b = raw.reshape(-1, 20)
        d = b[:, :2].copy().view(np.float16).astype(np.float32)
        m = b[:, 2:4].copy().view(np.float16).astype(np.float32)
        qs = b[:, 4:]
        q = np.concatenate([(qs & 15), (qs >> 4)], axis=1).astype(np.float32)
        return (q * d + m).reshape(-1)[:n]
    if ggml_type == 12:
        return _dequant_q4k(raw, n)
    if ggml_type == 14:
        return _dequant_q6k(raw, n)
    raise NotImplementedError(f"host dequant of ggml type {ggml_type}")


def _dequant_q4k(raw, n):
    b = raw.reshape(-1, 144)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
    sc = b[:, 4:16].astype(np.int32)
    qs = b[:, 16:]
    out = np.empty((b.shape[0], 256), np.float32)
    for j in range(8):
        if j < 4:
            s, m = sc[:, j] & 63, sc[:, j + 4] & 63
        else:
            s = (sc[:, j + 4] & 15) | ((sc[:, j - 4] >> 6) << 4)
            m = (sc[:, j + 4] >> 4) | ((sc[:, j] >> 6) << 4)
        q = qs[:, (j >> 1) * 32: (j >> 1) * 32 + 32]
        q = (q >> 4) if j & 1 else (q & 15)
        out[:, j * 32:(j + 1) * 32] = (d * s)[:, None] * q - (dmin * m)[:, None]
    return out.reshape(-1)[:n]


def _dequant_q6k(raw, n):
    b = raw.reshape(-1, 210)
    ql, qh = b[:, :128].astype(np.int32), b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = b[:, 208:210].copy().view(np.float16).astype(np.float32)[:, 0]
    out = np.empty((b.shape[0], 256), np.float32)
    for half in range(2):
        L, H, S = ql[:, 64 * half: 64 * half + 64], qh[:, 32 * half: 32 * half + 32], sc[:, 8 * half: 8 * half + 8]
        for qd in range(4):
            byte = L[:, 32 * (qd & 1): 32 * (qd & 1) + 32]
            low = (byte >> 4) if qd >= 2 else (byte & 15)
            hi = (H >> (2 * qd)) & 3
            q = (low | (hi << 4)) - 32
            scale = np.repeat(S[:, 2 * qd: 2 * qd + 2], 16, axis=1)
            out[:, 128 * half + 32 * qd: 128 * half + 32 * qd + 32] = d[:, None] * scale * q
    return out.reshape(-1)[:n]


def quantize_host(x: np.ndarray, ggml_type: int) -> bytes:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if ggml_type == 0:
        return x.tobytes()
    if ggml_type == 1:
        return x.astype(np.float16).tobytes()
    if ggml_type == 30:
        u = x.view(np.uint32)
        return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16).tobytes()
    if ggml_type == 8:
        b = x.reshape(-1, 32)
        amax = np.abs(b).max(axis=1, keepdims=True)
        d = (amax / 127.0).astype(np.float32)
        q = np.where(d > 0, np.round(b / np.where(d > 0, d, 1)), 0).astype(np.int8)
        out = np.empty((b.shape[0], 34), np.uint8)
        out[:, :2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 2:] = q.view(np.uint8)
        return out.tobytes()
    if ggml_type == 2:
        b = x.reshape(-1, 32)
        idx = np.abs(b).argmax(axis=1)
        mx = b[np.arange(b.shape[0]), idx]
        d = (mx / -8.0).astype(np.float32)
        inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
        q = np.clip(np.floor(b * inv[:, None] + 8.5), 0, 15).astype(np.uint8)
        out = np.empty((b.shape[0], 18), np.uint8)
        out[:, :2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
        out[:, 2:] = q[:, :16] | (q[:, 16:] << 4)
        return out.tobytes()
    if ggml_type == 12:
        return _quant_q4k(x)
    if ggml_type == 14:
        return _quant_q6k(x)
    raise NotImplementedError(f"host quantisation to ggml type {ggml_type}")


def _quant_q4k(x: np.ndarray) -> bytes:
    """Q4_K blocks (256 weights: fp16 d, dmin; 8 x 6-bit (scale, min) packed in 12 bytes; 4-bit q):
    w = d s_j q - dmin m_j per 32-weight sub-block j (the layout _dequant_q4k reads)."""
    b = x.reshape(-1, 8, 32)
    lo = np.minimum(b.min(axis=2), 0.0)
    a = (b.max(axis=2) - lo) / 15.0
    d = a.max(axis=1) / 63.0
    dmin = (-lo).max(axis=1) / 63.0
    d16, dm16 = d.astype(np.float16), dmin.astype(np.float16)
    df, dmf = d16.astype(np.float32), dm16.astype(np.float32)
    s = np.clip(np.round(a / np.where(df > 0, df, 1)[:, None]), 0, 63).astype(np.int32)
    m = np.clip(np.round(-lo / np.where(dmf > 0, dmf, 1)[:, None]), 0, 63).astype(np.int32)
    step = (df[:, None] * s)[:, :, None]
    off = (dmf[:, None] * m)[:, :, None]
    q = np.clip(np.round((b + off) / np.where(step > 0, step, 1)), 0, 15).astype(np.uint8)
    sc = np.zeros((b.shape[0], 12), np.uint8)
    for j in range(4):
        sc[:, j] = (s[:, j] & 63) | ((s[:, j + 4] >> 4) << 6)
        sc[:, j + 4] = (m[:, j] & 63) | ((m[:, j + 4] >> 4) << 6)
        sc[:, j + 8] = (s[:, j + 4] & 15) | ((m[:, j + 4] & 15) << 4)
    qs = np.empty((b.shape[0], 128), np.uint8)
    for k in range(4):
        qs[:, 32 * k: 32 * k + 32] = q[:, 2 * k] | (q[:, 2 * k + 1] << 4)
    out = np.empty((b.shape[0], 144), np.uint8)
    out[:, 0:2] = d16.view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dm16.view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = sc
    out[:, 16:] = qs
    return out.tobytes()


def _quant_q6k(x: np.ndarray) -> bytes:
    """Q6_K blocks (256 weights: 6-bit q as 128 low-nibble + 64 high-2-bit bytes, 16 int8 sub-block
    scales, fp16 d): w = d sc_j (q - 32) per 16-weight sub-block (the layout _dequant_q6k reads)."""
    b = x.reshape(-1, 16, 16)
    amax = np.abs(b).max(axis=2)
    sf = amax / 31.0
    d = sf.max(axis=1) / 127.0
    d16 = d.astype(np.float16)
    df = d16.astype(np.float32)
    sc = np.clip(np.round(sf / np.where(df > 0, df, 1)[:, None]), -128, 127).astype(np.int8)
    step = (df[:, None] * sc.astype(np.float32))[:, :, None]
    q = (np.clip(np.round(b / np.where(step != 0, step, 1)), -32, 31) + 32).astype(np.int32).reshape(-1, 256)
    ql = np.zeros((q.shape[0], 128), np.int32)
    qh = np.zeros((q.shape[0], 64), np.int32)
    for half in range(2):
        for qd in range(4):
            v = q[:, 128 * half + 32 * qd: 128 * half + 32 * qd + 32]
            col = 64 * half + 32 * (qd & 1)
            ql[:, col: col + 32] |= (v & 15) << (4 if qd >= 2 else 0)
            qh[:, 32 * half: 32 * half + 32] |= ((v >> 4) & 3) << (2 * qd)
    out = np.empty((q.shape[0], 210), np.uint8)
    out[:, :128] = ql.astype(np.uint8)
    out[:, 128:192] = qh.astype(np.uint8)
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = d16.view(np.uint8).reshape(-1, 2)
    return out.tobytes()


# ----------------------------------------------------------------- writer --
class GGUFWriter:
    def __init__(self, path: str, arch: str, alignment: int = 32):
        self.path = path
        self.alignment = alignment
        self.kv: List[Tuple[str, int, Any]] = []
        self.tensors: List[Tuple[str, Tuple[int, ...], int, bytes]] = []
        self.add("general.architecture", arch)
        self.add("general.alignment", alignment, _U32)

    def add(self, key: str, value, vtype: Optional[int] = None):
        if vtype is None:
            if isinstance(value, bool):
                vtype = _BOOL
            elif isinstance(value, int):
                vtype = _U32 if 0 <= value < 2 ** 32 else _I64
            elif isinstance(value, float):
                vtype = _F32
            elif isinstance(value, str):
                vtype = _STR
            elif isinstance(value, (list, tuple)):
                vtype = _ARR
            else:
                raise TypeError(key)
        self.kv.append((key, vtype, value))

    def add_tensor(self, name: str, arr: np.ndarray, type_name: str = "F32"):
        tid, be, _ = GGML_TYPES[type_name]
        assert arr.size % be == 0, (name, arr.shape, type_name)
        self.tensors.append((name, tuple(arr.shape), tid, quantize_host(arr, tid)))

    @staticmethod
    def _str(b: io.BytesIO, s: str):
        e = s.encode()
        b.write(struct.pack("<Q", len(e)))
        b.write(e)

    def _val(self, b, t, v):
        if t == _STR:
            self._str(b, v)
        elif t == _ARR:
            if all(isinstance(x, str) for x in v):
                b.write(struct.pack("<IQ", _STR, len(v)))
                for x in v:
                    self._str(b, x)
            elif all(isinstance(x, float) for x in v):
                b.write(struct.pack("<IQ", _F32, len(v)))
                b.write(np.asarray(v, np.float32).tobytes())
            else:
                b.write(struct.pack("<IQ", _I32, len(v)))
                b.write(np.asarray(v, np.int32).tobytes())
        else:
            b.write(struct.pack(_SCALAR[t], v))

    def write(self):
        b = io.BytesIO()
        b.write(GGUF_MAGIC)
        b.write(struct.pack("<IQQ", 3, len(self.tensors), len(self.kv)))
        for k, t, v in self.kv:
            self._str(b, k)
            b.write(struct.pack("<I", t))
            self._val(b, t, v)
        off = 0
        offsets = []
        for name, shape, tid, data in self.tensors:
            self._str(b, name)
            ne = tuple(reversed(shape))
            b.write(struct.pack("<I", len(ne)))
            b.write(struct.pack(f"<{len(ne)}Q", *ne))
            b.write(struct.pack("<IQ", tid, off))
            offsets.append(off)
            off = (off + len(data) + self.alignment - 1) // self.alignment * self.alignment
        pad = (-b.tell()) % self.alignment
        b.write(b"\0" * pad)
        with open(self.path, "wb") as f:
            f.write(b.getvalue())
            for (name, shape, tid, data), o in zip(self.tensors, offsets):
                f.write(data)
                f.write(b"\0" * ((-len(data)) % self.alignment))
