"""Causal decoder (llama architecture) for the splainference completion daemon.

The reference completion daemon drives llama.cpp (/root/reference/
splainference.cpp:181-400: prefill, then one llama_decode per sampled token,
top-p 0.9 / temperature 0.7 / seeded dist sampler chain, :272-279).  This is
the MI355X replacement, demo-grade as SURVEY §2.1 N8 scopes it:

* weights: GGUF arch "llama" (token_embd, blk.N.{attn_norm, attn_q, attn_k,
  attn_v, attn_output, ffn_norm, ffn_gate, ffn_up, ffn_down}, output_norm,
  output) dequantised on the device, or random init (``DecoderConfig``);
* every projection (q|k|v fused, o + residual, gate|up + SwiGLU, down +
  residual, LM head) runs on the gfx950 MFMA GEMM (``nomic_gemm``) with its
  fused epilogues; RMSNorm and RoPE (llama "normal" adjacent-pair rotation, as
  llama.cpp applies for arch llama, in place on the q|k GEMM output) are the
  HIP kernels of ``csrc/hip/decoder_kernels.hip``, and so is the per-token
  decode attention over the KV cache (``dec_attn_decode``), the causal prefill
  attention of a fresh or continued prompt over the cache (``dec_attn_prefill_kv``,
  head dim 64 / 128) and the nucleus sampler (``dec_sample``);
* tokenizer: the GGUF's own -- SentencePiece score merging (model "llama") or
  byte-level BPE over the merges (model "gpt2"), models/llm_tokenizer.py -- or,
  for random init, bytes 0..255 + BOS/EOS.

On a host without a GPU the same module runs entirely in torch on the CPU
(``device="cpu"``) so the daemon's label state machine is testable anywhere;
on a GPU box the projections MUST go through the HIP GEMM (no silent fallback).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

BYTE_BOS, BYTE_EOS = 256, 257


@dataclass
class DecoderConfig:
    vocab: int = 384          # 256 bytes + BOS/EOS, padded to a multiple of 128
    d: int = 512
    layers: int = 4
    heads: int = 8
    kv_heads: int = 8
    ffn: int = 1536
    eps: float = 1e-5
    rope_base: float = 10000.0
    n_ctx: int = 2048

    @property
    def head_dim(self) -> int:
        return self.d // self.heads


class ByteTokenizer:
    """bytes 0..255, BOS 256, EOS 257 (random-init demo vocabulary)."""
    bos_id, eos_id = BYTE_BOS, BYTE_EOS

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        return ([self.bos_id] if add_bos else []) + list(text.encode("utf-8"))

    def piece(self, tok: int) -> bytes:
        return bytes([tok]) if tok < 256 else b""

    def is_eog(self, tok: int) -> bool:
        return tok == self.eos_id

    def printable_mask(self, vocab: int) -> torch.Tensor:
        m = torch.zeros(vocab, dtype=torch.bool)
        m[32:127] = True
        m[10] = True
        m[self.eos_id] = True
        return m


def random_decoder_weights(cfg: DecoderConfig, seed: int = 0, std: float = 0.02) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    f = lambda *s: (rng.standard_normal(s) * std).astype(np.float32)  # noqa: E731
    kvd = cfg.kv_heads * cfg.head_dim
    w = {"token_embd.weight": f(cfg.vocab, cfg.d), "output_norm.weight": np.ones(cfg.d, np.float32),
         "output.weight": f(cfg.vocab, cfg.d)}
    for i in range(cfg.layers):
        p = f"blk.{i}."
        w[p + "attn_norm.weight"] = np.ones(cfg.d, np.float32)
        w[p + "attn_q.weight"] = f(cfg.d, cfg.d)
        w[p + "attn_k.weight"] = f(kvd, cfg.d)
        w[p + "attn_v.weight"] = f(kvd, cfg.d)
        w[p + "attn_output.weight"] = f(cfg.d, cfg.d)
        w[p + "ffn_norm.weight"] = np.ones(cfg.d, np.float32)
        w[p + "ffn_gate.weight"] = f(cfg.ffn, cfg.d)
        w[p + "ffn_up.weight"] = f(cfg.ffn, cfg.d)
        w[p + "ffn_down.weight"] = f(cfg.d, cfg.ffn)
    return w


def gguf_quant_kind(g) -> str:
    """"q4" when most projection weights (2-D blk.* tensors) of a GGUF are 4-bit types (Q4_0, Q4_1,
    Q4_K), else "bf16"."""
    proj = [t for n, t in g.tensors.items() if n.startswith("blk.") and len(t.shape) == 2]
    q4 = sum(t.nelems for t in proj if t.ggml_type in (2, 3, 12))
    return "q4" if proj and q4 * 2 > sum(t.nelems for t in proj) else "bf16"


def config_from_gguf(g) -> DecoderConfig:
    a = g.arch() or "llama"
    get = lambda k, d: g.get(f"{a}.{k}", d)  # noqa: E731
    tok = g.tensors["token_embd.weight"]
    d = int(get("embedding_length", 4096))
    heads = int(get("attention.head_count", 32))
    return DecoderConfig(vocab=int(tok.shape[0]), d=d, layers=int(get("block_count", 32)), heads=heads,
                         kv_heads=int(get("attention.head_count_kv", heads)), ffn=int(get("feed_forward_length", 11008)),
                         eps=float(get("attention.layer_norm_rms_epsilon", 1e-5)),
                         rope_base=float(get("rope.freq_base", 10000.0)), n_ctx=int(get("context_length", 2048)))


class Q4Weight:
    """A projection W [N, K] resident as Q4G32 (csrc/hip/decoder_kernels.hip): 4-bit nibbles
    ``q`` uint8 [N, K/2] plus one bf16 (d, m) pair per 32-k group ``sm`` int32 [N, K/32], w = d q + m;
    0.625 B per weight instead of 2.  Decode reads it with dec_gemv_q4; prefill dequantises one matrix
    at a time into a bf16 scratch for the MFMA GEMM.  The role of llama.cpp's Q4 weights in the
    reference's llama_decode (splainference.cpp:272-330)."""

    def __init__(self, q: torch.Tensor, sm: torch.Tensor):
        self.q, self.sm = q, sm
        self.shape = (q.shape[0], q.shape[1] * 2)

    @classmethod
    def quantize(cls, L, w: torch.Tensor) -> "Q4Weight":
        from .nomic import _chk, _stream
        w = w.to(torch.bfloat16).contiguous()
        N, K = w.shape
        q = torch.empty((N, K // 2), dtype=torch.uint8, device=w.device)
        sm = torch.empty((N, K // 32), dtype=torch.int32, device=w.device)
        _chk(L.dec_q4_quantize(w.data_ptr(), N, K, q.data_ptr(), sm.data_ptr(), _stream()), "q4_quantize")
        return cls(q, sm)

    def dequant(self, L, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        from .nomic import _chk, _stream
        N, K = self.shape
        if out is None:
            out = torch.empty((N, K), dtype=torch.bfloat16, device=self.q.device)
        _chk(L.dec_q4_dequant(self.q.data_ptr(), self.sm.data_ptr(), N, K, out.data_ptr(), _stream()), "q4_dequant")
        return out

    def nbytes(self) -> int:
        return self.q.numel() + self.sm.numel() * 4

    bits = 4


class Q8Weight(Q4Weight):
    """Q8G32: one byte per weight (u in 0..255) and the same bf16 (d, m) pair per 32-k group,
    w = d u + m; 1.125 B per weight.  Holds the tensors a mostly-4-bit GGUF keeps at more than 4
    bits (a Q4_K_M file's Q6_K attn_v / ffn_down / output), so they are not re-gridded below the
    file's precision.  Decode reads it with dec_gemv_q8, prefill dequantises with dec_q8_dequant."""
    bits = 8

    def __init__(self, q: torch.Tensor, sm: torch.Tensor):
        self.q, self.sm = q, sm
        self.shape = (q.shape[0], q.shape[1])

    @classmethod
    def quantize(cls, L, w: torch.Tensor) -> "Q8Weight":
        from .nomic import _chk, _stream
        w = w.to(torch.bfloat16).contiguous()
        N, K = w.shape
        q = torch.empty((N, K), dtype=torch.uint8, device=w.device)
        sm = torch.empty((N, K // 32), dtype=torch.int32, device=w.device)
        _chk(L.dec_q8_quantize(w.data_ptr(), N, K, q.data_ptr(), sm.data_ptr(), _stream()), "q8_quantize")
        return cls(q, sm)

    def dequant(self, L, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        from .nomic import _chk, _stream
        N, K = self.shape
        if out is None:
            out = torch.empty((N, K), dtype=torch.bfloat16, device=self.q.device)
        _chk(L.dec_q8_dequant(self.q.data_ptr(), self.sm.data_ptr(), N, K, out.data_ptr(), _stream()), "q8_dequant")
        return out


# GGUF tensor types stored at <= 4 bits per weight (Q4_0, Q4_1, Q2_K, Q3_K, Q4_K, IQ2/IQ3/IQ4, IQ1):
# Q4G32 keeps them at no loss of grid resolution; every other type (Q5_x, Q6_K, Q8_0, F16, BF16,
# F32) goes to Q8G32
GGML_LE4 = {2, 3, 10, 11, 12, 16, 17, 18, 19, 20, 21, 22, 23, 29}


class CausalLM:
    def __init__(self, cfg: DecoderConfig, tensors: Dict[str, torch.Tensor], device: str = "cuda",
                 quant: str = "bf16", ggml_types: Optional[Dict[str, int]] = None):
        """quant "q4": every projection (qkv, o, up|gate, down, LM head) is kept as a Q4Weight
        (GPU only) -- except those whose source GGUF tensors (``ggml_types``, name -> GGML type)
        hold more than 4 bits per weight, which are kept as Q8Weight; "bf16": bf16 weights."""
        if quant not in ("bf16", "q4"):
            raise ValueError(f"quant must be bf16 or q4, not {quant!r}")
        self.cfg = cfg
        self.device = device
        self.hip = device != "cpu"
        self.quant = quant if self.hip else "bf16"
        dt = torch.bfloat16 if self.hip else torch.float32
        T = lambda n: tensors[n].to(device=device, dtype=dt).contiguous()  # noqa: E731
        self.emb = T("token_embd.weight")
        self.norm_out = T("output_norm.weight").float()
        head = tensors.get("output.weight", tensors["token_embd.weight"])
        vpad = (cfg.vocab + 127) // 128 * 128
        hw = torch.zeros((vpad, cfg.d), dtype=dt, device=device)
        hw[: cfg.vocab] = head.to(device=device, dtype=dt)
        self.head = hw
        self.layers = []
        if self.hip:
            self._declare()
        gt = ggml_types or {}

        def Q(t, *names):
            if self.quant != "q4":
                return t
            wide = any(n in gt and gt[n] not in GGML_LE4 for n in names)
            return (Q8Weight if wide else Q4Weight).quantize(self.L, t)

        self.head = Q(self.head, "output.weight" if "output.weight" in tensors else "token_embd.weight")
        for i in range(cfg.layers):
            p = f"blk.{i}."
            qkv = torch.cat([T(p + "attn_q.weight"), T(p + "attn_k.weight"), T(p + "attn_v.weight")], 0)
            gate, up = T(p + "ffn_gate.weight"), T(p + "ffn_up.weight")
            # SwiGLU epilogue layout: rows interleaved [up16 | gate16] (nomic_api.h NOMIC_EPI_SWIGLU)
            from .nomic import pack_upgate
            ug = pack_upgate(up, gate)
            self.layers.append({"n1": T(p + "attn_norm.weight").float(),
                                "qkv": Q(qkv.contiguous(), p + "attn_q.weight", p + "attn_k.weight", p + "attn_v.weight"),
                                "o": Q(T(p + "attn_output.weight"), p + "attn_output.weight"),
                                "n2": T(p + "ffn_norm.weight").float(),
                                "ug": Q(ug.contiguous(), p + "ffn_gate.weight", p + "ffn_up.weight"),
                                "down": Q(T(p + "ffn_down.weight"), p + "ffn_down.weight")})
            del qkv, gate, up, ug
        self._q4_scratch: Optional[torch.Tensor] = None
        hd = cfg.head_dim
        inv = 1.0 / (cfg.rope_base ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
        ang = torch.arange(cfg.n_ctx, dtype=torch.float64)[:, None] * inv[None, :]
        self.cos = ang.cos().float().to(device)
        self.sin = ang.sin().float().to(device)
        # KV cache: one [layers, 2, n_ctx, kv_heads, head_dim] buffer allocated on first use and
        # written in place (no per-token torch.cat regrowth: decode stays O(1) copies per token)
        self.kv: Optional[torch.Tensor] = None
        self.pos = 0
        self.attn_kernel = True  # HIP prefill / decode attention (False: torch SDPA, for A/B only)
        if self.hip:
            ok = all(n % 128 == 0 for n in (cfg.d + 2 * cfg.kv_heads * hd, cfg.d, 2 * cfg.ffn, vpad)) \
                and cfg.d % 64 == 0 and cfg.ffn % 64 == 0
            if not ok:
                raise ValueError("decoder dims must be multiples of 128 (N) / 64 (K) for the MFMA GEMM")
        # HIP attention where the kernels take the head dim (prefill: 64 / 128, decode: any multiple of
        # 64 up to 256); other head dims (e.g. 80, 96) run those layers' attention on torch SDPA
        self.prefill_kernel = hd in (64, 128)
        self.decode_kernel = hd % 64 == 0 and hd <= 256

    def _declare(self):
        """ctypes signatures of the decoder kernels (csrc/hip/decoder_kernels.hip)."""
        from .nomic import _lib
        self.L = _lib()
        if not getattr(self.L, "_dec_declared", False):
            P, c_long, c_int, c_float = ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_float
            self.L.dec_rmsnorm.argtypes = [P, c_long, P, c_long, c_int, c_float, P, c_long, P]
            self.L.dec_rmsnorm.restype = c_int
            self.L.dec_rope.argtypes = [P, c_long, c_long, c_int, c_int, c_int, P, P, P]
            self.L.dec_rope.restype = c_int
            self.L.dec_attn_decode.argtypes = [P, P, P, c_long, c_int, c_int, c_int, c_int, c_float, P, P]
            self.L.dec_attn_decode.restype = c_int
            self.L.dec_attn_decode_st.argtypes = [P, P, P, c_long, c_int, c_int, c_int, c_int, c_float, P, P, P]
            self.L.dec_attn_decode_st.restype = c_int
            self.L.dec_attn_decode_ws.argtypes = [P, P, P, c_long, c_int, c_int, c_int, c_int, c_float, P, P, P, P]
            self.L.dec_attn_decode_ws.restype = c_int
            self.L.dec_attn_prefill.argtypes = [P, P, P, P, c_int, c_int, c_int, c_float, P]
            self.L.dec_attn_prefill.restype = c_int
            self.L.dec_attn_prefill_kv.argtypes = [P, c_long, P, P, c_long, c_int, c_int, c_int, c_int, c_int, c_float,
                                                   P, c_long, P]
            self.L.dec_attn_prefill_kv.restype = c_int
            self.L.dec_gemv.argtypes = [c_int, P, P, c_float, P, c_int, c_int, P, P, P]
            self.L.dec_gemv.restype = c_int
            self.L.dec_embed_tok.argtypes = [P, c_int, P, P, P]
            self.L.dec_embed_tok.restype = c_int
            self.L.dec_rope_kv.argtypes = [P, c_int, c_int, c_int, P, P, P, P, P, c_long, P]
            self.L.dec_rope_kv.restype = c_int
            self.L.dec_sample.argtypes = [P, c_int, P, c_float, c_float, ctypes.c_uint64, P, c_int, P, P]
            self.L.dec_sample.restype = c_int
            self.L.dec_sample_ws.argtypes = [P, c_int, P, c_float, c_float, ctypes.c_uint64, P, c_int, P, P, P]
            self.L.dec_sample_ws.restype = c_int
            self.L.dec_sample_ws_floats.argtypes = []
            self.L.dec_sample_ws_floats.restype = c_long
            self.L.dec_gemv_q4.argtypes = [c_int, P, P, c_float, P, P, c_int, c_int, P, P, P]
            self.L.dec_gemv_q4.restype = c_int
            self.L.dec_q4_quantize.argtypes = [P, c_long, c_int, P, P, P]
            self.L.dec_q4_quantize.restype = c_int
            self.L.dec_q4_dequant.argtypes = [P, P, c_long, c_int, P, P]
            self.L.dec_q4_dequant.restype = c_int
            self.L.dec_gemv_q8.argtypes = [c_int, P, P, c_float, P, P, c_int, c_int, P, P, P]
            self.L.dec_gemv_q8.restype = c_int
            self.L.dec_q8_quantize.argtypes = [P, c_long, c_int, P, P, P]
            self.L.dec_q8_quantize.restype = c_int
            self.L.dec_q8_dequant.argtypes = [P, P, c_long, c_int, P, P]
            self.L.dec_q8_dequant.restype = c_int
            self.L._dec_declared = True

    @classmethod
    def random(cls, cfg: DecoderConfig, seed: int = 0, device: str = "cuda", quant: str = "bf16") -> "CausalLM":
        return cls(cfg, {k: torch.from_numpy(v) for k, v in random_decoder_weights(cfg, seed).items()}, device,
                   quant=quant)

    @classmethod
    def from_gguf(cls, path: str, device: str = "cuda", quant: str = "auto"):
        """quant "auto": Q4G32 when most projection weights of the file are 4-bit GGUF types
        (Q4_0 / Q4_1 / Q4_K), with the file's wider tensors (a Q4_K_M file's Q6_K) on Q8G32; else bf16."""
        from .gguf import GGUFFile
        g = GGUFFile(path)
        cfg = config_from_gguf(g)
        if quant == "auto":
            quant = gguf_quant_kind(g)
        tensors = {n: torch.from_numpy(np.ascontiguousarray(g.to_numpy_f32(n))) for n in g.tensors}
        from .llm_tokenizer import tokenizer_from_gguf
        tok = tokenizer_from_gguf(g) or ByteTokenizer()  # SPM / BPE by tokenizer.ggml.model
        if not hasattr(tok, "chat_template"):
            tok.chat_template = None  # rendered by splainference.build_prompt
        types = {n: t.ggml_type for n, t in g.tensors.items()}
        return cls(cfg, tensors, device, quant=quant if device != "cpu" else "bf16", ggml_types=types), tok

    # ------------------------------------------------------------- pieces --
    def _mm(self, mode: int, x: torch.Tensor, w, out_cols: int, res: Optional[torch.Tensor] = None):
        """x [M, K] @ w[N, K]^T with a fused epilogue; HIP MFMA on the GPU, torch on the CPU."""
        M, K = x.shape
        if isinstance(w, Q4Weight):  # prefill: dequantise into the shared bf16 scratch
            n_el = w.shape[0] * w.shape[1]
            if self._q4_scratch is None or self._q4_scratch.numel() < n_el:
                self._q4_scratch = torch.empty(n_el, dtype=torch.bfloat16, device=self.device)
            w = w.dequant(self.L, self._q4_scratch[:n_el].view(w.shape))
        if not self.hip:
            if mode == 2:
                up, gate = self._split_ug(x @ w.T)
                return up * torch.nn.functional.silu(gate)
            y = x @ w.T
            return y + res if res is not None else y
        from .nomic import _chk, _stream
        Mp = (M + 127) // 128 * 128
        if Mp != M:
            xp = torch.zeros((Mp, K), dtype=x.dtype, device=x.device)
            xp[:M] = x
            x = xp
        x = x.contiguous()
        f32 = mode == 4
        out = torch.empty((Mp, out_cols), dtype=torch.float32 if f32 else torch.bfloat16, device=x.device)
        rp = None
        if res is not None:
            rp = torch.zeros((Mp, out_cols), dtype=torch.bfloat16, device=x.device)
            rp[:M] = res
        _chk(self.L.nomic_gemm(mode, x.data_ptr(), K, w.data_ptr(), K, M, w.shape[0], K, out.data_ptr(), out_cols,
                               None if rp is None else rp.data_ptr(), out_cols, None, None, 0, _stream()), "gemm")
        return out[:M]

    @staticmethod
    def _split_ug(y: torch.Tensor):
        g = y.reshape(y.shape[0], -1, 2, 16)  # pack_upgate: [up16 | gate16] per 16 outputs
        return g[:, :, 0].reshape(y.shape[0], -1), g[:, :, 1].reshape(y.shape[0], -1)

    def _rms(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        if self.hip:  # dec_rmsnorm (csrc/hip/decoder_kernels.hip): one wave per row
            from .nomic import _chk, _stream
            x = x.contiguous()
            out = torch.empty_like(x)
            _chk(self.L.dec_rmsnorm(x.data_ptr(), x.shape[1], w.data_ptr(), x.shape[0], x.shape[1], self.cfg.eps,
                                    out.data_ptr(), x.shape[1], _stream()), "rmsnorm")
            return out
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.cfg.eps) * w
        return y.to(x.dtype)

    def _rope(self, t: torch.Tensor, pos: torch.Tensor) -> torch.Tensor:
        # llama "normal" rotation: adjacent pairs (x[2i], x[2i+1])
        c, s = self.cos[pos][:, None, :], self.sin[pos][:, None, :]
        tf = t.float()
        x1, x2 = tf[..., 0::2], tf[..., 1::2]
        out = torch.stack([x1 * c - x2 * s, x1 * s + x2 * c], -1).flatten(-2)
        return out.to(t.dtype)

    def reset(self):
        self.pos = 0

    @torch.no_grad()
    def forward(self, ids: List[int]) -> torch.Tensor:
        """Append tokens to the KV cache; returns fp32 logits of the last position."""
        cfg = self.cfg
        hd, H, KVH = cfg.head_dim, cfg.heads, cfg.kv_heads
        n = len(ids)
        if self.pos + n > cfg.n_ctx:
            raise ValueError("context window exceeded")
        pos = torch.arange(self.pos, self.pos + n, device=self.device)
        x = self.emb[torch.tensor(ids, device=self.device)]
        for li, lw in enumerate(self.layers):
            h = self._rms(x, lw["n1"])
            qkv = self._mm(0, h, lw["qkv"], cfg.d + 2 * KVH * hd)
            if self.hip:  # RoPE in place over the q|k columns (dec_rope)
                from .nomic import _chk, _stream
                _chk(self.L.dec_rope(qkv.data_ptr(), qkv.stride(0), n, cfg.d + KVH * hd, hd, self.pos,
                                     self.cos.data_ptr(), self.sin.data_ptr(), _stream()), "rope")
            q = qkv[:, : cfg.d].reshape(n, H, hd)
            k = qkv[:, cfg.d: cfg.d + KVH * hd].reshape(n, KVH, hd)
            v = qkv[:, cfg.d + KVH * hd:].reshape(n, KVH, hd)
            if not self.hip:
                q, k = self._rope(q, pos), self._rope(k, pos)
            if self.kv is None:
                self.kv = torch.empty((cfg.layers, 2, cfg.n_ctx, KVH, hd), dtype=qkv.dtype, device=self.device)
            self.kv[li, 0, self.pos: self.pos + n] = k
            self.kv[li, 1, self.pos: self.pos + n] = v
            L_ = self.pos + n
            if self.hip and self.attn_kernel and self.prefill_kernel and n > 1:
                # prompt prefill, fresh or continuing a live cache: causal MFMA attention of the n new
                # queries over cache rows 0 .. pos+n-1 (dec_attn_prefill_kv, hd 64 / 128)
                from .nomic import _chk, _stream
                a = torch.empty((n, cfg.d), dtype=qkv.dtype, device=self.device)
                _chk(self.L.dec_attn_prefill_kv(qkv.data_ptr(), qkv.stride(0), self.kv[li, 0].data_ptr(),
                                                self.kv[li, 1].data_ptr(), KVH * hd, n, self.pos, H, KVH, hd,
                                                hd ** -0.5, a.data_ptr(), cfg.d, _stream()), "attn_prefill")
            elif self.hip and self.attn_kernel and self.decode_kernel and n == 1:
                # per-token decode: dec_attn_decode (one workgroup per q head, split-L online softmax)
                from .nomic import _chk, _stream
                a = torch.empty((1, cfg.d), dtype=qkv.dtype, device=self.device)
                qrow = qkv[0, : cfg.d].contiguous()
                _chk(self.L.dec_attn_decode(qrow.data_ptr(), self.kv[li, 0].data_ptr(), self.kv[li, 1].data_ptr(),
                                            KVH * hd, L_, H, KVH, hd, hd ** -0.5, a.data_ptr(), _stream()),
                     "attn_decode")
            else:
                K_, V_ = self.kv[li, 0, :L_], self.kv[li, 1, :L_]
                qh, kh, vh = q.transpose(0, 1), K_.transpose(0, 1), V_.transpose(0, 1)
                # causal over the cache: query i (absolute position pos + i) sees keys 0..pos+i; a single
                # decode token sees the whole cache, so no mask is needed
                # a fresh prompt (pos 0) is plain causal: is_causal lets torch pick its fused kernel instead
                # of the materialised-mask path
                fresh = n > 1 and L_ == n
                mask = None if n == 1 or fresh else \
                    torch.ones((n, L_), dtype=torch.bool, device=self.device).tril(L_ - n)
                a = torch.nn.functional.scaled_dot_product_attention(qh.unsqueeze(0), kh.unsqueeze(0),
                                                                     vh.unsqueeze(0), attn_mask=mask,
                                                                     is_causal=fresh, enable_gqa=KVH != H)[0]
                a = a.transpose(0, 1).reshape(n, cfg.d).contiguous()
            x = self._mm(1, a, lw["o"], cfg.d, res=x)
            h = self._rms(x, lw["n2"])
            f = self._mm(2, h, lw["ug"], cfg.ffn)
            x = self._mm(1, f.contiguous(), lw["down"], cfg.d, res=x)
        self.pos += n
        h = self._rms(x[-1:], self.norm_out)
        logits = self._mm(4, h, self.head, self.head.shape[0])
        return logits[0, : cfg.vocab].float()


class DecodeEngine:
    """Token generation with no host compute in the loop (K18): prompt prefill on the MFMA GEMMs
    and the causal MFMA attention, then per token ONE replay of a HIP graph holding the whole
    decode step -- embedding row, per layer (RMSNorm+QKV GEMV, RoPE + KV-cache append, decode
    attention, o GEMV + residual, RMSNorm+up|gate GEMV + SwiGLU, down GEMV + residual), final
    RMSNorm + LM-head GEMV and the top-p / temperature sampler (dec_sample).  Every kernel reads
    the position and the input token from a device state {pos, token, step}, so the captured
    arguments never change; the host reads back only the sampled token id (pinned memory).
    Reference: splainference.cpp:272-365 (sampler chain, llama_decode per token)."""

    def __init__(self, model: "CausalLM", top_p: float = 0.9, temp: float = 0.7, seed: int = 0xFFFFFFFF,
                 mask: Optional[torch.Tensor] = None, use_graph: bool = True):
        assert model.hip, "DecodeEngine runs on the GPU"
        if not model.decode_kernel:
            raise ValueError(f"head dim {model.cfg.head_dim}: the graph decode engine needs a multiple of 64 "
                             "up to 256 (use CausalLM.forward)")
        m, cfg = model, model.cfg
        self.m, self.top_p, self.temp, self.seed = m, float(top_p), float(temp), int(seed) & 0xFFFFFFFFFFFFFFFF
        dev = m.device
        e = dict(device=dev, dtype=torch.bfloat16)
        kvd = cfg.kv_heads * cfg.head_dim
        self.st = torch.zeros(4, dtype=torch.int32, device=dev)      # pos, token, step
        self.xa = torch.empty(cfg.d, **e)
        self.xb = torch.empty(cfg.d, **e)
        self.qkv = torch.empty(cfg.d + 2 * kvd, **e)
        self.attn = torch.empty(cfg.d, **e)
        self.ffn = torch.empty(cfg.ffn, **e)
        self.logits = torch.empty(m.head.shape[0], dtype=torch.float32, device=dev)
        self.attn_ws = torch.empty(cfg.heads * 32 * (cfg.head_dim + 2), dtype=torch.float32, device=dev)  # split-L
        self.samp_ws = torch.empty(m.L.dec_sample_ws_floats(), dtype=torch.float32, device=dev)  # multi-block sampler
        self.host_tok = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.mask = mask[: cfg.vocab].to(device=dev, dtype=torch.uint8).contiguous() if mask is not None else None
        if m.kv is None:
            m.kv = torch.empty((cfg.layers, 2, cfg.n_ctx, cfg.kv_heads, cfg.head_dim), dtype=torch.bfloat16, device=dev)
        self.use_graph = use_graph
        self.graphs = {}  # attention span (512 or the capacity) -> captured decode step
        self.steps = 0

    def _enqueue_step(self, span: int = 0):
        from .nomic import _chk, _stream
        m, cfg, L = self.m, self.m.cfg, self.m.L
        s = _stream()
        H, KVH, hd = cfg.heads, cfg.kv_heads, cfg.head_dim
        P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        _chk(L.dec_embed_tok(m.emb.data_ptr(), cfg.d, self.st.data_ptr(), self.xa.data_ptr(), s), "embed_tok")

        def gemv(mode, x, rms, w, N, K, res, out, what):
            rp = rms.data_ptr() if rms is not None else None
            if isinstance(w, Q4Weight):  # 4-bit: 0.625 B per weight streamed (dec_gemv_q4); 8-bit: 1.125 B
                _chk((L.dec_gemv_q8 if w.bits == 8 else L.dec_gemv_q4)(mode, x.data_ptr(), rp, cfg.eps, w.q.data_ptr(), w.sm.data_ptr(), N, K,
                                   P(res), out.data_ptr(), s), what)
            else:
                _chk(L.dec_gemv(mode, x.data_ptr(), rp, cfg.eps, w.data_ptr(), N, K, P(res), out.data_ptr(), s), what)

        for li, lw in enumerate(m.layers):
            gemv(0, self.xa, lw["n1"], lw["qkv"], lw["qkv"].shape[0], cfg.d, None, self.qkv, "gemv qkv")
            kc, vc = m.kv[li, 0], m.kv[li, 1]
            _chk(L.dec_rope_kv(self.qkv.data_ptr(), H, KVH, hd, m.cos.data_ptr(), m.sin.data_ptr(), self.st.data_ptr(),
                               kc.data_ptr(), vc.data_ptr(), KVH * hd, s), "rope_kv")
            # L = the span the step is captured for (<= 512: one workgroup per head group; else the
            # capacity, sizing the split-L grid); the length itself is read on the device
            _chk(L.dec_attn_decode_ws(self.qkv.data_ptr(), kc.data_ptr(), vc.data_ptr(), KVH * hd, span or cfg.n_ctx, H, KVH,
                                      hd, hd ** -0.5, self.attn.data_ptr(), self.st.data_ptr(),
                                      self.attn_ws.data_ptr(), s), "attn_decode")
            gemv(1, self.attn, None, lw["o"], cfg.d, cfg.d, self.xa, self.xb, "gemv o")
            gemv(2, self.xb, lw["n2"], lw["ug"], lw["ug"].shape[0], cfg.d, None, self.ffn, "gemv up|gate")
            gemv(1, self.ffn, None, lw["down"], cfg.d, cfg.ffn, self.xb, self.xa, "gemv down")
        gemv(4, self.xa, m.norm_out, m.head, m.head.shape[0], cfg.d, None, self.logits, "gemv head")
        self._sample(self.logits, inc_pos=1)

    def _sample(self, logits: torch.Tensor, inc_pos: int):
        from .nomic import _chk, _stream
        m = self.m
        _chk(m.L.dec_sample_ws(logits.data_ptr(), m.cfg.vocab, self.mask.data_ptr() if self.mask is not None else None,
                               self.top_p, self.temp, self.seed, self.st.data_ptr(), inc_pos, self.host_tok.data_ptr(),
                               self.samp_ws.data_ptr(), _stream()), "sample")

    def _step(self):
        # two captured steps: up to 512 cached keys the single-workgroup attention kernel, past that
        # the split-L one sized for the cache capacity (a split grid costs ~9 us more per layer on
        # short caches: profiles/r2_decode_splits_gqa.jsonl); the host knows the position
        span = self.m.cfg.n_ctx if self.m.pos + 1 > 512 else min(512, self.m.cfg.n_ctx)
        if not self.use_graph:
            self._enqueue_step(span)
            return
        g = self.graphs.get(span)
        if g is None:
            # warm up once outside capture (first-launch code-object loading), then capture
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            saved = self.st.clone()
            with torch.cuda.stream(side):
                self._enqueue_step(span)
            torch.cuda.current_stream().wait_stream(side)
            self.st.copy_(saved)  # the warm-up step is undone: same state, cache row rewritten next
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._enqueue_step(span)
            self.graphs[span] = g
        g.replay()

    def first_token(self, ids: List[int]) -> int:
        """Prefill the prompt (KV cache rows 0..n-1) and sample the first token on the device."""
        m = self.m
        m.reset()
        logits = m.forward(ids)
        self.st[0] = len(ids)
        self.st[1] = 0
        self._sample(logits.contiguous(), inc_pos=0)
        torch.cuda.current_stream().synchronize()
        return int(self.host_tok[0])

    def next_token(self) -> int:
        """One decode step on the device: consume the last sampled token, return the next one."""
        self._step()
        torch.cuda.current_stream().synchronize()
        self.m.pos += 1
        self.steps += 1
        return int(self.host_tok[0])


class Sampler:
    """top-p 0.9 -> temperature 0.7 -> seeded categorical (reference :272-279)."""

    def __init__(self, top_p: float = 0.9, temp: float = 0.7, seed: int = 0xFFFFFFFF, mask=None):
        self.top_p, self.temp, self.seed = top_p, temp, seed
        self.g = torch.Generator().manual_seed(seed)
        self.mask = mask

    def __call__(self, logits: torch.Tensor) -> int:
        lg = logits.detach().float().cpu()
        if self.mask is not None:
            lg = lg.masked_fill(~self.mask[: lg.shape[0]], -math.inf)
        p = torch.softmax(lg, -1)
        sp, si = torch.sort(p, descending=True)
        keep = torch.cumsum(sp, 0) - sp < self.top_p
        keep[0] = True
        lg2 = torch.full_like(lg, -math.inf)
        lg2[si[keep]] = lg[si[keep]]
        probs = torch.softmax(lg2 / self.temp, -1)
        return int(torch.multinomial(probs, 1, generator=self.g).item())
