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
  decode attention over the KV cache (``dec_attn_decode``); prompt prefill
  attention and the sampler use torch ops on the same device -- the decode
  step is latency-bound and not a benchmark path;
* tokenizer: greedy longest-match over the GGUF vocabulary (SentencePiece
  "▁" spaces, <0xNN> byte fallback) or, for random init, bytes 0..255 + BOS/EOS.

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

    def printable_mask(self, vocab: int) -> torch.Tensor:
        m = torch.zeros(vocab, dtype=torch.bool)
        m[32:127] = True
        m[10] = True
        m[self.eos_id] = True
        return m


class VocabTokenizer:
    """Greedy longest-match over a GGUF vocabulary (SentencePiece conventions)."""

    def __init__(self, tokens: List[str], bos: int, eos: int):
        self.tokens = tokens
        self.bos_id, self.eos_id = bos, eos
        self.index: Dict[str, int] = {t: i for i, t in enumerate(tokens)}
        self.maxlen = max((len(t) for t in tokens), default=1)
        self.byte_ids = {b: self.index.get(f"<0x{b:02X}>") for b in range(256)}

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        s = "▁" + text.replace(" ", "▁")
        out = [self.bos_id] if add_bos else []
        i = 0
        while i < len(s):
            for L in range(min(self.maxlen, len(s) - i), 0, -1):
                t = self.index.get(s[i:i + L])
                if t is not None:
                    out.append(t)
                    i += L
                    break
            else:
                for b in s[i].encode("utf-8"):
                    bid = self.byte_ids.get(b)
                    if bid is not None:
                        out.append(bid)
                i += 1
        return out

    def piece(self, tok: int) -> bytes:
        t = self.tokens[tok] if 0 <= tok < len(self.tokens) else ""
        if len(t) == 6 and t.startswith("<0x") and t.endswith(">"):
            return bytes([int(t[3:5], 16)])
        if t.startswith("<") and t.endswith(">"):
            return b""
        return t.replace("▁", " ").encode("utf-8")

    def printable_mask(self, vocab: int) -> Optional[torch.Tensor]:
        return None


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


class CausalLM:
    def __init__(self, cfg: DecoderConfig, tensors: Dict[str, torch.Tensor], device: str = "cuda"):
        self.cfg = cfg
        self.device = device
        self.hip = device != "cpu"
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
        for i in range(cfg.layers):
            p = f"blk.{i}."
            qkv = torch.cat([T(p + "attn_q.weight"), T(p + "attn_k.weight"), T(p + "attn_v.weight")], 0)
            gate, up = T(p + "ffn_gate.weight"), T(p + "ffn_up.weight")
            # SwiGLU epilogue layout: rows interleaved [up16 | gate16] (nomic_api.h NOMIC_EPI_SWIGLU)
            from .nomic import pack_upgate
            ug = pack_upgate(up, gate)
            self.layers.append({"n1": T(p + "attn_norm.weight").float(), "qkv": qkv.contiguous(),
                                "o": T(p + "attn_output.weight"), "n2": T(p + "ffn_norm.weight").float(),
                                "ug": ug.contiguous(), "gate": gate, "up": up, "down": T(p + "ffn_down.weight")})
        hd = cfg.head_dim
        inv = 1.0 / (cfg.rope_base ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
        ang = torch.arange(cfg.n_ctx, dtype=torch.float64)[:, None] * inv[None, :]
        self.cos = ang.cos().float().to(device)
        self.sin = ang.sin().float().to(device)
        # KV cache: one [layers, 2, n_ctx, kv_heads, head_dim] buffer allocated on first use and
        # written in place (no per-token torch.cat regrowth: decode stays O(1) copies per token)
        self.kv: Optional[torch.Tensor] = None
        self.pos = 0
        self.attn_kernel = True  # single-token decode through dec_attn_decode (False: SDPA, for A/B)
        if self.hip:
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
                self.L._dec_declared = True
            ok = all(n % 128 == 0 for n in (cfg.d + 2 * cfg.kv_heads * hd, cfg.d, 2 * cfg.ffn, vpad)) \
                and cfg.d % 64 == 0 and cfg.ffn % 64 == 0
            if not ok:
                raise ValueError("decoder dims must be multiples of 128 (N) / 64 (K) for the MFMA GEMM")

    @classmethod
    def random(cls, cfg: DecoderConfig, seed: int = 0, device: str = "cuda") -> "CausalLM":
        return cls(cfg, {k: torch.from_numpy(v) for k, v in random_decoder_weights(cfg, seed).items()}, device)

    @classmethod
    def from_gguf(cls, path: str, device: str = "cuda"):
        from .gguf import GGUFFile, dequant_host
        g = GGUFFile(path)
        cfg = config_from_gguf(g)
        tensors = {n: torch.from_numpy(dequant_host(g, n)) for n in g.tensors}
        tokens = g.get("tokenizer.ggml.tokens")
        tok = VocabTokenizer(list(tokens), int(g.get("tokenizer.ggml.bos_token_id", 1)),
                             int(g.get("tokenizer.ggml.eos_token_id", 2))) if tokens else ByteTokenizer()
        return cls(cfg, tensors, device), tok

    # ------------------------------------------------------------- pieces --
    def _mm(self, mode: int, x: torch.Tensor, w: torch.Tensor, out_cols: int, res: Optional[torch.Tensor] = None):
        """x [M, K] @ w[N, K]^T with a fused epilogue; HIP MFMA on the GPU, torch on the CPU."""
        M, K = x.shape
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
            if self.hip and self.attn_kernel and n == 1 and hd % 64 == 0 and hd <= 256:
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
                mask = None if n == 1 else torch.ones((n, L_), dtype=torch.bool, device=self.device).tril(L_ - n)
                a = torch.nn.functional.scaled_dot_product_attention(qh.unsqueeze(0), kh.unsqueeze(0),
                                                                     vh.unsqueeze(0), attn_mask=mask,
                                                                     enable_gqa=KVH != H)[0]
                a = a.transpose(0, 1).reshape(n, cfg.d).contiguous()
            x = self._mm(1, a, lw["o"], cfg.d, res=x)
            h = self._rms(x, lw["n2"])
            f = self._mm(2, h, lw["ug"], cfg.ffn)
            x = self._mm(1, f.contiguous(), lw["down"], cfg.d, res=x)
        self.pos += n
        h = self._rms(x[-1:], self.norm_out)
        logits = self._mm(4, h, self.head, self.head.shape[0])
        return logits[0, : cfg.vocab].float()


class Sampler:
    """top-p 0.9 -> temperature 0.7 -> seeded categorical (reference :272-279)."""

    def __init__(self, top_p: float = 0.9, temp: float = 0.7, seed: int = 0xFFFFFFFF, mask=None):
        self.top_p, self.temp = top_p, temp
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
