"""Nomic-BERT (nomic-embed-text-v1.5 architecture) on hand-written gfx950 kernels.

Replaces the llama.cpp decode used by the reference embedding daemon
(/root/reference/splinference.cpp:196-287: one sequence per llama_decode, mean
pooling forced at :431-437) with a batched, varlen, bf16 encoder:

  embed+LN  ->  12 x [ QKV GEMM (+RoPE epilogue) -> flash attention ->
                       O-proj GEMM (+residual epilogue) -> LN ->
                       up|gate GEMM (+SwiGLU epilogue) -> down GEMM (+residual) -> LN ]
  -> mean pool -> (optionally) vectors written straight into arena slots.

Architecture facts (GGUF arch "nomic-bert", SURVEY §2.12, re-checked from the
GGUF metadata at load): 12 layers, d=768, 12 heads x 64, SwiGLU MLP 3072,
NEOX rotary (base 1000) on q/k, post-LayerNorm (eps 1e-12), non-causal,
token-type row 0 added to the token embedding, no absolute positions.

``NomicReference`` is an independent fp32 PyTorch implementation used as the
numerics oracle in tests (the HF remote code is not available offline).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _native as N
from ..utils.tracing import trace_range
from .gguf import DEVICE_DEQUANT, GGUFFile, GGUFWriter, dequant_host

EPI_STORE, EPI_RESIDUAL, EPI_SWIGLU, EPI_ROPE, EPI_F32 = 0, 1, 2, 3, 4
# post-LayerNorm folded into the neighbouring GEMMs (csrc/include/nomic_api.h)
EPI_ROPE_FOLD, EPI_SWIGLU_FOLD, EPI_RES_STATS, EPI_RES_LN_STATS = 5, 6, 7, 8


@dataclass
class NomicConfig:
    vocab: int = 30528
    d: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    eps: float = 1e-12
    rope_base: float = 1000.0
    n_ctx: int = 2048
    type_vocab: int = 2

    @property
    def head_dim(self) -> int:
        return self.d // self.heads

    @classmethod
    def from_gguf(cls, g: GGUFFile) -> "NomicConfig":
        a = g.arch() or "nomic-bert"
        get = lambda k, d: g.get(f"{a}.{k}", d)  # noqa: E731
        tok = g.tensors.get("token_embd.weight")
        return cls(vocab=tok.shape[0] if tok else 30528, d=int(get("embedding_length", 768)),
                   layers=int(get("block_count", 12)), heads=int(get("attention.head_count", 12)),
                   ffn=int(get("feed_forward_length", 3072)), eps=float(get("attention.layer_norm_epsilon", 1e-12)),
                   rope_base=float(get("rope.freq_base", 1000.0)), n_ctx=int(get("context_length", 2048)))


def _lib():
    L = N.hip_lib()
    if not getattr(L, "_nomic_declared", False):
        P, c_long, c_int, c_float = ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_float
        L.nomic_gemm.argtypes = [c_int, P, c_long, P, c_long, c_long, c_int, c_int, P, c_long, P, c_long, P, P, c_int, P]
        L.nomic_gemm.restype = c_int
        L.nomic_gemm_ln.argtypes = [c_int, P, c_long, P, c_long, c_long, c_int, c_int, P, c_long, P, c_long, P, P,
                                    c_int, P, c_int, c_float, P, P, P, P, P, P]
        L.nomic_gemm_ln.restype = c_int
        L.nomic_gemm_res_ln.argtypes = [P, c_long, P, c_long, c_long, c_int, c_int, P, c_long, P, P, c_float, P,
                                        c_long, P]
        L.nomic_gemm_res_ln.restype = c_int
        L.nomic_gemm_res_ln_set_variant.argtypes = [c_int]
        L.nomic_gemm_res_ln_set_variant.restype = c_int
        L.nomic_row_stats.argtypes = [P, c_int, c_long, c_float, P, P]
        L.nomic_row_stats.restype = c_int
        L.nomic_gemm_set_variant.argtypes = [c_int]
        L.nomic_gemm_set_variant.restype = c_int
        L.nomic_attention_set_variant.argtypes = [c_int]
        L.nomic_attention_set_variant.restype = c_int
        L.nomic_embed_ln.argtypes = [P, c_long, P, P, P, P, c_float, P, P]
        L.nomic_embed_ln.restype = c_int
        L.nomic_layernorm.argtypes = [P, c_long, P, P, c_float, P, P]
        L.nomic_layernorm.restype = c_int
        L.nomic_attention.argtypes = [P, P, P, P, c_int, c_int, c_float, P]
        L.nomic_attention.restype = c_int
        L.nomic_mean_pool.argtypes = [P, P, c_int, P, c_int, N.Arena, P, P, P, P]
        L.nomic_mean_pool.restype = c_int
        L.nomic_dequant.argtypes = [c_int, P, c_long, P, P]
        L.nomic_dequant.restype = c_int
        L._nomic_declared = True
    return L


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: HIP launch failed ({rc})")


def _stream():
    return torch.cuda.current_stream().cuda_stream


# ================================================================ weights ==
GGUF_NAMES = {
    "tok": "token_embd.weight", "type": "token_types.weight",
    "emb_g": "token_embd_norm.weight", "emb_b": "token_embd_norm.bias",
}
LAYER_NAMES = {
    "wqkv": "attn_qkv.weight", "wo": "attn_output.weight",
    "ln1_g": "attn_output_norm.weight", "ln1_b": "attn_output_norm.bias",
    "wup": "ffn_up.weight", "wgate": "ffn_gate.weight", "wdown": "ffn_down.weight",
    "ln2_g": "layer_output_norm.weight", "ln2_b": "layer_output_norm.bias",
}


def random_weights(cfg: NomicConfig, seed: int = 0, std: float = 0.02) -> Dict[str, np.ndarray]:
    """Random-init fp32 weights in GGUF (numpy) orientation: linear = [out, in]."""
    rng = np.random.default_rng(seed)
    f = lambda *s: (rng.standard_normal(s) * std).astype(np.float32)  # noqa: E731
    w = {GGUF_NAMES["tok"]: f(cfg.vocab, cfg.d), GGUF_NAMES["type"]: f(cfg.type_vocab, cfg.d),
         GGUF_NAMES["emb_g"]: (1 + f(cfg.d) * 5).astype(np.float32), GGUF_NAMES["emb_b"]: f(cfg.d)}
    for i in range(cfg.layers):
        p = f"blk.{i}."
        w[p + "attn_qkv.weight"] = f(3 * cfg.d, cfg.d)
        w[p + "attn_output.weight"] = f(cfg.d, cfg.d)
        w[p + "attn_output_norm.weight"] = (1 + f(cfg.d) * 5).astype(np.float32)
        w[p + "attn_output_norm.bias"] = f(cfg.d)
        w[p + "ffn_up.weight"] = f(cfg.ffn, cfg.d)
        w[p + "ffn_gate.weight"] = f(cfg.ffn, cfg.d)
        w[p + "ffn_down.weight"] = f(cfg.d, cfg.ffn)
        w[p + "layer_output_norm.weight"] = (1 + f(cfg.d) * 5).astype(np.float32)
        w[p + "layer_output_norm.bias"] = f(cfg.d)
    return w


def write_gguf(path: str, cfg: NomicConfig, weights: Dict[str, np.ndarray], vocab: Optional[List[str]] = None,
               linear_type: str = "F16") -> None:
    """Write a nomic-bert GGUF (linears in `linear_type`, norms/embeddings F32/F16)."""
    w = GGUFWriter(path, "nomic-bert")
    a = "nomic-bert"
    w.add("general.name", "nomic-embed-text-v1.5 (random init)")
    w.add(f"{a}.context_length", cfg.n_ctx)
    w.add(f"{a}.embedding_length", cfg.d)
    w.add(f"{a}.feed_forward_length", cfg.ffn)
    w.add(f"{a}.attention.head_count", cfg.heads)
    w.add(f"{a}.attention.layer_norm_epsilon", float(cfg.eps))
    w.add(f"{a}.block_count", cfg.layers)
    w.add(f"{a}.rope.freq_base", float(cfg.rope_base))
    w.add(f"{a}.attention.causal", False)
    w.add(f"{a}.pooling_type", 1)
    if vocab is not None:
        w.add("tokenizer.ggml.model", "bert")
        w.add("tokenizer.ggml.tokens", vocab)
        w.add("tokenizer.ggml.token_type", [1] * len(vocab))
        ids = {t: i for i, t in enumerate(vocab)}
        for key, tok in (("bos", "[CLS]"), ("eos", "[SEP]"), ("seperator", "[SEP]"), ("unknown", "[UNK]"),
                         ("padding", "[PAD]")):
            if tok in ids:
                w.add(f"tokenizer.ggml.{key}_token_id", ids[tok])
    for name, arr in weights.items():
        lin = arr.ndim == 2 and not name.startswith("token_")
        w.add_tensor(name, arr, linear_type if lin else ("F16" if name == "token_embd.weight" else "F32"))
    w.write()


def pack_upgate(up: torch.Tensor, gate: torch.Tensor) -> torch.Tensor:
    """SWIGLU epilogue weight layout (nomic_api.h NOMIC_EPI_SWIGLU): per 16 outputs,
    16 up rows then 16 gate rows, so one MFMA lane holds up[o] and gate[o]."""
    F, d = up.shape
    return torch.stack([up.reshape(F // 16, 16, d), gate.reshape(F // 16, 16, d)], 1).reshape(2 * F, d)


_QKV_PERM = torch.cat([torch.arange(0, 16), torch.arange(32, 48), torch.arange(16, 32), torch.arange(48, 64)])


def pack_qkv(w: torch.Tensor) -> torch.Tensor:
    """ROPE epilogue weight layout (NOMIC_EPI_ROPE): the rows of every 64-wide head
    reordered [d0-15 | d32-47 | d16-31 | d48-63], so a NEOX pair (d, d+32) sits in one
    lane; the kernel writes the output back in the natural order."""
    n, d = w.shape
    return w.reshape(n // 64, 64, d)[:, _QKV_PERM.to(w.device)].reshape(n, d)


def fold_ln(w: torch.Tensor, g: torch.Tensor, b: torch.Tensor):
    """LayerNorm folded into the linear that consumes it: LN(h) w^T = rstd (h w'^T - mean c1) + c2
    with w' = w diag(g) (bf16), c1 = w' 1 and c2 = w b (fp32; c1 from the ROUNDED w', so the mean
    term cancels exactly what the GEMM accumulates).  w [N, K] in kernel (packed) row order."""
    wf = (w.float() * g.float()[None, :]).to(torch.bfloat16).contiguous()
    c1 = wf.float().sum(1).contiguous()
    c2 = (w.float() @ b.float()).contiguous()
    return wf, c1, c2


class NomicWeights:
    """Device-resident bf16 weights in kernel layout (plus the LN-folded copies the fused
    forward uses: ``wqkv_f`` folds the previous layer's output LN, ``wupgate_f`` this layer's
    attention-output LN)."""

    def __init__(self, cfg: NomicConfig, tensors: Dict[str, torch.Tensor], device="cuda"):
        self.cfg = cfg
        bf = lambda t: t.to(device=device, dtype=torch.bfloat16).contiguous()  # noqa: E731
        self.tok = bf(tensors[GGUF_NAMES["tok"]])
        self.type_row = bf(tensors[GGUF_NAMES["type"]][0])
        self.emb_g, self.emb_b = bf(tensors[GGUF_NAMES["emb_g"]]), bf(tensors[GGUF_NAMES["emb_b"]])
        self.layers = []
        for i in range(cfg.layers):
            p = f"blk.{i}."
            t = {k: tensors[p + v] for k, v in LAYER_NAMES.items()}
            self.layers.append({
                "wqkv": bf(pack_qkv(t["wqkv"])), "wo": bf(t["wo"]), "wupgate": bf(pack_upgate(t["wup"], t["wgate"])),
                "wdown": bf(t["wdown"]),
                "ln1_g": bf(t["ln1_g"]), "ln1_b": bf(t["ln1_b"]), "ln2_g": bf(t["ln2_g"]), "ln2_b": bf(t["ln2_b"]),
            })
        for i, lw in enumerate(self.layers):
            lw["wupgate_f"], lw["ug_c1"], lw["ug_c2"] = fold_ln(lw["wupgate"], lw["ln1_g"], lw["ln1_b"])
            if i > 0:
                prev = self.layers[i - 1]
                lw["wqkv_f"], lw["qkv_c1"], lw["qkv_c2"] = fold_ln(lw["wqkv"], prev["ln2_g"], prev["ln2_b"])

    @classmethod
    def from_numpy(cls, cfg, weights: Dict[str, np.ndarray], device="cuda"):
        return cls(cfg, {k: torch.from_numpy(v) for k, v in weights.items()}, device)

    @classmethod
    def from_gguf(cls, g: GGUFFile, cfg: Optional[NomicConfig] = None, device="cuda"):
        cfg = cfg or NomicConfig.from_gguf(g)
        L = _lib()
        out = {}
        for name, info in g.tensors.items():
            if info.ggml_type in DEVICE_DEQUANT:
                raw = torch.from_numpy(np.ascontiguousarray(g.raw(name))).to(device)
                dst = torch.empty(info.nelems, dtype=torch.bfloat16, device=device)
                _chk(L.nomic_dequant(info.ggml_type, raw.data_ptr(), info.nelems, dst.data_ptr(), _stream()),
                     f"dequant {name}")
                out[name] = dst.view(info.shape)
            else:
                out[name] = torch.from_numpy(dequant_host(g.raw(name), info.ggml_type, info.nelems)
                                             .reshape(info.shape)).to(device)
        return cls(cfg, out, device)


# ============================================================== reference ==
class NomicReference(torch.nn.Module):
    """Plain fp32 PyTorch nomic-bert forward (oracle for kernel numerics)."""

    def __init__(self, cfg: NomicConfig, weights: Dict[str, np.ndarray], device="cpu"):
        super().__init__()
        self.cfg = cfg
        self.w = {k: torch.from_numpy(np.asarray(v, np.float32)).to(device) for k, v in weights.items()}

    def rope(self, x, pos):  # x [T, H, 64]
        hd = self.cfg.head_dim
        inv = self.cfg.rope_base ** (-torch.arange(0, hd, 2, dtype=torch.float64, device=x.device) / hd)
        ang = pos[:, None].double() * inv[None, :]
        c, s = torch.cos(ang).float()[:, None, :], torch.sin(ang).float()[:, None, :]
        x1, x2 = x[..., : hd // 2], x[..., hd // 2:]
        return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)

    def forward(self, ids: torch.Tensor, cu: Sequence[int]) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        F = torch.nn.functional
        x = w["token_embd.weight"][ids] + w["token_types.weight"][0]
        x = F.layer_norm(x, (cfg.d,), w["token_embd_norm.weight"], w["token_embd_norm.bias"], cfg.eps)
        pos = torch.cat([torch.arange(cu[i + 1] - cu[i]) for i in range(len(cu) - 1)]).to(ids.device)
        H, hd = cfg.heads, cfg.head_dim
        for i in range(cfg.layers):
            p = f"blk.{i}."
            qkv = x @ w[p + "attn_qkv.weight"].T
            q, k, v = qkv.split(cfg.d, dim=1)
            q = self.rope(q.view(-1, H, hd), pos)
            k = self.rope(k.view(-1, H, hd), pos)
            v = v.view(-1, H, hd)
            outs = []
            for s in range(len(cu) - 1):
                a, b = cu[s], cu[s + 1]
                att = torch.einsum("qhd,khd->hqk", q[a:b], k[a:b]) / math.sqrt(hd)
                outs.append(torch.einsum("hqk,khd->qhd", att.softmax(-1), v[a:b]))
            o = torch.cat(outs).reshape(-1, cfg.d)
            x = F.layer_norm(o @ w[p + "attn_output.weight"].T + x, (cfg.d,), w[p + "attn_output_norm.weight"],
                             w[p + "attn_output_norm.bias"], cfg.eps)
            up = x @ w[p + "ffn_up.weight"].T
            gate = x @ w[p + "ffn_gate.weight"].T
            h = (up * F.silu(gate)) @ w[p + "ffn_down.weight"].T
            x = F.layer_norm(h + x, (cfg.d,), w[p + "layer_output_norm.weight"], w[p + "layer_output_norm.bias"],
                             cfg.eps)
        return torch.stack([x[cu[s]: cu[s + 1]].mean(0) for s in range(len(cu) - 1)])


# ================================================================ encoder ==
class Batch:
    """A packed varlen batch: token ids, sequence offsets, positions, q-blocks."""

    def __init__(self, seqs: Sequence[Sequence[int]], device="cuda", qblock: int = 128):
        lens = [len(s) for s in seqs]
        assert all(n > 0 for n in lens), "empty sequence"
        self.B = len(seqs)
        self.T = sum(lens)
        self.T_pad = (self.T + 127) // 128 * 128
        self.cu_host = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        self.max_len = max(lens)
        ids = np.zeros(self.T_pad, np.int32)
        ids[: self.T] = np.concatenate([np.asarray(s, np.int32) for s in seqs])
        pos = np.zeros(self.T_pad, np.int32)
        pos[: self.T] = np.concatenate([np.arange(n, dtype=np.int32) for n in lens])
        qb = np.asarray([(i, q0) for i, n in enumerate(lens) for q0 in range(0, n, qblock)], np.int32).reshape(-1)
        self.nqb = qb.size // 2
        self._ids_host, self._device, self._qblock, self._parts = ids, device, qblock, {}
        if str(device) == "cpu":
            self.ids, self.pos = torch.from_numpy(ids), torch.from_numpy(pos)
            self.cu, self.qblocks = torch.from_numpy(self.cu_host), torch.from_numpy(qb)
            return
        # one pinned staging buffer and ONE asynchronous host->device copy for ids | pos | cu | qblocks:
        # a pageable .to(device) blocks the host until every kernel queued before it has run, which
        # serialised the next batch's host work (tokenizer, packing) behind the current encoder
        # pass.  The caching host allocator keeps the pinned block until the copy has completed.
        parts = (ids, pos, self.cu_host, qb)
        span = [(p.size + 3) // 4 * 4 for p in parts]  # every part starts 16-B aligned
        host = torch.empty(sum(span), dtype=torch.int32, pin_memory=True)
        hv = host.numpy()
        o = 0
        for p, n in zip(parts, span):
            hv[o: o + p.size] = p
            o += n
        dev = host.to(device, non_blocking=True)
        o = 0
        views = []
        for p, n in zip(parts, span):
            views.append(dev[o: o + p.size])
            o += n
        self.ids, self.pos, self.cu, self.qblocks = views

    def split(self, parts: int):
        """[(sub-batch, first row)]: the documents cut into `parts` contiguous groups of about equal token
        counts, each a Batch of its own whose rows are rows [first, first + T) of this batch (cached)."""
        if parts in self._parts:
            return self._parts[parts]
        lens = np.diff(self.cu_host)
        cum = np.cumsum(lens)
        cuts = [0] + [int(np.searchsorted(cum, self.T * j / parts, side="left")) + 1 for j in range(1, parts)] + [self.B]
        out = []
        for j in range(parts):
            d0, d1 = cuts[j], cuts[j + 1]
            if d1 <= d0:
                continue
            r0, r1 = int(self.cu_host[d0]), int(self.cu_host[d1])
            seqs = [self._ids_host[self.cu_host[d]: self.cu_host[d + 1]].tolist() for d in range(d0, d1)]
            out.append((Batch(seqs, self._device, self._qblock), r0))
        self._parts[parts] = out
        return out


class NomicEncoder:
    """Batched bf16 forward on the gfx950 kernels (no torch compute in the hot path)."""

    def __init__(self, weights: NomicWeights, max_tokens: int = 1 << 17):
        self._split_streams = None
        self.w = weights
        self.cfg = weights.cfg
        self.L = _lib()
        cfg = self.cfg
        # RoPE table [n_pos][hd/2] of (cos, sin)
        npos = max(cfg.n_ctx, 8192)
        inv = cfg.rope_base ** (-np.arange(0, cfg.head_dim, 2, dtype=np.float64) / cfg.head_dim)
        ang = np.arange(npos, dtype=np.float64)[:, None] * inv[None, :]
        tab = np.stack([np.cos(ang), np.sin(ang)], axis=-1).astype(np.float32)
        self.rope = torch.from_numpy(tab.reshape(npos, -1)).cuda()
        self._ws_tokens = 0
        self._ensure(max_tokens)

    def _ensure(self, T_pad: int):
        if T_pad <= self._ws_tokens:
            return
        cfg = self.cfg
        e = dict(dtype=torch.bfloat16, device="cuda")
        self.x = torch.empty((T_pad, cfg.d), **e)
        self.h = torch.empty((T_pad, cfg.d), **e)
        self.attn = torch.empty((T_pad, cfg.d), **e)
        self.qkv = torch.empty((T_pad, 3 * cfg.d), **e)
        self.ffn = torch.empty((T_pad, cfg.ffn), **e)
        self.h2 = torch.empty((T_pad, cfg.d), **e)
        f = dict(dtype=torch.float32, device="cuda")
        self.part1 = torch.empty((T_pad, 2 * (cfg.d // 128)), **f)  # (mean, M2) per 128 columns of h1
        self.part2 = torch.empty((T_pad, 2 * (cfg.d // 128)), **f)  # ... of h2
        self._ws_tokens = T_pad

    def _gemm(self, mode, A, W, M, out, res=None, pos=None):
        N_, K = W.shape
        _chk(self.L.nomic_gemm(mode, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), M,
                               N_, K, out.data_ptr(), out.stride(0), res.data_ptr() if res is not None else None,
                               res.stride(0) if res is not None else 0, self.rope.data_ptr(),
                               pos.data_ptr() if pos is not None else None, 2 * self.cfg.d, _stream()), "gemm")

    def _gemm_ln(self, mode, A, W, M, out, res=None, pos=None, pin=None, c1=None, c2=None, ln=None, part=None):
        N_, K = W.shape
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        _chk(self.L.nomic_gemm_ln(mode, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), M, N_, K,
                                  out.data_ptr(), out.stride(0), ptr(res), res.stride(0) if res is not None else 0,
                                  self.rope.data_ptr(), ptr(pos), 2 * self.cfg.d, ptr(pin),
                                  pin.shape[1] // 2 if pin is not None else 0, self.cfg.eps, ptr(c1), ptr(c2),
                                  ptr(ln[0]) if ln else None, ptr(ln[1]) if ln else None, ptr(part), _stream()),
             f"gemm_ln({mode})")

    # Schedules of the post-LN layers (K15 / K16-down), all on hand-written kernels:
    #   "fused"  (default) residual GEMM + residual add + LayerNorm in one row-complete kernel
    #            (csrc/hip/gemm_rln.hip): x = LN(a W^T + x) in place, no separate LN pass;
    #   "split"  the residual GEMM (EPI_RESIDUAL) then the LayerNorm kernel (round-1 schedule);
    #   "folded" every post-LN folded into the neighbouring GEMMs (measured slower,
    #            profiles/r2_encoder_ln_fold.md).
    # NOMIC_SCHEDULE overrides; NOMIC_LN_FOLD=1 is the old spelling of "folded".
    schedule = os.environ.get("NOMIC_SCHEDULE", "folded" if os.environ.get("NOMIC_LN_FOLD", "0") != "0" else "fused")

    # NOMIC_SPLIT=N (N > 1): the batch's documents in N groups, each group's layer chain on its own
    # stream, issued layer by layer in turn, so one group's kernels fill the CUs another group's
    # kernel leaves idle (a GEMM's last partial wave of tiles, its prologue burst / epilogue tail)
    split_parts = int(os.environ.get("NOMIC_SPLIT", "1"))

    def hidden(self, b: Batch) -> torch.Tensor:
        """Final-layer hidden states [T, 768] (bf16) for a packed batch."""
        if self.split_parts > 1 and self.schedule == "fused" and b.B >= 2 * self.split_parts:
            return self._hidden_split(b, self.split_parts)
        if self.schedule == "folded":
            return self._hidden_folded(b)
        if self.schedule == "split":
            return self._hidden_unfused(b)
        if self.schedule != "fused":
            raise ValueError(f"unknown encoder schedule {self.schedule!r}")
        return self._hidden_fused(b)

    def _res_ln(self, A, W, M, x, g, beta):
        """x[:M] = LN(A W^T + x) * g + beta in place (row-complete MFMA kernel, gemm_rln.hip)."""
        N_, K = W.shape
        _chk(self.L.nomic_gemm_res_ln(A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), M, N_, K, x.data_ptr(),
                                      x.stride(0), g.data_ptr(), beta.data_ptr(), self.cfg.eps, x.data_ptr(),
                                      x.stride(0), _stream()), "gemm_res_ln")

    def _hidden_fused(self, b: Batch) -> torch.Tensor:
        """The shipped schedule: 5 kernels per layer, every one hand-written for gfx950 --
        QKV+RoPE GEMM, varlen attention, o-proj+residual+LN, up|gate+SwiGLU GEMM, down+residual+LN."""
        cfg, L, w = self.cfg, self.L, self.w
        assert b.max_len <= self.rope.shape[0]
        self._ensure(b.T_pad)
        s = _stream()
        T = b.T
        x, attn, qkv, ffn = self.x, self.attn, self.qkv, self.ffn
        _chk(L.nomic_embed_ln(b.ids.data_ptr(), T, w.tok.data_ptr(), w.type_row.data_ptr(), w.emb_g.data_ptr(),
                              w.emb_b.data_ptr(), cfg.eps, x.data_ptr(), s), "embed_ln")
        scale = 1.0 / math.sqrt(cfg.head_dim)
        for lw in w.layers:
            self._gemm(EPI_ROPE, x, lw["wqkv"], T, qkv, pos=b.pos)
            _chk(L.nomic_attention(qkv.data_ptr(), attn.data_ptr(), b.cu.data_ptr(), b.qblocks.data_ptr(), b.nqb,
                                   cfg.heads, scale, s), "attention")
            self._res_ln(attn, lw["wo"], T, x, lw["ln1_g"], lw["ln1_b"])
            self._gemm(EPI_SWIGLU, x, lw["wupgate"], T, ffn)
            self._res_ln(ffn, lw["wdown"], T, x, lw["ln2_g"], lw["ln2_b"])
        return x[:T]

    def _hidden_split(self, b: Batch, parts: int) -> torch.Tensor:
        """The fused schedule over `parts` document groups on their own streams (NOMIC_SPLIT); every
        group works on its own rows of the shared workspaces, so the hidden states land in rows [0, T)
        exactly as the one-stream forward leaves them."""
        cfg, L, w = self.cfg, self.L, self.w
        assert b.max_len <= self.rope.shape[0]
        self._ensure(b.T_pad)
        subs = b.split(parts)
        if self._split_streams is None or len(self._split_streams) < len(subs):
            self._split_streams = [torch.cuda.Stream() for _ in subs]
        cur = torch.cuda.current_stream()
        streams = self._split_streams[: len(subs)]
        for st in streams:
            st.wait_stream(cur)
        scale = 1.0 / math.sqrt(cfg.head_dim)
        views = []
        for (sb, r0), st in zip(subs, streams):
            views.append((sb, st, self.x[r0:], self.attn[r0:], self.qkv[r0:], self.ffn[r0:]))
        for sb, st, x, attn, qkv, ffn in views:
            with torch.cuda.stream(st):
                _chk(L.nomic_embed_ln(sb.ids.data_ptr(), sb.T, w.tok.data_ptr(), w.type_row.data_ptr(),
                                      w.emb_g.data_ptr(), w.emb_b.data_ptr(), cfg.eps, x.data_ptr(), st.cuda_stream),
                     "embed_ln")
        for lw in w.layers:
            for sb, st, x, attn, qkv, ffn in views:
                with torch.cuda.stream(st):
                    s_ = st.cuda_stream
                    T = sb.T
                    self._gemm(EPI_ROPE, x, lw["wqkv"], T, qkv, pos=sb.pos)
                    _chk(L.nomic_attention(qkv.data_ptr(), attn.data_ptr(), sb.cu.data_ptr(), sb.qblocks.data_ptr(),
                                           sb.nqb, cfg.heads, scale, s_), "attention")
                    self._res_ln(attn, lw["wo"], T, x, lw["ln1_g"], lw["ln1_b"])
                    self._gemm(EPI_SWIGLU, x, lw["wupgate"], T, ffn)
                    self._res_ln(ffn, lw["wdown"], T, x, lw["ln2_g"], lw["ln2_b"])
        for st in streams:
            cur.wait_stream(st)
        return self.x[: b.T]

    def _hidden_folded(self, b: Batch) -> torch.Tensor:
        """The forward with every post-LN folded into the GEMMs around it (K15): the residual GEMMs
        write raw sums h1 / h2 plus 128-column partial row statistics; the next projection combines
        them into (mean, rstd) per row in its prologue and runs on raw h against LN-folded weights,
        and the next residual GEMM normalises its residual operand on the fly.  One LayerNorm pass
        per forward (the final one, for pooling) instead of two per layer."""
        cfg, L, w = self.cfg, self.L, self.w
        assert b.max_len <= self.rope.shape[0]
        self._ensure(b.T_pad)
        s = _stream()
        T = b.T
        x, h1, h2, attn, qkv, ffn = self.x, self.h, self.h2, self.attn, self.qkv, self.ffn
        p1, p2 = self.part1, self.part2
        _chk(L.nomic_embed_ln(b.ids.data_ptr(), T, w.tok.data_ptr(), w.type_row.data_ptr(), w.emb_g.data_ptr(),
                              w.emb_b.data_ptr(), cfg.eps, x.data_ptr(), s), "embed_ln")
        scale = 1.0 / math.sqrt(cfg.head_dim)
        prev = None
        for lw in w.layers:
            if prev is None:
                self._gemm(EPI_ROPE, x, lw["wqkv"], T, qkv, pos=b.pos)
            else:
                self._gemm_ln(EPI_ROPE_FOLD, h2, lw["wqkv_f"], T, qkv, pos=b.pos, pin=p2, c1=lw["qkv_c1"],
                              c2=lw["qkv_c2"])
            _chk(L.nomic_attention(qkv.data_ptr(), attn.data_ptr(), b.cu.data_ptr(), b.qblocks.data_ptr(), b.nqb,
                                   cfg.heads, scale, s), "attention")
            if prev is None:
                self._gemm_ln(EPI_RES_STATS, attn, lw["wo"], T, h1, res=x, part=p1)
            else:
                self._gemm_ln(EPI_RES_LN_STATS, attn, lw["wo"], T, h1, res=h2, pin=p2,
                              ln=(prev["ln2_g"], prev["ln2_b"]), part=p1)
            self._gemm_ln(EPI_SWIGLU_FOLD, h1, lw["wupgate_f"], T, ffn, pin=p1, c1=lw["ug_c1"], c2=lw["ug_c2"])
            self._gemm_ln(EPI_RES_LN_STATS, ffn, lw["wdown"], T, h2, res=h1, pin=p1, ln=(lw["ln1_g"], lw["ln1_b"]),
                          part=p2)
            prev = lw
        _chk(L.nomic_layernorm(h2.data_ptr(), T, prev["ln2_g"].data_ptr(), prev["ln2_b"].data_ptr(), cfg.eps,
                               x.data_ptr(), s), "ln_final")
        return x[:T]

    def _hidden_unfused(self, b: Batch) -> torch.Tensor:
        """Split schedule: the residual GEMM, then a LayerNorm kernel (NOMIC_SCHEDULE=split)."""
        cfg, L, w = self.cfg, self.L, self.w
        assert b.max_len <= self.rope.shape[0]
        self._ensure(b.T_pad)
        s = _stream()
        T = b.T
        x, h, attn, qkv, ffn = self.x, self.h, self.attn, self.qkv, self.ffn
        _chk(L.nomic_embed_ln(b.ids.data_ptr(), T, w.tok.data_ptr(), w.type_row.data_ptr(), w.emb_g.data_ptr(),
                              w.emb_b.data_ptr(), cfg.eps, x.data_ptr(), s), "embed_ln")
        scale = 1.0 / math.sqrt(cfg.head_dim)
        for lw in w.layers:
            self._gemm(EPI_ROPE, x, lw["wqkv"], T, qkv, pos=b.pos)
            _chk(L.nomic_attention(qkv.data_ptr(), attn.data_ptr(), b.cu.data_ptr(), b.qblocks.data_ptr(), b.nqb,
                                   cfg.heads, scale, s), "attention")
            self._gemm(EPI_RESIDUAL, attn, lw["wo"], T, h, res=x)
            _chk(L.nomic_layernorm(h.data_ptr(), T, lw["ln1_g"].data_ptr(), lw["ln1_b"].data_ptr(), cfg.eps,
                                   x.data_ptr(), s), "ln1")
            self._gemm(EPI_SWIGLU, x, lw["wupgate"], T, ffn)
            self._gemm(EPI_RESIDUAL, ffn, lw["wdown"], T, h, res=x)
            _chk(L.nomic_layernorm(h.data_ptr(), T, lw["ln2_g"].data_ptr(), lw["ln2_b"].data_ptr(), cfg.eps,
                                   x.data_ptr(), s), "ln2")
        return x[:T]

    def embed(self, b: Batch, normalize: bool = False, arena=None, slots: Optional[torch.Tensor] = None,
              hashes: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
        """Mean-pooled [B, 768] fp32; with arena+slots the vectors are also written
        into the arena slots under the seqlock (returns (vectors, status))."""
        with trace_range("nomic.encoder"):
            self.hidden(b)
        if out is None:
            out = torch.empty((b.B, self.cfg.d), dtype=torch.float32, device="cuda")
        status = None
        desc = N.Arena()
        if arena is not None:
            desc = arena.desc
            status = torch.empty(b.B, dtype=torch.int32, device="cuda")
        _chk(self.L.nomic_mean_pool(self.x.data_ptr(), b.cu.data_ptr(), b.B, out.data_ptr(), int(normalize), desc,
                                    slots.data_ptr() if slots is not None else None,
                                    hashes.data_ptr() if hashes is not None else None,
                                    status.data_ptr() if status is not None else None, _stream()), "mean_pool")
        return (out, status) if arena is not None else out

    def flops(self, b: Batch) -> float:
        cfg = self.cfg
        lin = 2 * b.T * cfg.d * (3 * cfg.d + cfg.d + 2 * cfg.ffn + cfg.ffn) * cfg.layers
        lens = np.diff(b.cu_host)
        att = 4 * float((lens.astype(np.float64) ** 2).sum()) * cfg.d * cfg.layers
        return lin + att


def smoke_embed(arena, keys: torch.Tensor) -> None:
    """Tiny end-to-end check used by __graft_entry__.smoke(): random-init
    encoder embeds a few sequences straight into the arena slots."""
    cfg = NomicConfig(layers=2)
    w = NomicWeights.from_numpy(cfg, random_weights(cfg, seed=1))
    enc = NomicEncoder(w, max_tokens=1024)
    n = min(4, keys.shape[0])
    rng = np.random.default_rng(0)
    b = Batch([rng.integers(0, cfg.vocab, size=7 + 5 * i).tolist() for i in range(n)])
    st, idx = arena.meta("find", keys[:n])
    from ..parallel.sharded import GpuShard
    hashes = GpuShard(arena).hash_keys(keys[:n])
    vec, status = enc.embed(b, arena=arena, slots=idx, hashes=hashes)
    torch.cuda.synchronize()
    assert (status == 0).all(), status
    st2, back = arena.get_embeddings(keys[:n])
    assert torch.equal(back, vec), "slot vectors differ from pooled output"
    assert torch.isfinite(vec).all()
