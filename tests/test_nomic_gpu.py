"""Numerics of the gfx950 Nomic-BERT kernels against plain fp32 PyTorch."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (a - b).norm().item() / max(b.norm().item(), 1e-12)


@pytest.fixture(scope="module")
def L0():
    import torch  # noqa: F401
    from libsplinter_amd.models.nomic import _lib
    return _lib()


@pytest.fixture(params=[256, 128, 0], ids=["gemm256", "gemm128", "gemm_auto"])
def L(L0, request):
    """Run each GEMM numerics test on every kernel (NOMIC_GEMM 256 / 128) and the auto choice (a mode
    or shape the chosen kernel does not take runs on the next one that does)."""
    prev = L0.nomic_gemm_set_variant(request.param)
    yield L0
    L0.nomic_gemm_set_variant(prev)


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 768, 768), (1000, 2304, 768), (257, 768, 3072),
                                   (4096, 2304, 768)])
def test_gemm_store_and_residual(L, M, N, K):
    import torch
    from libsplinter_amd.models.nomic import _chk, _stream
    torch.manual_seed(0)
    Mp = (M + 127) // 128 * 128
    A = torch.randn(Mp, K, device="cuda").bfloat16()
    W = torch.randn(N, K, device="cuda").bfloat16() * 0.05
    R = torch.randn(Mp, N, device="cuda").bfloat16()
    ref = A[:M].float() @ W.float().T
    out = torch.zeros(Mp, N, device="cuda", dtype=torch.bfloat16)
    _chk(L.nomic_gemm(0, A.data_ptr(), K, W.data_ptr(), K, M, N, K, out.data_ptr(), N, None, 0, None, None, 0,
                      _stream()), "gemm")
    assert _rel(out[:M].float(), ref) < 5e-3
    assert (out[M:] == 0).all(), "rows past M must not be written"
    _chk(L.nomic_gemm(1, A.data_ptr(), K, W.data_ptr(), K, M, N, K, out.data_ptr(), N, R.data_ptr(), N, None, None,
                      0, _stream()), "gemm")
    assert _rel(out[:M].float(), ref + R[:M].float()) < 5e-3
    outf = torch.zeros(Mp, N, device="cuda")
    _chk(L.nomic_gemm(4, A.data_ptr(), K, W.data_ptr(), K, M, N, K, outf.data_ptr(), N, None, 0, None, None, 0,
                      _stream()), "gemm")
    assert _rel(outf[:M], ref) < 1e-5


def test_gemm_asymmetric_identity(L):
    """A = I with an asymmetric W catches a transposed C write (guide §3)."""
    import torch
    from libsplinter_amd.models.nomic import _chk, _stream
    K = 128
    A = torch.eye(128, K, device="cuda").bfloat16()
    W = (torch.arange(128 * K, device="cuda", dtype=torch.float32).reshape(128, K) % 97).bfloat16()
    out = torch.zeros(128, 128, device="cuda")
    _chk(L.nomic_gemm(4, A.data_ptr(), K, W.data_ptr(), K, 128, 128, K, out.data_ptr(), 128, None, 0, None, None, 0,
                      _stream()), "gemm")
    assert torch.equal(out, W.float().T)


def test_gemm_swiglu_and_rope(L):
    import torch
    from libsplinter_amd.models.nomic import NomicEncoder, NomicReference, _chk, _stream
    torch.manual_seed(1)
    M, K, F = 200, 768, 3072
    Mp = 256
    x = torch.randn(Mp, K, device="cuda").bfloat16()
    up = torch.randn(F, K, device="cuda") * 0.03
    gate = torch.randn(F, K, device="cuda") * 0.03
    from libsplinter_amd.models.nomic import pack_qkv, pack_upgate
    ug = pack_upgate(up, gate).bfloat16()
    out = torch.empty(Mp, F, device="cuda", dtype=torch.bfloat16)
    _chk(L.nomic_gemm(2, x.data_ptr(), K, ug.data_ptr(), K, M, 2 * F, K, out.data_ptr(), F, None, 0, None, None, 0,
                      _stream()), "swiglu")
    xf = x[:M].float()
    ref = (xf @ up.bfloat16().float().T) * torch.nn.functional.silu(xf @ gate.bfloat16().float().T)
    assert _rel(out[:M].float(), ref) < 1e-2
    # RoPE epilogue vs reference rotation
    wqkv = (torch.randn(3 * K, K, device="cuda") * 0.03).bfloat16()
    pos = torch.randint(0, 2000, (Mp,), device="cuda", dtype=torch.int32)
    from libsplinter_amd.models.nomic import NomicConfig
    cfg = NomicConfig()
    inv = cfg.rope_base ** (-np.arange(0, 64, 2) / 64)
    ang = np.arange(8192)[:, None] * inv[None, :]
    tab = torch.from_numpy(np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32).reshape(8192, -1)).cuda()
    qkv = torch.empty(Mp, 3 * K, device="cuda", dtype=torch.bfloat16)
    wpk = pack_qkv(wqkv)
    _chk(L.nomic_gemm(3, x.data_ptr(), K, wpk.data_ptr(), K, M, 3 * K, K, qkv.data_ptr(), 3 * K, None, 0,
                      tab.data_ptr(), pos.data_ptr(), 2 * K, _stream()), "rope")
    raw = xf @ wqkv.float().T
    ref_m = NomicReference(cfg, {}, "cuda")
    q = ref_m.rope(raw[:, :K].reshape(M, 12, 64), pos[:M].long()).reshape(M, K)
    k = ref_m.rope(raw[:, K:2 * K].reshape(M, 12, 64), pos[:M].long()).reshape(M, K)
    ref = torch.cat([q, k, raw[:, 2 * K:]], 1)
    assert _rel(qkv[:M].float(), ref) < 1e-2


def test_gemm256_swiglu_epilogue(L0):
    """The 256^2 kernel's SwiGLU epilogue against fp32, with a partial last row tile (M = 1000)."""
    import torch
    from libsplinter_amd.models.nomic import _chk, _stream, pack_upgate
    torch.manual_seed(3)
    M, K, F = 1000, 768, 1024
    x = torch.randn(1024, K, device="cuda").bfloat16()
    up = torch.randn(F, K, device="cuda") * 0.03
    gate = torch.randn(F, K, device="cuda") * 0.03
    ug = pack_upgate(up, gate).bfloat16()
    out = torch.full((1024, F), 7.0, device="cuda", dtype=torch.bfloat16)
    L = L0
    pv = L.nomic_gemm_set_variant(256)
    try:
        _chk(L.nomic_gemm(2, x.data_ptr(), K, ug.data_ptr(), K, M, 2 * F, K, out.data_ptr(), F, None, 0, None, None,
                          0, _stream()), "swiglu256")
        torch.cuda.synchronize()
    finally:
        L.nomic_gemm_set_variant(pv)
    xf = x[:M].float()
    ref = (xf @ up.bfloat16().float().T) * torch.nn.functional.silu(xf @ gate.bfloat16().float().T)
    assert _rel(out[:M].float(), ref) < 1e-2
    assert (out[M:].float() == 7.0).all()  # rows past M are never written


def test_gemm_layernorm_fold_modes(L):
    """Post-LN folded into the GEMMs (nomic_api.h modes 5-8) vs fp32 torch: residual sums with
    128-column partial statistics -> (mean, rstd) per row; the residual normalised on the fly;
    SwiGLU and RoPE projections of LN(h) computed from raw h against LN-folded weights."""
    import torch
    from libsplinter_amd.models.nomic import (NomicConfig, NomicReference, _chk, _stream, fold_ln, pack_qkv,
                                              pack_upgate)
    F_ = torch.nn.functional
    torch.manual_seed(3)
    M, K, F, eps = 300, 768, 3072, 1e-12
    Mp = 384
    nul = None

    def gemm_ln(mode, A, W, out, res=None, pos=None, tab=None, pin=None, c1=None, c2=None, g=None, b=None,
                part=None):
        p = lambda t: t.data_ptr() if t is not None else nul  # noqa: E731
        _chk(L.nomic_gemm_ln(mode, A.data_ptr(), A.stride(0), W.data_ptr(), W.stride(0), M, W.shape[0], W.shape[1],
                             out.data_ptr(), out.stride(0), p(res), res.stride(0) if res is not None else 0, p(tab),
                             p(pos), 2 * K, p(pin), K // 128 if pin is not None else 0, eps, p(c1), p(c2), p(g), p(b),
                             p(part), _stream()), f"mode {mode}")

    def partials(t):  # (mean, M2) per 128 columns, as a stats-mode producer writes them
        v = t.float().reshape(t.shape[0], -1, 128)
        mu = v.mean(2)
        return torch.stack([mu, ((v - mu[..., None]) ** 2).sum(2)], 2).reshape(t.shape[0], -1).contiguous()

    # raw residual stream with a per-row offset (the fold must cancel the mean exactly)
    h = (torch.randn(Mp, K, device="cuda") * 1.5 + torch.randn(Mp, 1, device="cuda") * 2).bfloat16()
    g = (1 + 0.3 * torch.randn(K, device="cuda")).bfloat16()
    bb = (0.1 * torch.randn(K, device="cuda")).bfloat16()
    hf = h[:M].float()
    xln = F_.layer_norm(hf, (K,), g.float(), bb.float(), eps)
    ph = partials(h)

    # 7: out = A W^T + R, partial stats -> row_stats
    A = torch.randn(Mp, K, device="cuda").bfloat16()
    W = (torch.randn(K, K, device="cuda") * 0.03).bfloat16()
    out = torch.zeros(Mp, K, device="cuda", dtype=torch.bfloat16)
    part = torch.zeros(Mp, 2 * (K // 128), device="cuda")
    gemm_ln(7, A, W, out, res=h, part=part)
    ref = A[:M].float() @ W.float().T + hf
    assert _rel(out[:M].float(), ref) < 5e-3
    assert (out[M:] == 0).all()
    st_got = torch.zeros(Mp, 2, device="cuda")
    _chk(L.nomic_row_stats(part.data_ptr(), K // 128, M, eps, st_got.data_ptr(), _stream()), "row_stats")
    o = out[:M].float()
    torch.testing.assert_close(st_got[:M, 0], o.mean(1), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(st_got[:M, 1], torch.rsqrt(o.var(1, unbiased=False) + eps), rtol=1e-3, atol=1e-4)

    # 8: out = A W^T + LN(h) with h's statistics
    gemm_ln(8, A, W, out, res=h, pin=ph, g=g, b=bb, part=part)
    assert _rel(out[:M].float(), A[:M].float() @ W.float().T + xln) < 5e-3

    # 6: SwiGLU of LN(h) from raw h and folded weights
    up = (torch.randn(F, K, device="cuda") * 0.03).bfloat16()
    gate = (torch.randn(F, K, device="cuda") * 0.03).bfloat16()
    wf, c1, c2 = fold_ln(pack_upgate(up, gate), g, bb)
    ffn = torch.empty(Mp, F, device="cuda", dtype=torch.bfloat16)
    gemm_ln(6, h, wf, ffn, pin=ph, c1=c1, c2=c2)
    ref = (xln @ up.float().T) * F_.silu(xln @ gate.float().T)
    assert _rel(ffn[:M].float(), ref) < 1.5e-2

    # 5: RoPE'd qkv of LN(h)
    cfg = NomicConfig()
    wqkv = (torch.randn(3 * K, K, device="cuda") * 0.03).bfloat16()
    pos = torch.randint(0, 2000, (Mp,), device="cuda", dtype=torch.int32)
    inv = cfg.rope_base ** (-np.arange(0, 64, 2) / 64)
    ang = np.arange(8192)[:, None] * inv[None, :]
    tab = torch.from_numpy(np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32).reshape(8192, -1)).cuda()
    wf, c1, c2 = fold_ln(pack_qkv(wqkv), g, bb)
    qkv = torch.empty(Mp, 3 * K, device="cuda", dtype=torch.bfloat16)
    gemm_ln(5, h, wf, qkv, pos=pos, tab=tab, pin=ph, c1=c1, c2=c2)
    raw = xln @ wqkv.float().T
    rm = NomicReference(cfg, {}, "cuda")
    q = rm.rope(raw[:, :K].reshape(M, 12, 64), pos[:M].long()).reshape(M, K)
    k = rm.rope(raw[:, K:2 * K].reshape(M, 12, 64), pos[:M].long()).reshape(M, K)
    assert _rel(qkv[:M].float(), torch.cat([q, k, raw[:, 2 * K:]], 1)) < 1.5e-2
    # a fold mode without its operands is refused, never launched
    assert L.nomic_gemm_ln(6, h.data_ptr(), K, wf.data_ptr(), K, M, 3 * K, K, qkv.data_ptr(), 3 * K, None, 0, None,
                           None, 0, None, 0, eps, None, None, None, None, None, _stream()) != 0


@pytest.mark.parametrize("variant", [13, 6])
@pytest.mark.parametrize("spike", [False, True])
def test_attention_varlen(L0, variant, spike):
    L = L0
    import torch
    from libsplinter_amd.models.nomic import Batch, _chk, _stream
    torch.manual_seed(2)
    lens = [1, 17, 64, 65, 127, 128, 129, 200, 513]
    b = Batch([[0] * n for n in lens], qblock=128)
    T = b.T
    qkv = torch.randn(b.T_pad, 3 * 768, device="cuda").bfloat16()
    if spike:  # a late key that dominates one query's row: forces the online-max rescale path
        s0 = int(b.cu_host[8])
        qkv[s0 + 3, :64] = 4.0
        qkv[s0 + 450, 768:768 + 64] = 4.0
    out = torch.zeros(b.T_pad, 768, device="cuda", dtype=torch.bfloat16)
    prev = L.nomic_attention_set_variant(variant)
    try:
        _chk(L.nomic_attention(qkv.data_ptr(), out.data_ptr(), b.cu.data_ptr(), b.qblocks.data_ptr(), b.nqb, 12,
                               1 / 8.0, _stream()), "attn")
    finally:
        L.nomic_attention_set_variant(prev)
    q, k, v = qkv[:T].float().split(768, 1)
    refs = []
    for i in range(len(lens)):
        a, e = b.cu_host[i], b.cu_host[i + 1]
        qq, kk, vv = (t[a:e].reshape(-1, 12, 64) for t in (q, k, v))
        p = (torch.einsum("qhd,khd->hqk", qq, kk) / 8.0).softmax(-1)
        refs.append(torch.einsum("hqk,khd->qhd", p, vv).reshape(-1, 768))
    assert _rel(out[:T].float(), torch.cat(refs)) < 1e-2


def test_layernorm_and_embed(L0):
    L = L0
    import torch
    from libsplinter_amd.models.nomic import _chk, _stream
    torch.manual_seed(3)
    T = 777
    x = torch.randn(T, 768, device="cuda").bfloat16() * 3 + 1
    g = (1 + 0.1 * torch.randn(768, device="cuda")).bfloat16()
    bb = (0.1 * torch.randn(768, device="cuda")).bfloat16()
    out = torch.empty_like(x)
    _chk(L.nomic_layernorm(x.data_ptr(), T, g.data_ptr(), bb.data_ptr(), 1e-12, out.data_ptr(), _stream()), "ln")
    ref = torch.nn.functional.layer_norm(x.float(), (768,), g.float(), bb.float(), 1e-12)
    assert _rel(out.float(), ref) < 5e-3
    tok = torch.randn(1000, 768, device="cuda").bfloat16()
    trow = torch.randn(768, device="cuda").bfloat16()
    ids = torch.randint(0, 1000, (T,), device="cuda", dtype=torch.int32)
    _chk(L.nomic_embed_ln(ids.data_ptr(), T, tok.data_ptr(), trow.data_ptr(), g.data_ptr(), bb.data_ptr(), 1e-12,
                          out.data_ptr(), _stream()), "embed")
    ref = torch.nn.functional.layer_norm(tok[ids.long()].float() + trow.float(), (768,), g.float(), bb.float(), 1e-12)
    assert _rel(out.float(), ref) < 5e-3


@pytest.fixture(params=[222, 232], ids=["rln222", "rln232"])
def rln_variant(L0, request):
    """Both row-complete residual+LN kernel forms (the residual added in the epilogue, and during
    the K loop at K = 768)."""
    prev = L0.nomic_gemm_res_ln_set_variant(request.param)
    yield request.param
    L0.nomic_gemm_res_ln_set_variant(prev)


@pytest.mark.parametrize("M,K", [(128, 768), (300, 768), (1, 3072), (257, 3072), (32768, 768), (4100, 3072)])
def test_gemm_residual_layernorm_row_complete(L0, M, K, rln_variant):
    """nomic_gemm_res_ln (gemm_rln.hip): x = LN(A W^T + x) * g + b in place, against fp32, with a
    row tail (M % 128 != 0), a single row, the shipped 32768-row o-proj shape and the down shape;
    rows past M untouched; asymmetric operands and non-trivial gamma/beta."""
    import torch
    from libsplinter_amd.models.nomic import _chk, _stream
    torch.manual_seed(M + K)
    N = 768
    Mp = (M + 127) // 128 * 128 + 128
    A = (torch.rand(Mp, K, device="cuda") * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) * (1.0 / math.sqrt(K))).bfloat16()
    X = (torch.randn(Mp, N, device="cuda") + torch.linspace(-2, 2, N, device="cuda")).bfloat16()
    g = (1 + 0.3 * torch.randn(N, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(N, device="cuda")).bfloat16()
    ref = torch.nn.functional.layer_norm(A[:M].float() @ W.float().T + X[:M].float(), (N,), g.float(), b.float(),
                                         1e-12)
    tail = X[M:].clone()
    _chk(L0.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, N, K, X.data_ptr(), N, g.data_ptr(),
                              b.data_ptr(), 1e-12, X.data_ptr(), N, _stream()), "gemm_res_ln")
    torch.cuda.synchronize()
    assert _rel(X[:M].float(), ref) < 6e-3
    assert (X[:M].float() - ref).abs().max().item() < 0.08
    assert torch.equal(X[M:], tail), "rows past M must not be written"
    # out-of-place with a separate residual gives the same bits
    X2 = torch.empty_like(X)
    R = (torch.randn(Mp, N, device="cuda")).bfloat16()
    ref2 = torch.nn.functional.layer_norm(A[:M].float() @ W.float().T + R[:M].float(), (N,), g.float(), b.float(),
                                          1e-12)
    _chk(L0.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, N, K, R.data_ptr(), N, g.data_ptr(),
                              b.data_ptr(), 1e-12, X2.data_ptr(), N, _stream()), "gemm_res_ln")
    assert _rel(X2[:M].float(), ref2) < 6e-3
    # shapes the kernel does not take are refused, not launched
    assert L0.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, 512, K, X.data_ptr(), N, g.data_ptr(),
                                b.data_ptr(), 1e-12, X.data_ptr(), N, _stream()) != 0
    assert L0.nomic_gemm_res_ln(A.data_ptr(), K, W.data_ptr(), K, M, N, 48, X.data_ptr(), N, g.data_ptr(),
                                b.data_ptr(), 1e-12, X.data_ptr(), N, _stream()) != 0


@pytest.mark.parametrize("schedule", ["fused", "split", "folded"])
def test_encoder_matches_fp32_reference(schedule):
    import torch
    from libsplinter_amd.models.nomic import (Batch, NomicConfig, NomicEncoder, NomicReference, NomicWeights,
                                              random_weights)
    cfg = NomicConfig(layers=3)
    w = random_weights(cfg, seed=5)
    enc = NomicEncoder(NomicWeights.from_numpy(cfg, w), max_tokens=4096)
    enc.schedule = schedule
    rng = np.random.default_rng(0)
    seqs = [rng.integers(0, cfg.vocab, size=n).tolist() for n in (5, 40, 129, 300)]
    b = Batch(seqs)
    got = enc.embed(b)
    ref = NomicReference(cfg, w, "cuda")(torch.from_numpy(np.concatenate(seqs)).cuda().long(), b.cu_host.tolist())
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=1)
    assert cos.min().item() > 0.999, cos
    assert _rel(got, ref) < 3e-2


def test_gguf_roundtrip_device_dequant(tmp_path):
    import torch
    from libsplinter_amd.models.gguf import GGUFFile
    from libsplinter_amd.models.nomic import NomicConfig, NomicWeights, random_weights, write_gguf
    cfg = NomicConfig(layers=1, vocab=512)
    w = random_weights(cfg, seed=9)
    for lt in ("F16", "Q8_0", "Q4_0"):
        p = str(tmp_path / f"m_{lt}.gguf")
        write_gguf(p, cfg, w, vocab=[f"t{i}" for i in range(cfg.vocab)], linear_type=lt)
        g = GGUFFile(p)
        assert NomicConfig.from_gguf(g).layers == 1
        nw = NomicWeights.from_gguf(g)
        host = torch.from_numpy(g.to_numpy_f32("blk.0.attn_qkv.weight")).cuda()
        from libsplinter_amd.models.nomic import pack_qkv
        assert torch.equal(nw.layers[0]["wqkv"].float(), pack_qkv(host).bfloat16().float()), lt  # kernel layout
        assert _rel(host, torch.from_numpy(w["blk.0.attn_qkv.weight"]).cuda()) < (0.2 if lt == "Q4_0" else 2e-2)


def test_pool_writes_into_arena_slots(uniq):
    import torch
    from libsplinter_amd.ops.arena import HbmArena, pack_keys, pack_values
    from libsplinter_amd.models.nomic import smoke_embed
    a = HbmArena.create(uniq, slots=256, max_val=64, embeddings=True)
    try:
        K = pack_keys([f"doc{i}" for i in range(8)], 16)
        V, Ln = pack_values([b"x"] * 8, 16)
        a.set(K, V, Ln)
        smoke_embed(a, K)
    finally:
        a.close()


def _random_blocks(ggml_type, nblocks, rng):
    """Random GGML blocks of `ggml_type` with finite f16 scales: every bit of the quant payload
    varies, so the device decoder is checked against the host reference on the whole layout."""
    from libsplinter_amd.models.gguf import TYPE_BY_ID
    _, _, bsz = TYPE_BY_ID[ggml_type]
    raw = rng.integers(0, 256, size=(nblocks, bsz), dtype=np.uint8)

    def f16(cols, lo, hi):
        v = rng.uniform(lo, hi, size=(nblocks, len(cols) // 2)).astype(np.float16)
        raw[:, cols] = v.view(np.uint8).reshape(nblocks, -1)

    if ggml_type == 2:        # Q4_0: d | qs[16]
        f16([0, 1], -0.05, 0.05)
    elif ggml_type == 3:      # Q4_1: d, m | qs[16]
        f16([0, 1, 2, 3], -0.05, 0.05)
    elif ggml_type == 8:      # Q8_0: d | qs[32]
        f16([0, 1], -0.01, 0.01)
    elif ggml_type == 12:     # Q4_K: d, dmin | scales[12] | qs[128]
        f16([0, 1, 2, 3], 0.0, 0.01)
    elif ggml_type == 14:     # Q6_K: ql[128] qh[64] scales[16] | d
        f16([208, 209], -0.01, 0.01)
    return raw


def test_device_dequant_matches_host_reference_all_types():
    """nomic_dequant (HIP) vs gguf.dequant_host (numpy, written from the GGML block layouts:
    ggml-quants.c dequantize_row_q4_0/q4_1/q8_0/q4_K/q6_K) on random blocks, every device type.
    Real nomic-embed-text Q4 GGUFs are Q4_K_M (Q4_K + Q6_K tensors)."""
    import torch
    from libsplinter_amd.models.gguf import dequant_host
    from libsplinter_amd.models import nomic
    from libsplinter_amd import _native as N
    from libsplinter_amd.ops.arena import _stream
    L = nomic._lib()
    del N
    rng = np.random.default_rng(5)
    for t, per in ((2, 32), (3, 32), (8, 32), (12, 256), (14, 256)):
        nb = 4096 if per == 32 else 512
        raw = _random_blocks(t, nb, rng)
        n = nb * per
        ref = dequant_host(raw.reshape(-1), t, n)
        src = torch.from_numpy(raw.reshape(-1).copy()).cuda()
        dst = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        rc = L.nomic_dequant(t, src.data_ptr(), n, dst.data_ptr(), _stream())
        assert rc == 0, (t, rc)
        torch.cuda.synchronize()
        want = torch.from_numpy(ref)
        got = dst.float().cpu()
        # the device may contract d*s*q - dmin*m into an FMA: at most one bf16 step apart
        tol = want.abs() * 2.0 ** -7 + 1e-7
        assert ((got - want).abs() <= tol).all(), (t, (got - want).abs().max().item())
        assert (got == want.to(torch.bfloat16).float()).float().mean() > 0.99, t
    for t, make in ((0, lambda x: x.astype(np.float32)), (1, lambda x: x.astype(np.float16)),
                    (30, lambda x: (x.astype(np.float32).view(np.uint32) >> 16).astype(np.uint16))):
        x = rng.standard_normal(8192).astype(np.float32)
        raw = make(x).view(np.uint8)
        ref = dequant_host(raw, t, 8192)
        src = torch.from_numpy(raw.copy()).cuda()
        dst = torch.empty(8192, dtype=torch.bfloat16, device="cuda")
        assert L.nomic_dequant(t, src.data_ptr(), 8192, dst.data_ptr(), _stream()) == 0
        torch.cuda.synchronize()
        assert torch.equal(dst.float().cpu(), torch.from_numpy(ref).to(torch.bfloat16).float()), t
    # K-quant lengths must be whole 256-element superblocks
    bad = torch.zeros(144, dtype=torch.uint8, device="cuda")
    out = torch.empty(32, dtype=torch.bfloat16, device="cuda")
    assert L.nomic_dequant(12, bad.data_ptr(), 32, out.data_ptr(), _stream()) != 0


@pytest.mark.parametrize("schedule", ["fused", "split"])
def test_full_encoder_shipped_shape_matches_fp32(schedule):
    """The shipped shape: all 12 layers, 64 documents x 512 tokens (the bench batch), bf16 gfx950
    kernels vs an fp32 torch forward of the same random-init nomic-bert weights; "fused" is the
    shipped schedule (the row-complete residual+LN kernel), "split" the residual-epilogue GEMM +
    LayerNorm kernel pair."""
    import torch
    from libsplinter_amd.models.nomic import (Batch, NomicConfig, NomicEncoder, NomicReference, NomicWeights,
                                              random_weights)
    cfg = NomicConfig(layers=12)
    w = random_weights(cfg, seed=11)
    b_docs, seq = 64, 512
    enc = NomicEncoder(NomicWeights.from_numpy(cfg, w), max_tokens=b_docs * seq)
    enc.schedule = schedule
    rng = np.random.default_rng(1)
    seqs = [rng.integers(1000, cfg.vocab, size=seq).tolist() for _ in range(b_docs)]
    b = Batch(seqs)
    got = enc.embed(b)
    ref_model = NomicReference(cfg, w, "cuda")
    ids = torch.from_numpy(np.concatenate(seqs)).cuda().long()
    with torch.no_grad():
        ref = ref_model(ids, b.cu_host.tolist())
    cos = torch.nn.functional.cosine_similarity(got.float(), ref.float(), dim=1)
    assert cos.min().item() > 0.999, cos.min().item()
    assert _rel(got, ref) < 3e-2
