"""splainference: the reference label state machine (WAITING -> SERVICING -> READY),
streaming append, truncation at max_val_sz, system prompt; and (GPU) the MFMA
decoder path against the CPU torch path of the same weights."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WAITING, SERVICING, READY = 0x1000000000000000, 0x2000000000000000, 0x4000000000000000


def test_state_machine_cpu(uniq):
    from libsplinter_amd import Store, unlink
    s = Store.create(uniq, slots=128, max_val=512, embeddings=False)
    try:
        s.set("req", "hello there")
        s.set_label("req", WAITING)
        s.set("long", "x" * 400)  # prompt + completion overflow 512 B -> truncation path
        s.set_label("long", WAITING)
        s.set("other", "not a request")
        s.set("sys", "be brief")
        r = subprocess.run([sys.executable, "-m", "libsplinter_amd.daemons.splainference", "--oneshot",
                            "--random-init", "--device", "cpu", "--max-tokens", "64", "--system-prompt-key", "sys",
                            uniq, "none.gguf", "7"], cwd=ROOT, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        v = s.get("req")
        assert v.startswith(b"<system>\nbe brief\n<user>\nhello there\n<assistant>\n")
        assert len(v) > len(b"<system>\nbe brief\n<user>\nhello there\n<assistant>\n")
        b = s.snapshot("req")["bloom"]
        assert b & READY and not b & (WAITING | SERVICING)
        assert len(s.get("long")) <= 512 and s.snapshot("long")["bloom"] & READY
        assert not s.snapshot("other")["bloom"] & READY
        dbg = s.get("__debug").decode()
        assert "[DONE]: Completion written to key: req" in dbg
    finally:
        s.close()
        unlink(uniq)


@pytest.mark.gpu
@pytest.mark.parametrize("kv_heads,heads,d", [(8, 8, 512), (2, 8, 512), (2, 4, 512), (1, 2, 512), (8, 8, 768)])
def test_decoder_hip_matches_cpu(kv_heads, heads, d):
    """GPU forward (prefill, a continuation prefill over the live cache, then one decode step)
    against the fp32 CPU model; heads 4 gives head dim 128 (dec_attn_prefill_kv<128>); head dim
    256 runs prefill on SDPA and decode on dec_attn_decode, head dim 96 both on SDPA."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    cfg = DecoderConfig(layers=2, kv_heads=kv_heads, heads=heads, d=d)
    gpu = CausalLM.random(cfg, seed=3, device="cuda")
    cpu = CausalLM.random(cfg, seed=3, device="cpu")
    ids = [256] + list(b"the quick brown fox")
    lg, lc = gpu.forward(ids).cpu(), cpu.forward(ids)
    rel = (lg - lc).norm() / lc.norm()
    assert rel < 3e-2, float(rel)
    # a second prompt chunk continuing the cache (pos > 0: the new queries see the old keys)
    more = list(b" jumps over the lazy dog, again and again")
    lg, lc = gpu.forward(more).cpu(), cpu.forward(more)
    assert (lg - lc).norm() / lc.norm() < 3e-2
    # one decode step through the KV cache
    lg2, lc2 = gpu.forward([65]).cpu(), cpu.forward([65])
    assert (lg2 - lc2).norm() / lc2.norm() < 3e-2
    assert torch.argmax(lg2) == torch.argmax(lc2) or (lg2 - lc2).abs().max() < 0.05


@pytest.mark.gpu
def test_decoder_rmsnorm_rope_kernels_vs_fp32():
    """dec_rmsnorm / dec_rope (csrc/hip/decoder_kernels.hip) against fp32 torch references."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    cfg = DecoderConfig(layers=1)
    m = CausalLM.random(cfg, seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    for d in (cfg.d, 4096):  # register-resident rows and the wide-row second pass
        x = torch.randn((37, d), device="cuda", generator=g).to(torch.bfloat16)
        w = torch.randn((d,), device="cuda", generator=g)
        m.cfg.eps = 1e-5
        got = m._rms(x, w).float()
        xf = x.float()
        ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w
        assert (got - ref).abs().max() <= 2e-2 * ref.abs().max(), d
    hd, H, KVH = cfg.head_dim, cfg.heads, cfg.kv_heads
    n, pos0 = 19, 5
    ld = cfg.d + 2 * KVH * hd
    qkv = torch.randn((n, ld), device="cuda", generator=g).to(torch.bfloat16)
    before = qkv.clone()
    assert m.L.dec_rope(qkv.data_ptr(), ld, n, cfg.d + KVH * hd, hd, pos0, m.cos.data_ptr(), m.sin.data_ptr(),
                        None) == 0
    torch.cuda.synchronize()
    pos = torch.arange(pos0, pos0 + n, device="cuda")
    q = before[:, : cfg.d].reshape(n, H, hd).float()
    k = before[:, cfg.d: cfg.d + KVH * hd].reshape(n, KVH, hd).float()

    def rope(t):
        c, s = m.cos[pos][:, None, :], m.sin[pos][:, None, :]
        x1, x2 = t[..., 0::2], t[..., 1::2]
        return torch.stack([x1 * c - x2 * s, x1 * s + x2 * c], -1).flatten(-2)

    ref = torch.cat([rope(q).reshape(n, -1), rope(k).reshape(n, -1), before[:, cfg.d + KVH * hd:].float()], 1)
    assert (qkv.float() - ref).abs().max() < 3e-2
    assert torch.equal(qkv[:, cfg.d + KVH * hd:], before[:, cfg.d + KVH * hd:])  # v untouched


@pytest.mark.gpu
@pytest.mark.parametrize("hd,H,KVH", [(128, 32, 8), (64, 8, 8), (128, 16, 2), (256, 8, 1), (64, 16, 8), (192, 8, 4)])
def test_decoder_attn_decode_kernel_vs_fp32(hd, H, KVH):
    """dec_attn_decode (csrc/hip/decoder_kernels.hip) against an fp32 softmax(q k^T) v reference,
    cache lengths on both sides of the 64-key chunk and 256-key workgroup boundaries; past 512 keys
    the split-L (flash-decoding) kernels + combine, also driven by the device-side length with a
    larger capacity (empty splits)."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(7)
    n_ctx = 5000
    kv = torch.randn((2, n_ctx, KVH, hd), device="cuda", generator=g).to(torch.bfloat16)
    q = torch.randn((H * hd,), device="cuda", generator=g).to(torch.bfloat16)
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    # (length, device-side length, capacity): up to 512 keys the grouped short-cache kernel, also driven by a
    # device-side length under a small capacity (a graph-captured step of a short context)
    for L, dev_len, cap in ((1, False, 0), (63, False, 0), (64, False, 0), (65, False, 0), (257, False, 0),
                            (512, False, 0), (1100, False, 0), (4097, False, 0), (5000, False, 0), (1, True, n_ctx),
                            (700, True, n_ctx), (5000, True, n_ctx), (1, True, 512), (300, True, 512),
                            (512, True, 512)):
        out = torch.full((H * hd,), float("nan"), device="cuda").to(torch.bfloat16)
        if dev_len:
            st[0] = L - 1
            assert m.L.dec_attn_decode_st(q.data_ptr(), kv[0].data_ptr(), kv[1].data_ptr(), KVH * hd, cap, H, KVH,
                                          hd, hd ** -0.5, out.data_ptr(), st.data_ptr(), None) == 0
        else:
            assert m.L.dec_attn_decode(q.data_ptr(), kv[0].data_ptr(), kv[1].data_ptr(), KVH * hd, L, H, KVH, hd,
                                       hd ** -0.5, out.data_ptr(), None) == 0
        torch.cuda.synchronize()
        qf = q.float().reshape(H, hd)
        kf = kv[0, :L].float().repeat_interleave(H // KVH, 1)  # [L, H, hd]
        vf = kv[1, :L].float().repeat_interleave(H // KVH, 1)
        p = torch.softmax(torch.einsum("hd,lhd->hl", qf, kf) * hd ** -0.5, -1)
        ref = torch.einsum("hl,lhd->hd", p, vf).reshape(-1)
        err = (out.float() - ref).abs().max()
        assert err < 2e-2 * max(1.0, ref.abs().max().item()), (L, dev_len, float(err))


def test_decoder_kv_cache_matches_full_recompute_cpu():
    """Prefill + token-by-token decode through the preallocated KV cache (GQA: 8 q heads over
    2 kv heads) gives the logits of one full forward over the same tokens."""
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=2, heads=8, kv_heads=2), seed=3, device="cpu")
    ids = [256] + list(b"hello world")
    full = m.forward(ids + [65, 66])
    m.reset()
    m.forward(ids)
    m.forward([65])
    inc = m.forward([66])
    assert (full - inc).abs().max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("H,KVH,n", [(8, 8, 300), (8, 2, 129), (12, 4, 64)])
def test_decoder_prefill_attention_causal_vs_fp32(H, KVH, n):
    """dec_attn_prefill (k_attn2<CAUSAL>, grouped-query) against fp32 causal softmax(q k^T) v."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    hd = 64
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn((n, (H + 2 * KVH) * hd), device="cuda", generator=g).to(torch.bfloat16)
    out = torch.full((n, H * hd), float("nan"), device="cuda").to(torch.bfloat16)
    cu = torch.tensor([0, n], dtype=torch.int32, device="cuda")
    qb = torch.tensor([v for q0 in range(0, n, 128) for v in (0, q0)], dtype=torch.int32, device="cuda")
    assert m.L.dec_attn_prefill(qkv.data_ptr(), out.data_ptr(), cu.data_ptr(), qb.data_ptr(), qb.numel() // 2, H, KVH,
                                hd ** -0.5, None) == 0
    torch.cuda.synchronize()
    q = qkv[:, : H * hd].float().reshape(n, H, hd)
    k = qkv[:, H * hd:(H + KVH) * hd].float().reshape(n, KVH, hd).repeat_interleave(H // KVH, 1)
    v = qkv[:, (H + KVH) * hd:].float().reshape(n, KVH, hd).repeat_interleave(H // KVH, 1)
    s = torch.einsum("qhd,khd->hqk", q, k) * hd ** -0.5
    s = s.masked_fill(torch.ones(n, n, dtype=torch.bool, device="cuda").triu(1), float("-inf"))
    ref = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(n, -1)
    assert (out.float() - ref).abs().max() < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize("hd,H,KVH", [(64, 8, 2), (128, 32, 8), (128, 4, 4)])
def test_decoder_prefill_kv_causal_vs_fp32(hd, H, KVH):
    """dec_attn_prefill_kv (k_prefill_attn<hd>): n new queries at absolute positions pos0 .. pos0+n-1
    over cache rows 0 .. pos0+n-1, against fp32 causal softmax(q k^T) v; chunk sizes across the
    128-row q-block and the key-tile boundaries, fresh (pos0 = 0) and continuation prompts."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(9)
    n_ctx = 1024
    kv = torch.randn((2, n_ctx, KVH, hd), device="cuda", generator=g).to(torch.bfloat16)
    for n, pos0 in ((2, 0), (129, 0), (300, 0), (5, 37), (64, 200), (257, 511), (33, 990)):
        ldq = (H + 2 * KVH) * hd  # q inside a fused q|k|v row, as the QKV GEMM writes it
        qkv = torch.randn((n, ldq), device="cuda", generator=g).to(torch.bfloat16)
        out = torch.full((n, H * hd), float("nan"), device="cuda").to(torch.bfloat16)
        assert m.L.dec_attn_prefill_kv(qkv.data_ptr(), ldq, kv[0].data_ptr(), kv[1].data_ptr(), KVH * hd, n, pos0, H,
                                       KVH, hd, hd ** -0.5, out.data_ptr(), H * hd, None) == 0
        torch.cuda.synchronize()
        L = pos0 + n
        q = qkv[:, : H * hd].float().reshape(n, H, hd)
        k = kv[0, :L].float().repeat_interleave(H // KVH, 1)
        v = kv[1, :L].float().repeat_interleave(H // KVH, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) * hd ** -0.5
        qpos = torch.arange(pos0, L, device="cuda")[:, None]
        s = s.masked_fill(torch.arange(L, device="cuda")[None, :] > qpos, float("-inf"))
        ref = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(n, -1)
        err = (out.float() - ref).abs().max().item()
        assert err < 3e-2, (n, pos0, err)
    assert m.L.dec_attn_prefill_kv(qkv.data_ptr(), ldq, kv[0].data_ptr(), kv[1].data_ptr(), KVH * hd, 4, 0, H, KVH, 96,
                                   1.0, out.data_ptr(), H * hd, None) != 0  # head dim 96: refused


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", [(512, 1536), (1536, 512), (4096, 200)])
def test_dec_gemv_modes_vs_fp32(K, N):
    """dec_gemv (M = 1 projections of a decode step): store / residual / SwiGLU / fp32, with and
    without the fused RMSNorm, against fp32 torch."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    from libsplinter_amd.models.nomic import pack_upgate
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(K, device="cuda", generator=g).to(torch.bfloat16)
    W = (torch.randn((N, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    rw = torch.rand(K, device="cuda", generator=g) + 0.5
    res = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    xf = x.float()
    xn = (xf * torch.rsqrt(xf.pow(2).mean() + 1e-5) * rw).to(torch.bfloat16).float()
    for rms in (False, True):
        xin = xn if rms else xf
        for mode in (0, 1, 4):
            out = torch.empty(N, device="cuda", dtype=torch.float32 if mode == 4 else torch.bfloat16)
            assert m.L.dec_gemv(mode, x.data_ptr(), rw.data_ptr() if rms else None, 1e-5, W.data_ptr(), N, K,
                                res.data_ptr(), out.data_ptr(), None) == 0
            torch.cuda.synchronize()
            ref = W.float() @ xin + (res.float() if mode == 1 else 0)
            assert (out.float() - ref).abs().max() < 2e-2 * max(1.0, ref.abs().max().item()), (rms, mode)
    if N % 32 == 0:
        up = W[: N // 2]
        gate = (torch.randn((N // 2, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        ug = pack_upgate(up, gate).contiguous()
        out = torch.empty(N // 2, device="cuda", dtype=torch.bfloat16)
        assert m.L.dec_gemv(2, x.data_ptr(), None, 0.0, ug.data_ptr(), N, K, None, out.data_ptr(), None) == 0
        torch.cuda.synchronize()
        u, gg = up.float() @ xf, gate.float() @ xf
        ref = u * torch.nn.functional.silu(gg)
        assert (out.float() - ref).abs().max() < 2e-2 * max(1.0, ref.abs().max().item())


def _q4_host_dequant(q, sm):
    """Host decoder of the Q4G32 planes (decoder_kernels.hip): nibble 2j low / 2j+1 high of byte j,
    one bf16 (d, m) pair per 32-k group, w = d q + m."""
    import torch
    qi = q.to(torch.int32)
    nib = torch.stack([qi & 15, qi >> 4], -1).reshape(q.shape[0], -1).float()
    smi = sm.to(torch.int64) & 0xFFFFFFFF
    d = ((smi & 0xFFFF) << 16).to(torch.int32).view(torch.float32)
    m = ((smi >> 16) << 16).to(torch.int32).view(torch.float32)
    return nib * d.repeat_interleave(32, 1) + m.repeat_interleave(32, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", [(512, 1536), (1536, 512), (11008, 96)])
def test_q4_quant_dequant_and_gemv_q4_vs_fp32(K, N):
    """Q4G32 weights: dec_q4_quantize stays within half a grid step of every weight, dec_q4_dequant
    equals the host decoder of the planes, and dec_gemv_q4 (store / residual / fp32 / SwiGLU, with
    and without the fused RMSNorm) matches fp32 torch over the dequantised weights."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig, Q4Weight
    from libsplinter_amd.models.nomic import pack_upgate
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(12)
    W = (torch.randn((N, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    qw = Q4Weight.quantize(m.L, W)
    torch.cuda.synchronize()
    deq_host = _q4_host_dequant(qw.q, qw.sm)
    deq = qw.dequant(m.L)
    torch.cuda.synchronize()
    assert torch.allclose(deq.float(), deq_host, rtol=2 ** -8, atol=1e-7)
    Wg = W.float().reshape(N, K // 32, 32)
    step = ((Wg.amax(-1) - Wg.amin(-1)) / 15).repeat_interleave(32, 1)
    err = (deq_host - W.float()).abs()
    assert bool((err <= step * 0.6 + 1e-6).all()), float((err / step).max())
    x = torch.randn(K, device="cuda", generator=g).to(torch.bfloat16)
    rw = torch.rand(K, device="cuda", generator=g) + 0.5
    res = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    xf = x.float()
    xn = (xf * torch.rsqrt(xf.pow(2).mean() + 1e-5) * rw).to(torch.bfloat16).float()
    for rms in (False, True):
        xin = xn if rms else xf
        for mode in (0, 1, 4):
            out = torch.empty(N, device="cuda", dtype=torch.float32 if mode == 4 else torch.bfloat16)
            assert m.L.dec_gemv_q4(mode, x.data_ptr(), rw.data_ptr() if rms else None, 1e-5, qw.q.data_ptr(),
                                   qw.sm.data_ptr(), N, K, res.data_ptr(), out.data_ptr(), None) == 0
            torch.cuda.synchronize()
            ref = deq_host @ xin + (res.float() if mode == 1 else 0)
            tol = (1e-3 if mode == 4 else 1e-2) * max(1.0, ref.abs().max().item())
            assert (out.float() - ref).abs().max() < tol, (rms, mode, (out.float() - ref).abs().max().item())
    if N % 32 == 0:
        gate = (torch.randn((N // 2, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        ug = Q4Weight.quantize(m.L, pack_upgate(W[: N // 2], gate).contiguous())
        out = torch.empty(N // 2, device="cuda", dtype=torch.bfloat16)
        assert m.L.dec_gemv_q4(2, x.data_ptr(), None, 0.0, ug.q.data_ptr(), ug.sm.data_ptr(), N, K, None,
                               out.data_ptr(), None) == 0
        torch.cuda.synchronize()
        y = _q4_host_dequant(ug.q, ug.sm) @ xf
        yg = y.reshape(-1, 2, 16)
        u, gg = yg[:, 0].reshape(-1), yg[:, 1].reshape(-1)
        ref = u * torch.nn.functional.silu(gg)
        assert (out.float() - ref).abs().max() < 1e-2 * max(1.0, ref.abs().max().item())


def _q8_host_dequant(q, sm):
    """Host decoder of the Q8G32 planes: one byte u per weight, bf16 (d, m) per 32-k group, w = d u + m."""
    import torch
    smi = sm.to(torch.int64) & 0xFFFFFFFF
    d = ((smi & 0xFFFF) << 16).to(torch.int32).view(torch.float32)
    m = ((smi >> 16) << 16).to(torch.int32).view(torch.float32)
    return q.float() * d.repeat_interleave(32, 1) + m.repeat_interleave(32, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N", [(512, 1536), (4096, 96)])
def test_q8_quant_dequant_and_gemv_q8_vs_fp32(K, N):
    """Q8G32 weights (the >4-bit tensors of a mostly-4-bit GGUF): quantisation within half a 1/255
    grid step, dequant equal to the host decoder, and dec_gemv_q8 in every mode against fp32."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig, Q8Weight
    from libsplinter_amd.models.nomic import pack_upgate
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(13)
    W = (torch.randn((N, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    qw = Q8Weight.quantize(m.L, W)
    torch.cuda.synchronize()
    assert qw.nbytes() * 8 == N * K * 9  # 1.125 B per weight
    deq_host = _q8_host_dequant(qw.q, qw.sm)
    deq = qw.dequant(m.L)
    torch.cuda.synchronize()
    assert torch.allclose(deq.float(), deq_host, rtol=2 ** -8, atol=1e-7)
    Wg = W.float().reshape(N, K // 32, 32)
    step = ((Wg.amax(-1) - Wg.amin(-1)) / 255).repeat_interleave(32, 1)
    err = (deq_host - W.float()).abs()
    assert bool((err <= step * 0.6 + 2e-6).all()), float((err / step).max())
    x = torch.randn(K, device="cuda", generator=g).to(torch.bfloat16)
    rw = torch.rand(K, device="cuda", generator=g) + 0.5
    res = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    xf = x.float()
    xn = (xf * torch.rsqrt(xf.pow(2).mean() + 1e-5) * rw).to(torch.bfloat16).float()
    for rms in (False, True):
        xin = xn if rms else xf
        for mode in (0, 1, 4):
            out = torch.empty(N, device="cuda", dtype=torch.float32 if mode == 4 else torch.bfloat16)
            assert m.L.dec_gemv_q8(mode, x.data_ptr(), rw.data_ptr() if rms else None, 1e-5, qw.q.data_ptr(),
                                   qw.sm.data_ptr(), N, K, res.data_ptr(), out.data_ptr(), None) == 0
            torch.cuda.synchronize()
            ref = deq_host @ xin + (res.float() if mode == 1 else 0)
            tol = (1e-3 if mode == 4 else 1e-2) * max(1.0, ref.abs().max().item())
            assert (out.float() - ref).abs().max() < tol, (rms, mode)
    if N % 32 == 0:
        gate = (torch.randn((N // 2, K), device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        ug = Q8Weight.quantize(m.L, pack_upgate(W[: N // 2], gate).contiguous())
        out = torch.empty(N // 2, device="cuda", dtype=torch.bfloat16)
        assert m.L.dec_gemv_q8(2, x.data_ptr(), None, 0.0, ug.q.data_ptr(), ug.sm.data_ptr(), N, K, None,
                               out.data_ptr(), None) == 0
        torch.cuda.synchronize()
        yg = (_q8_host_dequant(ug.q, ug.sm) @ xf).reshape(-1, 2, 16)
        u, gg = yg[:, 0].reshape(-1), yg[:, 1].reshape(-1)
        ref = u * torch.nn.functional.silu(gg)
        assert (out.float() - ref).abs().max() < 1e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.gpu
def test_from_gguf_mixed_q4_q6k_keeps_wide_tensors_at_8_bits(tmp_path):
    """A Q4_K_M-shaped file (Q4_K projections, Q6_K ffn_down / attn_v / output): the Q6_K tensors
    load as Q8Weight, the rest as Q4Weight, and decode steps through both GEMVs track the bf16 model
    of the same dequantised tensors."""
    import numpy as np
    import torch
    from libsplinter_amd.models.decoder import (CausalLM, DecodeEngine, DecoderConfig, Q4Weight, Q8Weight,
                                                random_decoder_weights)
    from libsplinter_amd.models.gguf import GGUFFile, GGUFWriter
    cfg = DecoderConfig(vocab=384, d=256, layers=2, heads=4, kv_heads=2, ffn=512, n_ctx=256)
    w = random_decoder_weights(cfg, seed=5)
    path = str(tmp_path / "mixed.gguf")
    gw = GGUFWriter(path, "llama")
    for k, v in (("embedding_length", cfg.d), ("block_count", cfg.layers), ("attention.head_count", cfg.heads),
                 ("attention.head_count_kv", cfg.kv_heads), ("feed_forward_length", cfg.ffn),
                 ("context_length", cfg.n_ctx)):
        gw.add(f"llama.{k}", v)
    for n, a in w.items():
        wide = n.endswith(("ffn_down.weight", "attn_v.weight")) or n == "output.weight"
        gw.add_tensor(n, a, ("Q6_K" if wide else "Q4_K") if a.ndim == 2 and n != "token_embd.weight" else "F32")
    gw.write()
    m, _ = CausalLM.from_gguf(path, device="cuda")
    assert m.quant == "q4"
    lw = m.layers[0]
    assert isinstance(lw["down"], Q8Weight) and isinstance(lw["qkv"], Q8Weight) and isinstance(m.head, Q8Weight)
    assert type(lw["o"]) is Q4Weight and type(lw["ug"]) is Q4Weight
    g = GGUFFile(path)
    ref = CausalLM(m.cfg, {n: torch.from_numpy(np.ascontiguousarray(g.to_numpy_f32(n))) for n in g.tensors},
                   device="cuda")
    ids = [256] + list(b"mixed precision")
    eng = DecodeEngine(m, use_graph=False)
    eng.first_token(ids)
    ref.forward(ids)
    for t in (72, 101, 108):
        eng.st[1] = t
        eng._step()
        torch.cuda.synchronize()
        m.pos += 1
        r = ref.forward([t])
        got = eng.logits[: cfg.vocab]
        assert (got - r).norm() / r.norm() < 0.1


@pytest.mark.gpu
def test_decode_engine_q4_matches_eager_and_bf16():
    """A 4-bit model: DecodeEngine steps (dec_gemv_q4) give the logits of the eager forward (the MFMA
    GEMM over dequantised weights), and the 4-bit logits stay close to the bf16 model's; the
    projections occupy 0.625 B per weight."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecodeEngine, DecoderConfig, Q4Weight
    cfg = DecoderConfig(layers=2, kv_heads=2)
    eager = CausalLM.random(cfg, seed=4, device="cuda", quant="q4")
    mdl = CausalLM.random(cfg, seed=4, device="cuda", quant="q4")
    full = CausalLM.random(cfg, seed=4, device="cuda")
    lw = mdl.layers[0]
    assert isinstance(lw["down"], Q4Weight) and isinstance(mdl.head, Q4Weight)
    assert lw["down"].nbytes() * 16 == cfg.d * cfg.ffn * 10
    eng = DecodeEngine(mdl, use_graph=True)
    ids = [256] + list(b"prefill prompt of the test")
    eng.first_token(ids)
    eager.forward(ids)
    ref_bf16 = full.forward(ids)
    for t in (72, 101, 108, 108, 111):
        eng.st[1] = t
        eng._step()
        torch.cuda.synchronize()
        mdl.pos += 1
        ref = eager.forward([t])
        got = eng.logits[: cfg.vocab]
        assert (got - ref).norm() / ref.norm() < 3e-2
        ref_bf16 = full.forward([t])
        assert (got - ref_bf16).norm() / ref_bf16.norm() < 0.3


@pytest.mark.gpu
def test_dec_sample_nucleus_temperature_distribution():
    """dec_sample: greedy at tiny temperature, never outside the top-p nucleus, and draw
    frequencies that follow the renormalised tempered nucleus distribution."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    V = 384
    p = torch.tensor([0.4, 0.25, 0.15, 0.08, 0.05] + [0.07 / (V - 5)] * (V - 5), dtype=torch.float64)
    perm = torch.randperm(V, generator=torch.Generator().manual_seed(3))
    logits = torch.empty(V, dtype=torch.float64)
    logits[perm] = p.log()
    lg = logits.float().cuda()
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    host = torch.zeros(1, dtype=torch.int32, pin_memory=True)

    def draw(top_p, temp, n):
        out = []
        for _ in range(n):
            assert m.L.dec_sample(lg.data_ptr(), V, None, top_p, temp, 1234, st.data_ptr(), 0, host.data_ptr(),
                                  None) == 0
            torch.cuda.synchronize()
            out.append(int(host[0]))
        return out

    assert set(draw(1.0, 1e-4, 20)) == {int(perm[0])}
    toks = draw(0.9, 0.7, 3000)
    nucleus = [int(perm[i]) for i in range(4)]  # 0.4 + 0.25 + 0.15 + 0.08 = 0.88 < 0.9 -> 5 tokens
    nucleus.append(int(perm[4]))
    assert set(toks) <= set(nucleus)
    q = p[:5] ** (1 / 0.7)
    q = q / q.sum()
    for i in range(5):
        f = toks.count(int(perm[i])) / len(toks)
        assert abs(f - float(q[i])) < 0.04, (i, f, float(q[i]))


@pytest.mark.gpu
@pytest.mark.parametrize("V", [50000, 128256])
def test_dec_sample_multiblock_distribution(V):
    """dec_sample_ws past 4096 tokens (the 64-block k_sb_* chain): greedy at tiny temperature,
    never outside the top-p nucleus, tempered nucleus frequencies, with the top tokens scattered
    over different blocks; top_p = 1 keeps every token eligible."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    p = torch.tensor([0.4, 0.25, 0.15, 0.08, 0.05] + [0.07 / (V - 5)] * (V - 5), dtype=torch.float64)
    perm = torch.randperm(V, generator=torch.Generator().manual_seed(5))
    logits = torch.empty(V, dtype=torch.float64)
    logits[perm] = p.log()
    lg = logits.float().cuda()
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    ws = torch.empty(m.L.dec_sample_ws_floats(), dtype=torch.float32, device="cuda")

    def draw(top_p, temp, n):
        out = []
        for _ in range(n):
            assert m.L.dec_sample_ws(lg.data_ptr(), V, None, top_p, temp, 4321, st.data_ptr(), 0, host.data_ptr(),
                                     ws.data_ptr(), None) == 0
            torch.cuda.synchronize()
            out.append(int(host[0]))
        return out

    assert set(draw(1.0, 1e-4, 10)) == {int(perm[0])}
    assert set(draw(0.9, 1e-4, 10)) == {int(perm[0])}
    toks = draw(0.9, 0.7, 2000)
    nucleus = [int(perm[i]) for i in range(5)]
    assert set(toks) <= set(nucleus)
    q = p[:5] ** (1 / 0.7)
    q = q / q.sum()
    for i in range(5):
        f = toks.count(int(perm[i])) / len(toks)
        assert abs(f - float(q[i])) < 0.04, (i, f, float(q[i]))
    wide = draw(1.0, 1.0, 400)  # whole vocabulary eligible: the 7 % tail shows up
    assert any(t not in nucleus for t in wide)


@pytest.mark.gpu
def test_decode_engine_steps_match_eager_forward():
    """A decode step of DecodeEngine (GEMVs, RoPE + KV append, device-state attention) gives the
    logits of the eager forward through the MFMA GEMMs, token by token (teacher forcing)."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecodeEngine, DecoderConfig
    cfg = DecoderConfig(layers=2, kv_heads=2)
    eager = CausalLM.random(cfg, seed=4, device="cuda")
    mdl = CausalLM.random(cfg, seed=4, device="cuda")
    eng = DecodeEngine(mdl, use_graph=False)
    ids = [256] + list(b"prefill prompt of the test")
    eng.first_token(ids)
    eager.forward(ids)
    for t in (72, 101, 108, 108, 111):
        eng.st[1] = t
        eng._step()
        torch.cuda.synchronize()
        mdl.pos += 1
        ref = eager.forward([t])
        got = eng.logits[: cfg.vocab]
        assert (got - ref).norm() / ref.norm() < 3e-2


@pytest.mark.gpu
def test_decode_engine_crosses_split_boundary():
    """Graph-replayed decode steps across the 512-key boundary where DecodeEngine switches from the
    single-workgroup attention graph to the split-L graph (capacity 2048) match the eager forward."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecodeEngine, DecoderConfig
    cfg = DecoderConfig(layers=2, kv_heads=2, n_ctx=2048)
    eager = CausalLM.random(cfg, seed=6, device="cuda")
    mdl = CausalLM.random(cfg, seed=6, device="cuda")
    eng = DecodeEngine(mdl, use_graph=True)
    ids = [256] + [int(b) for b in (b"abcdefghij" * 51)[:505]]
    eng.first_token(ids)
    eager.forward(ids)
    for i in range(16):  # cache lengths 507 .. 522
        t = 97 + i % 26
        eng.st[1] = t
        eng._step()
        torch.cuda.synchronize()
        mdl.pos += 1
        ref = eager.forward([t])
        got = eng.logits[: cfg.vocab]
        assert (got - ref).norm() / ref.norm() < 3e-2, i
    assert len(eng.graphs) == 2


@pytest.mark.gpu
def test_decode_engine_graph_replay_equals_eager_launches():
    """The captured HIP graph replays exactly the launched step: same seed and prompt give the
    same tokens; prints per-token latency of both."""
    import time
    from libsplinter_amd.models.decoder import ByteTokenizer, CausalLM, DecodeEngine, DecoderConfig
    cfg = DecoderConfig()
    mask = ByteTokenizer().printable_mask(cfg.vocab)
    ids = [256] + list(b"<user>\nhello\n<assistant>\n")
    res = {}
    for graph in (False, True):
        eng = DecodeEngine(CausalLM.random(cfg, seed=2, device="cuda"), seed=99, mask=mask, use_graph=graph)
        toks = [eng.first_token(ids)]
        eng.next_token()  # warm-up / capture outside the timed loop
        toks.append(int(eng.host_tok[0]))
        t0 = time.perf_counter()
        for _ in range(40):
            toks.append(eng.next_token())
        res[graph] = (toks, (time.perf_counter() - t0) / 40 * 1e3)
    print(f"decode ms/token: launches {res[False][1]:.3f}, graph {res[True][1]:.3f}")
    assert res[True][0] == res[False][0]
    assert all(32 <= t < 127 or t in (10, 257) for t in res[True][0])


@pytest.mark.gpu
def test_state_machine_gpu_decode_engine(uniq):
    """The daemon on the GPU path (prefill on MFMA + causal HIP attention, graph-replayed decode
    steps with the device sampler): label machine and streamed completion as on the CPU."""
    from libsplinter_amd import Store, unlink
    s = Store.create(uniq, slots=128, max_val=512, embeddings=False)
    try:
        s.set("req", "hello there")
        s.set_label("req", WAITING)
        r = subprocess.run([sys.executable, "-m", "libsplinter_amd.daemons.splainference", "--oneshot",
                            "--random-init", "--device", "cuda", "--max-tokens", "48", uniq, "none.gguf", "7"],
                           cwd=ROOT, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        v = s.get("req")
        head = b"<user>\nhello there\n<assistant>\n"
        assert v.startswith(head) and len(v) > len(head)
        assert all(32 <= c < 127 or c == 10 for c in v[len(head):])
        b = s.snapshot("req")["bloom"]
        assert b & READY and not b & (WAITING | SERVICING)
    finally:
        s.close()
        unlink(uniq)


def test_from_gguf_llama_q4_cpu(tmp_path):
    """CausalLM.from_gguf on a llama GGUF with Q4_0 projections: the weights are the host-dequantised
    blocks, quant="auto" picks q4 for a mostly-4-bit file (bf16 for an F16 one), and the CPU
    forward equals a model built from the same dequantised tensors."""
    import numpy as np
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig, gguf_quant_kind, random_decoder_weights
    from libsplinter_amd.models.gguf import GGUFFile, GGUFWriter
    cfg = DecoderConfig(vocab=384, d=128, layers=2, heads=2, kv_heads=1, ffn=256, n_ctx=64)
    w = random_decoder_weights(cfg, seed=3)
    for proj_type, kind in (("Q4_0", "q4"), ("F16", "bf16")):
        path = str(tmp_path / f"llama_{proj_type}.gguf")
        gw = GGUFWriter(path, "llama")
        for k, v in (("embedding_length", cfg.d), ("block_count", cfg.layers), ("attention.head_count", cfg.heads),
                     ("attention.head_count_kv", cfg.kv_heads), ("feed_forward_length", cfg.ffn),
                     ("context_length", cfg.n_ctx)):
            gw.add(f"llama.{k}", v)
        gw.add("llama.rope.freq_base", 10000.0)
        gw.add("llama.attention.layer_norm_rms_epsilon", 1e-5)
        for n, a in w.items():
            gw.add_tensor(n, a, proj_type if n.startswith("blk.") and a.ndim == 2 else "F32")
        gw.write()
        g = GGUFFile(path)
        assert gguf_quant_kind(g) == kind
        m, tok = CausalLM.from_gguf(path, device="cpu")
        assert m.cfg.d == cfg.d and m.cfg.layers == cfg.layers and m.cfg.kv_heads == cfg.kv_heads
        ref = CausalLM(m.cfg, {n: torch.from_numpy(np.ascontiguousarray(g.to_numpy_f32(n))) for n in g.tensors},
                       device="cpu")
        ids = [1, 5, 9, 200]
        assert torch.allclose(m.forward(ids), ref.forward(ids))
        if kind == "q4":
            assert not np.array_equal(g.to_numpy_f32("blk.0.ffn_down.weight"), w["blk.0.ffn_down.weight"])


def test_chat_template_families():
    """build_prompt: the GGUF chat template families llama.cpp detects by marker, and the
    reference's bare fallback (splainference.cpp:132-169)."""
    from libsplinter_amd.daemons.splainference import build_prompt
    assert build_prompt("", "hi") == "<user>\nhi\n<assistant>\n"
    assert build_prompt("sys", "hi", "{{ unknown }}") == "<system>\nsys\n<user>\nhi\n<assistant>\n"
    assert build_prompt("sys", "hi", "{% ... %}<|im_start|>{{ role }}") == (
        "<|im_start|>system\nsys<|im_end|>\n<|im_start|>user\nhi<|im_end|>\n<|im_start|>assistant\n")
    assert build_prompt("", "hi", "<|start_header_id|>").endswith(
        "<|start_header_id|>assistant<|end_header_id|>\n\n")
    assert build_prompt("s", "hi", "<start_of_turn>") == "<start_of_turn>user\ns\n\nhi<end_of_turn>\n<start_of_turn>model\n"
    assert build_prompt("", "hi", "[INST] {{ x }} [/INST]") == "[INST] hi [/INST]"
    assert build_prompt("s", "hi", "<|user|>...<|end|>...<|assistant|>").startswith("<|system|>\ns<|end|>\n")
    assert build_prompt("", "hi", "<|user|>\n{{ m }}</s>").endswith("<|assistant|>\n")
