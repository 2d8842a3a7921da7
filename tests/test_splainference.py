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
@pytest.mark.parametrize("kv_heads", [8, 2])
def test_decoder_hip_matches_cpu(kv_heads):
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    cfg = DecoderConfig(layers=2, kv_heads=kv_heads)
    gpu = CausalLM.random(cfg, seed=3, device="cuda")
    cpu = CausalLM.random(cfg, seed=3, device="cpu")
    ids = [256] + list(b"the quick brown fox")
    lg, lc = gpu.forward(ids).cpu(), cpu.forward(ids)
    rel = (lg - lc).norm() / lc.norm()
    assert rel < 3e-2, float(rel)
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
@pytest.mark.parametrize("hd,H,KVH", [(128, 32, 8), (64, 8, 8), (128, 16, 2)])
def test_decoder_attn_decode_kernel_vs_fp32(hd, H, KVH):
    """dec_attn_decode (csrc/hip/decoder_kernels.hip) against an fp32 softmax(q k^T) v reference,
    cache lengths on both sides of the 64-key chunk and 256-key workgroup boundaries."""
    import torch
    from libsplinter_amd.models.decoder import CausalLM, DecoderConfig
    m = CausalLM.random(DecoderConfig(layers=1), seed=1, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(7)
    n_ctx = 1100
    kv = torch.randn((2, n_ctx, KVH, hd), device="cuda", generator=g).to(torch.bfloat16)
    q = torch.randn((H * hd,), device="cuda", generator=g).to(torch.bfloat16)
    for L in (1, 63, 64, 65, 257, 1100):
        out = torch.full((H * hd,), float("nan"), device="cuda").to(torch.bfloat16)
        assert m.L.dec_attn_decode(q.data_ptr(), kv[0].data_ptr(), kv[1].data_ptr(), KVH * hd, L, H, KVH, hd,
                                   hd ** -0.5, out.data_ptr(), None) == 0
        torch.cuda.synchronize()
        qf = q.float().reshape(H, hd)
        kf = kv[0, :L].float().repeat_interleave(H // KVH, 1)  # [L, H, hd]
        vf = kv[1, :L].float().repeat_interleave(H // KVH, 1)
        p = torch.softmax(torch.einsum("hd,lhd->hl", qf, kf) * hd ** -0.5, -1)
        ref = torch.einsum("hl,lhd->hd", p, vf).reshape(-1)
        err = (out.float() - ref).abs().max()
        assert err < 2e-2 * max(1.0, ref.abs().max().item()), (L, float(err))


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
