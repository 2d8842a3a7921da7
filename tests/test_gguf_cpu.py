"""GGUF reader/writer and the fp32 reference encoder (CPU)."""
import numpy as np
import pytest

from libsplinter_amd.models.gguf import GGUFFile, GGUFWriter, dequant_host, quantize_host


def test_writer_reader_roundtrip(tmp_path):
    p = str(tmp_path / "t.gguf")
    w = GGUFWriter(p, "nomic-bert")
    w.add("nomic-bert.block_count", 12)
    w.add("nomic-bert.rope.freq_base", 1000.0)
    w.add("tokenizer.ggml.tokens", ["[PAD]", "[UNK]", "▁hello"])
    w.add("nomic-bert.attention.causal", False)
    rng = np.random.default_rng(0)
    a = rng.standard_normal((64, 96)).astype(np.float32)
    w.add_tensor("a.f32", a, "F32")
    w.add_tensor("a.f16", a, "F16")
    w.add_tensor("a.q8", a, "Q8_0")
    w.add_tensor("a.q4", a, "Q4_0")
    w.write()
    g = GGUFFile(p)
    assert g.arch() == "nomic-bert" and g.version == 3
    assert g.get("nomic-bert.block_count") == 12
    assert g.get("tokenizer.ggml.tokens") == ["[PAD]", "[UNK]", "▁hello"]
    assert g.get("nomic-bert.attention.causal") is False
    assert g.tensors["a.f32"].shape == (64, 96)
    np.testing.assert_array_equal(g.to_numpy_f32("a.f32"), a)
    np.testing.assert_allclose(g.to_numpy_f32("a.f16"), a, rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(g.to_numpy_f32("a.q8"), a, atol=np.abs(a).max() / 100)
    assert np.abs(g.to_numpy_f32("a.q4") - a).max() < np.abs(a).max() / 6


def test_q4k_q6k_host_decoders_shape():
    rng = np.random.default_rng(1)
    raw = rng.integers(0, 255, size=144 * 3, dtype=np.uint8)
    raw[0:2] = np.array([0x3c00], np.uint16).view(np.uint8)  # d = 1.0
    out = dequant_host(raw, 12, 256 * 3)
    assert out.shape == (768,) and np.isfinite(out[:256]).all()
    raw6 = rng.integers(0, 255, size=210 * 2, dtype=np.uint8)
    out6 = dequant_host(raw6, 14, 512)
    assert out6.shape == (512,)


def test_reference_encoder_cpu_properties():
    import torch
    from libsplinter_amd.models.nomic import NomicConfig, NomicReference, random_weights
    cfg = NomicConfig(layers=2, vocab=300)
    w = random_weights(cfg, seed=3)
    m = NomicReference(cfg, w)
    rng = np.random.default_rng(0)
    s1 = rng.integers(0, 300, size=9)
    s2 = rng.integers(0, 300, size=23)
    both = m(torch.from_numpy(np.concatenate([s1, s2])).long(), [0, 9, 32])
    one = m(torch.from_numpy(s2).long(), [0, 23])
    # sequences in one packed batch never attend to each other
    assert torch.allclose(both[1], one[0], atol=1e-5)
    assert both.shape == (2, 768)


def test_host_k_quant_roundtrip():
    """Host Q4_K / Q6_K writers (the layouts the readers and the device dequant decode): relative
    RMS error of a 4-bit and a 6-bit grid on Gaussian weights."""
    import numpy as np
    from libsplinter_amd.models.gguf import dequant_host, quantize_host
    a = (np.random.default_rng(0).standard_normal(8 * 256) * 0.02).astype(np.float32)
    for t, tol in ((12, 0.1), (14, 0.03)):
        raw = np.frombuffer(quantize_host(a, t), np.uint8)
        e = dequant_host(raw, t, a.size) - a
        assert np.sqrt((e ** 2).mean()) / a.std() < tol, t
