"""SentencePiece (score merging) and byte-level BPE (merge ranks) prompt tokenizers of the
completion daemon (models/llm_tokenizer.py), on synthetic vocabularies whose expected ids are
derived by hand from the algorithms (parity with llama.cpp itself: unpinned, no llama.cpp here).
Reference call: llama_tokenize(add_special=true, parse_special=true), splainference.cpp:236-250."""
import pytest

from libsplinter_amd.models.llm_tokenizer import (T_BYTE, T_CONTROL, T_NORMAL, BpeTokenizer, SpmTokenizer,
                                                  gpt2_byte_map, tokenizer_from_gguf)


def _spm():
    toks, scores, types = ["<unk>", "<s>", "</s>"], [0.0, 0.0, 0.0], [2, T_CONTROL, T_CONTROL]
    for b in range(256):
        toks.append(f"<0x{b:02X}>")
        scores.append(0.0)
        types.append(T_BYTE)
    pieces = {"▁": -10, "h": -10, "e": -10, "l": -10, "o": -10, "w": -10, "r": -10, "d": -10, "a": -10,
              "ll": -1, "llo": -2, "he": -3, "▁he": -4, "▁hello": -1.5, "or": -2.5, "▁w": -6, "▁wor": -5,
              "ld": -7, "▁world": -4.5, "aa": -1}
    for p, s in pieces.items():
        toks.append(p)
        scores.append(float(s))
        types.append(T_NORMAL)
    toks.append("<|im_start|>")
    scores.append(0.0)
    types.append(T_CONTROL)
    return SpmTokenizer(toks, scores, types, bos=1, eos=2)


def test_spm_score_merging_order():
    t = _spm()
    ix = t.index
    # ll(-1) -> llo(-2) -> or(-2.5) -> he(-3) -> ▁he(-4) -> ▁hello(-1.5) -> ▁w(-6) -> ▁wor(-5) -> ld(-7) -> ▁world
    assert t.encode("hello world") == [1, ix["▁hello"], ix["▁world"]]
    assert t.encode("hello world", add_bos=False) == [ix["▁hello"], ix["▁world"]]
    # equal scores: the leftmost pair merges first
    assert t.encode("aaa", add_bos=False) == [ix["▁"], ix["aa"], ix["a"]]
    assert b"".join(t.piece(i) for i in t.encode("hello world", add_bos=False)) == b" hello world"


def test_spm_byte_fallback_and_specials():
    t = _spm()
    ix = t.index
    # é has no piece: its UTF-8 bytes C3 A9 as <0xC3> <0xA9>
    assert t.encode("hé", add_bos=False) == [ix["▁"], ix["h"], ix["<0xC3>"], ix["<0xA9>"]]
    assert b"".join(t.piece(i) for i in t.encode("hé", add_bos=False)) == " hé".encode()
    # parse_special: the control token is matched verbatim, and the text after it gets the space prefix
    assert t.encode("<|im_start|>hello") == [1, ix["<|im_start|>"], ix["▁hello"]]
    # without parse_special the marker is plain text (byte fallback for < | _ ...)
    assert ix["<|im_start|>"] not in t.encode("<|im_start|>hello", parse_special=False)
    assert t.is_eog(2) and not t.is_eog(ix["▁hello"])


def _bpe(pre="gpt2"):
    m = gpt2_byte_map()
    sp = m[ord(" ")]  # 'Ġ'
    singles = [m[b] for b in range(256)]
    merges = ["h e", "l l", "ll o", "he llo", f"{sp} w", "o r", f"{sp}w or", "l d", f"{sp}wor ld", "b c", "a b"]
    words = ["he", "ll", "llo", "hello", f"{sp}w", "or", f"{sp}wor", "ld", f"{sp}world", "bc", "ab", "xyz"]
    toks = singles + words + ["<|eot_id|>", "<|begin_of_text|>"]
    types = [T_NORMAL] * (len(toks) - 2) + [T_CONTROL, T_CONTROL]
    return BpeTokenizer(toks, merges, types, bos=len(toks) - 1, eos=None, add_bos=True, pre=pre,
                        eot=len(toks) - 2)


def test_bpe_merge_ranks():
    t = _bpe()
    ix, sp = t.index, gpt2_byte_map()[32]
    # pre-split "hello" | " world"; h e -> l l -> ll o -> he llo ; Ġ w -> o r -> Ġw or -> l d -> Ġwor ld
    assert t.encode("hello world") == [t.bos_id, ix["hello"], ix[f"{sp}world"]]
    # rank order, not position: "b c" (rank 9) beats "a b" (rank 10)
    assert t.encode("abc", add_bos=False) == [ix["a"], ix["bc"]]
    assert b"".join(t.piece(i) for i in t.encode("hello world", add_bos=False)) == b"hello world"
    # bytes of non-ASCII text go through the printable byte map and come back exactly
    ids = t.encode("héllo ✓", add_bos=False)
    assert b"".join(t.piece(i) for i in ids) == "héllo ✓".encode()


def test_bpe_ignore_merges_and_specials():
    ix = _bpe().index
    # "xyz" is a vocab token no merge reaches: gpt2 spells it out, llama-3's pre-tokenizer takes it whole
    assert _bpe("gpt2").encode("xyz", add_bos=False) == [ix["x"], ix["y"], ix["z"]]
    assert _bpe("llama-bpe").encode("xyz", add_bos=False) == [ix["xyz"]]
    t = _bpe("llama-bpe")
    ids = t.encode("hello<|eot_id|>hello")
    assert ids == [t.bos_id, ix["hello"], ix["<|eot_id|>"], ix["hello"]]
    assert t.is_eog(ix["<|eot_id|>"])
    # llama-3 regex: digits in groups of at most three
    assert [t.piece(i) for i in t.encode("12345", add_bos=False)] == [b"1", b"2", b"3", b"4", b"5"]
    assert len(t._re.findall("12345")) == 2


def test_tokenizer_from_gguf(tmp_path):
    import numpy as np
    from libsplinter_amd.models.gguf import GGUFFile, GGUFWriter
    spm = _spm()
    p = str(tmp_path / "spm.gguf")
    w = GGUFWriter(p, "llama")
    w.add("tokenizer.ggml.model", "llama")
    w.add("tokenizer.ggml.tokens", spm.tokens)
    w.add("tokenizer.ggml.scores", [float(s) for s in spm.scores])
    w.add("tokenizer.ggml.token_type", spm.types)
    w.add("tokenizer.ggml.bos_token_id", 1)
    w.add("tokenizer.ggml.eos_token_id", 2)
    w.add_tensor("dummy", np.zeros(4, np.float32))
    w.write()
    t = tokenizer_from_gguf(GGUFFile(p))
    assert isinstance(t, SpmTokenizer) and t.encode("hello world") == spm.encode("hello world")
    bpe = _bpe("llama-bpe")
    p = str(tmp_path / "bpe.gguf")
    w = GGUFWriter(p, "llama")
    w.add("tokenizer.ggml.model", "gpt2")
    w.add("tokenizer.ggml.pre", "llama-bpe")
    w.add("tokenizer.ggml.tokens", bpe.tokens)
    w.add("tokenizer.ggml.merges", [f"{a} {b}" for (a, b), _ in sorted(bpe.ranks.items(), key=lambda kv: kv[1])])
    w.add("tokenizer.ggml.token_type", bpe.types)
    w.add("tokenizer.ggml.bos_token_id", bpe.bos_id)
    w.add("tokenizer.ggml.add_bos_token", True)
    w.add_tensor("dummy", np.zeros(4, np.float32))
    w.write()
    t = tokenizer_from_gguf(GGUFFile(p))
    assert isinstance(t, BpeTokenizer) and t.ignore_merges
    assert t.encode("hello world<|eot_id|>") == bpe.encode("hello world<|eot_id|>")
    w = GGUFWriter(str(tmp_path / "x.gguf"), "llama")
    w.add("tokenizer.ggml.model", "t5")
    w.add("tokenizer.ggml.tokens", ["a"])
    w.add_tensor("dummy", np.zeros(4, np.float32))
    w.write()
    with pytest.raises(ValueError):
        tokenizer_from_gguf(GGUFFile(str(tmp_path / "x.gguf")))
