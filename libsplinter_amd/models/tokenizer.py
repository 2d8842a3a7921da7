"""WordPiece tokenizer (native C++, csrc/core/wordpiece.cpp) over a GGUF vocab.

Replaces llama.cpp's tokenizer in the embedding daemon (reference
splinference.cpp:210-217).  Accepts both the GGUF/llama.cpp convention
(word-initial pieces prefixed with U+2581) and the HF BERT "##" convention.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .. import _native as N


def _lib():
    L = N.core_lib()
    if not getattr(L, "_tok_declared", False):
        P = ctypes.c_void_p
        L.spl_tok_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int]
        L.spl_tok_create.restype = P
        L.spl_tok_free.argtypes = [P]
        L.spl_tok_is_wpm.argtypes = [P]
        L.spl_tok_encode.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t, P, ctypes.c_int, ctypes.c_int]
        L.spl_tok_encode.restype = ctypes.c_int
        L.spl_tok_encode_batch.argtypes = [P, ctypes.POINTER(ctypes.c_char_p), P, ctypes.c_int, P, ctypes.c_long, P,
                                           P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.spl_tok_encode_batch.restype = ctypes.c_int
        L._tok_declared = True
    return L


class WordPieceTokenizer:
    def __init__(self, tokens: Sequence[str], cls_id: Optional[int] = None, sep_id: Optional[int] = None,
                 unk_id: Optional[int] = None, pad_id: int = 0):
        self.tokens = list(tokens)
        idx = {t: i for i, t in enumerate(self.tokens)}
        self.cls_id = idx.get("[CLS]", -1) if cls_id is None else cls_id
        self.sep_id = idx.get("[SEP]", -1) if sep_id is None else sep_id
        self.unk_id = idx.get("[UNK]", 0) if unk_id is None else unk_id
        self.pad_id = pad_id
        self._L = _lib()
        arr = (ctypes.c_char_p * len(self.tokens))(*[t.encode("utf-8") for t in self.tokens])
        self._h = self._L.spl_tok_create(arr, len(self.tokens), self.cls_id, self.sep_id, self.unk_id)
        self.threads = min(16, os.cpu_count() or 4)

    @classmethod
    def from_gguf(cls, g) -> "WordPieceTokenizer":
        toks = g.get("tokenizer.ggml.tokens")
        if not toks:
            raise ValueError("GGUF has no tokenizer.ggml.tokens")
        return cls(toks, g.get("tokenizer.ggml.bos_token_id"), g.get("tokenizer.ggml.seperator_token_id",
                                                                   g.get("tokenizer.ggml.eos_token_id")),
                   g.get("tokenizer.ggml.unknown_token_id"), g.get("tokenizer.ggml.padding_token_id", 0))

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.spl_tok_free(self._h)
            self._h = None

    @property
    def vocab_size(self) -> int:
        return len(self.tokens)

    @property
    def wpm(self) -> bool:
        return bool(self._L.spl_tok_is_wpm(self._h))

    def encode(self, text, add_special: bool = True) -> List[int]:
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        n = self._L.spl_tok_encode(self._h, b, len(b), None, 0, int(add_special))
        out = np.zeros(max(n, 1), np.int32)
        self._L.spl_tok_encode(self._h, b, len(b), out.ctypes.data, n, int(add_special))
        return out[:n].tolist()

    def encode_batch(self, texts: Sequence, max_len: int, add_special: bool = True
                     ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """-> (ids_flat int32, offsets int64 [n+1], full_lens int32 [n]); each sequence is
        truncated to max_len ids (full_lens tells the untruncated count)."""
        bs = [t.encode("utf-8") if isinstance(t, str) else bytes(t) for t in texts]
        n = len(bs)
        ptrs = (ctypes.c_char_p * n)(*bs)
        lens = np.array([len(b) for b in bs], dtype=np.uint64)
        cap = sum(min(max_len, len(b) + 2) for b in bs) + 16 * n + 16
        while True:
            out = np.empty(cap, np.int32)
            offs = np.zeros(n + 1, np.int64)
            full = np.zeros(n, np.int32)
            got = self._L.spl_tok_encode_batch(self._h, ptrs, lens.ctypes.data, n, out.ctypes.data, cap,
                                               offs.ctypes.data, full.ctypes.data, max_len, int(add_special),
                                               self.threads)
            if got >= 0:
                return out[:got], offs, full
            cap *= 2

    def decode(self, ids: Sequence[int]) -> str:
        parts = []
        for i in ids:
            t = self.tokens[i]
            if t in ("[CLS]", "[SEP]", "[PAD]"):
                continue
            if t.startswith("▁"):
                parts.append(" " + t[1:])
            elif t.startswith("##"):
                parts.append(t[2:])
            elif self.wpm:
                parts.append(t)
            else:
                parts.append(" " + t)
        return "".join(parts).strip()


def synthetic_vocab(size: int = 30528, seed: int = 0) -> List[str]:
    """A BERT-shaped vocabulary for random-init models (no network for the real
    one): specials, single characters (word-initial and continuation forms) and
    frequent English fragments, padded with random letter n-grams, in the GGUF
    (U+2581) convention."""
    specials = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    chars = [chr(c) for c in range(33, 127) if not chr(c).isupper()]
    words = ("the of and to in is was for that on as with by he at from his it an were are which this be or has "
             "had not but first one their its new after who they have her she two been other when there all during "
             "into school time may years more most only over city some world would where later up such used many "
             "can state about national out known university united then made also between system data search "
             "vector memory store key value shared embed model text document query result token").split()
    out = list(specials)
    seen = set(out)

    def add(t):
        if t not in seen and len(out) < size:
            seen.add(t)
            out.append(t)

    for c in chars:
        add("▁" + c)
    for c in chars:
        add(c)
    for w in words:
        add("▁" + w)
    rng = np.random.default_rng(seed)
    letters = np.array(list("abcdefghijklmnopqrstuvwxyz"))
    while len(out) < size:
        k = int(rng.integers(2, 7))
        frag = "".join(rng.choice(letters, k))
        add(("▁" + frag) if rng.random() < 0.6 else frag)
    return out
