"""Prompt tokenizers of the completion daemon, chosen by the GGUF ``tokenizer.ggml.model``.

The reference tokenizes each prompt with ``llama_tokenize(vocab, prompt, add_special=true,
parse_special=true)`` (/root/reference/splainference.cpp:236-250) and turns sampled ids back into
text with ``llama_token_to_piece(..., special=true)`` (:314).  The two vocabularies llama-family
GGUF files carry are re-implemented here from their published algorithms:

* ``"llama"`` -- SentencePiece unigram-score merging (llama 1/2, Mistral, TinyLlama, Gemma):
  the text is split into UTF-8 characters, and the adjacent pair whose concatenation is a vocab
  token with the highest ``tokenizer.ggml.scores`` entry is merged first (ties: leftmost), until
  no merge applies; a final symbol that is not a token is re-split along its merge history, and a
  character with no token falls back to its ``<0xXX>`` byte tokens.  Spaces become U+2581 and a
  space is prefixed to every text run that starts the prompt or follows a special token
  (``tokenizer.ggml.add_space_prefix``, default on).
* ``"gpt2"`` -- byte-level BPE (llama 3, Qwen2, GPT-2 family): the text is pre-split with the
  regex named by ``tokenizer.ggml.pre``, every byte of a piece is mapped to its printable GPT-2
  code point, and the adjacent pair with the lowest ``tokenizer.ggml.merges`` rank is merged
  first (ties: leftmost).  With ``ignore_merges`` (llama-3's pre-tokenizer) a piece that is a
  whole vocab token is emitted as is.

Both split special tokens out of the text first (parse_special): CONTROL / USER_DEFINED /
UNKNOWN typed tokens, longest first, are matched verbatim and emitted as their ids.

Parity with llama.cpp's own tokenizer is unpinned (no llama.cpp and no real vocabularies here):
tests/test_llm_tokenizer.py checks the algorithms on synthetic vocab / score / merge fixtures
against hand-derived expected ids.
"""
from __future__ import annotations

import heapq
from typing import Dict, List, Optional, Sequence, Tuple

import torch

# tokenizer.ggml.token_type values (llama.cpp llama_token_type)
T_NORMAL, T_UNKNOWN, T_CONTROL, T_USER, T_UNUSED, T_BYTE = 1, 2, 3, 4, 5, 6

# pre-tokenizer regexes (tokenizer.ggml.pre): llama-3 family and the GPT-2 default
_PRE_LLAMA3 = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
               r"|\s*[\r\n]+|\s+(?!\S)|\s+")
_PRE_GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"
_PRE_QWEN2 = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
              r"|\s*[\r\n]+|\s+(?!\S)|\s+")
_PRE = {"llama3": (_PRE_LLAMA3, True), "llama-v3": (_PRE_LLAMA3, True), "llama-bpe": (_PRE_LLAMA3, True),
        "smaug-bpe": (_PRE_LLAMA3, False), "qwen2": (_PRE_QWEN2, False), "gpt-2": (_PRE_GPT2, False),
        "gpt2": (_PRE_GPT2, False), "default": (_PRE_GPT2, False)}


_EOG_TEXTS = {"<|eot_id|>", "<|im_end|>", "<|end|>", "<end_of_turn>", "<|endoftext|>", "<|eom_id|>", "</s>",
              "<|end_of_text|>"}


def gpt2_byte_map() -> Dict[int, str]:
    """GPT-2's reversible byte -> printable code point map: printable Latin-1 bytes map to
    themselves, the other 68 bytes to U+0100 onwards in byte order."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(0xA1, 0xAC + 1)) + list(range(0xAE, 0xFF + 1))
    out, extra = {}, 0
    for b in range(256):
        if b in keep:
            out[b] = chr(b)
        else:
            out[b] = chr(256 + extra)
            extra += 1
    return out


class _LlamaVocabBase:
    """Shared: id <-> text tables, token types, special-token partition, BOS/EOS, pieces."""

    def __init__(self, tokens: Sequence[str], types: Optional[Sequence[int]], bos: Optional[int], eos: Optional[int],
                 add_bos: bool, add_eos: bool, eot: Optional[int] = None):
        self.tokens = list(tokens)
        n = len(self.tokens)
        self.types = list(types) if types is not None and len(types) == n else [T_NORMAL] * n
        self.index: Dict[str, int] = {}
        for i, t in enumerate(self.tokens):
            self.index.setdefault(t, i)
        self.bos_id = bos if bos is not None else -1
        self.eos_id = eos if eos is not None else -1
        self.eot_id = eot
        self.add_bos, self.add_eos = add_bos, add_eos
        # parse_special: every CONTROL / USER_DEFINED / UNKNOWN token, longest text first
        self.specials: List[Tuple[str, int]] = sorted(
            ((t, i) for i, t in enumerate(self.tokens) if self.types[i] in (T_CONTROL, T_USER, T_UNKNOWN) and t),
            key=lambda p: (-len(p[0]), p[1]))
        self.chat_template = None
        # end of generation: EOS, EOT, and the end-of-turn control tokens of the chat families
        self.eog = {t for t in (self.eos_id, eot) if t is not None and t >= 0}
        for i, t in enumerate(self.tokens):
            if t in _EOG_TEXTS and self.types[i] in (T_CONTROL, T_USER):
                self.eog.add(i)

    def is_eog(self, tok: int) -> bool:
        return tok in self.eog

    def _partition(self, text: str) -> List[Tuple[bool, object]]:
        """[(is_special, text | id)]: special tokens matched verbatim, longest first."""
        frags: List[Tuple[bool, object]] = [(False, text)]
        for st, sid in self.specials:
            nxt: List[Tuple[bool, object]] = []
            for is_sp, v in frags:
                if is_sp or st not in v:
                    nxt.append((is_sp, v))
                    continue
                parts = v.split(st)
                for j, p in enumerate(parts):
                    if p:
                        nxt.append((False, p))
                    if j + 1 < len(parts):
                        nxt.append((True, sid))
            frags = nxt
        return frags

    def encode(self, text: str, add_bos: bool = True, parse_special: bool = True) -> List[int]:
        out: List[int] = []
        if add_bos and self.add_bos and self.bos_id >= 0:
            out.append(self.bos_id)
        frags = self._partition(text) if parse_special else [(False, text)]
        prev_special = True
        for is_sp, v in frags:
            if is_sp:
                out.append(int(v))
                prev_special = True
            else:
                self._encode_text(str(v), out, prev_special)
                prev_special = False
        if add_bos and self.add_eos and self.eos_id >= 0:
            out.append(self.eos_id)
        return out

    def printable_mask(self, vocab: int) -> Optional[torch.Tensor]:
        return None


class SpmTokenizer(_LlamaVocabBase):
    """tokenizer.ggml.model == "llama": SentencePiece score merging with byte fallback."""

    def __init__(self, tokens, scores: Optional[Sequence[float]], types=None, bos=1, eos=2, add_bos=True,
                 add_eos=False, add_space_prefix=True, eot=None):
        super().__init__(tokens, types, bos, eos, add_bos, add_eos, eot)
        n = len(self.tokens)
        self.scores = [float(s) for s in scores] if scores is not None and len(scores) == n else [0.0] * n
        self.add_space_prefix = add_space_prefix
        self.byte_ids: Dict[int, Optional[int]] = {}
        for b in range(256):
            t = self.index.get(f"<0x{b:02X}>")
            if t is None and b < 128:
                t = self.index.get(chr(b))
            self.byte_ids[b] = t

    def _encode_text(self, text: str, out: List[int], first: bool) -> None:
        if self.add_space_prefix and first:
            text = " " + text
        text = text.replace(" ", "▁")
        if not text:
            return
        sym = list(text)                     # one symbol per code point (UTF-8 character)
        n = len(sym)
        nxt = list(range(1, n)) + [-1]
        prv = list(range(-1, n - 1))
        alive = [True] * n
        heap: List[Tuple[float, int, int, str]] = []
        rev: Dict[str, Tuple[str, str]] = {}

        def bigram(a: int, b: int):
            if a < 0 or b < 0:
                return
            t = sym[a] + sym[b]
            tid = self.index.get(t)
            if tid is None:
                return
            heapq.heappush(heap, (-self.scores[tid], a, b, t))
            rev[t] = (sym[a], sym[b])

        for i in range(1, n):
            bigram(i - 1, i)
        while heap:
            _, a, b, t = heapq.heappop(heap)
            if not (alive[a] and alive[b]) or nxt[a] != b or sym[a] + sym[b] != t:
                continue  # one side merged since the pair was queued
            sym[a] = t
            alive[b] = False
            nxt[a] = nxt[b]
            if nxt[b] >= 0:
                prv[nxt[b]] = a
            bigram(prv[a], a)
            bigram(a, nxt[a])

        def emit(s: str):
            tid = self.index.get(s)
            if tid is not None:
                out.append(tid)
                return
            parts = rev.get(s)
            if parts is not None:
                emit(parts[0])
                emit(parts[1])
                return
            for byte in s.encode("utf-8"):
                bid = self.byte_ids.get(byte)
                if bid is not None:
                    out.append(bid)

        i = 0
        while i != -1:
            emit(sym[i])
            i = nxt[i]

    def piece(self, tok: int) -> bytes:
        if not 0 <= tok < len(self.tokens):
            return b""
        t, ty = self.tokens[tok], self.types[tok]
        if ty == T_BYTE or (len(t) == 6 and t.startswith("<0x") and t.endswith(">")):
            return bytes([int(t[3:5], 16)])
        if ty == T_USER or ty == T_CONTROL:
            return t.encode("utf-8")  # special=true pieces print control tokens too (reference :314)
        if ty == T_UNUSED:
            return b""
        return t.replace("▁", " ").encode("utf-8")


class BpeTokenizer(_LlamaVocabBase):
    """tokenizer.ggml.model == "gpt2": byte-level BPE over tokenizer.ggml.merges."""

    def __init__(self, tokens, merges: Sequence[str], types=None, bos=None, eos=None, add_bos=False, add_eos=False,
                 pre: str = "default", eot=None):
        super().__init__(tokens, types, bos, eos, add_bos, add_eos, eot)
        import regex
        pat, self.ignore_merges = _PRE.get(pre or "default", _PRE["default"])
        self.pre = pre
        self._re = regex.compile(pat)
        self.ranks: Dict[Tuple[str, str], int] = {}
        for r, m in enumerate(merges):
            a, sep, b = m.partition(" ")
            if sep and (a, b) not in self.ranks:
                self.ranks[(a, b)] = r
        self.b2u = gpt2_byte_map()
        self.u2b = {u: b for b, u in self.b2u.items()}

    def _bpe(self, word: str, out: List[int]) -> None:
        if self.ignore_merges and word in self.index:
            out.append(self.index[word])
            return
        sym = list(word)
        n = len(sym)
        nxt = list(range(1, n)) + [-1]
        prv = list(range(-1, n - 1))
        alive = [True] * n
        heap: List[Tuple[int, int, int, str, str]] = []

        def bigram(a: int, b: int):
            if a < 0 or b < 0:
                return
            r = self.ranks.get((sym[a], sym[b]))
            if r is not None:
                heapq.heappush(heap, (r, a, b, sym[a], sym[b]))

        for i in range(1, n):
            bigram(i - 1, i)
        while heap:
            _, a, b, sa, sb = heapq.heappop(heap)
            if not (alive[a] and alive[b]) or nxt[a] != b or sym[a] != sa or sym[b] != sb:
                continue
            sym[a] = sa + sb
            alive[b] = False
            nxt[a] = nxt[b]
            if nxt[b] >= 0:
                prv[nxt[b]] = a
            bigram(prv[a], a)
            bigram(a, nxt[a])
        i = 0
        while i != -1:
            s = sym[i]
            tid = self.index.get(s)
            if tid is not None:
                out.append(tid)
            else:  # no token for the merged text: its single byte-symbols, where they exist
                for ch in s:
                    t1 = self.index.get(ch)
                    if t1 is not None:
                        out.append(t1)
            i = nxt[i]

    def _encode_text(self, text: str, out: List[int], first: bool) -> None:
        for m in self._re.finditer(text):
            w = m.group(0)
            if w:
                self._bpe("".join(self.b2u[b] for b in w.encode("utf-8")), out)

    def piece(self, tok: int) -> bytes:
        if not 0 <= tok < len(self.tokens):
            return b""
        t, ty = self.tokens[tok], self.types[tok]
        if ty in (T_CONTROL, T_USER):
            return t.encode("utf-8")
        if ty == T_UNUSED:
            return b""
        try:
            return bytes(self.u2b[c] for c in t)
        except KeyError:
            return t.encode("utf-8")


def tokenizer_from_gguf(g):
    """The GGUF's own tokenizer: SPM for model "llama", byte-level BPE for "gpt2"; None when the
    file carries no vocabulary.  Unknown models raise (no silent greedy fallback)."""
    tokens = g.get("tokenizer.ggml.tokens")
    if not tokens:
        return None
    model = g.get("tokenizer.ggml.model", "llama")
    types = g.get("tokenizer.ggml.token_type")
    bos, eos = g.get("tokenizer.ggml.bos_token_id"), g.get("tokenizer.ggml.eos_token_id")
    eot = g.get("tokenizer.ggml.eot_token_id")
    if model == "llama":
        tok = SpmTokenizer(list(tokens), g.get("tokenizer.ggml.scores"), types,
                           int(bos) if bos is not None else 1, int(eos) if eos is not None else 2,
                           bool(g.get("tokenizer.ggml.add_bos_token", True)),
                           bool(g.get("tokenizer.ggml.add_eos_token", False)),
                           bool(g.get("tokenizer.ggml.add_space_prefix", True)), eot)
    elif model == "gpt2":
        tok = BpeTokenizer(list(tokens), list(g.get("tokenizer.ggml.merges") or []), types,
                           int(bos) if bos is not None else None, int(eos) if eos is not None else None,
                           bool(g.get("tokenizer.ggml.add_bos_token", False)),
                           bool(g.get("tokenizer.ggml.add_eos_token", False)), g.get("tokenizer.ggml.pre", "default"),
                           eot)
    else:
        raise ValueError(f"tokenizer.ggml.model {model!r}: only 'llama' (SentencePiece) and 'gpt2' (BPE) decoders")
    tok.chat_template = g.get("tokenizer.chat_template", None)
    return tok
