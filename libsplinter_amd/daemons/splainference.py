#!/usr/bin/env python3
"""splainference — the completion sidecar, on the MI355X causal decoder.

Contract kept from the reference daemon (/root/reference/splainference.cpp):
  argv    [--oneshot] [--n-ctx N] [--system-prompt-key KEY] <bus> <gguf> <group>  (:410-454)
  labels  0x1000000000000000 WAITING (client posts + bumps) ->
          0x2000000000000000 SERVICING (set before the first token, :232-234) ->
          0x4000000000000000 READY (on completion or failure, :390-392)
  request odd epoch = skip (writer active); the value is read with an epoch
          check (:191-210); the slot is overwritten with the formatted prompt
          (:269) and the completion is APPENDED as it streams: a flush at a
          word boundary (piece starts with ' ' or contains '\\n') or every 8
          tokens (:86, :102-109, :332-364), truncated at max_val_sz (:336-345)
  prompt  the GGUF chat template's family is detected by its markers (chatml, llama 3,
          gemma, phi 3, zephyr, llama 2 / mistral), as llama_chat_apply_template does;
          otherwise the reference's bare fallback "<system>/<user>/<assistant>" (:132-169)
  shard   0x5F1A WILLNEED prio 200, re-bid every 32 appended tokens, WILLNEED
          madvise of the request slot (:39-62, :222-230, :359-363)
  done    ctime backfill with the processing delta (:282, :383-387), "__debug"
          chatter (:94-100), cold-start sweep of WAITING keys (:542-551), then
          poll the signal group every 50 ms (:570-592)
Extra flags: --random-init (no GGUF: random llama weights, byte vocabulary,
printable-byte sampling), --max-tokens (cap per request), --seed.
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import time
from typing import Optional

LABEL_WAITING = 0x1000000000000000
LABEL_SERVICING = 0x2000000000000000
LABEL_READY = 0x4000000000000000
SHARD_ID = 0x5F1A
SHARD_DUR_LIVE = 1 << 30
SHARD_PRIO_LIVE = 200
SHARD_REBID_TOKENS = 32
TOKEN_FLUSH_MAX = 8
POSIX_MADV_WILLNEED = 3
INTENT_WILLNEED = 1

_running = True


def _stop(*_):
    global _running
    _running = False


def debug_post(store, msg: str) -> None:
    line = msg + "\n"
    try:
        store.append("__debug", line)
    except OSError:
        try:
            store.set("__debug", line)
        except OSError:
            pass


def build_prompt(system_msg: str, user_msg: str, template: Optional[str] = None) -> str:
    """The reference renders the model's GGUF chat template with llama_chat_apply_template and
    falls back to a bare "<system>/<user>/<assistant>" layout (splainference.cpp:132-169).
    llama.cpp recognises templates by marker substrings rather than evaluating the jinja; the
    families below follow the same detection, anything else takes the bare fallback."""
    t = template or ""
    sys_ = system_msg
    if "<|im_start|>" in t:  # chatml
        out = f"<|im_start|>system\n{sys_}<|im_end|>\n" if sys_ else ""
        return out + f"<|im_start|>user\n{user_msg}<|im_end|>\n<|im_start|>assistant\n"
    if "<|start_header_id|>" in t:  # llama 3
        out = f"<|start_header_id|>system<|end_header_id|>\n\n{sys_}<|eot_id|>" if sys_ else ""
        return out + (f"<|start_header_id|>user<|end_header_id|>\n\n{user_msg}<|eot_id|>"
                      "<|start_header_id|>assistant<|end_header_id|>\n\n")
    if "<start_of_turn>" in t:  # gemma: the system text is prepended to the user turn
        body = f"{sys_}\n\n{user_msg}" if sys_ else user_msg
        return f"<start_of_turn>user\n{body}<end_of_turn>\n<start_of_turn>model\n"
    if "<|assistant|>" in t and "<|end|>" in t:  # phi 3
        out = f"<|system|>\n{sys_}<|end|>\n" if sys_ else ""
        return out + f"<|user|>\n{user_msg}<|end|>\n<|assistant|>\n"
    if "<|user|>" in t and "</s>" in t:  # zephyr
        out = f"<|system|>\n{sys_}</s>\n" if sys_ else ""
        return out + f"<|user|>\n{user_msg}</s>\n<|assistant|>\n"
    if "[INST]" in t:  # llama 2 / mistral
        if sys_:
            return f"[INST] <<SYS>>\n{sys_}\n<</SYS>>\n\n{user_msg} [/INST]"
        return f"[INST] {user_msg} [/INST]"
    out = ""
    if system_msg:
        out += "<system>\n" + system_msg + "\n"
    return out + "<user>\n" + user_msg + "\n<assistant>\n"


def is_word_boundary(piece: bytes) -> bool:
    return bool(piece) and (piece[:1] in (b" ", b"\n") or b"\n" in piece)


class Splainference:
    def __init__(self, store, model, tokenizer, sampler, system_prompt_key=None, max_tokens: int = 256):
        self.store, self.model, self.tok, self.sampler = store, model, tokenizer, sampler
        self.system_prompt_key = system_prompt_key
        self.max_tokens = max_tokens
        self.engine = None
        if getattr(model, "hip", False) and getattr(model, "decode_kernel", True):
            from ..models.decoder import DecodeEngine
            self.engine = DecodeEngine(model, sampler.top_p, sampler.temp, sampler.seed, sampler.mask)

    def _read_request(self, key: str):
        s = self.store
        start = s.epoch(key)
        if start & 1:
            debug_post(s, f"[splainference][SKIP]: {key} has odd epoch (writer active).")
            return None, start
        raw = s.raw(key) if s.backend != "hbm" else None
        if raw is not None:
            view, ep = raw
            val = bytes(view)
            if ep != start or s.epoch(key) != start:
                debug_post(s, f"[splainference][SKIP]: {key} epoch shifted during read.")
                return None, start
        else:
            val = s.get(key) or b""
            if s.epoch(key) != start:
                debug_post(s, f"[splainference][SKIP]: {key} epoch shifted during read.")
                return None, start
        if not val:
            debug_post(s, f"[splainference][SKIP]: {key} is empty.")
            return None, start
        return val.decode("utf-8", "replace"), start

    def _finish(self, key: str) -> None:
        self.store.unset_label(key, LABEL_SERVICING)
        self.store.set_label(key, LABEL_READY)
        self.store.bump(key)

    def process(self, key: str) -> int:
        s = self.store
        user_msg, start = self._read_request(key)
        if user_msg is None:
            return 0
        system_msg = ""
        if self.system_prompt_key:
            v = s.get(self.system_prompt_key)
            system_msg = v.decode("utf-8", "replace") if v else ""
        prompt = build_prompt(system_msg, user_msg, getattr(self.tok, "chat_template", None))
        debug_post(s, f"[splainference][START]: Processing key: {key}")
        s.shard_rebid(SHARD_ID, INTENT_WILLNEED, SHARD_PRIO_LIVE, SHARD_DUR_LIVE)
        try:
            s.madvise(SHARD_ID, POSIX_MADV_WILLNEED, 0)
        except OSError:
            pass
        s.unset_label(key, LABEL_WAITING)
        s.set_label(key, LABEL_SERVICING)
        s.bump(key)
        ids = self.tok.encode(prompt)
        if not ids:
            debug_post(s, f"[splainference][ERROR]: Tokenization failed for key: {key}")
            self._finish(key)
            return 0
        max_val = s.max_val
        pb = prompt.encode("utf-8")[:max_val]
        s.set(key, pb)
        written = len(pb)
        t0 = time.perf_counter_ns()
        self.model.reset()
        ctx_room = self.model.cfg.n_ctx - len(ids)
        if ctx_room <= 0:
            debug_post(s, f"[splainference][ERROR]: Prefill decode failed for key: {key}")
            self._finish(key)
            return 0
        eng = self.engine
        if eng is not None:  # GPU: prefill + device sampler, then one graph replay per token
            t = eng.first_token(ids)
        else:
            logits = self.model.forward(ids)
        chunk, run, rebid, oom = b"", 0, 0, False
        for _ in range(min(self.max_tokens, ctx_room)):
            if not _running:
                break
            if eng is None:
                t = self.sampler(logits)
            if self.tok.is_eog(t):  # EOS / EOT / end-of-turn (llama_vocab_is_eog, reference :310)
                break
            piece = self.tok.piece(t)
            chunk += piece
            run += 1
            if eng is not None:
                t = eng.next_token()
            else:
                logits = self.model.forward([t])
            if (is_word_boundary(piece) or run >= TOKEN_FLUSH_MAX) and chunk:
                if written + len(chunk) > max_val:
                    debug_post(s, f"[splainference][WARN]: Slot full, truncating completion: {key}")
                    if max_val - written > 0:
                        s.append(key, chunk[: max_val - written])
                    oom = True
                    break
                written = s.append(key, chunk)
                chunk, run = b"", 0
                rebid += TOKEN_FLUSH_MAX
                if rebid >= SHARD_REBID_TOKENS:
                    s.shard_rebid(SHARD_ID, INTENT_WILLNEED, SHARD_PRIO_LIVE, SHARD_DUR_LIVE)
                    rebid = 0
        if chunk and not oom and max_val - written > 0:
            s.append(key, chunk[: max_val - written])
        from ..store import TIME_CTIME
        s.set_time(key, TIME_CTIME, int(time.time()), (time.perf_counter_ns() - t0) // 1000)
        self._finish(key)
        debug_post(s, f"[splainference][DONE]: Completion written to key: {key}")
        return start

    def waiting(self):
        return [k for k, _ in self.store.enumerate(LABEL_WAITING)]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="splainference")
    ap.add_argument("--oneshot", action="store_true")
    ap.add_argument("--n-ctx", type=int, default=0)
    ap.add_argument("--system-prompt-key", default=None)
    ap.add_argument("--random-init", action="store_true")
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0xFFFFFFFF)
    ap.add_argument("--poll-ms", type=int, default=50)
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is present) or cpu")
    ap.add_argument("--quant", default="auto", choices=["auto", "bf16", "q4"],
                    help="weights in HBM: q4 = 4-bit Q4G32 (decode streams 0.625 B per weight), bf16, or auto "
                         "(q4 for a 4-bit GGUF, bf16 otherwise; --random-init: bf16)")
    ap.add_argument("bus")
    ap.add_argument("gguf")
    ap.add_argument("group", type=int)
    a = ap.parse_args(argv)
    if not 0 <= a.group < 64:
        print("Error: signal_group_id must be 0-63.", file=sys.stderr)
        return 1
    import torch
    from ..store import Store
    from ..models.decoder import ByteTokenizer, CausalLM, DecoderConfig, Sampler
    signal.signal(signal.SIGINT, _stop)
    signal.signal(signal.SIGTERM, _stop)
    try:
        store = Store.open(a.bus)
    except OSError:
        print(f"Failed to connect to Splinter bus: {a.bus}", file=sys.stderr)
        return 1
    try:
        store.shard_claim(SHARD_ID, INTENT_WILLNEED, SHARD_PRIO_LIVE, SHARD_DUR_LIVE)
    except OSError:
        print("[Warn]: could not claim a shard bid slot (table full?); continuing without cooperative advisement.")
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    print(f"[Startup]: Loading {'random-init decoder' if a.random_init else 'GGUF model `' + a.gguf + '`'} "
          f"on {device} ...", flush=True)
    if a.random_init:
        cfg = DecoderConfig()
        if a.n_ctx > 0:
            cfg.n_ctx = a.n_ctx
        q = "q4" if a.quant == "q4" and device != "cpu" else "bf16"
        model, tok = CausalLM.random(cfg, device=device, quant=q), ByteTokenizer()
    else:
        model, tok = CausalLM.from_gguf(a.gguf, device=device, quant=a.quant)
        if a.n_ctx > 0:
            model.cfg.n_ctx = min(a.n_ctx, model.cos.shape[0])
    print(f"[Startup]: context window = {model.cfg.n_ctx} tokens, {model.quant} weights.", flush=True)
    sampler = Sampler(seed=a.seed, mask=tok.printable_mask(model.cfg.vocab))
    d = Splainference(store, model, tok, sampler, a.system_prompt_key, a.max_tokens)
    pending = d.waiting()
    if pending:
        print(f"[Startup]: {len(pending)} waiting key(s) found at cold start.", flush=True)
        for k in pending:
            d.process(k)
    if a.oneshot:
        store.shard_release(SHARD_ID)
        store.close()
        return 0
    last = store.signal_count(a.group)
    print(f"[Active]: Watching signal group {a.group} (count: {last})", flush=True)
    debug_post(store, "[splainference][Active]: Completion daemon online.")
    while _running:
        cur = store.signal_count(a.group)
        if cur == last:
            time.sleep(a.poll_ms / 1e3)
            continue
        for k in d.waiting():
            if not _running:
                break
            d.process(k)
        last = cur
    print("\n[Signal]: Shutting down splainference safely...")
    debug_post(store, "[splainference]: Daemon shutting down.")
    store.shard_release(SHARD_ID)
    store.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
