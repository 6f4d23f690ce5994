"""Tokenizers + chat templates for the served model families.

The byte-level BPE vocabularies (128,256 ids for Llama-3, 32,000 for Mixtral) are
trained offline by tools/train_tokenizer.py and shipped gzip'd next to this file;
the `tokenizers` (Rust) library does encode/decode.  The chat templates reproduce
the Llama-3 header format and the Mistral [INST] format, so a request is
``[system, user]`` exactly as ag2 sent it to Groq.
"""
from __future__ import annotations

import functools
import gzip
from pathlib import Path

from tokenizers import Tokenizer as _HFTok

_DIR = Path(__file__).resolve().parent


def _bytes_to_unicode() -> dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


_U2B = {u: b for b, u in _bytes_to_unicode().items()}


class Tokenizer:
    def __init__(self, flavor: str = "llama3", path: str | None = None):
        """path: a real checkpoint's ``tokenizer.json`` (HF tokenizers format);
        default: the shipped synthetic vocabulary of the flavor."""
        if path:
            self._tok = _HFTok.from_file(str(path))
        else:
            with gzip.open(_DIR / f"{flavor}_synth.json.gz", "rb") as f:
                self._tok = _HFTok.from_str(f.read().decode())
        self.flavor = flavor
        self.path = str(path) if path else None      # to rebuild it in another process
        self.vocab_size = self._tok.get_vocab_size()
        self._content_prefixes: list[str] = []
        self._raw_prefixes: dict[str, tuple[list[int], int]] = {}
        if flavor == "llama3":
            self.bos_id = self._tok.token_to_id("<|begin_of_text|>")
            self.eot_id = self._tok.token_to_id("<|eot_id|>")
            self.eos_ids = (self._tok.token_to_id("<|end_of_text|>"), self.eot_id)
            self._hdr_start = self._tok.token_to_id("<|start_header_id|>")
            self._hdr_end = self._tok.token_to_id("<|end_header_id|>")
        else:
            self.bos_id = self._tok.token_to_id("<s>")
            self.eot_id = self._tok.token_to_id("</s>")
            self.eos_ids = (self.eot_id,)

    # -------------------------------------------------------------- encode/decode
    def encode(self, text: str) -> list[int]:
        for raw, (ids, last_start) in self._raw_prefixes.items():
            if text.startswith(raw) and self._splits_at(text, last_start, len(raw)):
                return ids + self._tok.encode(text[len(raw):], add_special_tokens=False).ids
        return self._tok.encode(text, add_special_tokens=False).ids

    def register_prefix(self, prefix: str) -> None:
        """Declare a long string that many messages start with (the RFQ extraction
        template is ~84 % of every user message).  chat_ids() then encodes it once:
        BPE never merges across pre-tokenizer splits, so when the text's pre-token
        boundaries include the end of the prefix, encode(prefix + rest) ==
        encode(prefix) + encode(rest) exactly; the boundary is checked per text."""
        if prefix and prefix not in self._content_prefixes:
            self._content_prefixes.append(prefix)

    def _splits_at(self, text: str, start: int, pos: int) -> bool:
        """True if the pre-tokenizer puts a boundary at ``pos`` in ``text`` (``start`` =
        beginning of the pre-token that ends at ``pos`` in the cached prefix)."""
        pre = self._tok.pre_tokenizer
        if pre is None:
            return True
        window = text[start:pos + 64]
        return any(end == pos - start for _, (_, end) in pre.pre_tokenize_str(window))

    def _cache_raw_prefix(self, raw: str) -> None:
        if raw in self._raw_prefixes or len(self._raw_prefixes) >= 64:
            return
        pre = self._tok.pre_tokenizer
        last_start = pre.pre_tokenize_str(raw)[-1][1][0] if pre is not None else 0
        self._raw_prefixes[raw] = (self._tok.encode(raw, add_special_tokens=False).ids,
                                   last_start)

    def _encode_segment(self, seg: str, content_at: int = 0) -> list[int]:
        """encode(seg) where a registered content prefix may start at ``content_at``."""
        for p in self._content_prefixes:
            if seg.startswith(p, content_at):
                self._cache_raw_prefix(seg[:content_at + len(p)])
                break
        return self.encode(seg)

    def encode_batch(self, texts: list[str]) -> list[list[int]]:
        return [e.ids for e in self._tok.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids, skip_special: bool = True) -> str:
        return self._tok.decode(list(ids), skip_special_tokens=skip_special)

    @functools.lru_cache(maxsize=1)
    def token_bytes_table(self) -> list[bytes | None]:
        """Raw bytes of every id (None for special/added tokens)."""
        out: list[bytes | None] = [None] * self.vocab_size
        added = {t.content for t in self._tok.get_added_tokens_decoder().values()}
        for s, i in self._tok.get_vocab(with_added_tokens=True).items():
            if s in added or i >= self.vocab_size:
                continue
            try:
                out[i] = bytes(_U2B[c] for c in s)
            except KeyError:
                out[i] = None
        return out

    # ------------------------------------------------------------- chat template
    def chat_ids(self, messages: list[dict], add_generation_prompt: bool = True) -> list[int]:
        if self.flavor == "llama3":
            ids = [self.bos_id]
            for m in messages:
                ids += [self._hdr_start] + self.encode(m["role"]) + [self._hdr_end]
                ids += self._encode_segment("\n\n" + m["content"].strip(), 2) + [self.eot_id]
            if add_generation_prompt:
                ids += [self._hdr_start] + self.encode("assistant") + [self._hdr_end]
                ids += self.encode("\n\n")
            return ids
        # Mistral/Mixtral: system text is folded into the first user turn
        sys_txt = "".join(m["content"] for m in messages if m["role"] == "system")
        ids = [self.bos_id]
        for m in messages:
            if m["role"] == "user":
                body = (sys_txt + "\n\n" + m["content"]) if sys_txt else m["content"]
                sys_txt = ""
                ids += self._encode_segment(f"[INST] {body} [/INST]",
                                            len(body) - len(m["content"]) + 7)
            elif m["role"] == "assistant":
                ids += self.encode(m["content"]) + [self.eot_id]
        return ids

    def shared_prefix_len(self, a: list[int], b: list[int]) -> int:
        n = 0
        for x, y in zip(a, b):
            if x != y:
                break
            n += 1
        return n


@functools.lru_cache(maxsize=4)
def get_tokenizer(flavor: str = "llama3", path: str | None = None) -> Tokenizer:
    return Tokenizer(flavor, path)


def flavor_for_vocab(vocab_size: int) -> str:
    return "mixtral" if vocab_size == 32000 else "llama3"
