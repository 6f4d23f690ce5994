"""Train the synthetic byte-level BPE tokenizers shipped with the engine.

No Llama-3 / Mixtral tokenizer asset exists offline, so the
engine ships byte-level BPE vocabularies of the *same sizes* trained here on local
text: English docstrings/docs from the Python stdlib and /usr/share/doc, the
extraction prompt, and a synthetic RFQ corpus with extraction-JSON completions.

* llama3 flavour: 128,000 BPE ids + 256 special ids = 128,256 (Llama-3 layout:
  <|begin_of_text|>=128000, <|end_of_text|>=128001, <|start_header_id|>=128006,
  <|end_header_id|>=128007, <|eot_id|>=128009), Llama-3 pre-tokenizer regex.
* mixtral flavour: 32,000 ids with <unk>=0, <s>=1, </s>=2.

Output: gzip'd tokenizer.json files under replisense_rfq_amd/engine/tokenizer/.
Usage: python tools/train_tokenizer.py [--max-mb 60]
"""
from __future__ import annotations

import argparse
import gzip
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers  # noqa: E402

from replisense_rfq_amd.service.prompt import EXTRACTION_PROMPT_TEMPLATE, SYSTEM_MESSAGE  # noqa: E402
from replisense_rfq_amd.utils import synth  # noqa: E402

LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
                r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
OUT = ROOT / "replisense_rfq_amd" / "engine" / "tokenizer"


def text_sources(max_bytes: int):
    budget = max_bytes
    for base in ("/usr/lib/python3.10", "/usr/share/doc"):
        for dirpath, _, files in sorted(os.walk(base)):
            for f in sorted(files):
                if not (f.endswith((".py", ".txt", ".md", ".rst")) or f in ("README", "NEWS")):
                    continue
                try:
                    data = Path(dirpath, f).read_text(encoding="utf-8", errors="ignore")
                except OSError:
                    continue
                budget -= len(data)
                yield data
                if budget <= 0:
                    return


def rfq_sources(n_docs: int):
    for i in range(n_docs):
        d = synth.make_rfq(i)
        yield EXTRACTION_PROMPT_TEMPLATE + '\n"""\n' + d.text + '\n"""'
        yield synth.reference_like_completion(d, seed=i)
    yield SYSTEM_MESSAGE


def train(vocab: int, specials_front: list[str], corpus_mb: int, n_docs: int) -> Tokenizer:
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
    ])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(
        vocab_size=vocab, min_frequency=2, special_tokens=specials_front,
        initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)

    def it():
        yield from rfq_sources(n_docs)
        yield from text_sources(corpus_mb << 20)

    tok.train_from_iterator(it(), trainer=trainer)
    return tok


def llama3(corpus_mb: int, n_docs: int) -> Tokenizer:
    tok = train(128000, [], corpus_mb, n_docs)
    n = tok.get_vocab_size()
    fill = [f"<|filler_{i}|>" for i in range(128000 - n)]
    special = ["<|begin_of_text|>", "<|end_of_text|>", "<|reserved_special_token_0|>",
               "<|reserved_special_token_1|>", "<|reserved_special_token_2|>",
               "<|reserved_special_token_3|>", "<|start_header_id|>", "<|end_header_id|>",
               "<|reserved_special_token_4|>", "<|eot_id|>"]
    special += [f"<|reserved_special_token_{i}|>" for i in range(5, 5 + 256 - len(special))]
    tok.add_special_tokens(fill + special)
    assert tok.get_vocab_size() == 128256, tok.get_vocab_size()
    assert tok.token_to_id("<|begin_of_text|>") == 128000
    assert tok.token_to_id("<|eot_id|>") == 128009
    return tok


def mixtral(corpus_mb: int, n_docs: int) -> Tokenizer:
    tok = train(32000, ["<unk>", "<s>", "</s>"], corpus_mb, n_docs)
    n = tok.get_vocab_size()
    if n < 32000:
        tok.add_special_tokens([f"<filler_{i}>" for i in range(32000 - n)])
    assert tok.get_vocab_size() == 32000 and tok.token_to_id("<s>") == 1
    return tok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mb", type=int, default=48)
    ap.add_argument("--docs", type=int, default=20000)
    args = ap.parse_args()
    OUT.mkdir(parents=True, exist_ok=True)
    for name, fn in (("llama3", llama3), ("mixtral", mixtral)):
        tok = fn(args.max_mb, args.docs)
        data = tok.to_str().encode()
        with open(OUT / f"{name}_synth.json.gz", "wb") as raw, \
                gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
            f.write(data)
        print(f"{name}: vocab={tok.get_vocab_size()} -> {len(data) / 1e6:.1f} MB json")


if __name__ == "__main__":
    main()
