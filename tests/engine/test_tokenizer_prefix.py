"""Registered-prefix encoding (Tokenizer.register_prefix) must be token-identical to
encoding the whole message, including documents whose first characters would merge
with the end of the prompt template under BPE."""
import pytest

from replisense_rfq_amd.engine.tokenizer import get_tokenizer
from replisense_rfq_amd.service.extract import build_messages
from replisense_rfq_amd.service.prompt import register_prompt_prefix
from replisense_rfq_amd.utils import synth

ODD_STARTS = ["", " ", "  leading spaces", "\n\nblank lines", "\"quoted\"", "'s", "123 units",
              "été", "\t tab", "a", "!!!", "\"\"\"\n", "ÄÖÜ Kugellager 6204-2RS"]


@pytest.mark.parametrize("flavor", ["llama3", "mixtral"])
def test_prefix_cache_matches_plain_encoding(flavor):
    plain = get_tokenizer(flavor)
    cached = get_tokenizer(flavor)
    register_prompt_prefix(cached)
    texts = [synth.make_rfq(i).text for i in range(20)] + ODD_STARTS
    texts += [s + synth.make_rfq(99).text for s in ODD_STARTS]
    for t in texts:
        msgs = build_messages(t)
        assert cached.chat_ids(msgs) == plain.chat_ids(msgs), repr(t[:40])
    assert cached._raw_prefixes, "prefix was never cached"
