"""C++ CLIP tokenizer (the product, csrc/host/tokenizer.cpp) and the oracle restatement
(oracle/tokenizer_ref.py) vs golden ids from the `tokenizers` 0.22.2 wheel — the crate
version the reference pins (Cargo.lock:2807-2808) — configured as src/text.rs:76-85.
Bar: bit-exact ids and masks."""
import json
import os

import numpy as np
import pytest

from oracle.tokenizer_ref import ClipTokenizerRef

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOK = os.path.join(GOLD, "clip_synth_tokenizer.json")


def golden():
    with open(os.path.join(GOLD, "tokenizer_golden.json"), encoding="utf-8") as f:
        return json.load(f)


def cpp(ctx, pad=0):
    from open_clip_inference.engine import Tokenizer
    return Tokenizer(TOK, ctx, pad)


@pytest.mark.parametrize("case", range(4))
def test_cpp_tokenizer_matches_tokenizers_golden(case):
    g = golden()
    c = g["cases"][case]
    ids, mask = cpp(c["context_length"]).encode_batch(g["texts"], lowercase=c["lowercase"])
    assert ids.tolist() == c["ids"]
    assert mask.tolist() == c["mask"]


@pytest.mark.parametrize("case", range(4))
def test_oracle_tokenizer_matches_tokenizers_golden(case):
    g = golden()
    c = g["cases"][case]
    ref = ClipTokenizerRef(TOK, c["context_length"], 0)
    for i, t in enumerate(g["texts"]):
        ids, mask = ref.encode(t, c["lowercase"])
        assert ids == c["ids"][i], t
        assert mask == c["mask"][i], t


def test_truncation_keeps_eot_at_last_slot():
    """> ctx tokens: content truncated to ctx-2, EOT at index ctx-1 (src/text.rs:81-85)."""
    t = cpp(77)
    ids, mask = t.encode_batch([" ".join(["word"] * 300)])
    eot = t.token_id("<|endoftext|>")
    assert ids[0, 76] == eot and ids[0, 0] == t.token_id("<|startoftext|>")
    assert mask.sum() == 77
    assert int(np.argmax(ids[0])) == 76


def test_padding_and_pad_id_lookup():
    t = cpp(16, pad=3)
    ids, mask = t.encode_batch(["a photo"])
    n = int(mask.sum())
    assert (ids[0, n:] == 3).all() and (mask[0, n:] == 0).all()
    from open_clip_inference.engine import Tokenizer
    from open_clip_inference.error import ConfigError
    with pytest.raises(ConfigError, match="No pad token"):  # no "<pad>" in the vocab (src/text.rs:70-73)
        Tokenizer(TOK, 16, None)


def test_embedded_nul_and_invalid_utf8():
    from open_clip_inference import _lib
    from open_clip_inference.error import TokenizerError
    t = cpp(16)
    a, _ = t.encode_batch(["x\x00y"])
    assert (a[0] != 0).sum() > 2
    import ctypes
    arr = (ctypes.c_char_p * 1)(b"\xff\xfe")
    ids = np.empty((1, 16), np.int64)
    rc = _lib.lib().clipgpu_tokenize(t._h, arr, None, 1, 0, ids.ctypes.data, ids.ctypes.data)
    assert rc == 5 and "UTF-8" in _lib.lib().clipgpu_last_error().decode()
    with pytest.raises(TokenizerError):
        _lib.check(rc)


def test_empty_batch_is_ok_at_tokenizer_level():
    ids, mask = cpp(16).encode_batch([])
    assert ids.shape == (0, 16)


def test_cpp_matches_tokenizers_live_fuzz():
    """Random Unicode-heavy strings vs the live tokenizers wheel (when importable)."""
    tokenizers = pytest.importorskip("tokenizers")
    from hypothesis import given, settings, strategies as st
    ref = tokenizers.Tokenizer.from_file(TOK)
    ref.enable_padding(length=32, pad_id=0)
    ref.enable_truncation(max_length=32)
    tok = cpp(32)
    alphabet = st.characters(blacklist_categories=("Cs",), max_codepoint=0x2FFFF)

    @settings(max_examples=300, deadline=None)
    @given(st.lists(st.text(alphabet=alphabet, max_size=40), min_size=1, max_size=4))
    def check(texts):
        enc = ref.encode_batch(texts)
        ids, mask = tok.encode_batch(texts)
        assert ids.tolist() == [e.ids for e in enc]
        assert mask.tolist() == [e.attention_mask for e in enc]

    check()


# SentencePiece-style BPE tokenizer.json forms (SigLIP2's Gemma tokenizer, README.md:72-80;
# Llama-2's Prepend + Replace; Metaspace): synthetic files and goldens from the tokenizers wheel
# (tests/golden/make_sp_tokenizers.py).
SP_FILES = ["gemma_synth_tokenizer.json", "spm_prepend_tokenizer.json", "metaspace_tokenizer.json"]


def sp_golden():
    with open(os.path.join(GOLD, "sp_tokenizer_golden.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.mark.parametrize("case", range(12))
def test_cpp_sentencepiece_bpe_matches_tokenizers_golden(case):
    """Byte fallback (<0xXX> pieces), fuse_unk, no / Metaspace pre-tokenizer, Prepend / Replace
    normalizers, TemplateProcessing with <bos> before and / or <eos> after $A, truncation to
    ctx - added tokens, Fixed(ctx) padding with pad id 0: bit-exact ids and masks."""
    from open_clip_inference.engine import Tokenizer
    g = sp_golden()
    c = g["cases"][case]
    tok = Tokenizer(os.path.join(GOLD, c["file"]), c["context_length"], 0)
    ids, mask = tok.encode_batch(g["texts"], lowercase=c["lowercase"])
    bad = [i for i in range(len(g["texts"])) if ids[i].tolist() != c["ids"][i]]
    assert not bad, [(g["texts"][i][:40], ids[i].tolist()[:12], c["ids"][i][:12]) for i in bad[:3]]
    assert mask.tolist() == c["mask"]


@pytest.mark.parametrize("name", SP_FILES)
def test_cpp_sentencepiece_bpe_matches_tokenizers_live_fuzz(name):
    tokenizers = pytest.importorskip("tokenizers")
    from hypothesis import given, settings, strategies as st
    from open_clip_inference.engine import Tokenizer
    path = os.path.join(GOLD, name)
    ref = tokenizers.Tokenizer.from_file(path)
    ref.enable_padding(length=48, pad_id=0)
    ref.enable_truncation(max_length=48)
    tok = Tokenizer(path, 48, 0)
    alphabet = st.characters(blacklist_categories=("Cs",), max_codepoint=0x2FFFF)
    words = st.sampled_from(["<bos>", "<eos>", "<mask>", " ", "  ", "▁", "the", "photo", "Straße", "日本"])

    @settings(max_examples=250, deadline=None)
    @given(st.lists(st.lists(st.one_of(st.text(alphabet=alphabet, max_size=12), words), max_size=6).map("".join),
                    min_size=1, max_size=4))
    def check(texts):
        enc = ref.encode_batch(texts)
        ids, mask = tok.encode_batch(texts)
        assert ids.tolist() == [e.ids for e in enc], texts
        assert mask.tolist() == [e.attention_mask for e in enc]

    check()


def test_ignore_merges_looks_up_the_bare_word(tmp_path):
    """Byte-level BPE with ignore_merges and an end_of_word_suffix: a word found in the vocab as is
    (without the suffix) is one token, whatever the merges would make of it (tokenizers 0.22.2
    BPE::tokenize_with_cache).  The CLIP-structured synthetic file with ignore_merges on
    and bare-word entries added, live against the wheel."""
    tokenizers = pytest.importorskip("tokenizers")
    from open_clip_inference.engine import Tokenizer
    with open(TOK, encoding="utf-8") as f:
        tj = json.load(f)
    vocab = tj["model"]["vocab"]
    added = ["photo", "zebra", "xq"]  # bare (suffix-less) entries
    for w in added:
        vocab.setdefault(w, max(vocab.values()) + 1)
    tj["model"]["ignore_merges"] = True
    path = str(tmp_path / "tokenizer.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(tj, f)
    ref = tokenizers.Tokenizer.from_file(path)
    ref.enable_padding(length=24, pad_id=0)
    ref.enable_truncation(max_length=24)
    texts = ["a photo of a zebra", "photo", "xq xqq photos", "the zebra's photo", "a photograph"]
    enc = ref.encode_batch(texts)
    assert vocab["photo"] in enc[1].ids  # the wheel takes the bare entry
    ids, mask = Tokenizer(path, 24, 0).encode_batch(texts)
    assert ids.tolist() == [e.ids for e in enc]
    assert mask.tolist() == [e.attention_mask for e in enc]
