#!/usr/bin/env python3
"""Regenerate the SentencePiece-style tokenizer fixtures under tests/golden/ (SigLIP2 text tower).

Run in the dev container (needs the `tokenizers` 0.22.2 wheel, the crate version the reference
pins, Cargo.lock:2807-2808):
    python tests/golden/make_sp_tokenizers.py

The reference's TextEmbedder loads whatever tokenizer.json the model folder holds
(src/text.rs:62-85, Tokenizer::from_file); for the SigLIP2 models (README.md:72-80) that is a
Gemma tokenizer (256k SentencePiece BPE with byte fallback), not available offline.  These
fixtures are synthetic files with the structures such tokenizers use, with merges trained here by
the `tokenizers` BpeTrainer on Python stdlib docstrings:

  gemma_synth_tokenizer.json   Gemma: normalizer Replace(" " -> "▁"), no pre-tokenizer, BPE with
                               byte_fallback + fuse_unk over <pad> <eos> <bos> <unk> <mask>, the 256
                               <0xXX> byte pieces and the trained pieces, TemplateProcessing <bos> $A
  spm_prepend_tokenizer.json   Llama-2 style: normalizer Sequence[Prepend("▁"), Replace(" " -> "▁")],
                               TemplateProcessing <bos> $A <eos>
  metaspace_tokenizer.json     Metaspace pre-tokenizer (replacement "▁", prepend_scheme "first",
                               split true), no normalizer, TemplateProcessing $A <eos>
  sp_tokenizer_golden.json     ids / attention masks from the `tokenizers` wheel configured as
                               src/text.rs:76-85 does (Fixed(ctx) padding with pad id 0, truncation
                               max_length = ctx), for ctx 64 and 16, lowercase false / true
                               (src/text.rs:115-117: str::to_lowercase first).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import TEXTS, corpus  # noqa: E402

SPECIALS = ["<pad>", "<eos>", "<bos>", "<unk>", "<mask>"]
EXTRA_TEXTS = ["▁already▁has▁metaspace", "  leading and trailing  ", "<bos>inline special<eos>", "<mask>",
               "x" * 300, "🙂" * 40, "á é combining", "日本語のテキスト、句読点。", "﻿BOM"]


def trained_pieces():
    from tokenizers import Tokenizer, models, normalizers, trainers
    tok = Tokenizer(models.BPE(unk_token="<unk>", byte_fallback=True, fuse_unk=True))
    tok.normalizer = normalizers.Replace(" ", "▁")
    trainer = trainers.BpeTrainer(vocab_size=5000, min_frequency=2, limit_alphabet=400, show_progress=False,
                                  special_tokens=[])
    tok.train_from_iterator(corpus() + TEXTS, trainer)
    t = json.loads(tok.to_str())
    merges = [m if isinstance(m, list) else m.split(" ") for m in t["model"]["merges"]]
    pieces = sorted(t["model"]["vocab"].items(), key=lambda kv: kv[1])
    return [p for p, _ in pieces], merges


def build(kind, pieces, merges):
    vocab = {}
    for s in SPECIALS:
        vocab[s] = len(vocab)
    for b in range(256):
        vocab["<0x%02X>" % b] = len(vocab)
    for p in pieces:
        if p not in vocab:
            vocab[p] = len(vocab)
    kept = [[a, b] for a, b in merges if a in vocab and b in vocab and a + b in vocab]
    added = [{"id": vocab[s], "content": s, "single_word": False, "lstrip": False, "rstrip": False,
              "normalized": False, "special": True} for s in SPECIALS]

    def special(tok):
        return {"SpecialToken": {"id": tok, "type_id": 0}}

    seq = {"Sequence": {"id": "A", "type_id": 0}}
    if kind == "gemma":
        normalizer = {"type": "Replace", "pattern": {"String": " "}, "content": "▁"}
        pre = None
        single = [special("<bos>"), seq]
    elif kind == "spm_prepend":
        normalizer = {"type": "Sequence", "normalizers": [{"type": "Prepend", "prepend": "▁"},
                                                          {"type": "Replace", "pattern": {"String": " "},
                                                           "content": "▁"}]}
        pre = None
        single = [special("<bos>"), seq, special("<eos>")]
    else:
        normalizer = None
        pre = {"type": "Metaspace", "replacement": "▁", "prepend_scheme": "first", "split": True}
        single = [seq, special("<eos>")]
    used = sorted({p["SpecialToken"]["id"] for p in single if "SpecialToken" in p})
    spec = {
        "version": "1.0", "truncation": None, "padding": None, "added_tokens": added,
        "normalizer": normalizer, "pre_tokenizer": pre,
        "post_processor": {"type": "TemplateProcessing", "single": single, "pair": single + single[-1:],
                           "special_tokens": {s: {"id": s, "ids": [vocab[s]], "tokens": [s]} for s in used}},
        "decoder": {"type": "Sequence", "decoders": [
            {"type": "Replace", "pattern": {"String": "▁"}, "content": " "}, {"type": "ByteFallback"},
            {"type": "Fuse"}]},
        "model": {"type": "BPE", "dropout": None, "unk_token": "<unk>", "continuing_subword_prefix": None,
                  "end_of_word_suffix": None, "fuse_unk": True, "byte_fallback": True, "ignore_merges": False,
                  "vocab": vocab, "merges": [" ".join(m) for m in kept]},
    }
    return json.dumps(spec, ensure_ascii=False)


def goldens(files, ctx_list=(64, 16)):
    from tokenizers import Tokenizer
    texts = TEXTS + EXTRA_TEXTS
    out = {"tokenizers_version": __import__("tokenizers").__version__, "texts": texts, "cases": []}
    for name in files:
        tok = Tokenizer.from_file(os.path.join(HERE, name))
        for ctx in ctx_list:
            tok.enable_padding(length=ctx, pad_id=0)
            tok.enable_truncation(max_length=ctx)
            for lower in (False, True):
                src = [t.lower() for t in texts] if lower else texts  # Python lower == Rust to_lowercase here
                enc = tok.encode_batch(src)
                out["cases"].append({"file": name, "context_length": ctx, "lowercase": lower,
                                     "ids": [e.ids for e in enc], "mask": [e.attention_mask for e in enc]})
    return out


def main():
    from tokenizers import Tokenizer
    pieces, merges = trained_pieces()
    files = []
    for kind, name in (("gemma", "gemma_synth_tokenizer.json"), ("spm_prepend", "spm_prepend_tokenizer.json"),
                       ("metaspace", "metaspace_tokenizer.json")):
        s = build(kind, pieces, merges)
        Tokenizer.from_str(s)  # must load in the reference's tokenizers
        with open(os.path.join(HERE, name), "w", encoding="utf-8") as f:
            f.write(s)
        files.append(name)
    g = goldens(files)
    with open(os.path.join(HERE, "sp_tokenizer_golden.json"), "w", encoding="utf-8") as f:
        json.dump(g, f, ensure_ascii=False)


if __name__ == "__main__":
    main()
