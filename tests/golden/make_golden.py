#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/.

Run in the dev container (needs `tokenizers` 0.22.2, Pillow, transformers):
    python tests/golden/make_golden.py

Fixtures (data only — inputs and expected outputs):
  clip_synth_tokenizer.json  CLIP-structured tokenizer.json (NFC / \\s+ / lowercase normalizer,
                             CLIP split regex + ByteLevel, BPE with </w>, RobertaProcessing
                             BOS/EOT as the two highest ids) whose merges were trained here with
                             the `tokenizers` BpeTrainer on Python stdlib docstrings.  The real
                             49408-entry CLIP vocab is not available offline.
  tokenizer_golden.json      ids / attention masks from the `tokenizers` 0.22.2 wheel (the crate
                             version the reference pins, Cargo.lock:2807-2808) configured exactly
                             as src/text.rs:76-85 does (Fixed(ctx) padding, truncation max_length=ctx),
                             plus the lowercase=true variant (src/text.rs:115-117).
  preprocess_golden.npz      Pillow 12.2 BICUBIC resize with the reference crop box
                             (src/vision.rs:184-192) of assets/img/cat_face.jpg and of seeded
                             synthetic images, u8 [S,S,3].
  embed_golden.npz           oracle (fp64 restatement) embeddings for seeded weights/inputs, and the
                             HF transformers CLIP embeddings of the same weights/inputs (pin).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

REF_ASSETS = "/root/reference/assets/img"

CLIP_SPLIT = ("<\\|startoftext\\|>|<\\|endoftext\\|>|'s|'t|'re|'ve|'m|'ll|'d|[\\p{L}]+|[\\p{N}]|"
              "[^\\s\\p{L}\\p{N}]+")

TEXTS = [
    "A photo of a cat", "A photo of a dog", "A photo of a beignet", "", " ", "a",
    "Hello, World!!  How's it going?", "I'LL be there; we've done it, they're here, you'd know.",
    "don't stop 'til you get enough", "3.14159 is pi; 42 is the answer; 2024-10-15",
    "Café naïve résumé — coöperate", "Café (decomposed e + acute)", "ﬁﬂ ligatures ﬀ",
    "tab\tseparated\nnew line\r\nand   many    spaces nbsp　ideographic",
    "ΣΑΣ ΟΔΥΣΣΕΥΣ σίσυφος", "İstanbul IŞIK ǅ ǈ", "Straße GROSS ẞ", "漢字かなカナ 한국어 조선말",
    "emoji 😀🎉👍🏽 family 👨‍👩‍👧", "عربي مرحبا", "हिन्दी नमस्ते", "<|endoftext|> special inside",
    "prefix<|startoftext|>suffix", "email@example.com http://x.y/z?q=1&r=2#frag", "@@@### $$$ %%% ^^^",
    "ALL CAPS SENTENCE WITH NUMBERS 123 456", "mixed123letters456and789digits",
    " ".join(["word%d" % i for i in range(120)]),
    "a " * 200, "supercalifragilisticexpialidocious antidisestablishmentarianism",
    "\u0000control\u0007chars\u001b", "zero​width‍joiner", "Ωmega ℃ № ™ ½ ² ⅷ",
]


def corpus():
    import pkgutil
    import importlib
    docs = []
    for m in sorted(["os", "sys", "json", "re", "collections", "itertools", "functools", "typing", "string",
                     "textwrap", "argparse", "logging", "unittest", "email", "http", "urllib", "pathlib",
                     "datetime", "decimal", "fractions", "random", "statistics", "csv", "sqlite3", "zipfile",
                     "tarfile", "shutil", "subprocess", "threading", "asyncio", "socket", "ssl", "hashlib",
                     "inspect", "dis", "ast", "tokenize", "pickle", "copy", "pprint", "heapq", "bisect",
                     "difflib", "calendar", "locale", "gettext", "codecs", "unicodedata", "io", "time"]):
        try:
            mod = importlib.import_module(m)
        except Exception:
            continue
        docs.append(mod.__doc__ or "")
        for name in dir(mod):
            obj = getattr(mod, name, None)
            d = getattr(obj, "__doc__", None)
            if isinstance(d, str):
                docs.append(d)
    docs += ["a photo of a %s" % w for w in ("cat", "dog", "beignet", "car", "beetle", "palace", "coast",
                                              "sunset", "cliff", "plate", "rock", "beach")]
    return docs


def make_tokenizer():
    from tokenizers import Tokenizer, models, normalizers, pre_tokenizers, trainers, Regex
    tok = Tokenizer(models.BPE(end_of_word_suffix="</w>"))
    tok.normalizer = normalizers.Sequence([normalizers.NFC(), normalizers.Replace(Regex(r"\s+"), " "),
                                           normalizers.Lowercase()])
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(CLIP_SPLIT), behavior="removed", invert=True),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    trainer = trainers.BpeTrainer(vocab_size=6000, min_frequency=2, end_of_word_suffix="</w>",
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), show_progress=False)
    tok.train_from_iterator(corpus(), trainer)
    trained = json.loads(tok.to_str())
    merges = trained["model"]["merges"]
    merges = [m if isinstance(m, list) else m.split(" ") for m in merges]
    # CLIP-like id layout: 256 byte chars, 256 byte chars + </w>, merge results, then BOS/EOT.
    alpha = sorted(pre_tokenizers.ByteLevel.alphabet())
    vocab = {}
    for c in alpha:
        vocab[c] = len(vocab)
    for c in alpha:
        vocab[c + "</w>"] = len(vocab)
    kept = []
    for a, b in merges:
        if a in vocab and b in vocab:
            kept.append([a, b])
            if a + b not in vocab:
                vocab[a + b] = len(vocab)
    bos, eot = len(vocab), len(vocab) + 1
    vocab["<|startoftext|>"] = bos
    vocab["<|endoftext|>"] = eot
    spec = {
        "version": "1.0", "truncation": None, "padding": None,
        "added_tokens": [
            {"id": bos, "content": "<|startoftext|>", "single_word": False, "lstrip": False, "rstrip": False,
             "normalized": True, "special": True},
            {"id": eot, "content": "<|endoftext|>", "single_word": False, "lstrip": False, "rstrip": False,
             "normalized": True, "special": True}],
        "normalizer": {"type": "Sequence", "normalizers": [
            {"type": "NFC"}, {"type": "Replace", "pattern": {"Regex": "\\s+"}, "content": " "},
            {"type": "Lowercase"}]},
        "pre_tokenizer": {"type": "Sequence", "pretokenizers": [
            {"type": "Split", "pattern": {"Regex": CLIP_SPLIT}, "behavior": "Removed", "invert": True},
            {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": False}]},
        "post_processor": {"type": "RobertaProcessing", "sep": ["<|endoftext|>", eot],
                           "cls": ["<|startoftext|>", bos], "trim_offsets": False, "add_prefix_space": False},
        "decoder": {"type": "ByteLevel", "add_prefix_space": True, "trim_offsets": True, "use_regex": True},
        "model": {"type": "BPE", "dropout": None, "unk_token": "<|endoftext|>", "continuing_subword_prefix": "",
                  "end_of_word_suffix": "</w>", "fuse_unk": False, "byte_fallback": False,
                  "ignore_merges": False, "vocab": vocab, "merges": [" ".join(m) for m in kept]},
    }
    s = json.dumps(spec, ensure_ascii=False)
    Tokenizer.from_str(s)  # must load in the reference's tokenizers
    with open(os.path.join(HERE, "clip_synth_tokenizer.json"), "w", encoding="utf-8") as f:
        f.write(s)
    return s, bos, eot


def tokenizer_goldens(tok_json, ctx_list=(77, 16)):
    from tokenizers import Tokenizer
    out = {"tokenizers_version": __import__("tokenizers").__version__, "texts": TEXTS, "cases": []}
    for ctx in ctx_list:
        for lower in (False, True):
            t = Tokenizer.from_str(tok_json)
            t.enable_padding(length=ctx, pad_id=0)       # PaddingStrategy::Fixed(ctx), pad_id
            t.enable_truncation(max_length=ctx)          # TruncationParams { max_length: ctx, ..Default }
            texts = [x.lower() for x in TEXTS] if lower else TEXTS  # Python lower ~ Rust to_lowercase
            enc = t.encode_batch(texts, add_special_tokens=True)
            out["cases"].append({"context_length": ctx, "lowercase": lower,
                                 "ids": [e.ids for e in enc], "mask": [e.attention_mask for e in enc]})
    with open(os.path.join(HERE, "tokenizer_golden.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False)


def pillow_resize(rgb, S, mode="shortest", interp="bicubic"):
    from PIL import Image
    H, W = rgb.shape[:2]
    im = Image.fromarray(rgb)
    if mode == "squash":
        box = (0, 0, W, H)
    else:
        scale = S / min(W, H)
        cw = S / scale
        x0, y0 = (W - cw) / 2.0, (H - cw) / 2.0
        # f64 round-off can put the box 1e-14 outside the image; clamp (as csrc/host/preprocess.cpp)
        box = (max(0.0, x0), max(0.0, y0), min(float(W), x0 + cw), min(float(H), y0 + cw))
    f = {"bicubic": Image.BICUBIC, "bilinear": Image.BILINEAR}[interp]
    return np.asarray(im.resize((S, S), f, box=box))


def preprocess_goldens():
    from PIL import Image
    from oracle.weights import synth_images_u8
    data = {}
    cat = os.path.join(REF_ASSETS, "cat_face.jpg")
    if os.path.exists(cat):
        rgb = np.asarray(Image.open(cat).convert("RGB"))
        data["cat_face_224"] = pillow_resize(rgb, 224)
        data["cat_face_shape"] = np.array(rgb.shape)
        # small decoded crop so CPU tests can exercise the C++ resizer on real photo content
        data["cat_face_crop"] = np.ascontiguousarray(rgb[::16, ::16][:160, :200])
        data["cat_face_crop_224"] = pillow_resize(data["cat_face_crop"], 224)
        data["cat_face_crop_64_bilinear"] = pillow_resize(data["cat_face_crop"], 64, interp="bilinear")
    # synthetic sources are regenerated from their seed by the tests (not stored)
    for (h, w) in ((389, 517), (300, 200), (64, 64), (97, 301), (50, 40)):
        img = synth_images_u8(h * 1000 + w, 1, max(h, w))[0][:h, :w].copy()
        data[f"synth_{h}x{w}_64"] = pillow_resize(img, 64)
        data[f"synth_{h}x{w}_64_squash"] = pillow_resize(img, 64, mode="squash")
    np.savez_compressed(os.path.join(HERE, "preprocess_golden.npz"), **data)


def embed_goldens():
    from oracle import clip_ref, hf_pin, weights
    from oracle.model_spec import OPENAI_MEAN, OPENAI_STD, TINY_CFG, VIT_B_32_CFG, text_spec_from_cfg, \
        vision_spec_from_cfg
    out = {}
    for name, cfg, B in (("tiny", TINY_CFG, 3), ("b32", VIT_B_32_CFG, 2)):
        v = vision_spec_from_cfg(cfg["model_cfg"])
        t = text_spec_from_cfg(cfg["model_cfg"])
        u8 = weights.synth_images_u8(100, B, v.image_size)
        px = ((u8.astype(np.float32) / np.float32(255) - np.asarray(OPENAI_MEAN, np.float32))
              / np.asarray(OPENAI_STD, np.float32)).transpose(0, 3, 1, 2)
        P = weights.vision_weights(v, 1234)
        out[f"{name}_vision_oracle"] = clip_ref.encode_image(P, v, px)
        out[f"{name}_vision_hf"] = hf_pin.hf_encode_image(hf_pin.hf_vision(P, v), px)
        ids = weights.synth_token_ids(200, B + 1, t.context_length, t.vocab_size, t.vocab_size - 2,
                                      t.vocab_size - 1, random_eot=True)
        PT = weights.text_weights(t, 1234)
        out[f"{name}_text_ids"] = ids
        out[f"{name}_text_oracle"] = clip_ref.encode_text(PT, t, ids)
        out[f"{name}_text_hf"] = hf_pin.hf_encode_text(hf_pin.hf_text(PT, t), ids)
    np.savez_compressed(os.path.join(HERE, "embed_golden.npz"), **out)


if __name__ == "__main__":
    s, bos, eot = make_tokenizer()
    tokenizer_goldens(s)
    preprocess_goldens()
    embed_goldens()
    print("ok")
