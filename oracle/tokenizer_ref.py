"""Pure-Python restatement of the CLIP tokenizer pipeline — TEST INFRASTRUCTURE.

The reference tokenizes with HF ``tokenizers`` 0.22.2 (Cargo.lock:2807-2808),
configured in TextEmbedder::from_local_dir (src/text.rs:62-85) and driven by
TextEmbedder::tokenize (src/text.rs:110-139).  This restates that crate's
published algorithm for a CLIP tokenizer.json:

1. added tokens are split out (leftmost-longest; ``normalized`` ones after normalisation);
2. normalizer: NFC -> Replace(``\\s+`` -> " ") -> Lowercase (char-wise);
3. pre-tokenizer: Split(CLIP regex, Removed, invert=True) keeps the regex matches,
   then ByteLevel maps each UTF-8 byte to the GPT-2 byte alphabet;
4. BPE: chars of the word, ``</w>`` appended to the last; merge the lowest-rank
   adjacent pair (leftmost first) until none applies;
5. post-processor: [BOS] + tokens + [EOT]; truncation to context_length (content
   truncated to ctx - 2, right); padding Fixed(ctx) with pad_id, mask 1/0.
Pinned against the ``tokenizers`` wheel in tests/test_cpu_tokenizer.py.
"""
from __future__ import annotations

import json
import unicodedata

WHITE_SPACE = set([0x9, 0xA, 0xB, 0xC, 0xD, 0x20, 0x85, 0xA0, 0x1680, 0x2028, 0x2029, 0x202F, 0x205F, 0x3000]
                  + list(range(0x2000, 0x200B)))


def is_letter(ch):
    return unicodedata.category(ch)[0] == "L"


def is_number(ch):
    return unicodedata.category(ch)[0] == "N"


def is_space(ch):
    return ord(ch) in WHITE_SPACE


def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _match_at(s, i):
    """Length of the CLIP split regex match at position i (leftmost-first alternation), 0 if none."""
    for lit in ("<|startoftext|>", "<|endoftext|>", "'s", "'t", "'re", "'ve", "'m", "'ll", "'d"):
        if s.startswith(lit, i):
            return len(lit)
    n = len(s)
    if is_letter(s[i]):                          # [\p{L}]+
        j = i
        while j < n and is_letter(s[j]):
            j += 1
        return j - i
    if is_number(s[i]):                          # [\p{N}]
        return 1
    if not is_space(s[i]):                       # [^\s\p{L}\p{N}]+
        j = i
        while j < n and not (is_space(s[j]) or is_letter(s[j]) or is_number(s[j])):
            j += 1
        return j - i
    return 0


def clip_split(s):
    """Split(pattern, Removed, invert=True): keep the matches, drop the rest."""
    out, i = [], 0
    while i < len(s):
        k = _match_at(s, i)
        if k:
            out.append(s[i:i + k])
            i += k
        else:
            i += 1
    return out


class ClipTokenizerRef:
    def __init__(self, tokenizer_json: str, context_length: int, pad_id: int = 0):
        with open(tokenizer_json, encoding="utf-8") as f:
            d = json.load(f)
        m = d["model"]
        self.vocab = dict(m["vocab"])
        self.ranks = {}
        for r, mg in enumerate(m["merges"]):
            a, b = mg.split(" ") if isinstance(mg, str) else mg
            self.ranks.setdefault((a, b), r)
        self.eow = m.get("end_of_word_suffix") or ""
        self.unk = self.vocab.get(m.get("unk_token")) if m.get("unk_token") else None
        self.added = [(a["content"], a["id"], a.get("normalized", True)) for a in d.get("added_tokens", [])]
        for c, i, _ in self.added:
            self.vocab[c] = i
        pp = d["post_processor"]
        self.cls, self.sep = pp["cls"][1], pp["sep"][1]
        self.ctx = context_length
        self.pad_id = pad_id
        self.b2u = bytes_to_unicode()

    @staticmethod
    def normalize(s):
        s = unicodedata.normalize("NFC", s)
        out, i = [], 0
        while i < len(s):
            if is_space(s[i]):
                while i < len(s) and is_space(s[i]):
                    i += 1
                out.append(" ")
            else:
                out.append(s[i])
                i += 1
        return "".join(ch.lower() for ch in "".join(out))  # char-wise lowercase

    def _split_added(self, pieces, normalized):
        out = []
        for p in pieces:
            if isinstance(p, int):
                out.append(p)
                continue
            start = i = 0
            while i < len(p):
                best = None
                for c, tid, norm in self.added:
                    if norm == normalized and p.startswith(c, i) and (best is None or len(c) > len(best[0])):
                        best = (c, tid)
                if best:
                    if i > start:
                        out.append(p[start:i])
                    out.append(best[1])
                    i += len(best[0])
                    start = i
                else:
                    i += 1
            if start < len(p):
                out.append(p[start:])
        return out

    def bpe(self, word):
        syms = [self.b2u[b] for b in word.encode("utf-8")]
        if not syms:
            return []
        syms[-1] = syms[-1] + self.eow
        while len(syms) > 1:
            best = None
            for i in range(len(syms) - 1):
                r = self.ranks.get((syms[i], syms[i + 1]))
                if r is not None and (best is None or r < best[0]):
                    best = (r, i)
            if best is None:
                break
            i = best[1]
            syms[i:i + 2] = [syms[i] + syms[i + 1]]
        return [self.vocab.get(s, self.unk) for s in syms]

    def encode(self, text, lowercase=False):
        if lowercase:
            text = text.lower()
        pieces = self._split_added([text], False)
        pieces = [p if isinstance(p, int) else self.normalize(p) for p in pieces]
        pieces = self._split_added(pieces, True)
        ids = []
        for p in pieces:
            if isinstance(p, int):
                ids.append(p)
            else:
                for w in clip_split(p):
                    ids += self.bpe(w)
        ids = [self.cls] + ids[:self.ctx - 2] + [self.sep]
        mask = [1] * len(ids) + [0] * (self.ctx - len(ids))
        ids = ids + [self.pad_id] * (self.ctx - len(ids))
        return ids, mask
