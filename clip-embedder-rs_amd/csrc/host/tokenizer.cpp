// BPE tokenizer (host, C++).
//
// Replaces the HF `tokenizers` 0.22.2 pipeline the reference drives in
// TextEmbedder (src/text.rs:62-85 setup, :110-139 tokenize) for the BPE tokenizer.json forms of
// the models it runs -- CLIP's byte-level BPE and the SentencePiece-style BPE of SigLIP2's Gemma
// tokenizer (README.md:72-80):
//   added tokens split out (normalized flag honoured, leftmost-longest)
//   normalizer     Sequence of NFC, Lowercase, Replace (Regex \s+ or a string), Prepend, Strip
//                  (CLIP: NFC, \s+ -> " ", Lowercase; Gemma: " " -> "▁"; Llama-2: Prepend "▁", " " -> "▁")
//   pre_tokenizer  CLIP: Sequence[Split(CLIP regex, Removed, invert), ByteLevel(no prefix, no regex)];
//                  none (the normalized text is one word); Metaspace(replacement, prepend_scheme
//                  always / first / never, split)
//   model          BPE: lowest-rank-first merges over byte-level chars or Unicode chars,
//                  end_of_word_suffix / continuing_subword_prefix, unk (fuse_unk), byte_fallback
//                  (<0xXX> pieces), ignore_merges
//   post_processor RobertaProcessing / BertProcessing / TemplateProcessing (any special tokens
//                  before and after $A)
//   truncation     max_length = context_length (content truncated to ctx - added tokens, right)
//   padding        Fixed(context_length), pad_id, right; attention mask 1/0
// Optional str::to_lowercase of the input first (tokenizer_needs_lowercase,
// src/text.rs:115-117; Rust's final-sigma rule applied).
// Unicode tables: tools/gen_unicode_tables.py (classes + lowercase probed from the tokenizers
// wheel's own onig/Rust tables; NFC data from Unicode 13.0).  Pinned against the
// Python `tokenizers` 0.22.2 wheel (same crate version as Cargo.lock:2807-2808)
// by tests/test_cpu_tokenizer.py on committed fixtures.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <queue>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/clipgpu.h"
#include "api_util.hpp"
#include "json.hpp"

namespace clipgpu {
namespace uni {
#include "unicode_tables.inc"

template <size_t N>
static bool in_ranges(const uint32_t (&r)[N][2], uint32_t cp) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (cp < r[mid][0]) hi = mid;
    else if (cp > r[mid][1]) lo = mid + 1;
    else return true;
  }
  return false;
}
bool is_letter(uint32_t cp) { return in_ranges(kLetterRanges, cp); }
bool is_number(uint32_t cp) { return in_ranges(kNumberRanges, cp); }
bool is_space(uint32_t cp) { return in_ranges(kSpaceRanges, cp); }  // onig \s

template <size_t N, size_t W>
static const uint32_t* find_row(const uint32_t (&t)[N][W], uint32_t cp) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (t[mid][0] < cp) lo = mid + 1;
    else hi = mid;
  }
  return (lo < N && t[lo][0] == cp) ? t[lo] : nullptr;
}

void lower_char(uint32_t cp, std::u32string& out) {
  const uint32_t* r = find_row(kLower, cp);
  if (!r) { out.push_back(cp); return; }
  out.push_back(r[2]);
  if (r[1] == 2) out.push_back(r[3]);
}

int ccc(uint32_t cp) {
  const uint32_t* r = find_row(kCCC, cp);
  return r ? (int)r[1] : 0;
}

constexpr uint32_t SBase = 0xAC00, LBase = 0x1100, VBase = 0x1161, TBase = 0x11A7;
constexpr uint32_t LCount = 19, VCount = 21, TCount = 28, NCount = VCount * TCount, SCount = LCount * NCount;

void decompose(uint32_t cp, std::u32string& out) {
  if (cp >= SBase && cp < SBase + SCount) {
    const uint32_t s = cp - SBase;
    out.push_back(LBase + s / NCount);
    out.push_back(VBase + (s % NCount) / TCount);
    if (s % TCount) out.push_back(TBase + s % TCount);
    return;
  }
  const uint32_t* r = find_row(kDecomp, cp);
  if (!r) { out.push_back(cp); return; }
  decompose(r[1], out);
  if (r[2]) decompose(r[2], out);
}

uint32_t compose_pair(uint32_t a, uint32_t b) {
  if (a >= LBase && a < LBase + LCount && b >= VBase && b < VBase + VCount)
    return SBase + ((a - LBase) * VCount + (b - VBase)) * TCount;
  if (a >= SBase && a < SBase + SCount && (a - SBase) % TCount == 0 && b > TBase && b < TBase + TCount)
    return a + (b - TBase);
  size_t lo = 0, hi = sizeof(kComp) / sizeof(kComp[0]);
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (kComp[mid][0] < a || (kComp[mid][0] == a && kComp[mid][1] < b)) lo = mid + 1;
    else hi = mid;
  }
  const size_t N = sizeof(kComp) / sizeof(kComp[0]);
  return (lo < N && kComp[lo][0] == a && kComp[lo][1] == b) ? kComp[lo][2] : 0;
}

std::u32string nfc(const std::u32string& s) {
  std::u32string d;
  d.reserve(s.size());
  for (uint32_t c : s) decompose(c, d);
  // canonical ordering: stable sort each run of non-starters by ccc
  for (size_t i = 0; i < d.size();) {
    if (ccc(d[i]) == 0) { ++i; continue; }
    size_t j = i;
    while (j < d.size() && ccc(d[j]) != 0) ++j;
    std::stable_sort(d.begin() + i, d.begin() + j, [](uint32_t a, uint32_t b) { return ccc(a) < ccc(b); });
    i = j;
  }
  // canonical composition
  std::u32string out;
  out.reserve(d.size());
  int starter = -1;
  int last_cc = -1;
  for (uint32_t c : d) {
    const int cc = ccc(c);
    if (starter >= 0) {
      const bool blocked = last_cc != -1 && (last_cc == 0 ? true : last_cc >= cc);
      const bool adjacent = (int)out.size() - 1 == starter;
      if (adjacent || !blocked) {
        const uint32_t comp = compose_pair(out[starter], c);
        if (comp && (adjacent || last_cc < cc)) {
          out[starter] = comp;
          continue;
        }
      }
    }
    if (cc == 0) {
      starter = (int)out.size();
      last_cc = -1;
    } else {
      last_cc = cc;
    }
    out.push_back(c);
    if (cc == 0) last_cc = -1;
  }
  return out;
}
}  // namespace uni

namespace {

std::u32string utf8_decode(const std::string& s) {
  std::u32string out;
  out.reserve(s.size());
  size_t i = 0;
  while (i < s.size()) {
    const unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 0x6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 0xE) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 0x1E) { cp = c & 0x07; n = 4; }
    else throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: invalid UTF-8 input");
    if (i + n > s.size()) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: truncated UTF-8 input");
    for (int k = 1; k < n; ++k) {
      const unsigned char cc = (unsigned char)s[i + k];
      if ((cc >> 6) != 0x2) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: invalid UTF-8 input");
      cp = (cp << 6) | (cc & 0x3F);
    }
    out.push_back(cp);
    i += n;
  }
  return out;
}

void utf8_append(std::string& out, uint32_t cp) {
  if (cp < 0x80) out += (char)cp;
  else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) {
    out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
  } else {
    out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
    out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
  }
}

std::string utf8_encode(const std::u32string& s) {
  std::string out;
  out.reserve(s.size());
  for (uint32_t c : s) utf8_append(out, c);
  return out;
}

// Rust str::to_lowercase (with the Final_Sigma rule) — src/text.rs:115-117.
std::u32string rust_to_lowercase(const std::u32string& s) {
  std::u32string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == 0x3A3) {
      bool before = false, after = false;
      for (size_t j = i; j-- > 0;) { if (uni::is_letter(s[j])) { before = true; break; } if (uni::ccc(s[j]) == 0 && s[j] != 0x27) break; }
      for (size_t j = i + 1; j < s.size(); ++j) { if (uni::is_letter(s[j])) { after = true; break; } if (uni::ccc(s[j]) == 0 && s[j] != 0x27) break; }
      out.push_back(before && !after ? 0x3C2 : 0x3C3);
      continue;
    }
    uni::lower_char(s[i], out);
  }
  return out;
}

struct AddedToken {
  std::u32string content;
  int64_t id;
  bool normalized;
};

enum NormKind { N_NFC, N_LOWER, N_REPLACE_WS, N_REPLACE_STR, N_STRIP, N_PREPEND };
struct NormStep {
  NormKind kind;
  std::u32string from, to;
};

}  // namespace
}  // namespace clipgpu

struct clipgpu_tokenizer {
  std::unordered_map<std::string, int64_t> vocab;
  std::unordered_map<uint64_t, std::pair<int32_t, int64_t>> merges;  // (a,b) -> (rank, merged id)
  std::vector<clipgpu::AddedToken> added;
  std::vector<clipgpu::NormStep> norm;
  std::string eow = "</w>", cont_prefix;
  int64_t unk = -1;
  std::vector<int64_t> tmpl_pre, tmpl_post;  // post_processor: special ids before / after $A
  int ctx = 77;
  int64_t pad_id = 0;
  bool byte_level = false, add_prefix_space = false, clip_split = false;
  bool byte_fallback = false, fuse_unk = false, ignore_merges = false;
  // Metaspace pre-tokenizer: ' ' -> replacement, prepend_scheme 0 never / 1 first / 2 always,
  // split on the replacement (MergedWithNext)
  bool metaspace = false, ms_split = true;
  int ms_prepend = 2;
  std::u32string ms_repl = U"\u2581";
  int64_t byte_piece[256];  // byte_fallback: id of "<0xXX>" (-1: absent)
  uint32_t byte2cp[256];
};

namespace clipgpu {
namespace {

using json::Value;

const char* kClipPattern1 =
    "<\\|startoftext\\|>|<\\|endoftext\\|>|'s|'t|'re|'ve|'m|'ll|'d|[\\p{L}]+|[\\p{N}]|[^\\s\\p{L}\\p{N}]+";
const char* kClipPattern2 = "'s|'t|'re|'ve|'m|'ll|'d|[\\p{L}]+|[\\p{N}]|[^\\s\\p{L}\\p{N}]+";

void init_bytes(clipgpu_tokenizer& t) {
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
  bool in[256] = {false};
  for (int b : bs) { in[b] = true; t.byte2cp[b] = (uint32_t)b; }
  int n = 0;
  for (int b = 0; b < 256; ++b)
    if (!in[b]) t.byte2cp[b] = 256 + n++;
}

void parse_normalizer(clipgpu_tokenizer& t, const Value* n) {
  if (!n || n->is_null()) return;
  const std::string type = n->get("type") ? n->get("type")->as_str("") : "";
  if (type == "Sequence") {
    const Value* list = n->get("normalizers");
    if (list) for (auto& s : list->arr) parse_normalizer(t, s.get());
  } else if (type == "NFC") {
    t.norm.push_back({N_NFC, {}, {}});
  } else if (type == "Lowercase") {
    t.norm.push_back({N_LOWER, {}, {}});
  } else if (type == "Replace") {
    const Value* pat = n->get("pattern");
    const std::string content = n->get("content") ? n->get("content")->as_str("") : "";
    if (pat && pat->get("Regex") && pat->get("Regex")->as_str("") == "\\s+") {
      t.norm.push_back({N_REPLACE_WS, {}, utf8_decode(content)});
    } else if (pat && pat->get("String")) {
      t.norm.push_back({N_REPLACE_STR, utf8_decode(pat->get("String")->as_str("")), utf8_decode(content)});
    } else {
      throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported Replace normalizer pattern");
    }
  } else if (type == "Strip") {
    t.norm.push_back({N_STRIP, {}, {}});
  } else if (type == "Prepend") {
    t.norm.push_back({N_PREPEND, {}, utf8_decode(n->get("prepend") ? n->get("prepend")->as_str("") : "")});
  } else {
    throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported normalizer " + type);
  }
}

void parse_pretok(clipgpu_tokenizer& t, const Value* p, bool& have_split) {
  if (!p || p->is_null()) return;  // none: the normalized text is one word
  const std::string type = p->get("type") ? p->get("type")->as_str("") : "";
  if (type == "Sequence") {
    const Value* list = p->get("pretokenizers");
    if (list) for (auto& s : list->arr) parse_pretok(t, s.get(), have_split);
  } else if (type == "Split") {
    const Value* pat = p->get("pattern");
    const std::string re = (pat && pat->get("Regex")) ? pat->get("Regex")->as_str("") : "";
    const std::string beh = p->get("behavior") ? p->get("behavior")->as_str("") : "";
    const bool inv = p->get("invert") ? p->get("invert")->as_bool(false) : false;
    if ((re != kClipPattern1 && re != kClipPattern2) || beh != "Removed" || !inv)
      throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported Split pre-tokenizer (CLIP pattern expected)");
    have_split = true;
    t.clip_split = true;
  } else if (type == "ByteLevel") {
    if (p->get("use_regex") && p->get("use_regex")->as_bool(true) && !have_split)
      throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: ByteLevel(use_regex=true) without CLIP Split");
    t.byte_level = true;
    t.add_prefix_space = p->get("add_prefix_space") ? p->get("add_prefix_space")->as_bool(false) : false;
  } else if (type == "Metaspace") {
    t.metaspace = true;
    if (const Value* r = p->get("replacement")) t.ms_repl = utf8_decode(r->as_str("\xe2\x96\x81"));
    if (t.ms_repl.size() != 1) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: Metaspace replacement must be one char");
    const std::string scheme = p->get("prepend_scheme") ? p->get("prepend_scheme")->as_str("always")
                               : (p->get("add_prefix_space") && !p->get("add_prefix_space")->as_bool(true) ? "never"
                                                                                                         : "always");
    if (scheme == "always") t.ms_prepend = 2;
    else if (scheme == "first") t.ms_prepend = 1;
    else if (scheme == "never") t.ms_prepend = 0;
    else throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: Metaspace prepend_scheme " + scheme);
    t.ms_split = p->get("split") ? p->get("split")->as_bool(true) : true;
  } else {
    throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported pre_tokenizer " + type);
  }
}

int64_t special_id(const Value* pair) {  // ["<|endoftext|>", 49407]
  if (!pair || pair->arr.size() != 2) return -1;
  return (int64_t)pair->arr[1]->as_num(-1);
}

void parse_post(clipgpu_tokenizer& t, const Value* p) {
  if (!p || p->is_null()) return;
  const std::string type = p->get("type") ? p->get("type")->as_str("") : "";
  if (type == "RobertaProcessing" || type == "BertProcessing") {
    const int64_t cls = special_id(p->get("cls")), sep = special_id(p->get("sep"));
    if (cls >= 0) t.tmpl_pre.push_back(cls);
    if (sep >= 0) t.tmpl_post.push_back(sep);
  } else if (type == "TemplateProcessing") {
    const Value* single = p->get("single");
    const Value* st = p->get("special_tokens");
    if (!single || !st) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: bad TemplateProcessing");
    int seen_a = 0;
    for (auto& piece : single->arr) {
      if (const Value* sp = piece->get("SpecialToken")) {
        const Value* e = st->get(sp->get("id") ? sp->get("id")->as_str("") : "");
        if (!e || !e->get("ids")) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: TemplateProcessing special token without ids");
        for (auto& id : e->get("ids")->arr) (seen_a ? t.tmpl_post : t.tmpl_pre).push_back((int64_t)id->as_num(-1));
      } else if (piece->get("Sequence")) {
        ++seen_a;
      } else {
        throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported TemplateProcessing piece");
      }
    }
    if (seen_a != 1) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported TemplateProcessing layout");
  } else {
    throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unsupported post_processor " + type);
  }
}

std::u32string normalize(const clipgpu_tokenizer& t, const std::u32string& in) {
  std::u32string s = in;
  for (const NormStep& st : t.norm) {
    std::u32string o;
    switch (st.kind) {
      case N_NFC: s = uni::nfc(s); continue;
      case N_LOWER:
        for (uint32_t c : s) uni::lower_char(c, o);
        break;
      case N_REPLACE_WS:
        for (size_t i = 0; i < s.size();) {
          if (uni::is_space(s[i])) {
            while (i < s.size() && uni::is_space(s[i])) ++i;
            o += st.to;
          } else {
            o.push_back(s[i++]);
          }
        }
        break;
      case N_REPLACE_STR:
        for (size_t i = 0; i < s.size();) {
          if (!st.from.empty() && s.compare(i, st.from.size(), st.from) == 0) {
            o += st.to;
            i += st.from.size();
          } else {
            o.push_back(s[i++]);
          }
        }
        break;
      case N_PREPEND:  // tokenizers Prepend: non-empty strings only
        if (!s.empty()) o = st.to + s;
        break;
      case N_STRIP: {
        size_t a = 0, b = s.size();
        while (a < b && uni::is_space(s[a])) ++a;
        while (b > a && uni::is_space(s[b - 1])) --b;
        o = s.substr(a, b - a);
        break;
      }
    }
    s.swap(o);
  }
  return s;
}

// Pieces of text: either an added-token id (>= 0) or raw text to process.  origin: the piece
// starts at offset 0 of the input (Metaspace prepend_scheme "first").
struct Piece {
  int64_t id;
  std::u32string text;
  bool origin = false;
};

void split_added(const clipgpu_tokenizer& t, std::vector<Piece>& pieces, bool normalized_pass) {
  std::vector<Piece> out;
  for (Piece& p : pieces) {
    if (p.id >= 0) { out.push_back(p); continue; }
    const std::u32string& s = p.text;
    size_t start = 0, i = 0;
    while (i < s.size()) {
      int best = -1;
      size_t best_len = 0;
      for (size_t k = 0; k < t.added.size(); ++k) {
        const AddedToken& a = t.added[k];
        if (a.normalized != normalized_pass || a.content.empty()) continue;
        if (a.content.size() > best_len && s.compare(i, a.content.size(), a.content) == 0) {
          best = (int)k;
          best_len = a.content.size();
        }
      }
      if (best >= 0) {
        if (i > start) out.push_back({-1, s.substr(start, i - start), p.origin && start == 0});
        out.push_back({t.added[best].id, {}, false});
        i += best_len;
        start = i;
      } else {
        ++i;
      }
    }
    if (start < s.size()) out.push_back({-1, s.substr(start), p.origin && start == 0});
  }
  pieces.swap(out);
}

// CLIP split regex (leftmost-first alternation), matches kept, the rest removed.
void clip_pretokenize(const std::u32string& s, std::vector<std::u32string>& words) {
  static const std::u32string st = U"<|startoftext|>", en = U"<|endoftext|>";
  static const char32_t* contractions[] = {U"'s", U"'t", U"'re", U"'ve", U"'m", U"'ll", U"'d"};
  size_t i = 0;
  const size_t n = s.size();
  while (i < n) {
    if (s.compare(i, st.size(), st) == 0) { words.push_back(st); i += st.size(); continue; }
    if (s.compare(i, en.size(), en) == 0) { words.push_back(en); i += en.size(); continue; }
    bool done = false;
    if (s[i] == U'\'') {
      for (const char32_t* c : contractions) {
        const std::u32string cs(c);
        if (s.compare(i, cs.size(), cs) == 0) {
          words.push_back(cs);
          i += cs.size();
          done = true;
          break;
        }
      }
      if (done) continue;
    }
    const uint32_t c = s[i];
    if (uni::is_letter(c)) {
      size_t j = i;
      while (j < n && uni::is_letter(s[j])) ++j;
      words.push_back(s.substr(i, j - i));
      i = j;
    } else if (uni::is_number(c)) {
      words.push_back(s.substr(i, 1));
      ++i;
    } else if (!uni::is_space(c)) {
      size_t j = i;
      while (j < n && !uni::is_space(s[j]) && !uni::is_letter(s[j]) && !uni::is_number(s[j])) ++j;
      words.push_back(s.substr(i, j - i));
      i = j;
    } else {
      ++i;
    }
  }
}

int64_t lookup(const clipgpu_tokenizer& t, const std::string& s) {
  auto it = t.vocab.find(s);
  return it == t.vocab.end() ? -1 : it->second;
}

struct Sym { int64_t id; int prev, next; size_t len; };

// Lowest-rank-first merges over a word's symbols (tokenizers Word::merge_all without dropout).
void bpe_merge(const clipgpu_tokenizer& t, std::vector<Sym>& syms, std::vector<int64_t>& out) {
  if (syms.empty()) return;
  for (size_t i = 0; i < syms.size(); ++i) {
    syms[i].prev = (int)i - 1;
    syms[i].next = i + 1 < syms.size() ? (int)i + 1 : -1;
  }
  struct Cand {
    int32_t rank;
    int pos;
    int64_t new_id;
    bool operator<(const Cand& o) const { return rank != o.rank ? rank > o.rank : pos > o.pos; }  // min-heap
  };
  auto key = [](int64_t a, int64_t b) { return ((uint64_t)(uint32_t)a << 32) | (uint32_t)b; };
  std::priority_queue<Cand> pq;
  for (size_t i = 0; i + 1 < syms.size(); ++i) {
    auto it = t.merges.find(key(syms[i].id, syms[i + 1].id));
    if (it != t.merges.end()) pq.push({it->second.first, (int)i, it->second.second});
  }
  while (!pq.empty()) {
    const Cand c = pq.top();
    pq.pop();
    Sym& a = syms[c.pos];
    if (a.len == 0 || a.next < 0) continue;
    Sym& b = syms[a.next];
    auto it = t.merges.find(key(a.id, b.id));
    if (it == t.merges.end() || it->second.second != c.new_id) continue;  // stale
    a.id = c.new_id;
    a.len += b.len;
    b.len = 0;
    const int bnext = b.next;
    a.next = bnext;
    if (bnext >= 0) syms[bnext].prev = c.pos;
    if (a.prev >= 0) {
      auto jt = t.merges.find(key(syms[a.prev].id, a.id));
      if (jt != t.merges.end()) pq.push({jt->second.first, a.prev, jt->second.second});
    }
    if (a.next >= 0) {
      auto jt = t.merges.find(key(a.id, syms[a.next].id));
      if (jt != t.merges.end()) pq.push({jt->second.first, c.pos, jt->second.second});
    }
  }
  for (int i = 0; i >= 0 && i < (int)syms.size(); i = syms[i].next) out.push_back(syms[i].id);
}

// Byte-level BPE word (CLIP): every byte is one char of the GPT-2 byte alphabet.
void bpe_word(const clipgpu_tokenizer& t, const std::string& word_bytes, std::vector<int64_t>& out) {
  std::vector<std::string> chars;
  for (unsigned char b : word_bytes) {
    std::string c;
    utf8_append(c, t.byte2cp[b]);
    chars.push_back(c);
  }
  if (chars.empty()) return;
  if (t.ignore_merges) {
    std::string whole;
    for (auto& c : chars) whole += c;
    // tokenizers' BPE::tokenize_with_cache looks up the bare word, without end_of_word_suffix
    // (as bpe_chars does; test_ignore_merges_looks_up_the_bare_word)
    const int64_t id = lookup(t, whole);
    if (id >= 0) { out.push_back(id); return; }
  }
  std::vector<Sym> syms;
  for (size_t i = 0; i < chars.size(); ++i) {
    std::string s = (i > 0 ? t.cont_prefix : std::string()) + chars[i];
    if (i + 1 == chars.size()) s += t.eow;
    int64_t id = lookup(t, s);
    if (id < 0) {
      if (t.unk < 0) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unknown symbol and no unk token");
      id = t.unk;
    }
    syms.push_back({id, 0, 0, 1});
  }
  bpe_merge(t, syms, out);
}

// BPE word over Unicode chars (SentencePiece-style tokenizer.json, e.g. Gemma): a char missing
// from the vocab falls back to its UTF-8 bytes as <0xXX> pieces (byte_fallback) or becomes unk
// (consecutive unks fused with fuse_unk), as tokenizers' BPE::merge_word does.
void bpe_chars(const clipgpu_tokenizer& t, const std::u32string& w, std::vector<int64_t>& out) {
  if (w.empty()) return;
  if (t.ignore_merges) {
    const int64_t id = lookup(t, utf8_encode(w));
    if (id >= 0) { out.push_back(id); return; }
  }
  std::vector<Sym> syms;
  int64_t pend_unk = -1;  // a pending (fusable) unk symbol
  size_t pend_len = 0;
  for (size_t i = 0; i < w.size(); ++i) {
    std::string c;
    utf8_append(c, w[i]);
    const size_t byte_len = c.size();
    std::string sym = (i > 0 ? t.cont_prefix : std::string()) + c;
    if (i + 1 == w.size()) sym += t.eow;
    const int64_t id = lookup(t, sym);
    if (id >= 0) {
      if (pend_unk >= 0) { syms.push_back({pend_unk, 0, 0, pend_len}); pend_unk = -1; }
      syms.push_back({id, 0, 0, byte_len});
      continue;
    }
    if (t.byte_fallback) {
      bool all = true;
      for (unsigned char b : sym) all = all && t.byte_piece[b] >= 0;
      if (all) {  // (tokenizers leaves a pending unk in place here)
        for (unsigned char b : sym) syms.push_back({t.byte_piece[b], 0, 0, 1});
        continue;
      }
    }
    if (t.unk < 0) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: unknown symbol and no unk token");
    if (pend_unk >= 0 && t.fuse_unk) {
      pend_len += byte_len;
    } else {
      if (pend_unk >= 0) syms.push_back({pend_unk, 0, 0, pend_len});
      pend_unk = t.unk;
      pend_len = byte_len;
    }
  }
  if (pend_unk >= 0) syms.push_back({pend_unk, 0, 0, pend_len});
  bpe_merge(t, syms, out);
}

// Metaspace pre-tokenizer: ' ' -> replacement, the replacement prepended (scheme), then (split)
// one word per replacement char, merged with what follows it (MergedWithNext).
void metaspace_words(const clipgpu_tokenizer& t, std::u32string s, bool origin, std::vector<std::u32string>& words) {
  const char32_t r = t.ms_repl[0];
  for (auto& c : s)
    if (c == U' ') c = r;
  if ((t.ms_prepend == 2 || (t.ms_prepend == 1 && origin)) && (s.empty() || s[0] != r)) s.insert(s.begin(), r);
  if (!t.ms_split) {
    if (!s.empty()) words.push_back(s);
    return;
  }
  size_t start = 0;
  for (size_t i = 1; i <= s.size(); ++i)
    if (i == s.size() || s[i] == r) {
      if (i > start) words.push_back(s.substr(start, i - start));
      start = i;
    }
}

void encode_one(const clipgpu_tokenizer& t, const std::string& text, bool lowercase, int64_t* ids, int64_t* mask) {
  std::u32string u = utf8_decode(text);
  if (lowercase) u = rust_to_lowercase(u);
  std::vector<Piece> pieces{{-1, u, true}};
  split_added(t, pieces, false);
  for (Piece& p : pieces)
    if (p.id < 0) p.text = normalize(t, p.text);
  split_added(t, pieces, true);
  std::vector<int64_t> content;
  for (const Piece& p : pieces) {
    if (p.id >= 0) { content.push_back(p.id); continue; }
    std::u32string s = p.text;
    if (t.byte_level && t.add_prefix_space && !s.empty() && s[0] != U' ') s.insert(s.begin(), U' ');
    std::vector<std::u32string> words;
    if (t.clip_split) clip_pretokenize(s, words);
    else if (t.metaspace) metaspace_words(t, s, p.origin, words);
    else if (!s.empty()) words.push_back(s);  // no pre-tokenizer: one word
    for (const auto& w : words) {
      if (t.byte_level) bpe_word(t, utf8_encode(w), content);
      else bpe_chars(t, w, content);
    }
  }
  const int n_special = (int)(t.tmpl_pre.size() + t.tmpl_post.size());
  const size_t keep = (size_t)std::max(0, t.ctx - n_special);
  if (content.size() > keep) content.resize(keep);  // TruncationParams: LongestFirst, Right
  std::vector<int64_t> seq(t.tmpl_pre);
  seq.insert(seq.end(), content.begin(), content.end());
  seq.insert(seq.end(), t.tmpl_post.begin(), t.tmpl_post.end());
  if ((int)seq.size() > t.ctx) seq.resize(t.ctx);
  for (int i = 0; i < t.ctx; ++i) {
    const bool real = i < (int)seq.size();
    ids[i] = real ? seq[i] : t.pad_id;
    mask[i] = real ? 1 : 0;
  }
}

}  // namespace
}  // namespace clipgpu

using namespace clipgpu;

extern "C" {

int clipgpu_tokenizer_create(const char* path, int context_length, int64_t pad_id, clipgpu_tokenizer** out) {
  return guarded([&]() {
    if (!out) throw ClipErr(CLIPGPU_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (!path) throw ClipErr(CLIPGPU_ERR_INVALID, "path is NULL");
    if (context_length < 2) throw ClipErr(CLIPGPU_ERR_INVALID, "context_length must be >= 2");
    json::ValuePtr root;
    try {
      root = json::parse_file(path);
    } catch (const std::runtime_error& e) {
      throw ClipErr(std::string(e.what()).rfind("IO", 0) == 0 ? CLIPGPU_ERR_IO : CLIPGPU_ERR_TOKENIZER, e.what());
    }
    std::unique_ptr<clipgpu_tokenizer> t(new clipgpu_tokenizer());
    t->ctx = context_length;
    init_bytes(*t);
    const Value* model = root->get("model");
    if (!model || !model->get("type") || model->get("type")->as_str("") != "BPE")
      throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: only BPE tokenizer.json models are supported");
    const Value* vocab = model->get("vocab");
    if (!vocab) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: BPE model without vocab");
    t->vocab.reserve(vocab->items.size() * 2);
    for (auto& kv : vocab->items) t->vocab[kv.first] = (int64_t)kv.second->as_num(-1);
    if (const Value* e = model->get("end_of_word_suffix")) t->eow = e->as_str("");
    else t->eow.clear();
    if (const Value* c = model->get("continuing_subword_prefix")) t->cont_prefix = c->as_str("");
    if (const Value* u = model->get("unk_token")) {
      if (u->kind == Value::STR) t->unk = lookup(*t, u->str);
    }
    auto flag = [&](const char* k) { const Value* f = model->get(k); return f && !f->is_null() && f->as_bool(false); };
    t->byte_fallback = flag("byte_fallback");
    t->fuse_unk = flag("fuse_unk");
    t->ignore_merges = flag("ignore_merges");
    for (int b = 0; b < 256; ++b) {
      char name[8];
      std::snprintf(name, sizeof(name), "<0x%02X>", b);
      t->byte_piece[b] = lookup(*t, name);
    }
    const Value* merges = model->get("merges");
    if (merges) {
      int32_t rank = 0;
      t->merges.reserve(merges->arr.size() * 2);
      for (auto& m : merges->arr) {
        std::string a, b;
        if (m->kind == Value::STR) {
          const size_t sp = m->str.find(' ');
          if (sp == std::string::npos) throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: bad merge entry");
          a = m->str.substr(0, sp);
          b = m->str.substr(sp + 1);
        } else if (m->kind == Value::ARR && m->arr.size() == 2) {
          a = m->arr[0]->as_str("");
          b = m->arr[1]->as_str("");
        } else {
          throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: bad merge entry");
        }
        const int64_t ia = lookup(*t, a), ib = lookup(*t, b), im = lookup(*t, a + b);
        if (ia < 0 || ib < 0 || im < 0)
          throw ClipErr(CLIPGPU_ERR_TOKENIZER, "Tokenization error: merge '" + a + " " + b + "' not in vocab");
        const uint64_t k = ((uint64_t)(uint32_t)ia << 32) | (uint32_t)ib;
        if (!t->merges.count(k)) t->merges[k] = {rank, im};
        ++rank;
      }
    }
    if (const Value* at = root->get("added_tokens")) {
      for (auto& a : at->arr) {
        AddedToken tok;
        tok.content = utf8_decode(a->get("content") ? a->get("content")->as_str("") : "");
        tok.id = a->get("id") ? (int64_t)a->get("id")->as_num(-1) : -1;
        tok.normalized = a->get("normalized") ? a->get("normalized")->as_bool(true) : true;
        if (tok.id >= 0 && !tok.content.empty()) {
          t->added.push_back(tok);
          t->vocab[utf8_encode(tok.content)] = tok.id;  // get_vocab(with_added_tokens = true)
        }
      }
    }
    parse_normalizer(*t, root->get("normalizer"));
    bool have_split = false;
    parse_pretok(*t, root->get("pre_tokenizer"), have_split);
    parse_post(*t, root->get("post_processor"));
    if (pad_id >= 0) {
      t->pad_id = pad_id;
    } else {  // src/text.rs:70-73
      const int64_t p = lookup(*t, "<pad>");
      if (p < 0) throw ClipErr(CLIPGPU_ERR_CONFIG, "Configuration error: No pad token found in tokenizer");
      t->pad_id = p;
    }
    *out = t.release();
  });
}

void clipgpu_tokenizer_destroy(clipgpu_tokenizer* t) { delete t; }

int clipgpu_tokenize(clipgpu_tokenizer* t, const char* const* texts, const int64_t* lengths, int64_t n,
                     int lowercase, int64_t* ids, int64_t* mask) {
  return guarded([&]() {
    if (!t) throw ClipErr(CLIPGPU_ERR_INVALID, "tokenizer is NULL");
    if (n < 0 || (n > 0 && (!texts || !ids || !mask))) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL buffer");
    for (int64_t i = 0; i < n; ++i) {
      if (!texts[i]) throw ClipErr(CLIPGPU_ERR_INVALID, "NULL text");
      const std::string text = lengths ? std::string(texts[i], (size_t)lengths[i]) : std::string(texts[i]);
      encode_one(*t, text, lowercase != 0, ids + i * t->ctx, mask + i * t->ctx);
    }
  });
}

int64_t clipgpu_tokenizer_token_id(const clipgpu_tokenizer* t, const char* token) {
  if (!t || !token) return -1;
  return lookup(*t, token);
}

int64_t clipgpu_tokenizer_vocab_size(const clipgpu_tokenizer* t) { return t ? (int64_t)t->vocab.size() : -1; }

}  // extern "C"
