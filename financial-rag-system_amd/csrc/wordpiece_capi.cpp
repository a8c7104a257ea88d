// wordpiece_capi.cpp — host-native BERT WordPiece tokenisation for ASCII text (the query strings
// of stage 1: main2.py:170-171 encode(list[str]) tokenises every batch; main.py:245
// CrossEncoder.predict tokenises (query, chunk) pairs). The rule set is exactly the one of the
// Rust `tokenizers` BertWordPieceTokenizer that ragmi.encoders.WordPiece wraps (and of
// oracle/wordpiece_ref.py), restricted to ASCII, where every Unicode rule collapses to a byte
// rule:
//   clean_text   drop NUL and control bytes (0x01-0x08, 0x0B, 0x0C, 0x0E-0x1F, 0x7F; Unicode
//                Cc/Cf/Co/Cn/Cs outside tab/newline/return), map ' ', \t, \n, \r to a space;
//   lowercase    A-Z -> a-z (when the checkpoint's tokenizer_config says do_lower_case);
//   accents, CJK no-ops on ASCII;
//   pre-tokenise split on spaces; every ASCII punctuation byte (33-47, 58-64, 91-96,
//                123-126) is a token of its own;
//   wordpiece    greedy longest match, continuation pieces prefixed "##"; a word longer than
//                100 chars, or with an unmatchable remainder, is one [UNK];
//   specials     [CLS] a [SEP] (b [SEP]), token types 0 / 1, truncation 'longest_first' to
//                max_length as tokenizers 0.22 does it (budget n = max_length - 3: the shorter
//                sequence keeps min(len, n / 2), ties count the first as shorter, the longer
//                one the rest; a single text keeps max_length - 2).
// A text (or pair) with any byte >= 0x80, or holding a literal special-token string such as
// "[MASK]" (matched to one id by the Rust tokenizer before normalisation), is NOT encoded
// here: it is flagged and the caller encodes it with the Rust tokenizer (Unicode
// normalisation tables and the added-token matcher stay out of this file).
// Why native: the Rust tokenizer's Python wrapper costs ~80 us per query string on one host
// thread (~2.5 ms per 32-query batch) and holds the GIL while it builds Encoding objects, which
// serialises a serving loop's kernel launches behind it; this path releases the GIL (ctypes)
// and costs ~1-2 us per string.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ragmi.h"
#include "../../include/ragmi_bert.h"
#include "common_host.hpp"

namespace {

// open-addressing hash of vocab pieces (FNV-1a) -> id
struct PieceTable {
  std::vector<char> arena;
  struct Slot {
    uint64_t h = 0;
    uint32_t off = 0, len = 0;
    int32_t id = -1;
  };
  std::vector<Slot> slots;
  uint64_t mask = 0;

  static uint64_t fnv(const char* p, size_t n, uint64_t h = 1469598103934665603ull) {
    for (size_t i = 0; i < n; ++i) {
      h ^= (unsigned char)p[i];
      h *= 1099511628211ull;
    }
    return h;
  }
  void init(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    slots.assign(cap, Slot{});
    mask = cap - 1;
  }
  // later duplicates overwrite (tokenizers' WordPiece::read_file inserts line by line)
  void put(const char* p, size_t n, int32_t id) {
    const uint64_t h = fnv(p, n);
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      Slot& s = slots[i];
      if (s.id < 0) {
        s.h = h;
        s.off = (uint32_t)arena.size();
        s.len = (uint32_t)n;
        s.id = id;
        arena.insert(arena.end(), p, p + n);
        return;
      }
      if (s.h == h && s.len == n && std::memcmp(arena.data() + s.off, p, n) == 0) {
        s.id = id;
        return;
      }
    }
  }
  // lookup of prefix (optional "##") + p[0..n)
  int32_t get(bool cont, const char* p, size_t n) const {
    uint64_t h = 1469598103934665603ull;
    if (cont) h = fnv("##", 2, h);
    h = fnv(p, n, h);
    const size_t len = n + (cont ? 2 : 0);
    for (uint64_t i = h & mask;; i = (i + 1) & mask) {
      const Slot& s = slots[i];
      if (s.id < 0) return -1;
      if (s.h == h && s.len == len) {
        const char* a = arena.data() + s.off;
        if ((!cont || (a[0] == '#' && a[1] == '#')) && std::memcmp(a + (cont ? 2 : 0), p, n) == 0)
          return s.id;
      }
    }
  }
};

inline bool is_punct(unsigned char c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) ||
         (c >= 123 && c <= 126);
}
inline bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_dropped(unsigned char c) {   // NUL and the other ASCII control bytes
  return (c < 32 && !is_space(c)) || c == 127;
}

}  // namespace

struct rag_wordpiece {
  PieceTable vocab;
  int32_t cls = -1, sep = -1, unk = -1;
  int max_length = 512;
  bool lowercase = true;
};

namespace {

constexpr int kMaxWordChars = 100;

// ASCII text -> piece ids appended to out
void tokenize_ascii(const rag_wordpiece* t, const char* s, size_t n, std::vector<int32_t>& out) {
  std::string word;
  word.reserve(128);
  auto flush_word = [&]() {
    if (word.empty()) return;
    const size_t L = word.size();
    if (L > (size_t)kMaxWordChars) {
      out.push_back(t->unk);
      word.clear();
      return;
    }
    const size_t mark = out.size();
    size_t start = 0;
    while (start < L) {
      size_t end = L;
      int32_t id = -1;
      while (start < end) {
        id = t->vocab.get(start > 0, word.data() + start, end - start);
        if (id >= 0) break;
        --end;
      }
      if (id < 0) {                 // unmatchable remainder: the whole word is [UNK]
        out.resize(mark);
        out.push_back(t->unk);
        word.clear();
        return;
      }
      out.push_back(id);
      start = end;
    }
    word.clear();
  };
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = (unsigned char)s[i];
    if (is_dropped(c)) continue;
    if (is_space(c)) {
      flush_word();
      continue;
    }
    if (t->lowercase && c >= 'A' && c <= 'Z') c = (unsigned char)(c - 'A' + 'a');
    if (is_punct(c)) {
      flush_word();
      word.push_back((char)c);
      flush_word();
      continue;
    }
    word.push_back((char)c);
  }
  flush_word();
}

bool ascii(const char* s, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if ((unsigned char)s[i] >= 0x80) return false;
  return true;
}

// A literal special-token string inside the text ([PAD] [UNK] [CLS] [SEP] [MASK], the tokens
// BertWordPieceTokenizer registers as added special tokens): the Rust tokenizer maps it to ONE
// id before normalisation, where the byte rules above would split it into '[' word ']'. Such a
// text takes the fallback. Matched case-insensitively, which only sends a few more
// texts to the fallback than needed (special tokens match case-sensitively there).
bool has_special(const char* s, size_t n) {
  static const char* const kSpecial[] = {"pad]", "unk]", "cls]", "sep]", "mask]"};
  for (size_t i = 0; i < n; ++i) {
    if (s[i] != '[') continue;
    for (const char* sp : kSpecial) {
      const size_t L = std::strlen(sp);
      if (i + 1 + L > n) continue;
      bool eq = true;
      for (size_t k = 0; k < L && eq; ++k) {
        char c = s[i + 1 + k];
        if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
        eq = c == sp[k];
      }
      if (eq) return true;
    }
  }
  return false;
}

}  // namespace

extern "C" {

int rag_wordpiece_create(const char* vocab_txt, int64_t nbytes, int max_length, int lowercase,
                         rag_wordpiece_t** out) {
  ragmi::clear_error();
  if (!vocab_txt || nbytes < 0 || !out || max_length < 2)
    return ragmi::fail(RAG_EINVAL, "bad wordpiece arguments");
  *out = nullptr;
  auto* t = new rag_wordpiece();
  t->max_length = max_length;
  t->lowercase = lowercase != 0;
  // count lines first (table size), then insert "line.trim_end()" -> line index
  size_t lines = 0;
  for (int64_t i = 0; i < nbytes; ++i) lines += vocab_txt[i] == '\n';
  t->vocab.init(lines + 1);
  int32_t idx = 0;
  int64_t b = 0;
  while (b < nbytes) {
    int64_t e = b;
    while (e < nbytes && vocab_txt[e] != '\n') ++e;
    int64_t te = e;
    while (te > b && (vocab_txt[te - 1] == ' ' || vocab_txt[te - 1] == '\t' ||
                      vocab_txt[te - 1] == '\r' || vocab_txt[te - 1] == '\x0b' ||
                      vocab_txt[te - 1] == '\x0c'))
      --te;
    t->vocab.put(vocab_txt + b, (size_t)(te - b), idx++);
    b = e + 1;
  }
  t->cls = t->vocab.get(false, "[CLS]", 5);
  t->sep = t->vocab.get(false, "[SEP]", 5);
  t->unk = t->vocab.get(false, "[UNK]", 5);
  if (t->cls < 0 || t->sep < 0 || t->unk < 0) {
    delete t;
    return ragmi::fail(RAG_EINVAL, "vocab lacks [CLS], [SEP] or [UNK]");
  }
  *out = t;
  return RAG_OK;
}

int rag_wordpiece_destroy(rag_wordpiece_t* t) {
  delete t;
  return RAG_OK;
}

int rag_wordpiece_encode(const rag_wordpiece_t* t, const char* texts, const int64_t* text_off,
                         const char* pairs, const int64_t* pair_off, int n, int32_t* ids,
                         int32_t* types, int32_t* cu, int64_t cap, uint8_t* fallback) {
  ragmi::clear_error();
  if (!t || n < 0 || (n > 0 && (!texts || !text_off || !ids || !types || !cu || !fallback)) ||
      ((pairs == nullptr) != (pair_off == nullptr)))
    return ragmi::fail(RAG_EINVAL, "bad wordpiece encode arguments");
  std::vector<int32_t> a, bb;
  a.reserve(64);
  bb.reserve(512);
  int64_t T = 0;
  if (cu) cu[0] = 0;   // n == 0 may pass no output arrays
  for (int j = 0; j < n; ++j) {
    const char* s = texts + text_off[j];
    const size_t sn = (size_t)(text_off[j + 1] - text_off[j]);
    const char* p = pairs ? pairs + pair_off[j] : nullptr;
    const size_t pn = pairs ? (size_t)(pair_off[j + 1] - pair_off[j]) : 0;
    if (!ascii(s, sn) || (p && !ascii(p, pn)) || has_special(s, sn) || (p && has_special(p, pn))) {
      fallback[j] = 1;
      cu[j + 1] = (int32_t)T;
      continue;
    }
    fallback[j] = 0;
    a.clear();
    tokenize_ascii(t, s, sn, a);
    size_t ka = a.size(), kb = 0;
    if (p) {
      bb.clear();
      tokenize_ascii(t, p, pn, bb);
      const size_t budget = (size_t)std::max(t->max_length - 3, 0);
      kb = bb.size();
      if (ka + kb > budget) {
        if (ka > kb) {
          kb = std::min(kb, budget / 2);
          ka = budget - kb;
        } else {
          ka = std::min(ka, budget / 2);
          kb = budget - ka;
        }
      }
    } else {
      ka = std::min(ka, (size_t)std::max(t->max_length - 2, 0));
    }
    const int64_t len = (int64_t)ka + 2 + (p ? (int64_t)kb + 1 : 0);
    if (T + len > cap) return ragmi::fail(RAG_ERANGE, "token capacity exceeded");
    int32_t* o = ids + T;
    int32_t* y = types + T;
    *o++ = t->cls;
    *y++ = 0;
    for (size_t i = 0; i < ka; ++i) {
      *o++ = a[i];
      *y++ = 0;
    }
    *o++ = t->sep;
    *y++ = 0;
    if (p) {
      for (size_t i = 0; i < kb; ++i) {
        *o++ = bb[i];
        *y++ = 1;
      }
      *o++ = t->sep;
      *y++ = 1;
    }
    T += len;
    cu[j + 1] = (int32_t)T;
  }
  return RAG_OK;
}

}  // extern "C"
