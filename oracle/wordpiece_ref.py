"""TEST INFRASTRUCTURE ONLY (the checker; never imported by the product package).

Pure-Python restatement of BERT's uncased WordPiece tokenisation — the algorithm behind the
tokenizers of both reference models (bge-small-en-v1.5 and ms-marco-MiniLM-L-6-v2, loaded by
sentence-transformers' `SentenceTransformer` / `CrossEncoder` in the reference's
main.py:80-90 / main2.py:88-103; their tokenizer_config.json: BertTokenizer, do_lower_case
true). Restated from the published algorithm (Google BERT `tokenization.py`: BasicTokenizer +
WordpieceTokenizer; identical in transformers' BertTokenizer before the Rust port):

  basic:  drop NUL / U+FFFD / control chars, map whitespace to ' ' (clean_text); put spaces
          around CJK ideographs (tokenize_chinese_chars); split on whitespace; per token:
          lowercase, then NFD + drop Mn marks (strip_accents defaults to do_lower_case);
          split punctuation (ASCII 33-47, 58-64, 91-96, 123-126 or Unicode P*) into single
          tokens.
  wordpiece: per basic token, greedy longest-match-first against the vocab, continuation
          pieces prefixed '##'; a token longer than 100 chars, or with an unmatchable
          remainder, becomes [UNK] as a whole.
  specials: [CLS] a [SEP] / [CLS] a [SEP] b [SEP], token types 0 / 1; truncation
          'longest_first' to max_length (counting the specials) as the Rust `tokenizers`
          library does it (the fast tokenizer sentence-transformers loads): with budget
          n = max_length - 3, the shorter sequence keeps min(its length, n // 2) tokens (on
          equal lengths the first counts as the shorter) and the longer one the rest, both cut
          at the end. (The pre-Rust Python tokenizer's one-token-at-a-time loop differs on odd
          budgets; the rule here was checked against tokenizers 0.22 for every length pair
          below 30 and max_length 3..39 — tests/test_tokenizer_cpu.py keeps a sweep.)

ragmi.encoders.WordPiece (the product side) runs HuggingFace `tokenizers`; tests compare the
two id for id, and both with transformers.BertTokenizer.
"""
from __future__ import annotations

import unicodedata


def load_vocab(path: str) -> dict[str, int]:
    vocab = {}
    with open(path, encoding="utf-8") as f:
        for i, line in enumerate(f):
            tok = line.rstrip("\n")
            if tok and tok not in vocab:
                vocab[tok] = i
    return vocab


def _is_whitespace(c: str) -> bool:
    if c in (" ", "\t", "\n", "\r"):
        return True
    return unicodedata.category(c) == "Zs"


def _is_control(c: str) -> bool:
    if c in ("\t", "\n", "\r"):
        return False
    return unicodedata.category(c) in ("Cc", "Cf")


def _is_punctuation(c: str) -> bool:
    cp = ord(c)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return unicodedata.category(c).startswith("P")


def _is_cjk(cp: int) -> bool:
    return (0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0x20000 <= cp <= 0x2A6DF or
            0x2A700 <= cp <= 0x2B73F or 0x2B740 <= cp <= 0x2B81F or 0x2B820 <= cp <= 0x2CEAF or
            0xF900 <= cp <= 0xFAFF or 0x2F800 <= cp <= 0x2FA1F)


def basic_tokenize(text: str, lowercase=True, strip_accents=None, chinese=True) -> list[str]:
    out = []
    for c in text:
        cp = ord(c)
        if cp == 0 or cp == 0xFFFD or _is_control(c):
            continue
        out.append(" " if _is_whitespace(c) else c)
    text = "".join(out)
    if chinese:
        text = "".join(f" {c} " if _is_cjk(ord(c)) else c for c in text)
    if strip_accents is None:
        strip_accents = lowercase
    tokens = []
    for tok in text.split():
        if lowercase:
            tok = tok.lower()
        if strip_accents:
            tok = "".join(c for c in unicodedata.normalize("NFD", tok)
                          if unicodedata.category(c) != "Mn")
        cur = ""
        for c in tok:
            if _is_punctuation(c):
                if cur:
                    tokens.append(cur)
                    cur = ""
                tokens.append(c)
            else:
                cur += c
        if cur:
            tokens.append(cur)
    return tokens


def wordpiece(token: str, vocab: dict[str, int], unk="[UNK]", max_chars=100) -> list[str]:
    if len(token) > max_chars:
        return [unk]
    pieces, start = [], 0
    while start < len(token):
        end, cur = len(token), None
        while start < end:
            sub = token[start:end]
            if start > 0:
                sub = "##" + sub
            if sub in vocab:
                cur = sub
                break
            end -= 1
        if cur is None:
            return [unk]
        pieces.append(cur)
        start = end
    return pieces


def tokenize_ids(text: str, vocab: dict[str, int], **kw) -> list[int]:
    return [vocab[p] for t in basic_tokenize(text, **kw) for p in wordpiece(t, vocab)]


def _truncate_longest_first(a: list[int], b: list[int], budget: int):
    if len(a) + len(b) <= budget:
        return list(a), list(b)
    if len(a) > len(b):
        kb = min(len(b), budget // 2)
        return list(a[:budget - kb]), list(b[:kb])
    ka = min(len(a), budget // 2)
    return list(a[:ka]), list(b[:budget - ka])


def encode(text: str, vocab: dict[str, int], pair: str | None = None, max_length: int = 512,
           **kw) -> tuple[list[int], list[int]]:
    """(input_ids, token_type_ids) with specials and 'longest_first' truncation."""
    cls, sep = vocab["[CLS]"], vocab["[SEP]"]
    a = tokenize_ids(text, vocab, **kw)
    if pair is None:
        a = a[:max(max_length - 2, 0)]
        return [cls] + a + [sep], [0] * (len(a) + 2)
    b = tokenize_ids(pair, vocab, **kw)
    a, b = _truncate_longest_first(a, b, max(max_length - 3, 0))
    return [cls] + a + [sep] + b + [sep], [0] * (len(a) + 2) + [1] * (len(b) + 1)
