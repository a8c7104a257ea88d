"""Tokenisation parity (CPU): ragmi.encoders.WordPiece — what SentenceTransformer.encode and
CrossEncoder.predict tokenise with (reference main.py:80-90, 211-213, 241-247) — against
(1) transformers.BertTokenizer (5.15: the tokenizer class sentence-transformers loads for
bge-small-en-v1.5 and ms-marco-MiniLM-L-6-v2) built from the same vocab.txt, and (2) the
pure-Python restatement of BERT's BasicTokenizer + WordPiece (oracle/wordpiece_ref.py), id
for id, on text that exercises every normaliser rule: case, accents (NFD + Mn drop), CJK
spacing, control / zero-width / NUL characters, punctuation splitting, 100-char words,
unmatched pieces, empty strings, and pair truncation 'longest_first' at several lengths.
The real checkpoints' vocabularies are not available offline: the vocab is synthetic (words,
subwords, letters, digits, punctuation, accented and CJK characters)."""
import json
import os

import numpy as np
import pytest

import wordpiece_ref as R

WORDS = ("the revenue apple inc company net income fiscal year quarter risk factors financial "
         "report cafe societe resume naive tax billion million share equity operating cash flow "
         "un co operation related growth margin guidance tsmc nvda microsoft 10 k q 2023 "
         "semiconductor supply chain").split()
SUBS = "##ing ##ed ##s ##ly ##ation ##holder ##holders ##er ##al ##ity ##ness ##ive".split()
CJK = list("台積電中国公司收入")
ACCENTED = ["é", "##é", "ï", "##ï", "ç", "café"]


@pytest.fixture(scope="module")
def vocab_file(tmp_path_factory):
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    toks += [chr(c) for c in range(33, 127)]
    toks += ["##" + chr(c) for c in range(ord("a"), ord("z") + 1)]
    toks += ["##" + chr(c) for c in range(ord("0"), ord("9") + 1)]
    toks += WORDS + SUBS + CJK + ACCENTED
    seen, uniq = set(), []
    for t in toks:
        if t not in seen:
            seen.add(t)
            uniq.append(t)
    d = tmp_path_factory.mktemp("vocab")
    f = d / "vocab.txt"
    f.write_text("\n".join(uniq) + "\n", encoding="utf-8")
    return str(f)


TEXTS = [
    "Apple Inc. reported net income of $94.7 billion in fiscal year 2023.",
    "Café Société — Résumé of Risk Factors; naïve co-operation!",
    "台積電 (TSMC) revenue rose 10% in 2023Q4.",
    "Control\x00chars\x07 and\ttabs\nnewlines nbsp ​zero�width",
    "x" * 101 + " ok " + "y" * 100,
    "emoji \U0001F600 here, UPPERCASE Words and shareholders' equity of 1,234.56",
    "un-related growth: margin guidance (10-K), supply-chain risk...",
    "",
    "   leading and trailing   ",
    "Ελληνικά и кириллица mixed with NVDA",
]


def _hf(vocab_file, **kw):
    from transformers import BertTokenizer
    return BertTokenizer(vocab=R.load_vocab(vocab_file), **kw)


@pytest.mark.parametrize("text", TEXTS)
def test_single_text_ids(vocab_file, text):
    from ragmi.encoders import WordPiece
    vocab = R.load_vocab(vocab_file)
    ids, types, cu = WordPiece(vocab_file).encode_packed([text])
    want, want_t = R.encode(text, vocab)
    assert ids.tolist() == want and types.tolist() == want_t
    assert _hf(vocab_file)(text)["input_ids"] == want


@pytest.mark.parametrize("max_length", [8, 16, 24, 512])
def test_pairs_longest_first(vocab_file, max_length):
    from ragmi.encoders import WordPiece
    vocab = R.load_vocab(vocab_file)
    hf = _hf(vocab_file)
    wp = WordPiece(vocab_file, max_length)
    qs = [TEXTS[0], TEXTS[2], TEXTS[6], "", TEXTS[1]]
    cs = [TEXTS[1], TEXTS[6], TEXTS[6], TEXTS[5], ""]
    ids, types, cu = wp.encode_packed(qs, cs)
    for j, (q, c) in enumerate(zip(qs, cs)):
        got = ids[cu[j]:cu[j + 1]].tolist()
        got_t = types[cu[j]:cu[j + 1]].tolist()
        want, want_t = R.encode(q, vocab, pair=c, max_length=max_length)
        assert got == want and got_t == want_t, (q, c)
    # batched, as CrossEncoder.predict calls it (a single-pair call with an empty second
    # text would drop the pair altogether)
    h = hf(qs, cs, truncation="longest_first", max_length=max_length)
    for j, (q, c) in enumerate(zip(qs, cs)):
        want, want_t = R.encode(q, vocab, pair=c, max_length=max_length)
        assert h["input_ids"][j] == want and h["token_type_ids"][j] == want_t, (q, c)


@pytest.mark.parametrize("flags", [dict(do_lower_case=False), dict(strip_accents=False),
                                   dict(tokenize_chinese_chars=False)],
                         ids=["cased", "keep_accents", "no_cjk_split"])
def test_tokenizer_config_honoured(vocab_file, tmp_path, flags):
    """A checkpoint's tokenizer_config.json flags reach the normaliser (from_model_dir)."""
    from ragmi.encoders import WordPiece
    d = tmp_path / "model"
    d.mkdir()
    (d / "vocab.txt").write_text(open(vocab_file, encoding="utf-8").read(), encoding="utf-8")
    (d / "tokenizer_config.json").write_text(json.dumps(dict(flags, model_max_length=512)))
    wp = WordPiece.from_model_dir(str(d))
    vocab = R.load_vocab(vocab_file)
    kw = dict(lowercase=flags.get("do_lower_case", True), strip_accents=flags.get("strip_accents"),
              chinese=flags.get("tokenize_chinese_chars", True))
    hf = _hf(vocab_file, **flags)
    for text in TEXTS:
        ids, _, _ = wp.encode_packed([text])
        want, _ = R.encode(text, vocab, **kw)
        assert ids.tolist() == want, text
        assert hf(text)["input_ids"] == want, text


def test_max_seq_length_from_sentence_bert_config(vocab_file, tmp_path):
    from ragmi.encoders import WordPiece
    d = tmp_path / "m"
    d.mkdir()
    (d / "vocab.txt").write_text(open(vocab_file, encoding="utf-8").read(), encoding="utf-8")
    (d / "sentence_bert_config.json").write_text(json.dumps({"max_seq_length": 12}))
    wp = WordPiece.from_model_dir(str(d))
    ids, _, cu = wp.encode_packed([TEXTS[0]])
    assert wp.max_length == 12 and int(cu[-1]) == 12
    assert ids.tolist() == R.encode(TEXTS[0], R.load_vocab(vocab_file), max_length=12)[0]


def test_longest_first_rule_sweep(vocab_file):
    """The oracle's truncation rule against the product tokenizer for every pair of lengths
    below 24 and max_length 3..30 (single-token words: lengths are exact)."""
    from ragmi.encoders import WordPiece
    vocab = R.load_vocab(vocab_file)
    words = WORDS[:24]
    for ml in range(3, 31):
        wp = WordPiece(vocab_file, ml)
        qs, cs = [], []
        for n1 in range(24):
            for n2 in range(24):
                qs.append(" ".join(words[:n1]))
                cs.append(" ".join(words[:n2]))
        ids, types, cu = wp.encode_packed(qs, cs)
        for j, (q, c) in enumerate(zip(qs, cs)):
            want, want_t = R.encode(q, vocab, pair=c, max_length=ml)
            assert ids[cu[j]:cu[j + 1]].tolist() == want, (ml, q, c)
            assert types[cu[j]:cu[j + 1]].tolist() == want_t


def _fuzz_ascii(rng, n):
    """Random ASCII text: vocab words, case, digits, every punctuation byte, control bytes
    (tab / newline / return / NUL / BEL / VT / FF / DEL), runs of spaces, long words."""
    alpha = [chr(c) for c in range(128)]
    out = []
    for _ in range(n):
        parts = []
        for _ in range(int(rng.integers(0, 30))):
            r = rng.random()
            if r < 0.5:
                w = WORDS[int(rng.integers(len(WORDS)))]
                parts.append(w.upper() if rng.random() < 0.2 else w)
            elif r < 0.8:
                parts.append("".join(alpha[int(c)] for c in rng.integers(0, 128, int(rng.integers(1, 8)))))
            elif r < 0.9:
                parts.append("z" * int(rng.integers(95, 106)))     # around the 100-char limit
            else:
                parts.append(WORDS[int(rng.integers(len(WORDS)))] + "ing")
        out.append((" " if rng.random() < 0.8 else "\t").join(parts))
    return out


def test_native_ascii_path_matches_rust_and_oracle(vocab_file):
    """The host-native tokenizer (rag_wordpiece_encode, csrc/wordpiece_capi.cpp) against the
    Rust tokenizer and the pure-Python oracle on 400 fuzzed ASCII texts and 200 pairs at
    several max_length (truncation), id for id."""
    from ragmi.encoders import WordPiece
    vocab = R.load_vocab(vocab_file)
    rng = np.random.default_rng(17)
    texts = _fuzz_ascii(rng, 400)
    wp = WordPiece(vocab_file)
    assert wp._native is not None, "libragmi.so (rag_wordpiece_*) must be loadable on CPU"
    ids, types, cu = wp.encode_packed(texts)
    r_ids, r_types, r_cu = wp._encode_rust(texts)
    np.testing.assert_array_equal(cu, r_cu)
    np.testing.assert_array_equal(ids, r_ids)
    np.testing.assert_array_equal(types, r_types)
    for j in range(0, 400, 7):
        assert ids[cu[j]:cu[j + 1]].tolist() == R.encode(texts[j], vocab)[0]
    for ml in (9, 17, 40, 512):
        wpm = WordPiece(vocab_file, ml)
        qs, cs = texts[:200], texts[200:]
        a = wpm.encode_packed(qs, cs)
        b = wpm._encode_rust(qs, cs)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
        for j in range(0, 200, 11):
            want, want_t = R.encode(qs[j], vocab, pair=cs[j], max_length=ml)
            assert a[0][a[2][j]:a[2][j + 1]].tolist() == want
            assert a[1][a[2][j]:a[2][j + 1]].tolist() == want_t


def test_native_path_splices_non_ascii_in_order(vocab_file):
    """Mixed batches: non-ASCII entries go through the Rust tokenizer and land in place."""
    from ragmi.encoders import WordPiece
    wp = WordPiece(vocab_file)
    texts = [TEXTS[0], TEXTS[1], TEXTS[6], TEXTS[2], "", TEXTS[9], TEXTS[3]]
    a = wp.encode_packed(texts)
    b = wp._encode_rust(texts)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    pairs = [TEXTS[5], TEXTS[0], TEXTS[1], "", TEXTS[2], TEXTS[6], TEXTS[8]]
    a = wp.encode_packed(texts, pairs)
    b = wp._encode_rust(texts, pairs)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_native_vocab_rules(tmp_path):
    """Vocab file rules of tokenizers' WordPiece::read_file: trailing whitespace trimmed,
    later duplicates win; missing specials are refused."""
    import ctypes

    from ragmi import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    v = b"[PAD]\n[UNK]\n[CLS]\n[SEP]\nab \ncd\r\nab\n"
    _lib.check(L.rag_wordpiece_create(v, len(v), 512, 1, ctypes.byref(h)))
    t = b"ab cd"
    off = np.array([0, len(t)], np.int64)
    ids = np.zeros(16, np.int32)
    ty = np.zeros(16, np.int32)
    cu = np.zeros(2, np.int32)
    fb = np.zeros(1, np.uint8)
    _lib.check(L.rag_wordpiece_encode(h, t, off.ctypes.data_as(_lib.c_i64p), None, None, 1,
                                      ids.ctypes.data_as(_lib.c_i32p), ty.ctypes.data_as(_lib.c_i32p),
                                      cu.ctypes.data_as(_lib.c_i32p), 16,
                                      fb.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
    assert ids[:cu[1]].tolist() == [2, 6, 5, 3]       # "ab" -> line 6 (last wins), "cd" -> 5
    L.rag_wordpiece_destroy(h)
    bad = b"[PAD]\n[CLS]\n[SEP]\n"
    with pytest.raises(_lib.RagmiError):
        _lib.check(L.rag_wordpiece_create(bad, len(bad), 512, 1, ctypes.byref(h)))


def test_native_path_defers_literal_special_tokens(vocab_file):
    """the Rust tokenizer maps a literal "[MASK]" / "[SEP]" / ... in the text to ONE
    special-token id before normalisation; the native byte rules would split it into '[' word
    ']'. Texts and pairs holding one go to the fallback, so ids match the Rust path."""
    from ragmi.encoders import WordPiece
    wp = WordPiece(vocab_file, 64)
    texts = ["what is [MASK] here", "a [SEP] b", "[CLS][cls] Apple [UNK] inc [PAD]",
             "plain text only", "[mask] lower and [Sep] mixed", "bracket [ MASK ] spaced",
             "[MASKED] word", "net income"]
    pairs = ["x [SEP] y", "plain", "q", "[PAD] pad [PAD]", "r", "s", "t", "[MASK]"]
    a = wp.encode_packed(texts)
    b = wp._encode_rust(texts)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    a = wp.encode_packed(texts, pairs)
    b = wp._encode_rust(texts, pairs)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    # the special token really is one id on the Rust path (what the native split would miss)
    ids = wp._encode_rust(["what is [MASK] here"])[0].tolist()
    assert R.load_vocab(vocab_file)["[MASK]"] in ids
