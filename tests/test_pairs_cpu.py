"""CPU test of the device-side cross-encoder batch assembly (ragmi.pairs.build_pairs, pure
torch ops): against a per-pair loop restating BertTokenizer pair encoding
([CLS] q [SEP] c [SEP], types 0/1) with longest_first truncation of the chunk."""
import numpy as np
import torch


def reference(q_list, rows, c_toks, c_lens, max_len):
    ids, types, cu = [], [], [0]
    for b, q in enumerate(q_list):
        body = list(q[1:-1])                                   # drop the query's CLS/SEP
        for r in rows[b]:
            c = list(c_toks[r][:c_lens[r]])
            c = c[:max(0, max_len - 3 - len(body))]
            seq = [101] + body + [102] + c + [102]
            ids += seq
            types += [0] * (len(body) + 2) + [1] * (len(c) + 1)
            cu.append(cu[-1] + len(seq))
    return np.array(ids), np.array(types), np.array(cu)


def test_build_pairs_matches_loop():
    from ragmi.pairs import build_pairs
    rng = np.random.default_rng(0)
    B, K, R, L = 5, 4, 50, 40
    q_list = [np.r_[101, rng.integers(1000, 30000, n - 2), 102] for n in rng.integers(3, 12, B)]
    q_ids = torch.from_numpy(np.concatenate(q_list).astype(np.int32))
    q_cu = torch.from_numpy(np.r_[0, np.cumsum([len(q) for q in q_list])].astype(np.int32))
    c_toks = rng.integers(1000, 30000, (R, L)).astype(np.int16)
    c_lens = rng.integers(1, L + 1, R).astype(np.int32)
    rows = rng.integers(0, R, (B, K)).astype(np.int64)
    for max_len in (512, 24):                                   # 24: truncation is exercised
        ids, types, cu, mx = build_pairs(q_ids, q_cu, torch.from_numpy(rows),
                                         torch.from_numpy(c_toks), torch.from_numpy(c_lens),
                                         max_len=max_len)
        ri, rt, rc = reference(q_list, rows, c_toks, c_lens, max_len)
        np.testing.assert_array_equal(ids.numpy(), ri)
        np.testing.assert_array_equal(types.numpy(), rt)
        np.testing.assert_array_equal(cu.numpy(), rc)
        assert mx == int(np.diff(rc).max()) and mx <= max_len
        assert ids.dtype == torch.int32 and cu.dtype == torch.int32
