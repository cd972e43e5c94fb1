"""tests/common.np_rank (the numpy rank() used at full c2 size, where the C
oracle is too slow) against the C oracle's rank() on a small index: docnos and
fp64 score bits, both idf modes."""
import common
import numpy as np
import oracle_lib as O
import pytest


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_np_rank_equals_oracle(synth, idf_mode):
    n = 400
    c = synth.gen_corpus(n, V=2500, seed=19, len_lo=20, len_hi=120)
    ref = O.OracleIndex(c, synth.mapping_bytes(n), 1, 1)
    terms = sorted([t for t in ref.terms() if t[0] != (" ",)], key=lambda t: t[0][0].encode("utf-16-be", "surrogatepass"))
    names = [t[0][0] for t in terms]
    off = np.zeros(len(terms) + 1, np.int64)
    off[1:] = np.cumsum([len(t[3]) for t in terms])
    dn = np.array([d for t in terms for d, _ in t[3]], np.int32)
    tf = np.array([f for t in terms for _, f in t[3]], np.int32)
    df = np.diff(off)
    tq, qo = synth.queries_by_df(df.astype(np.int32), 150, seed=4)
    for q in range(150):
        ids = tq[qo[q]:qo[q + 1]].tolist()
        rd, rs = ref.query([names[t] for t in ids], 10, idf_mode, 0)
        d, s = common.np_rank(off, dn, tf, ids, ref.N, 10, idf_mode, df)
        assert d == rd and s == rs, q
