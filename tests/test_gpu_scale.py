"""The device path at BASELINE config scale.

* c2shard / c5shard: 50,000 docs of the c2 distribution (V_w = 2^20, 400-600
  tokens, ~1,000 query-side tiles... 49 tiles of 1024 docs) and 100,000 docs of
  the c5 distribution (V_w = 30,000, ~56 tokens, 98 tiles), generated in HBM by
  sme_synth_corpus, built on the device and compared with golden results the CPU
  oracle produced for the same corpus (tests/golden/scale_*.json, made by
  tools/gen_scale_golden.py): per-partition record digests, N / V / P / sum tf,
  and top-10 / top-100 query results -- docnos identical, fp64 scores bit-equal --
  for c3-drawn (by df), uniform and true-df-mode queries.
* c2 full size (1M docs, BASELINE configs[1]) in test_c2_full_properties:
  size-independent properties of the built index (sum tf = tokens + docid
  tokens, offsets monotone, reduce order (tf desc, docno asc), docno order of
  the query CSR) and c3-drawn queries over it (configs[2]'s distribution)
  checked against a numpy restatement of rank() over the index's own postings
  (tests/common.py np_rank), docnos and fp64 score bits.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _gold(name):
    path = os.path.join(GOLD, "scale_%s.json" % name)
    if not os.path.exists(path):
        pytest.fail("missing golden fixture %s (run tools/gen_scale_golden.py)" % path)
    return json.load(open(path))


def _build(sme, synth, g, idf_mode=0):
    c = g["config"]
    corpus = sme.DeviceCorpus(c["n"], V=c["V"], seed=c["seed"], len_lo=c["lo"], len_hi=c["hi"])
    ctx = sme.Context(1, c["R"], idf_mode)
    ctx.load_docno_mapping(synth.mapping_bytes(c["n"]))
    ix = ctx.build_device(corpus.ptr, corpus.nbytes)
    return corpus, ctx, ix


def _check_queries(ix, group):
    names = [q[0] for q in group["q"]]
    flat = sorted({t for tl in names for t in tl})
    ids = dict(zip(flat, ix.lookup(flat).tolist()))
    assert min(ids.values()) >= 0  # every golden query term is in the index
    terms = np.array([ids[t] for tl in names for t in tl], np.int32)
    qoff = np.zeros(len(names) + 1, np.int64)
    qoff[1:] = np.cumsum([len(tl) for tl in names])
    k = group["k"]
    dn, sc = ix.query_topk(terms, qoff, k)
    for q, (tl, d, s) in enumerate(group["q"]):
        assert dn[q, :len(d)].tolist() == d, (group["kind"], q, tl)
        assert [float(x).hex() for x in sc[q, :len(d)]] == s, (group["kind"], q, tl)
        assert (dn[q, len(d):] == -1).all()


@pytest.mark.parametrize("name", ["c2shard", "c5shard"])
def test_scale_build_and_queries(sme, synth, name):
    import common
    import hashlib
    g = _gold(name)
    corpus, ctx, ix = _build(sme, synth, g)
    assert hashlib.sha256(corpus.to_host()).hexdigest() == g["corpus_sha256"]
    assert (ix.N, ix.V, ix.P) == (g["N"], g["V"], g["P"])
    off, _, tf, df = ix.csr()
    assert int(tf.astype(np.int64).sum()) == g["sum_tf"]
    for p, h in enumerate(g["parts"]):
        assert common.canon_digest(ix.partition_records(p)) == h, p
    for group in g["queries"]:
        if group["idf_mode"] == 0:
            _check_queries(ix, group)
    ix.close()
    corpus.close()
    # true-df idf mode (log10(floor(N / df)))
    groups = [gr for gr in g["queries"] if gr["idf_mode"] == 1]
    if groups:
        corpus, ctx, ix = _build(sme, synth, g, idf_mode=1)
        for group in groups:
            _check_queries(ix, group)


@pytest.mark.parametrize("opts", [{"win_sample": 0}, {"cand_cap": 64}])
def test_scale_queries_window_modes(sme, synth, opts):
    """The window scorer without the sampled-window stages, and with short
    candidate lists (overflow re-runs), on the c2-shard golden: docnos and fp64
    score bits equal to the oracle's in every mode."""
    g = _gold("c2shard")
    corpus, ctx, ix = _build(sme, synth, g)
    for n, v in opts.items():
        ctx.set_option(n, v)
    for group in g["queries"]:
        if group["idf_mode"] == 0:
            _check_queries(ix, group)
    ix.close()
    corpus.close()


def test_c2_full_properties(sme, synth):
    import common
    n, V, seed, lo, hi = 1_000_000, 1 << 20, 42, 400, 600
    corpus = sme.DeviceCorpus(n, V=V, seed=seed, len_lo=lo, len_hi=hi)
    ctx = sme.Context(1, 1, 0)
    ctx.load_docno_mapping(synth.mapping_bytes(n))
    ix = ctx.build_device(corpus.ptr, corpus.nbytes)
    corpus.close()
    assert ix.N == n
    off, dn, tf, df = ix.csr()
    lens = synth.doc_lengths(0, n, seed, lo, hi)
    assert int(tf.astype(np.int64).sum()) == int(lens.sum()) + n  # every token + the docid term (T7)
    assert off[0] == 0 and off[-1] == ix.P and (np.diff(off) >= 1).all()
    newt = np.zeros(ix.P, bool)
    newt[off[:-1]] = True
    same = ~newt[1:]
    assert (((tf[1:] <= tf[:-1]) | ~same).all())  # tf desc inside a term
    assert (((tf[1:] != tf[:-1]) | (dn[1:] > dn[:-1]) | ~same).all())  # then docno asc
    o2, dd, _ = ix.weights()
    assert np.array_equal(o2, off) and ((dd[1:] > dd[:-1]) | ~same).all()
    del dd, newt, same
    terms, qoff = synth.queries_by_df(df, 300, seed=7)
    for k in (10, 100):
        got_d, got_s = ix.query_topk(terms, qoff, k)
        for q in range(0, 300, 3 if k == 10 else 15):
            rd, rs = common.np_rank(off, dn, tf, terms[qoff[q]:qoff[q + 1]].tolist(), ix.N, k)
            assert got_d[q, :len(rd)].tolist() == rd, (k, q)
            assert got_s[q, :len(rd)].tolist() == rs, (k, q)  # fp64 bit-equal
