"""Device path (libsme.so on gfx950) against the CPU oracle: tokenizer, index
records (bit-exact), CSR, and query top-k."""
import importlib
import json
import os
import random

import common
import numpy as np
import oracle_lib as O
import pytest

pytestmark = pytest.mark.gpu
KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_appendix_b.json")))


@pytest.fixture(scope="module")
def ctx(sme):
    return sme.Context(1, 1)


@pytest.mark.parametrize("text,expected", KAT["process_content"])
def test_device_process_content_kat(ctx, text, expected):
    assert ctx.process_content(text) == expected


@pytest.mark.parametrize("word,expected", KAT["stem"])
def test_device_stem_kat(ctx, word, expected):
    assert ctx.process_content(word) == ([] if O.is_stopword(word) else [expected])


def test_device_process_content_fuzz(ctx):
    rng = random.Random(1234)
    for i in range(300):
        doc = common.fuzz_doc(rng, "X%d" % i, rng.randint(1, 40))
        assert ctx.process_content(doc) == O.process_content(doc), doc


def _check_build(sme, corpus, mapping_ids, R=1, idf_mode=0, K=1, tiebreak=0, opts=None):
    mb = O.write_mapping(mapping_ids)
    ref = O.OracleIndex(corpus, mb, K, R)
    ctx = sme.Context(K, R, idf_mode, tiebreak=tiebreak)
    for name, v in (opts or {}).items():
        ctx.set_option(name, v)
    ctx.load_docno_mapping(mb)
    ix = ctx.build(corpus)
    assert ix.N == ref.N
    for p in range(R):
        common.compare_partitions(ix.partition_records(p), ref.partition_bytes(p))
    if K > 1:
        return ix, ref
    # CSR view equals the oracle's reduce output
    off, dn, tf, df = ix.csr()
    rterms = sorted([t for t in ref.terms() if t[0] != (" ",)], key=lambda t: t[0][0].encode("utf-16-be", "surrogatepass"))
    assert ix.V == len(rterms)
    assert ix.P == sum(len(t[3]) for t in rterms)
    for i, t in enumerate(rterms):
        assert ix.term(i) == t[0][0]
        got = list(zip(dn[off[i]:off[i + 1]].tolist(), tf[off[i]:off[i + 1]].tolist()))
        assert got == [tuple(p) for p in t[3]]
    return ix, ref


def test_build_kat(sme):
    _check_build(sme, KAT["index_corpus"].encode(), KAT["index_mapping"], R=1)
    _check_build(sme, KAT["index_corpus"].encode(), KAT["index_mapping"], R=10)


def test_build_synthetic(sme, synth):
    n = 400
    c = synth.gen_corpus(n, V=5000, seed=1, len_lo=50, len_hi=150)
    _check_build(sme, c, synth.docids(n), R=1)
    _check_build(sme, c, synth.docids(n), R=10)


def test_build_large_segments(sme, synth):
    """Terms with df > 8192 and tf up to ~20: every class of the segmented
    tf-desc sort (one wave, 4-wave and 16-wave blocks) against the reducer order."""
    n = 12000
    c = synth.gen_corpus(n, V=250, seed=11, len_lo=50, len_hi=150)
    ix, _ = _check_build(sme, c, synth.docids(n), R=3)
    off, _, _, _ = ix.csr()
    assert int(np.diff(off).max()) > 8192


@pytest.mark.parametrize("bits", [6, 8, 11])
def test_build_sort_digit_bits(sme, synth, bits):
    """The term sort's LSD digit width (sme_set_option "sort_digit_bits"): 2 to 4
    passes over the same pairs give the reducer's order."""
    n = 3000
    c = synth.gen_corpus(n, V=40000, seed=3, len_lo=40, len_hi=160)
    _check_build(sme, c, synth.docids(n), R=2, opts={"sort_digit_bits": bits})


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_build_fuzz(sme, seed):
    corpus, ids = common.fuzz_corpus(seed, 120)
    _check_build(sme, corpus, ids, R=1)
    _check_build(sme, corpus, ids, R=7)


def test_build_invalid_utf8_and_big_record(sme):
    rng = random.Random(7)
    docs = []
    for i in range(20):
        body = bytes(rng.choice([0x41, 0x62, 0x20, 0xC3, 0xA9, 0xE2, 0x82, 0xFF, 0xF0, 0x9F, 0x98, 0x80, 0x2E, 0x27])
                     for _ in range(rng.randint(0, 300)))
        docs.append(b"<DOC><DOCNO>U%02d</DOCNO>" % i + body + b" </DOC>\n")
    # one record with many distinct terms (global-table aggregation path)
    big = " ".join("t%05d" % i for i in range(5000)).encode()
    docs.append(b"<DOC><DOCNO>BIG</DOCNO>" + big + b"</DOC>")
    _check_build(sme, b"".join(docs), sorted(["U%02d" % i for i in range(20)] + ["BIG"]), R=3)


def test_build_big_records_interleaved(sme, synth):
    """Several records with more distinct terms than the LDS table holds, between
    ordinary ones (single-pass aggregation: their pairs are placed in their own
    regions by the global-table path, in docno order with their neighbours)."""
    rng = random.Random(5)
    docs, ids = [], []
    for i in range(40):
        did = "R%03d" % i
        ids.append(did)
        if i in (3, 17, 18, 39):
            words = ["b%04d" % rng.randrange(3000) for _ in range(2500)] + ["w%02d" % (i % 7)] * 3
        else:
            words = ["w%02d" % rng.randrange(60) for _ in range(rng.randint(20, 200))]
        docs.append(b"<DOC>\n<DOCNO>" + did.encode() + b"</DOCNO>\n" + " ".join(words).encode() + b"\n</DOC>\n")
    _check_build(sme, b"".join(docs), ids, R=3)


@pytest.mark.parametrize("dup", [False, True])
def test_build_high_tf(sme, dup):
    """A term repeated > 1023 times in a record (largest tf past the segmented
    counting sort's LDS counters): the reduce order comes from the composite
    (term, tf desc) radix sort; with a docid repeated across records the
    aggregation's pairs are unpacked and equal docnos merged (the reducer's sum)."""
    rng = random.Random(3)
    docs, ids = [], []
    for i in range(30):
        did = "H%02d" % (i if not (dup and i % 10 == 9) else i - 1)
        ids.append(did)
        words = ["w%02d" % rng.randrange(40) for _ in range(rng.randint(5, 60))]
        if i in (4, 21):
            words += ["flood"] * (1500 + 700 * (i == 21)) + ["w07"] * 1100
        docs.append(b"<DOC>\n<DOCNO>" + did.encode() + b"</DOCNO>\n" + " ".join(words).encode() + b"\n</DOC>\n")
    ix, _ = _check_build(sme, b"".join(docs), sorted(set(ids)), R=3)
    assert int(ix.csr()[2].max()) > 1023


def test_build_dotted_token_tf_past_u16(sme):
    """One dotted non-acronym raw token that splits into > 65535 copies of one
    term (TagTokenizer.tokenAcronymProcessing's split branch, TagTokenizer.java:
    508-522): the record has few raw tokens but a tf past the per-wave u16
    counters, so the aggregation must bound the term count, not the token count."""
    dotted = ".".join(["ab"] * 70000) + "." + ".".join(["cd"] * 3)
    docs = [b"<DOC>\n<DOCNO>X00</DOCNO>\nalpha beta " + dotted.encode() + b" gamma\n</DOC>\n",
            b"<DOC>\n<DOCNO>X01</DOCNO>\nab cd ab alpha\n</DOC>\n"]
    ix, _ = _check_build(sme, b"".join(docs), ["X00", "X01"], R=3)
    assert int(ix.csr()[2].max()) == 70000


def test_build_many_tiny_records(sme):
    """Thousands of records with 0-3 words (a few pairs each, some only the
    docid): a wave's 1024 pairs of the term sort's gather pass span hundreds of
    records, past its 48-record LDS table (the global walk takes over)."""
    rng = random.Random(11)
    docs, ids = [], []
    for i in range(3000):
        did = "T%05d" % i
        ids.append(did)
        words = ["t%03d" % rng.randrange(400) for _ in range(rng.randint(0, 3))]
        if i % 7 == 0:
            words = ["one", "two"]  # stopwords only
        docs.append(b"<DOC>\n<DOCNO>" + did.encode() + b"</DOCNO>\n" + " ".join(words).encode() + b"\n</DOC>\n")
    _check_build(sme, b"".join(docs), ids, R=2)


def test_build_nested_doc_tags(sme):
    """A <DOC> inside a record is content (XMLRecordReader reads to the next
    </DOC>); a start tag after the last </DOC> opens no record."""
    corpus = (b"<DOC><DOCNO>AX1</DOCNO> wolf <DOC><DOCNO>BX2</DOCNO> bear moose </DOC>"
              b"<DOC><DOCNO>CX3</DOCNO> wolf elk </DOC><DOC><DOCNO>DX4</DOCNO> lynx")
    ids = ["AX1", "BX2", "CX3", "DX4"]
    ix, ref = _check_build(sme, corpus, ids, R=1)
    assert ix.N == 2 and ix.V > 0
    _check_build(sme, corpus, ids, R=1, K=2)
    # all-stopword records: no postings at all
    ix, _ = _check_build(sme, b"<DOC><DOCNO>A</DOCNO> one two </DOC>", ["A"], R=1)
    assert (ix.V, ix.P) == (0, 0)


def test_build_empty_and_no_records(sme):
    with pytest.raises(sme.SmeError):
        ctx = sme.Context(1, 1)
        ctx.load_docno_mapping(O.write_mapping(["A"]))
        ctx.build(b"<DOC><DOCNO>A x </DOC>")  # getDocid throws in the reference
    ctx = sme.Context(1, 1)
    ctx.load_docno_mapping(O.write_mapping(["A"]))
    ix = ctx.build(b"no records here")
    assert (ix.N, ix.V, ix.P) == (0, 0, 0)


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_queries_vs_oracle(sme, synth, idf_mode):
    n = 300
    c = synth.gen_corpus(n, V=3000, seed=11, len_lo=40, len_hi=120)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, idf_mode=idf_mode)
    _, _, _, df = ix.csr()
    terms, qoff = synth.queries_by_df(df, 200, seed=7)
    terms[::17] = -1  # unknown terms are skipped
    dn, sc = ix.query_topk(terms, qoff, 10)
    names = [ix.term(i) for i in range(ix.V)]
    for q in range(len(qoff) - 1):
        tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]] if t >= 0]
        rd, rs = ref.query(tl, 10, idf_mode, 0)
        k = len(rd)
        assert dn[q, :k].tolist() == rd, q
        assert np.array_equal(sc[q, :k], np.array(rs)), q  # fp64 bit-exact (same op order)
        assert (dn[q, k:] == -1).all()


def _query_opts(ix, terms, qoff, k, **opts):
    """Query with context path options set (sme_set_option), then restore the defaults."""
    defaults = {"query_kernel": 0, "heavy_div": 128, "seed_tiles": 4, "query_order": 1, "cand_cap": 1024,
                "seed_m": 64, "win_sample": 1}
    try:
        for n, v in opts.items():
            ix.ctx.set_option(n, v)
        return ix.query_topk(terms, qoff, k)
    finally:
        for n in opts:
            ix.ctx.set_option(n, defaults[n])


def _query_both_kernels(ix, terms, qoff, k):
    """Default window-major scoring (seeded threshold, heavy impact rows for terms
    covering >= 1/32 of the docno span), the same on postings only, every term
    heavy, only full-span terms heavy, without seeds, with candidate lists so
    short that most queries overflow to the block-max sweep, the block-max sweep
    itself (4 / 0 / 8 seed tiles, batch order), and the streaming kernel
    (register lists for k <= 32, the LDS candidate list above): all identical bits."""
    dn, sc = ix.query_topk(terms, qoff, k)
    assert ix.ctx.last_build_profile()["query_kernel_name"] in ("k_query_win", "k_query")
    variants = [{"heavy_div": 0}, {"heavy_div": 1 << 30}, {"heavy_div": 1}, {"seed_m": 0}, {"cand_cap": 4},
                {"win_sample": 0}, {"cand_cap": 16, "seed_m": 0},
                {"cand_cap": 1, "heavy_div": 1}, {"query_kernel": 2}, {"query_kernel": 2, "seed_tiles": 0},
                {"query_kernel": 2, "seed_tiles": 8, "query_order": 0}, {"query_kernel": 2, "heavy_div": 0}]
    variants.append({"query_kernel": 1})
    for v in variants:
        dn2, sc2 = _query_opts(ix, terms, qoff, k, **v)
        assert np.array_equal(dn, dn2) and np.array_equal(sc, sc2), v
    return dn, sc


def test_queries_multi_tile(sme, synth):
    """Docnos spanning several 4096-document tiles, negative docnos (unmapped
    docids, T14) below the mapped ones, unknown terms, a query longer than the
    tiled kernel takes (falls back to the streaming kernel)."""
    n = 9000
    c = synth.gen_corpus(n, V=3000, seed=13, len_lo=8, len_hi=30)
    ids = synth.docids(n)
    mapped = [d for i, d in enumerate(ids) if i % 7 != 3]  # every 7th docid unmapped -> negative docno
    ix, ref = _check_build(sme, c, mapped, R=1)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    tu, ou = synth.queries_by_df(df, 60, seed=5, uniform=True)
    td_, od = synth.queries_by_df(df, 8, seed=6)
    tu[::11] = -1
    for terms, qoff in ((tu, ou), (td_, od)):
        dn, sc = _query_both_kernels(ix, terms, qoff, 10)
        for q in range(len(qoff) - 1):
            tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, 10, 0, 0)
            assert dn[q, :len(rd)].tolist() == rd, q
            assert np.array_equal(sc[q, :len(rd)], np.array(rs)), q
    # 64-term queries stay on the block-max kernel (more than its 16 heavy
    # slots: the rest take the posting path); the heaviest terms repeated push
    # every impact sum towards 64 x 254.  A 65-term query sends the whole batch
    # to the streaming kernel.
    heavy = np.argsort(-df, kind="stable")[:8].astype(np.int32)
    # k > 32 with a 65-term query: the streaming kernel's LDS candidate list
    # (round 3 returned SME_ENOTIMPL), several list compactions at k = 40
    for nlong, k in ((64, 10), (65, 10), (65, 40), (65, 100), (65, 448)):
        q64 = np.concatenate([np.repeat(heavy, 4), np.arange(nlong - 32, dtype=np.int32)])
        long_terms = np.concatenate([tu[:ou[3]], q64])
        long_off = np.concatenate([ou[:4], [ou[3] + nlong]]).astype(np.int64)
        dn, sc = ix.query_topk(long_terms, long_off, k)
        assert ix.ctx.last_build_profile()["query_kernel_name"] == ("k_query_win" if nlong == 64 else "k_query")
        for q in range(4):
            tl = [names[t] for t in long_terms[long_off[q]:long_off[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, k, 0, 0)
            assert dn[q, :len(rd)].tolist() == rd and np.array_equal(sc[q, :len(rd)], np.array(rs)), (nlong, k, q)
            assert (dn[q, len(rd):] == -1).all(), (nlong, k, q)
    # queries of more than 128 terms (up to 1024) take the LDS-list kernel at any k;
    # reference tie order holds the token index in 8 bits (<= 256 terms)
    rng = np.random.default_rng(17)
    for nlong, k in ((300, 10), (300, 100), (1024, 10)):
        ql = rng.integers(0, ix.V, size=nlong).astype(np.int32)
        long_terms = np.concatenate([tu[:ou[3]], ql])
        long_off = np.concatenate([ou[:4], [ou[3] + nlong]]).astype(np.int64)
        dn, sc = ix.query_topk(long_terms, long_off, k)
        assert ix.ctx.last_build_profile()["query_kernel_name"] == "k_query"
        for q in range(4):
            tl = [names[t] for t in long_terms[long_off[q]:long_off[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, k, 0, 0)
            assert dn[q, :len(rd)].tolist() == rd and np.array_equal(sc[q, :len(rd)], np.array(rs)), (nlong, k, q)
    too_long = np.zeros(1025, dtype=np.int32)
    with pytest.raises(sme.SmeError):
        ix.query_topk(too_long, np.array([0, 1025], dtype=np.int64), 10)


def test_queries_block_sum_past_16_bits(sme, synth):
    """A 16-document block whose sparse impact sum passes 2^16 in a window whose
    postings are too many to list: 27 rare terms in every document of two groups
    of 16 -- group A in window 0 (first stage), group B in window 3 (last stage),
    where one term occurs twice, so B outranks A and B's block must pass the gate
    that A's scores raised.  Its true sum (16 x (26 x 150 + 254) = 66,464) wraps to
    928 in 16 bits; the window kernel must still score B."""
    n = 17 * 4096
    rare = ["xq" + a + b for a in "bcdfg" for b in "hjklmn"][:27]
    fill = ["zub", "zuc", "zud", "zuf", "zug"]
    ids = synth.docids(n)
    A, B = set(range(16)), set(range(3 * 4096 + 32, 3 * 4096 + 48))
    docs = []
    for i in range(n):
        words = [fill[i % 5], fill[(i + 2) % 5]]
        if i in A:
            words += rare
        if i in B:
            words += rare + rare[:1]
        docs.append(b"<DOC>\n<DOCNO>%s</DOCNO>\n<TEXT>\n%s\n</TEXT>\n</DOC>\n" % (ids[i].encode(), " ".join(words).encode()))
    ix, ref = _check_build(sme, b"".join(docs), ids)
    names = [ix.term(i) for i in range(ix.V)]
    terms = np.array([names.index(w) for w in rare], dtype=np.int32)
    qoff = np.array([0, len(terms)], dtype=np.int64)
    dn, sc = ix.query_topk(terms, qoff, 10)
    assert ix.ctx.last_build_profile()["query_kernel_name"] == "k_query_win"
    rd, rs = ref.query(rare, 10, 0, 0)
    assert dn[0].tolist() == rd and np.array_equal(sc[0], np.array(rs))
    dn2, sc2 = _query_opts(ix, terms, qoff, 10, query_kernel=1)
    assert np.array_equal(dn, dn2) and np.array_equal(sc, sc2)


def test_queries_dense_rows(sme, synth):
    """Hot terms read from per-batch dense tf rows: a small vocabulary makes most
    terms dense, a few documents push one hot term's tf past 255 (its row is
    withdrawn, posting path), queries repeat terms and hold more dense terms
    than the kernel's dense slots; k = 10 and k = 16 instantiations."""
    n = 5000
    c = synth.gen_corpus(n, V=60, seed=21, len_lo=10, len_hi=50)
    blob, offs = synth.make_vocab(60, 21)
    hot = blob[offs[0]:offs[1]].decode()
    extra = b"".join(b"<DOC>\n<DOCNO>Z%04d</DOCNO>\n<TEXT>\n" % i + (hot + " ").encode() * (250 + 7 * i) +
                     b"\n</TEXT>\n</DOC>\n" for i in range(4))
    ix, ref = _check_build(sme, c + extra, synth.docids(n) + ["Z%04d" % i for i in range(4)], R=1)
    assert int(ix.csr()[2].max()) > 255
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    terms, qoff = synth.queries_by_df(df, 40, seed=3, qlen_lo=1, qlen_hi=12)
    terms[5] = terms[4]  # a repeated term
    for k in (10, 16):
        dn, sc = _query_both_kernels(ix, terms, qoff, k)
        for q in range(len(qoff) - 1):
            tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, k, 0, 0)
            assert dn[q, :len(rd)].tolist() == rd, (k, q)
            assert np.array_equal(sc[q, :len(rd)], np.array(rs)), (k, q)


def test_single_term_queries_match_reference_sort(sme, synth):
    """For single-term queries the reference's Collections.sort on DocScore
    leaves the stored (tf desc, docno asc) order: equal to the docno tie-break."""
    n = 200
    c = synth.gen_corpus(n, V=2000, seed=12, len_lo=40, len_hi=80)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1)
    for t in range(0, ix.V, max(1, ix.V // 50)):
        dn, sc = ix.query_topk(np.array([t], np.int32), np.array([0, 1], np.int64), 10)
        rd, rs = ref.query([ix.term(t)], 10, 0, 1)
        assert dn[0, :len(rd)].tolist() == rd


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_queries_reference_order(sme, synth, idf_mode):
    """SME_TIE_REFERENCE: the reference's printed order, checked against the
    oracle's Java 6 Collections.sort over the DocScore comparator (order 1,
    IntDocVectorsForwardIndex.java:195-215,363-365), not against the
    first-encounter restatement -- on both scoring kernels, every heavy-row
    setting, k = 10 / 100, several 1024-doc tiles, unknown and repeated terms.
    The tie words of the results must give back the same order when the
    results are merged (dist._merge_rows)."""
    import torch
    D = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.dist")
    n = 5000
    c = synth.gen_corpus(n, V=800, seed=31, len_lo=20, len_hi=90)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, idf_mode=idf_mode, tiebreak=1)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    terms, qoff = synth.queries_by_df(df, 120, seed=9, qlen_lo=1, qlen_hi=8)
    terms[::13] = -1
    terms[7] = terms[6]
    for k in (10, 100):
        dn, sc = _query_both_kernels(ix, terms, qoff, k)
        dn2, sc2, tie = ix.query_topk(terms, qoff, k, with_tie=True)
        assert np.array_equal(dn, dn2) and np.array_equal(sc, sc2)
        for q in range(len(qoff) - 1):
            tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, k, idf_mode, 1)
            assert dn[q, :len(rd)].tolist() == rd, (k, q)
            assert np.array_equal(sc[q, :len(rd)], np.array(rs)), (k, q)
        # shuffled halves of every row merge back into the same order by the tie words
        perm = np.random.default_rng(k).permutation(k)
        md, ms, _ = D._merge_rows(torch.from_numpy(sc[:, perm]), torch.from_numpy(dn[:, perm]), k,
                                  torch.from_numpy(tie[:, perm].astype(np.int64)))
        assert np.array_equal(md.numpy(), dn) and np.array_equal(ms.numpy(), sc)


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_queries_java7_timsort_order(sme, synth, idf_mode):
    """SME_TIE_JAVA7: rank()'s whole first-encounter list sorted by the JDK 7 GA
    ComparableTimSort over DocScore.compareTo (IntDocVectorsForwardIndex.java:
    195-222,363-365) on the device, held to the oracle's restatement (order 3):
    the same k documents and scores where Java prints a list, docno -2 rows
    where its TimSort throws IllegalArgumentException -- which must happen for
    some of these multi-term queries (profiles/t5_divergence.json: 13 % of c3
    top-10 queries in reference idf mode).  Unknown and repeated terms, k = 10 /
    100, lists past TimSort's 32-element binary-insertion cut."""
    n = 3000
    c = synth.gen_corpus(n, V=600, seed=37, len_lo=20, len_hi=90)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, idf_mode=idf_mode, tiebreak=2)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    terms, qoff = synth.queries_by_df(df, 150, seed=11, qlen_lo=1, qlen_hi=8)
    terms[::17] = -1
    terms[9] = terms[8]
    thrown = listed = 0
    for k in (10, 100):
        dn, sc = ix.query_topk(terms, qoff, k)
        for q in range(len(qoff) - 1):
            tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]] if t >= 0]
            rd, rs = ref.query(tl, k, idf_mode, 3)
            if rd is None:
                thrown += 1
                assert (dn[q] == -2).all(), (k, q)
                continue
            listed += 1
            assert dn[q, :len(rd)].tolist() == rd, (k, q)
            assert np.array_equal(sc[q, :len(rd)], np.array(rs)), (k, q)
            assert (dn[q, len(rd):] == -1).all()
    assert listed > 0
    if idf_mode == 0:
        assert thrown > 0  # the contract-violation path is exercised


def test_queries_reference_order_long(sme, synth):
    """SME_TIE_REFERENCE with queries of more than 256 terms (up to 1024): the
    tie key holds the token index in 10 bits above 22 tf bits for such a batch,
    and the order still equals the oracle's Java 6 Collections.sort; the tie
    words merge shuffled rows back into the same order."""
    import torch
    D = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.dist")
    n = 1500
    c = synth.gen_corpus(n, V=2500, seed=41, len_lo=20, len_hi=90)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, tiebreak=1)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    rng = np.random.default_rng(5)
    lens = [300, 2, 1024, 5, 700]
    terms = np.concatenate([rng.integers(0, ix.V, size=m) for m in lens]).astype(np.int32)
    qoff = np.zeros(len(lens) + 1, np.int64)
    qoff[1:] = np.cumsum(lens)
    for k in (10, 100):
        dn, sc, tie = ix.query_topk(terms, qoff, k, with_tie=True)
        for q in range(len(lens)):
            tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]]]
            rd, rs = ref.query(tl, k, 0, 1)
            assert dn[q, :len(rd)].tolist() == rd, (k, q)
            assert np.array_equal(sc[q, :len(rd)], np.array(rs)), (k, q)
        perm = np.random.default_rng(k).permutation(k)
        md, ms, _ = D._merge_rows(torch.from_numpy(sc[:, perm]), torch.from_numpy(dn[:, perm]), k,
                                  torch.from_numpy(tie[:, perm].astype(np.int64)))
        assert np.array_equal(md.numpy(), dn) and np.array_equal(ms.numpy(), sc)


def test_forward_index_facade(sme):
    indexer = sme.TermKGramDocIndexer(k=1, num_reduce_tasks=1)
    ix = indexer.run(KAT["index_corpus"].encode(), O.write_mapping(KAT["index_mapping"]))
    fw = sme.IntDocVectorsForwardIndex(ix)
    fw.getValue(["cat", "dog", "unknownterm"])
    assert fw.rank() == [1, 2]


@pytest.mark.parametrize("K,R", [(2, 1), (2, 10), (3, 4)])
def test_build_kgram_synthetic(sme, synth, K, R):
    n = 250
    c = synth.gen_corpus(n, V=600, seed=21, len_lo=1, len_hi=60)
    _check_build(sme, c, synth.docids(n), R=R, K=K)


@pytest.mark.parametrize("seed", [4, 5])
def test_build_kgram_fuzz(sme, seed):
    """K = 2 over markup, acronym splits (several terms per raw token), duplicate /
    missing docids, and a record with more distinct 2-grams than the wave table."""
    corpus, ids = common.fuzz_corpus(seed, 100)
    big = " ".join("g%04d" % i for i in range(1500)).encode()
    corpus += b"<DOC><DOCNO>" + ids[0].encode() + b"</DOCNO>" + big + b"</DOC>"
    _check_build(sme, corpus, ids, R=1, K=2)
    _check_build(sme, corpus, ids, R=3, K=2)


@pytest.mark.parametrize("K,R", [(2, 10), (3, 4), (5, 3)])
def test_build_kgram_ranked_keys(sme, synth, K, R):
    """The iterated-ranking gram keys (the path of K * ceil(log2 V) > 63, forced
    here by the kgram_rank option on a small vocabulary): byte-equal records."""
    n = 250
    c = synth.gen_corpus(n, V=600, seed=21, len_lo=1, len_hi=60)
    _check_build(sme, c, synth.docids(n), R=R, K=K, opts={"kgram_rank": 1})
    corpus, ids = common.fuzz_corpus(4, 100)
    _check_build(sme, corpus, ids, R=3, K=2, opts={"kgram_rank": 1})


def test_build_kgram_wide_vocabulary(sme, synth):
    """K = 4 over 1,500 documents of the c2 distribution (V ~ 2e5 terms: 4 x 18
    bits > 63, so the packed term-id keys cannot hold a gram and the device ranks
    them): records byte-equal to the oracle's TermKGramDocIndexer at R = 10."""
    n = 1500
    c = synth.gen_corpus(n, V=1 << 20, seed=42, len_lo=400, len_hi=600)
    ix, _ = _check_build(sme, c, synth.docids(n), R=10, K=4)
    assert ix.V > 100000


def test_kgram_queries_first_element_lookup(sme, synth):
    """K = 2: a query term resolves to the LAST 2-gram starting with it (the
    forward index's Hashtable), as the oracle's rank() does."""
    n = 150
    c = synth.gen_corpus(n, V=300, seed=8, len_lo=10, len_hi=50)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, K=2)
    firsts = sorted(set(ix.term(i) for i in range(ix.V)))[:60]
    rng = random.Random(5)
    for q in range(40):
        tl = [rng.choice(firsts) for _ in range(rng.randint(1, 3))]
        ids = ix.lookup(tl)
        dn, sc = ix.query_topk(ids.astype(np.int32), np.array([0, len(ids)], np.int64), 10)
        rd, rs = ref.query(tl, 10, 0, 0)
        assert dn[0, :len(rd)].tolist() == rd, (q, tl)
        assert np.array_equal(sc[0, :len(rd)], np.array(rs))


def _java_trim(s):
    b, e = 0, len(s)
    while b < e and ord(s[b]) <= 0x20:
        b += 1
    while e > b and ord(s[e - 1]) <= 0x20:
        e -= 1
    return s[b:e]


def _mutf8(s):
    raw = s.encode("utf-16-be", "surrogatepass")
    out = bytearray()
    for i in range(0, len(raw), 2):
        c = (raw[i] << 8) | raw[i + 1]
        if 1 <= c <= 0x7F:
            out.append(c)
        elif c > 0x7FF:
            out += bytes([0xE0 | (c >> 12), 0x80 | ((c >> 6) & 0x3F), 0x80 | (c & 0x3F)])
        else:
            out += bytes([0xC0 | (c >> 6), 0x80 | (c & 0x3F)])
    return bytes(out)


def _ref_number_documents(corpus):
    """NumberTrecDocuments (map getDocid -> Text, byte-order sort, distinct, 1..N)
    + writeDocnoData, restated from NumberTrecDocuments.java:82-107 and
    TrecDocnoMapping.java:92-125 over the oracle's record reader."""
    ids = set()
    for off, ln in O.split_records(corpus):
        text = corpus[off:off + ln].decode("utf-8", "replace")
        i = text.find("<DOCNO>")
        d = "" if i < 0 else _java_trim(text[i + 7:text.index("</DOCNO>", i)])
        ids.add(d.encode("utf-8", "surrogatepass"))
    out = bytearray(len(ids).to_bytes(4, "big"))
    for k in sorted(ids):
        m = _mutf8(k.decode("utf-8", "surrogatepass"))
        out += len(m).to_bytes(2, "big") + m
    return bytes(out)


def test_number_documents(sme, synth):
    ctx = sme.Context(1, 1)
    c = synth.gen_corpus(300, V=500, seed=4, len_lo=5, len_hi=30)
    m = ctx.number_documents(c)
    assert m == synth.mapping_bytes(300) == _ref_number_documents(c)
    fz, _ = common.fuzz_corpus(6, 150)  # duplicate, missing and unmapped docids, <<DOC>, unterminated tail
    assert ctx.number_documents(fz) == _ref_number_documents(fz)
    odd = (b"<DOC><DOCNO> caf\xc3\xa9 </DOCNO> x </DOC><DOC><DOCNO>\xf0\x9f\x98\x80z</DOCNO> y </DOC>"
           b"<DOC><DOCNO>\xc4\xb0d</DOCNO> z </DOC><DOC><DOCNO>a\xffb</DOCNO> w </DOC><DOC> none </DOC>"
           b"<DOC><DOCNO>ab</DOCNO></DOC><DOC><DOCNO>a</DOCNO></DOC><DOC><DOCNO>ab\x01</DOCNO></DOC>")
    assert ctx.number_documents(odd) == _ref_number_documents(odd)
    assert ctx.number_documents(b"no records") == b"\x00\x00\x00\x00"
    with pytest.raises(sme.SmeError):
        ctx.number_documents(b"<DOC><DOCNO>A x </DOC>")
    # the generated mapping drives the index build: docnos 1..N in docid order
    ctx.load_docno_mapping(ctx.number_documents(fz))
    ix = ctx.build(fz)
    assert ix.N == O.OracleIndex(fz, ctx.number_documents(fz), 1, 1).N


# ---- CharKGramTermIndexer on the device (C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:74-211) ----
def _check_chargram(sme, corpus, k, R):
    ref = O.OracleCharGram(corpus, k, R)
    ctx = sme.Context(k, R)
    out = ctx.build_chargram(corpus)
    assert (out.ngrams, out.npairs) == (ref.ngrams, ref.npairs)
    for p in range(R):
        assert out.partition_text(p) == ref.part_bytes(p), p
    return out


def test_chargram_kat(sme):
    corpus = b"<DOC><DOCNO>A</DOCNO> bats cats dog </DOC>\n<DOC><DOCNO>B</DOCNO> cat bat </DOC>"
    out = _check_chargram(sme, corpus, 2, 1)
    assert b"at\t[cat, bat]\n" in out.partition_text(0)


@pytest.mark.parametrize("k,R", [(1, 1), (2, 10), (3, 3), (5, 2), (6, 3), (9, 2), (14, 1)])
def test_chargram_fuzz(sme, k, R):
    corpus, _ = common.fuzz_corpus(20 + k, 120)
    _check_chargram(sme, corpus, k, R)


@pytest.mark.parametrize("k", [2, 3])
def test_chargram_synthetic(sme, synth, k):
    """Zipfian vocabulary: sets of thousands of terms (many JDK 6 resizes)."""
    c = synth.gen_corpus(300, V=4000, seed=31, len_lo=40, len_hi=120)
    _check_chargram(sme, c, k, 10)


def test_chargram_empty(sme):
    ctx = sme.Context(2, 3)
    out = ctx.build_chargram(b"no records")
    assert (out.ngrams, out.npairs) == (0, 0) and out.partition_text(2) == b""
    out = ctx.build_chargram(b"<DOC><DOCNO>A</DOCNO> the of </DOC>")  # stopwords only
    assert out.ngrams == 0


def _expected_weights(ix, idf_mode, N=None, df_override=None):
    """(1 + ln tf) * log10(N // df) per posting (IntDocVectorsForwardIndex.java:211,
    T2 int division), docno-ascending per term, from the reduce-order CSR."""
    import math
    off, dn, tf, df = ix.csr()
    N = ix.N if N is None else N
    exp = []
    for t in range(ix.V):
        d = 1 if idf_mode == 0 else int(df[t] if df_override is None else df_override[t])
        idf = math.log10(float(N // d))
        ps = sorted(zip(dn[off[t]:off[t + 1]].tolist(), tf[off[t]:off[t + 1]].tolist()))
        exp += [(1.0 + math.log(float(f))) * idf for _, f in ps]
    return np.array(exp, np.float64)


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_build_docid_split(sme, synth, idf_mode):
    """K6b: docid pairs beside the term sort (6-bit digits: 5,000 docid terms
    beside ~800 word terms take three LSD passes, the words alone two).  The
    split build's partition records and reduce-order CSR equal the oracle's,
    and its docno-order CSR, TF-IDF weights and query results equal those of
    the single sort (docid_split 0), in both idf modes."""
    n = 5000
    c = synth.gen_corpus(n, V=800, seed=23, len_lo=20, len_hi=90)
    ixs = []
    for split in (1, 0):
        ix, _ = _check_build(sme, c, synth.docids(n), R=3, idf_mode=idf_mode,
                             opts={"sort_digit_bits": 6, "docid_split": 2 * split})
        assert ("docid_pairs" in ix.ctx.last_build_profile()) == bool(split)  # the split ran (or not)
        ixs.append(ix)
    a, b = ixs
    for x, y in zip(a.weights(), b.weights()):
        assert np.array_equal(x, y)
    assert np.array_equal(a.weights()[2], _expected_weights(a, idf_mode))
    _, _, _, df = a.csr()
    terms, qoff = synth.queries_by_df(df, 200, seed=5)
    for k in (10, 100):
        d1, s1 = a.query_topk(terms, qoff, k)
        d2, s2 = b.query_topk(terms, qoff, k)
        assert np.array_equal(d1, d2) and np.array_equal(s1, s2)


@pytest.mark.parametrize("idf_mode", [0, 1])
def test_weight_pass_and_reweight(sme, synth, idf_mode):
    """The build's fused TF-IDF pass (k_weights) and sme_index_reweight with
    all-reduced statistics: every fp64 weight bit-equal to the reference formula."""
    import ctypes as C
    n = 600
    c = synth.gen_corpus(n, V=800, seed=17, len_lo=20, len_hi=90)
    ctx = sme.Context(1, 1, idf_mode)
    ctx.load_docno_mapping(synth.mapping_bytes(n))
    ix = ctx.build(c)
    off, dn, w = ix.weights()
    assert np.array_equal(off, ix.csr()[0])
    assert np.array_equal(w, _expected_weights(ix, idf_mode))
    # reweight with a larger global N and per-term df + 3 (as after a df all-reduce)
    df = ix.csr()[3].astype(np.int64) + 3
    L = sme.lib()
    d_df = C.c_void_p()
    assert L.sme_device_alloc(0, df.nbytes, C.byref(d_df)) == 0
    try:
        sme.memcpy(d_df.value, df.ctypes.data, df.nbytes)
        ix.reweight(7 * n, d_df.value)
        _, _, w2 = ix.weights()
        assert np.array_equal(w2, _expected_weights(ix, idf_mode, N=7 * n, df_override=df))
    finally:
        L.sme_device_free(d_df)


def test_query_term_id_bounds(sme, synth):
    """ids outside [-1, V) are rejected by the host entry point."""
    n = 50
    c = synth.gen_corpus(n, V=200, seed=3, len_lo=5, len_hi=30)
    ctx = sme.Context(1, 1)
    ctx.load_docno_mapping(synth.mapping_bytes(n))
    ix = ctx.build(c)
    for bad in (ix.V, ix.V + 5, -2):
        with pytest.raises(sme.SmeError):
            ix.query_topk(np.array([0, bad], np.int32), np.array([0, 2], np.int64), 10)
    dn, _ = ix.query_topk(np.array([0, -1], np.int32), np.array([0, 2], np.int64), 10)
    assert dn[0, 0] >= 0


def test_unsorted_mapping_file(sme, synth):
    """A mapping file that is not sorted (or repeats a docid): docno lookup falls
    back to binary search over the file's array, as Arrays.binarySearch does."""
    n = 40
    c = synth.gen_corpus(n, V=200, seed=4, len_lo=5, len_hi=30)
    ids = synth.docids(n)
    for m in (ids[::-1], ids[:20] + ids[10:], ids[5:] + ids[:5]):
        _check_build(sme, c, m, R=1)


@pytest.mark.parametrize("k", [50, 100, 448, 1000])
def test_queries_large_k(sme, synth, k):
    """top-k beyond the register lists: k = 50 / 100 / 448 (c5's top-100); k = 1000
    (above the window kernels' 448: the streaming kernel's LDS list, up to 1792)."""
    n = 3000
    c = synth.gen_corpus(n, V=400, seed=23, len_lo=5, len_hi=40)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    terms, qoff = synth.queries_by_df(df, 30, seed=9, qlen_lo=1, qlen_hi=6)
    dn, sc = _query_both_kernels(ix, terms, qoff, k)
    for q in range(len(qoff) - 1):
        tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]]]
        rd, rs = ref.query(tl, k, 0, 0)
        assert dn[q, :len(rd)].tolist() == rd, q
        assert np.array_equal(sc[q, :len(rd)], np.array(rs)), q
        assert (dn[q, len(rd):] == -1).all()
    if k > 448:
        assert ix.ctx.last_build_profile()["query_kernel_name"] == "k_query"
        with pytest.raises(sme.SmeError):
            ix.query_topk(terms, qoff, 1793)


def test_forward_index_on_device_output(sme, synth, tmp_path):
    """SURVEY 8f-1 composed with the device: libsme partition records ->
    SequenceFile part files -> BuildIntDocVectorsForwardIndex -> getValue through
    the forward index -> the reference's rank() arithmetic over those postings
    equals the device query_topk and the oracle (BuildIntDocVectorsForwardIndex
    .java:84-158, IntDocVectorsForwardIndex.java:93-122,148-223)."""
    import importlib
    import math
    SF = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.seqfile")
    n = 400
    c = synth.gen_corpus(n, V=1500, seed=41, len_lo=20, len_hi=90)
    ix, ref = _check_build(sme, c, synth.docids(n), R=3)
    table = SF.write_index_dir(ix, str(tmp_path / "idx"), sync=bytes(range(16)))
    SF.build_forward_index(table, str(tmp_path / "fwd"))
    fw = SF.ForwardIndex(str(tmp_path / "idx"), str(tmp_path / "fwd"))
    N = fw.get_value(b" ")[1]  # main(): N = df of the " " record
    assert N == ix.N
    _, _, _, df = ix.csr()
    terms, qoff = synth.queries_by_df(df, 40, seed=12, qlen_lo=1, qlen_hi=4)
    names = [ix.term(i) for i in range(ix.V)]
    dn, sc = ix.query_topk(terms, qoff, 10)
    for q in range(len(qoff) - 1):
        tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]]]
        acc = {}
        for t in tl:
            grams, sdf, posts = fw.get_value(t.encode())
            for d, tf in posts:  # score += (1 + ln tf) * log10(N / df): stored order
                w = (1.0 + math.log(tf)) * math.log10(N // sdf)
                acc[d] = acc[d] + w if d in acc else 0.0 + w
        top = sorted(acc.items(), key=lambda x: (-x[1], x[0]))[:10]
        assert dn[q, :len(top)].tolist() == [d for d, _ in top], q
        assert sc[q, :len(top)].tolist() == [s for _, s in top], q
        rd, rs = ref.query(tl, 10, 0, 0)
        assert [d for d, _ in top] == rd


def test_repl_contract(sme):
    """IntDocVectorsForwardIndex.main's loop (:284-320): 1-2 raw words are
    answered, an empty line or 3+ words end the session; docids printed when a
    mapping is given."""
    indexer = sme.TermKGramDocIndexer(k=1, num_reduce_tasks=1)
    mb = O.write_mapping(KAT["index_mapping"])
    ix = indexer.run(KAT["index_corpus"].encode(), mb)
    fw = sme.IntDocVectorsForwardIndex(ix)
    assert fw.query_line("  cat dog \n") == "cat dog: [1, 2]"
    assert fw.query_line("zebraword") == "zebraword: No results ..."
    assert fw.query_line("   ") is None
    assert fw.query_line("cat dog bird") is None
    fm = sme.IntDocVectorsForwardIndex(ix, mb)
    ids = [""] + list(KAT["index_mapping"])
    assert fm.query_line("cat dog") == "cat dog: " + ids[1] + " " + ids[2] + " "


@pytest.mark.parametrize("budget,cap", [(1, 1024), (8192, 4)])
def test_queries_table_budget(sme, synth, budget, cap):
    """Batches whose skip tables exceed the table budget (sme_set_option
    "query_table_budget") are split by query range, and queries that still
    overflow their candidate lists without room for the tile table run as their
    own compact batches: k = 100 over a uniform-vocabulary batch answers every
    query (no SME_ENOTIMPL), bit-identical to the default path and to the
    oracle's rank().  budget 1 splits down to single queries; 8 KiB fits the
    window table but not the tile table, and cand_cap 4 < k sends every query
    to that fallback."""
    n = 9000
    c = synth.gen_corpus(n, V=3000, seed=13, len_lo=8, len_hi=30)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1)
    _, _, _, df = ix.csr()
    names = [ix.term(i) for i in range(ix.V)]
    terms, qoff = synth.queries_by_df(df, 60, seed=5, uniform=True)
    k = 100
    dn0, sc0 = ix.query_topk(terms, qoff, k)
    try:
        ix.ctx.set_option("query_table_budget", budget)
        dn, sc = _query_opts(ix, terms, qoff, k, cand_cap=cap)
        prof = ix.ctx.last_build_profile()
    finally:
        ix.ctx.set_option("query_table_budget", 0)
    assert prof["query_kernel_name"] == "k_query_win"
    assert np.array_equal(dn, dn0) and np.array_equal(sc, sc0)
    for q in range(len(qoff) - 1):
        tl = [names[t] for t in terms[qoff[q]:qoff[q + 1]]]
        rd, rs = ref.query(tl, k, 0, 0)
        assert dn[q, :len(rd)].tolist() == rd, q
        assert np.array_equal(sc[q, :len(rd)], np.array(rs)), q
        assert (dn[q, len(rd):] == -1).all()


@pytest.mark.parametrize("long_query", [False, True])
def test_queries_tie_width_split(sme, synth, long_query):
    """SME_TIE_REFERENCE under a forced split (query_table_budget 1: down to one
    query per nested call, then overflow subsets with cand_cap 4): the tie
    words' tf width is the TOP-LEVEL batch's (22 bits when one of its queries
    has more than 256 terms, else 24) and the nested calls inherit it, so every
    tie word equals the unsplit run's -- doc shards merging tie words
    (dist.merge_topk_owner) never see two widths for one query."""
    n = 4000
    c = synth.gen_corpus(n, V=1500, seed=17, len_lo=10, len_hi=40)
    ix, ref = _check_build(sme, c, synth.docids(n), R=1, tiebreak=1)
    _, _, _, df = ix.csr()
    terms, qoff = synth.queries_by_df(df, 40, seed=3, qlen_lo=1, qlen_hi=8)
    if long_query:
        rng = np.random.default_rng(2)
        terms = np.concatenate([terms, rng.integers(0, ix.V, size=300).astype(np.int32)])
        qoff = np.concatenate([qoff, [qoff[-1] + 300]]).astype(np.int64)
    k = 10
    dn0, sc0, t0 = ix.query_topk(terms, qoff, k, with_tie=True)
    try:
        ix.ctx.set_option("query_table_budget", 1)
        ix.ctx.set_option("cand_cap", 4)
        dn, sc, t = ix.query_topk(terms, qoff, k, with_tie=True)
    finally:
        ix.ctx.set_option("query_table_budget", 0)
        ix.ctx.set_option("cand_cap", 1024)
    assert np.array_equal(dn, dn0) and np.array_equal(sc.view(np.int64), sc0.view(np.int64))
    assert np.array_equal(t, t0)
    # the width is visible in the words: token index j above tb bits of 2^tb - 1 - tf
    hit = dn0 >= 0
    tb = 22 if long_query else 24
    f = ((1 << tb) - 1) - (t0[hit].astype(np.int64) & ((1 << tb) - 1))
    assert hit.any() and ((f >= 1) & (f < 256)).all()


def test_c1_sample_on_device(sme, tmp_path):
    """c1 on the device: the committed 1,000-document sample through
    libsme (R = 10 reducers) -> partition records byte-equal to the oracle's ->
    SequenceFile part files -> forward index -> the REPL's 1-2 word queries:
    rank() over getValue's postings = device query_topk = the oracle's rank()."""
    import importlib
    import test_c1_plumbing as C1
    SF = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.seqfile")
    corpus, mapping = C1.c1()
    ref = O.OracleIndex(corpus, mapping, 1, 10)
    ctx = sme.Context(1, 10)
    ctx.load_docno_mapping(mapping)
    ix = ctx.build(corpus)
    assert ix.N == 1000
    for p in range(10):
        common.compare_partitions(ix.partition_records(p), ref.partition_bytes(p))
    table = SF.write_index_dir(ix, str(tmp_path / "idx"), sync=bytes(range(16)))
    SF.build_forward_index(table, str(tmp_path / "fwd"))
    fw = SF.ForwardIndex(str(tmp_path / "idx"), str(tmp_path / "fwd"))
    N = fw.get_value(b" ")[1]
    assert N == 1000
    queries = C1.c1_queries(ref.terms())
    ids = ix.lookup([t for tl in queries for t in tl]).astype(np.int32)
    qoff = np.zeros(len(queries) + 1, np.int64)
    qoff[1:] = np.cumsum([len(tl) for tl in queries])
    dn, sc = ix.query_topk(ids, qoff, 10)
    for q, tl in enumerate(queries):
        top = C1.rank_via_forward_index(fw, tl, N)
        rd, rs = ref.query(tl, 10, 0, 0)
        assert [d for d, _ in top] == rd and [s for _, s in top] == rs, tl
        assert dn[q, :len(rd)].tolist() == rd and sc[q, :len(rd)].tolist() == rs, tl


def _trec(docs):
    return "".join("<DOC>\n<DOCNO> %s </DOCNO>\n<TEXT>\n%s\n</TEXT>\n</DOC>\n" % (d, body) for d, body in docs).encode()


@pytest.mark.parametrize("case", ["ascending", "shuffled", "mixed_forms", "case_twins", "docid_in_text",
                                  "duplicates", "docid_in_other_text", "mixed_case"])
@pytest.mark.parametrize("docid_terms,bits", [(1, 11), (0, 11), (1, 6)])
def test_build_docid_terms(sme, synth, case, docid_terms, bits):
    """K4b: docid terms (T7) beside the word vocabulary.  A record's DOCNO token
    that is its own term (ASCII letters and digits ending in a digit, unchanged by
    Porter2) skips the per-distinct vocabulary work and is ranked by a merge with
    the sorted word terms when the docids ascend in file order; otherwise (docids
    out of order, two raw forms of one term, a docid term also a word term) the
    build stays on the general path.  Either way the partition records and the
    term strings equal the oracle's (TrecDocument.java:94-96: the DOCNO text is
    indexed), with the option on and off."""
    g = np.random.default_rng(hash(case) & 0xFFFF)
    words = ["alpha", "bravo", "charlie", "delta", "echo", "foxtrot", "golf", "hotel", "india", "kilo", "lima", "zulu",
             "running", "ponies", "x9", "abc123", "42"]
    n = 300
    ids = ["D%09d" % (1000 + 3 * i) for i in range(n)]
    bodies = [" ".join(g.choice(words, size=int(g.integers(5, 40)))) for _ in range(n)]
    if case == "shuffled":
        perm = g.permutation(n)
        ids = [ids[i] for i in perm]
    elif case == "mixed_forms":
        forms = ["LA%06d-%04d", "ab%d", "XY%d", "FT%dA", "doc.%d", "%d"]
        ids = sorted(forms[i % len(forms)] % ((i,) if forms[i % len(forms)].count("%") == 1 else (i, i)) for i in
                     range(n))
    elif case == "case_twins":
        ids = ["d%09d" % (1000 + 3 * i) if i == 7 else ids[i] for i in range(n)]
        ids[8] = "D%09d" % (1000 + 3 * 7)  # the same term as record 7's, another raw form
    elif case == "docid_in_text":
        bodies[5] += " " + ids[200].lower() + " " + ids[100]  # a word equal to a docid term; a docid in a body
    elif case == "duplicates":
        ids[11] = ids[10]
        ids[50] = ids[49]
    elif case == "docid_in_other_text":
        bodies[5] += " " + ids[100]  # record 5 holds two docid terms' pairs (K6b falls back to merged ids)
    elif case == "mixed_case":
        # docid terms ascend in file order, the mapping's (case-sensitive) docno order differs
        ids = [("A%07d" if i % 2 == 0 else "a%07d") % i for i in range(n)]
    c = _trec(list(zip(ids, bodies)))
    mapping = sorted(set(ids))
    # bits 6: the K6b split forced (docid_split 2), with more LSD passes than the words' two
    opts = {"docid_terms": docid_terms, "sort_digit_bits": bits, "docid_split": 2 if bits == 6 else 1}
    _check_build(sme, c, mapping, R=1, opts=opts)
    _check_build(sme, c, mapping, R=7, opts=opts)
