"""The CPU oracle against the known-answer tests of SURVEY.md Appendix B
(tests/golden/kat_appendix_b.json).  These pin the oracle before it is used
to check the device path."""
import json
import os

import oracle_lib as O
import pytest

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_appendix_b.json")))


@pytest.mark.parametrize("text,expected", KAT["process_content"])
def test_process_content(text, expected):
    assert O.process_content(text) == expected


@pytest.mark.parametrize("word,expected", KAT["stem"])
def test_stem(word, expected):
    assert O.stem(word) == expected


def test_stopwords():
    assert O.is_stopword("the") and O.is_stopword("cant") and not O.is_stopword("cat")
    # 8 listed stopwords contain '-', a split char: unreachable after tokenization (T9)
    assert O.process_content("no-one") == []  # "no" and "one" are both stopwords anyway
    assert O.is_stopword("no-one")


def _index():
    return O.OracleIndex(KAT["index_corpus"].encode(), O.write_mapping(KAT["index_mapping"]), 1, 1)


def test_index_records():
    ix = _index()
    got = [[list(g), df, [list(p) for p in posts]] for g, _, df, posts in ix.terms()]
    assert got == KAT["index_records_k1_r1"]


def test_index_record_bytes():
    import common
    recs = common.parse_records(_index().partition_bytes(0))
    cat = [r for r in recs if r[0] == (b"cat",)][0]
    assert cat[3].hex() == KAT["cat_record_hex"]


def test_partitions_r10():
    ix = O.OracleIndex(KAT["index_corpus"].encode(), O.write_mapping(KAT["index_mapping"]), 1, 10)
    parts = {g[0]: p for g, p, _, _ in ix.terms()}
    assert parts == KAT["partitions_r10"]


@pytest.mark.parametrize("terms,docs,scores", KAT["queries"])
def test_queries(terms, docs, scores):
    ix = _index()
    for order in (0, 1, 2):
        d, s = ix.query(terms, 10, 0, order)
        assert d == docs
        assert s == pytest.approx(scores, rel=1e-15)


def test_doc_counter_quirk():
    """T3: " " postings hold (0,0) for the first record of a map task, then the
    previous record's (docno, 1); df(" ") = N."""
    corpus = b"".join(b"<DOC><DOCNO>X%d</DOCNO> wolf </DOC>" % i for i in range(4))
    ix = O.OracleIndex(corpus, O.write_mapping(["X%d" % i for i in range(4)]), 1, 1)
    sp = ix.terms()[0]
    assert sp[0] == (" ",) and sp[2] == 4 and sp[3] == [(0, 0), (1, 1), (2, 1), (3, 1)]
    # two map tasks (splits): each starts with (0,0)
    ix2 = O.OracleIndex(corpus, O.write_mapping(["X%d" % i for i in range(4)]), 1, 1,
                        splits=[0, 60, len(corpus)])
    assert sorted(ix2.terms()[0][3]) == [(0, 0), (0, 0), (1, 1), (3, 1)]


def test_record_reader_quirks():
    # '<<DOC>' does not match (mismatch resets without re-testing the byte)
    assert O.split_records(b"<<DOC> a </DOC>") == []
    assert len(O.split_records(b"<<<DOC> a </DOC>")) == 1
    # '<</DOC>' misses the end tag; the record runs to the next </DOC>
    recs = O.split_records(b"<DOC> a <</DOC> b </DOC>")
    assert len(recs) == 1 and recs[0] == (0, 24)
    # unterminated record is dropped
    assert O.split_records(b"<DOC> a </DOC><DOC> b") == [(0, 14)]
    # a nested <DOC> is content of the enclosing record
    assert O.split_records(b"<DOC> a <DOC> b </DOC> c </DOC>") == [(0, 22)]


def test_docno_edge_cases():
    corpus = b"<DOC> nodocno </DOC><DOC><DOCNO>ZZZ</DOCNO> xray </DOC><DOC><DOCNO> A1 </DOCNO> yak </DOC>"
    ix = O.OracleIndex(corpus, O.write_mapping(["A1", "B2"]), 1, 1)
    t = {g[0]: posts for g, _, _, posts in ix.terms()}
    assert t["nodocno"] == [(0, 1)]      # docid "" -> binarySearch finds the "" sentinel at 0
    assert t["xray"] == [(-4, 1)]           # ZZZ absent -> -(insertion point 3) - 1 (T14)
    assert t["yak"] == [(1, 1)]            # trimmed docid
    with pytest.raises(RuntimeError):
        O.OracleIndex(b"<DOC><DOCNO>A1 x </DOC>", O.write_mapping(["A1"]), 1, 1)


def test_tf_desc_docno_asc_order():
    corpus = b"".join(b"<DOC><DOCNO>D%d</DOCNO> %s </DOC>" % (i, b" ".join([b"wolf"] * c))
                      for i, c in enumerate([1, 3, 2, 3, 1]))
    ix = O.OracleIndex(corpus, O.write_mapping(["D%d" % i for i in range(5)]), 1, 1)
    w = [p for g, _, _, p in ix.terms() if g == ("wolf",)][0]
    assert w == [(2, 3), (4, 3), (3, 2), (1, 1), (5, 1)]


def test_duplicate_docids_merge():
    corpus = b"<DOC><DOCNO>A</DOCNO> wolf wolf </DOC><DOC><DOCNO>B</DOCNO> wolf </DOC><DOC><DOCNO>A</DOCNO> wolf </DOC>"
    ix = O.OracleIndex(corpus, O.write_mapping(["A", "B"]), 1, 1)
    w = [p for g, _, _, p in ix.terms() if g == ("wolf",)][0]
    assert w == [(1, 3), (2, 1)]


# ---- CharKGramTermIndexer (C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:74-211) ----
def test_chargram_kat():
    """Hand-derived: "bats cats dog" then "cat bat", k=2, R=1.  The set of "at" is
    inserted bat-then-cat, but JDK 6 HashSet iteration puts cat (bucket 2 of 16:
    spread("cat".hashCode()=98262) & 15) before bat (bucket 10: spread(97301) & 15)."""
    corpus = b"<DOC><DOCNO>A</DOCNO> bats cats dog </DOC>\n<DOC><DOCNO>B</DOCNO> cat bat </DOC>"
    o = O.OracleCharGram(corpus, 2, 1)
    assert o.part_bytes(0) == (b"$b\t[bat]\n$c\t[cat]\n$d\t[dog]\nat\t[cat, bat]\nba\t[bat]\nca\t[cat]\n"
                               b"do\t[dog]\ng$\t[dog]\nog\t[dog]\nt$\t[cat, bat]\n")
    assert (o.ngrams, o.npairs) == (10, 12)


@pytest.mark.parametrize("k,R", [(1, 1), (2, 10), (3, 3), (4, 1)])
def test_chargram_oracle_vs_python(k, R):
    """The C oracle (direct JDK 6 HashMap simulation) against the pure-Python
    restatement on fuzzed corpora: sets > 12 and > 24 members (resizes), non-ASCII,
    surrogate pairs cut by a gram, markup."""
    import common
    import pyref_chargram as P
    corpus, _ = common.fuzz_corpus(7 + k, 60)
    o = O.OracleCharGram(corpus, k, R)
    exp = P.chargram_parts(corpus, k, R)
    for p in range(R):
        assert o.part_bytes(p) == exp[p], p


def _py_rank(ix, terms, k, idf_mode):
    """rank() restated in Python with the reference's list + indexOf accumulator
    (IntDocVectorsForwardIndex.java:192-213), forward-index lookup by the LAST
    term (global key order) whose first element matches (:107-120)."""
    import math
    recs = ix.terms()
    recs_sorted = sorted(recs, key=lambda r: [g.encode("utf-16-be", "surrogatepass") for g in r[0]])
    by_first = {}
    for r in recs_sorted:
        if r[0] != (" ",):
            by_first[r[0][0]] = r
    scores = []  # [docno, score]
    for t in terms:
        r = by_first.get(t)
        if r is None:
            continue
        df = r[2] if idf_mode == 0 else len(r[3])
        idf = math.log10(ix.N // df)
        for d, tf in r[3]:
            hit = [s for s in scores if s[0] == d]
            w = (1.0 + math.log(tf)) * idf
            if hit:
                hit[0][1] += w
            else:
                scores.append([d, 0.0 + w])
    scores.sort(key=lambda s: (-s[1], s[0]))
    return [s[0] for s in scores[:k]], [s[1] for s in scores[:k]]


@pytest.mark.parametrize("K", [1, 2])
def test_oracle_query_tables_vs_scan(K):
    """The oracle's hashed forward-index lookup and docno accumulator equal the
    O(V) scan and the list-indexOf accumulator they replace."""
    import common
    import random
    corpus, ids = common.fuzz_corpus(40 + K, 80)
    ix = O.OracleIndex(corpus, O.write_mapping(ids), K, 1)
    assert ix.lookup_selfcheck() == 0
    firsts = sorted({g[0] for g, _, _, _ in ix.terms() if g != (" ",)})
    rng = random.Random(K)
    for _ in range(40):
        tl = [rng.choice(firsts) for _ in range(rng.randint(1, 4))] + ["zz-absent"]
        for mode in (0, 1):
            d, s = ix.query(tl, 10, mode, 0)
            pd, ps = _py_rank(ix, tl, 10, mode)
            assert d == pd and s == ps, (tl, mode)
