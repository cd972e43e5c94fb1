"""Two independent readings of the tokenizer and stemmer must agree: the C oracle
(oracle/oracle_tok.c, oracle_stem.c) against the Python restatement written from
the Java (tests/pyref_tokenize.py) -- on the Appendix-B known answers, fuzzed
TREC documents, hypothesis-generated strings over the tokenizer's edge alphabet
(markup, entities, '.', apostrophes, uppercase, non-ASCII, Unicode spaces, long
tokens) and 200,000 synthetic vocabulary words through the stemmer alone.
(C/org/galagosearch/core/parse/TagTokenizer.java:155-709,
C/ivory/tokenize/GalagoTokenizer.java:139-183,
C/org/tartarus/snowball/ext/englishStemmer.java:1149-1317.)"""
import json
import os
import random

import common
import oracle_lib as O
import pyref_tokenize as P
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_appendix_b.json")))


@pytest.mark.parametrize("text,expected", KAT["process_content"])
def test_pyref_kat_process_content(text, expected):
    assert P.process_content(text) == expected


@pytest.mark.parametrize("word,expected", KAT["stem"])
def test_pyref_kat_stem(word, expected):
    assert P.stem(word) == expected


def test_pyref_vs_oracle_fuzz_docs():
    rng = random.Random(4242)
    for i in range(600):
        doc = common.fuzz_doc(rng, "P%d" % i, rng.randint(1, 60))
        assert P.process_content(doc) == O.process_content(doc), doc


def test_pyref_vs_oracle_fuzz_bytes():
    """Record bytes with invalid UTF-8 (Text.toString replacement) and markup."""
    rng = random.Random(99)
    pieces = [b"<", b">", b"&", b";", b".", b"'", b"A", b"b", b" ", b"\xc3", b"\xa9", b"\xe2\x82\xac", b"\xff",
              b"\xf0\x9f\x98\x80", b"\xed\xa0\x80", b"<!--", b"-->", b"<script>", b"</script>", b"amp", b"\xc2\xa0",
              b"x" * 40, b"\xe2\x80\xa8", b"<a href='x>y'>", b"\\"]
    for i in range(800):
        raw = b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 40)))
        assert P.process_content(raw) == O.process_content(raw), raw


def test_pyref_vs_oracle_stemmer_vocabulary(synth):
    blob, off = synth.make_vocab(200000, 5)
    words = [blob[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]
    rng = random.Random(3)
    words += ["".join(rng.choice("aeiouybcdlnrstgy'") for _ in range(rng.randint(1, 14))) for _ in range(20000)]
    bad = [w for w in words if P.stem(w) != O.stem(w)]
    assert not bad, bad[:20]


EDGE = st.sampled_from(list("<>&;.'-/!?=\"#_ \n\tAaBbZzYyEeSs019") +
                       ["é", "İ", "Σ", "ß", " ", " ", " ", "\U0001F600", "K",
                        "<!--", "-->", "<script>", "</script>", "<style>", "</style>", "&amp;", "&#1;", "<?", "?>",
                        "<b>", "</b>", "<a href=\"x\">", "ies", "ing", "ed", "ly", "sses", "ational", "y",
                        "a" * 20, "b." * 5, "x" * 99, "Q" * 100])


@settings(max_examples=3000, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(EDGE, max_size=60).map("".join))
def test_pyref_vs_oracle_hypothesis(text):
    assert P.process_content(text) == O.process_content(text)
    assert P.tag_tokenize(text) == O.tag_tokenize(text)
