"""The docid-term rule of the build's fast path (K4b, sme_build.hip
k_docid_slots), pinned on the oracle (CPU, not the device): a raw token of ASCII
letters and digits that ends in a digit is its own term -- lowercased, never a
stopword (GalagoTokenizer.java:35-125,152-156), unchanged by the 2010 Porter2
(englishStemmer.java: every rule matches a letter suffix or a whole letter
word) -- so the device may take such a DOCNO token's term straight from its
bytes.  GalagoTokenizer.processContent runs the whole chain."""
import random
import string

import oracle_lib as O
import pyref_stopwords


def test_no_stopword_ends_in_a_digit():
    assert not any(w[-1].isdigit() for w in pyref_stopwords.TERRIER_STOP_WORDS)


def test_alnum_ending_in_digit_is_its_own_term():
    rng = random.Random(17)
    alpha = string.ascii_letters + string.digits
    words = []
    for n in list(range(2, 49)) * 60:
        w = "".join(rng.choice(alpha) for _ in range(n - 1)) + rng.choice(string.digits)
        words.append(w)
    # suffix-shaped stems of Porter2 rules followed by a digit, and docid shapes
    for suf in ("sses", "ies", "ied", "ing", "ingly", "eed", "ational", "ful", "ness", "y", "e", "ll", "s", "us",
                "ss", "ly", "li", "ement", "ative", "ize", "ion", "skies", "dying", "news", "atlas"):
        for d in ("0", "7", "42"):
            words += [suf + d, "x" + suf + d, suf.upper() + d, "D000" + suf + d]
    words += ["D%09d" % i for i in range(0, 10 ** 9, 7919 * 12345)] + ["LA123190", "FT911", "a1", "Y2", "yy9"]
    for w in words:
        assert O.process_content(w) == [w.lower()], w
