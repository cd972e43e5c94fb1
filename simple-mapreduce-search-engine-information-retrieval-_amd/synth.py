"""Deterministic synthetic TREC corpora.

Layout of document d (0-based), docid D%09d so docids sort in generation
order and docno = d + 1:

    <DOC>\\n<DOCNO>D000000001</DOCNO>\\n<TEXT>\\n w w w ... \\n</TEXT>\\n</DOC>\\n

Tokens are words of a synthetic vocabulary (lowercase [a-z], lengths 3-12,
shorter at lower rank, no stopwords), drawn Zipf(s) by rank; single spaces,
a newline after every 12th token and after the last.  Randomness is
counter-based (splitmix64 of (seed, doc, position)), so the host (numpy) and
device (HIP, sme_gen_corpus_device) generators emit identical bytes.
"""
import functools
import math

import numpy as np

M64 = (1 << 64) - 1
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)

HEAD = b"<DOC>\n<DOCNO>D%09d</DOCNO>\n<TEXT>\n"
TAIL = b"</TEXT>\n</DOC>\n"
HEAD_LEN = len(HEAD % 0)
LINE_TOKENS = 12


def splitmix64(x):
    """Vectorised splitmix64 on numpy uint64 (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (np.asarray(x, dtype=np.uint64) + _GOLD)
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))


def _splitmix_int(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _stopwords():
    import os
    import re
    here = os.path.dirname(os.path.abspath(__file__))
    src = open(os.path.join(here, "csrc", "stopwords_tab.hpp")).read()
    chars = re.search(r'kStopChars\[\] = "([^"]*)"', src).group(1)
    offs = [int(x) for x in re.search(r"kStopOff\[[^\]]*\] = \{([^}]*)\}", src).group(1).split(",")]
    return {chars[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)}


@functools.lru_cache(maxsize=8)
def make_vocab(V, seed):
    """V distinct words; rank r has length min(12, 3 + floor(log2(r+1)/2))."""
    stop = _stopwords()
    words, seen = [], set()
    letters = "abcdefghijklmnopqrstuvwxyz"
    r = 0
    attempt = 0
    while len(words) < V:
        ln = min(12, 3 + int(math.log2(len(words) + 1) / 2))
        h = _splitmix_int((seed << 40) ^ (r << 8) ^ attempt)
        w = []
        for _ in range(ln):
            w.append(letters[h % 26])
            h //= 26
            if h < 26:
                h = _splitmix_int(h ^ (r << 20) ^ len(w))
        w = "".join(w)
        if w in seen or w in stop:
            attempt += 1
            continue
        seen.add(w)
        words.append(w)
        r += 1
        attempt = 0
    blob = "".join(words).encode()
    offs = np.zeros(V + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(w) for w in words])
    return blob, offs


@functools.lru_cache(maxsize=8)
def zipf_cdf(V, s=1.0):
    w = 1.0 / np.power(np.arange(1, V + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    c /= c[-1]
    c[-1] = 1.0
    return c


def _u01(keys):
    return (splitmix64(keys) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def doc_lengths(d0, d1, seed, lo, hi):
    d = np.arange(d0, d1, dtype=np.uint64)
    keys = (np.uint64(seed) << np.uint64(40)) + (d << np.uint64(12)) + np.uint64(4095)
    return (lo + (splitmix64(keys) % np.uint64(hi - lo + 1)).astype(np.int64))


def token_ranks(d, pos, seed, V, s=1.0):
    keys = (np.uint64(seed) << np.uint64(40)) + (d.astype(np.uint64) << np.uint64(12)) + pos.astype(np.uint64)
    return np.searchsorted(zipf_cdf(V, s), _u01(keys), side="right").astype(np.int64)


def gen_corpus(n_docs, V=1 << 20, seed=42, len_lo=400, len_hi=600, s=1.0, d0=0):
    """Documents d0 .. d0+n_docs-1 as bytes (host generator)."""
    blob, offs = make_vocab(V, seed)
    lens = doc_lengths(d0, d0 + n_docs, seed, len_lo, len_hi)
    T = int(lens.sum())
    doc_of = np.repeat(np.arange(d0, d0 + n_docs, dtype=np.int64), lens)
    starts = np.zeros(n_docs, dtype=np.int64)
    starts[1:] = np.cumsum(lens)[:-1]
    pos = np.arange(T, dtype=np.int64) - np.repeat(starts, lens)
    ranks = token_ranks(doc_of, pos, seed, V, s)
    blob_np = np.frombuffer(blob, dtype=np.uint8)
    wl = (offs[1:] - offs[:-1])[ranks]
    last = pos == np.repeat(lens, lens) - 1
    sep = np.where(last | ((pos + 1) % LINE_TOKENS == 0), ord("\n"), ord(" ")).astype(np.uint8)
    tok_bytes = wl + 1
    # per-doc byte sizes
    body = np.zeros(n_docs, dtype=np.int64)
    np.add.at(body, doc_of - d0, tok_bytes)
    doc_size = HEAD_LEN + body + len(TAIL)
    doc_off = np.zeros(n_docs + 1, dtype=np.int64)
    doc_off[1:] = np.cumsum(doc_size)
    out = np.zeros(int(doc_off[-1]), dtype=np.uint8)
    # headers / tails
    for i in range(n_docs):
        o = doc_off[i]
        out[o:o + HEAD_LEN] = np.frombuffer(HEAD % (d0 + i), dtype=np.uint8)
        out[doc_off[i + 1] - len(TAIL):doc_off[i + 1]] = np.frombuffer(TAIL, dtype=np.uint8)
    # token bytes
    tok_start = np.zeros(T, dtype=np.int64)
    cs = np.cumsum(tok_bytes)
    tok_start[1:] = cs[:-1]
    tok_start -= np.repeat(np.concatenate([[0], np.cumsum(body)[:-1]]), lens)
    tok_start += np.repeat(doc_off[:-1] + HEAD_LEN, lens)
    maxw = int(wl.max()) if T else 0
    for j in range(maxw):
        m = wl > j
        out[tok_start[m] + j] = blob_np[offs[ranks[m]] + j]
    out[tok_start + wl] = sep
    return out.tobytes()


def docids(n_docs, d0=0):
    return ["D%09d" % (d0 + i) for i in range(n_docs)]


def mapping_bytes(n_docs):
    """TrecDocnoMapping file for docids D000000000.. (already sorted)."""
    import struct
    ids = b"".join(struct.pack(">H", 10) + (b"D%09d" % i) for i in range(n_docs))
    return struct.pack(">i", n_docs) + ids


def queries_by_df(true_df, n_queries, seed=7, qlen_lo=2, qlen_hi=8, uniform=False):
    """c3 queries: |q| ~ U{lo..hi}; terms drawn proportional to df (or uniform)."""
    rng = np.random.default_rng(seed)
    ql = rng.integers(qlen_lo, qlen_hi + 1, size=n_queries)
    qoff = np.zeros(n_queries + 1, dtype=np.int64)
    qoff[1:] = np.cumsum(ql)
    V = len(true_df)
    if uniform:
        terms = rng.integers(0, V, size=int(qoff[-1]))
    else:
        p = true_df.astype(np.float64)
        c = np.cumsum(p)
        c /= c[-1]
        terms = np.searchsorted(c, rng.random(int(qoff[-1])), side="right")
        terms = np.minimum(terms, V - 1)
    return terms.astype(np.int32), qoff
