"""Helpers shared by the parity tests: record-stream parsing and fuzz corpora."""
import random
import struct


def parse_records(buf):
    """SequenceFile-body records -> list of (gram tuple of bytes, df_field, [(docno, tf)], raw bytes)."""
    out, i = [], 0
    while i < len(buf):
        rl, kl = struct.unpack_from(">ii", buf, i)
        rec = buf[i:i + 8 + rl]
        key = buf[i + 8:i + 8 + kl]
        val = buf[i + 8 + kl:i + 8 + rl]
        k = struct.unpack_from(">i", key, 0)[0]
        p, gram = 4, []
        for _ in range(k):
            ln = struct.unpack_from(">H", key, p)[0]
            gram.append(key[p + 2:p + 2 + ln])
            p += 2 + ln
        df = struct.unpack_from(">i", key, p)[0]
        assert p + 4 == kl
        n = struct.unpack_from(">i", val, 0)[0]
        posts = []
        if n > 0:
            cl = struct.unpack_from(">H", val, 4)[0]
            assert val[6:6 + cl] == b"sa.edu.kaust.io.PostingWritable"
            q = 6 + cl
            for j in range(n):
                posts.append(struct.unpack_from(">ii", val, q + 8 * j))
            assert q + 8 * n == len(val)
        out.append((tuple(gram), df, posts, rec))
        i += 8 + rl
    return out


def compare_partitions(a, b):
    """Bit-exact record comparison; the " " doc-counter record by (df, postings multiset)."""
    ra, rb = parse_records(a), parse_records(b)
    assert len(ra) == len(rb), (len(ra), len(rb))
    for x, y in zip(ra, rb):
        assert x[0] == y[0], (x[0], y[0])
        if x[0] == (b" ",):
            assert x[1] == y[1]
            assert sorted(x[2]) == sorted(y[2])
        else:
            assert x[3] == y[3], (x[0], x[2][:5], y[2][:5])


WORDS = ["apple", "Banana", "CHERRY", "don't", "U.S.A.", "ph.d.", "umass.edu", "e-mail", "AT&T", "the", "of",
         "running", "generously", "skies", "I.B.M.", "x1", "a.b.c.d.e", "hello.world.foo", "café",
         "İstanbul", "Σοφία", "naïve", "\U0001F600smile", "''quoted''",
         "O'Neil", "rock'n'roll", "3.14", "1,000", "C++", "a_b", "x~y", "tab\there", "long" * 30,
         "dots." * 30, "&amp;", "&AMP;", "&#169;", "&lt;tag&gt;", "&nosemi", "Straße", "KKelvin"]
MARKUP = ["<P>", "</P>", "<b>", "</b>", "<a href=\"x.html\">", "<img src='y' />", "<!-- comment <b> -->",
          "<!DOCTYPE html>", "<?xml version=\"1.0\"?>", "<script>var x = 'hidden';</script>",
          "<style>p { color: red }</style>", "<SCRIPT type=\"t\">HIDDEN</SCRIPT>", "<br/>", "<a<b>", "</ x >",
          "<HEADLINE>", "</HEADLINE>", "<script/>visible", "<tag attr=v>", "< spaced>"]


def fuzz_doc(rng, docid, n_tokens, hard=True):
    parts = []
    for _ in range(n_tokens):
        r = rng.random()
        if hard and r < 0.12:
            parts.append(rng.choice(MARKUP))
        elif hard and r < 0.5:
            parts.append(rng.choice(WORDS))
        else:
            ln = rng.randint(1, 10)
            parts.append("".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(ln)))
        parts.append(rng.choice([" ", " ", " ", "\n", ", ", ". ", "; ", "--", "/", "(", ")"]))
    body = "".join(parts)
    did = "" if docid is None else "<DOCNO> %s </DOCNO>\n" % docid
    return "<DOC>\n%s<TEXT>\n%s\n</TEXT>\n</DOC>\n" % (did, body)


def fuzz_corpus(seed, n_docs, hard=True, extra_docids=0, with_quirks=True):
    """Returns (corpus bytes, mapping docids sorted)."""
    rng = random.Random(seed)
    ids = ["FZ%06d-%02d" % (i, rng.randint(0, 99)) for i in range(n_docs)]
    docs = []
    for i, d in enumerate(ids):
        choice = rng.random()
        docid = d
        if with_quirks and choice < 0.03:
            docid = None  # no DOCNO -> docid "" -> docno 0
        elif with_quirks and choice < 0.06:
            docid = ids[rng.randrange(max(i, 1))]  # duplicate docid
        elif with_quirks and choice < 0.08:
            docid = "MISSING%d" % i  # not in mapping -> negative docno
        docs.append(fuzz_doc(rng, docid, rng.randint(0, 80), hard))
    body = "".join(docs)
    if with_quirks:
        body = "junk before <<DOC> x </DOC>\n" + body + "<DOC>\n<DOCNO>TAIL</DOCNO> unterminated"
    mapping = sorted(set(ids))
    return body.encode("utf-8"), mapping


def canon_digest(buf):
    """sha256 of a partition's record stream with the " " doc-counter record's
    postings sorted (their order is Hadoop-defined): equal digests
    <=> compare_partitions passes.  Only the " " record is parsed."""
    import hashlib
    import numpy as np
    h = hashlib.sha256()
    i, n = 0, len(buf)
    while i < n:
        rl, kl = struct.unpack_from(">ii", buf, i)
        if kl == 11 and buf[i + 8:i + 15] == b"\x00\x00\x00\x01\x00\x01 ":
            df = struct.unpack_from(">i", buf, i + 15)[0]
            val = buf[i + 8 + kl:i + 8 + rl]
            cnt = struct.unpack_from(">i", val, 0)[0]
            h.update(b"SPACE%d:" % df)
            if cnt > 0:
                cl = struct.unpack_from(">H", val, 4)[0]
                p = np.frombuffer(val, dtype=">i4", offset=6 + cl, count=2 * cnt).reshape(cnt, 2)
                order = np.lexsort((p[:, 1], p[:, 0]))
                h.update(p[order].astype(">i4").tobytes())
        else:
            h.update(buf[i:i + 8 + rl])
        i += 8 + rl
    return h.hexdigest()


def np_rank(off, dn, tf, terms_q, N, k, idf_mode=0, df=None):
    """rank() of IntDocVectorsForwardIndex (C/sa/edu/kaust/fwindex/
    IntDocVectorsForwardIndex.java:192-223) restated with numpy over a CSR (any
    posting order per term): for each query token in order, every posting adds
    (1 + ln tf) * log10(N / df) to its document's score -- one fp64 add per token
    and document, so a dense accumulator reproduces the JVM's sequential sum bit
    for bit (the first add is 0.0 + w = w).  1 + ln tf comes from libm log
    (math.log), as the device's shared LUT does.  Top-k by (score desc, docno
    asc).  Size-independent: used at full c2 size where the C oracle is too slow."""
    import math
    import numpy as np
    if not len(terms_q):
        return [], []
    dmin = min(int(dn[off[t]:off[t + 1]].min()) for t in terms_q if off[t + 1] > off[t]) \
        if any(off[t + 1] > off[t] for t in terms_q) else 0
    dmax = max(int(dn[off[t]:off[t + 1]].max()) for t in terms_q if off[t + 1] > off[t]) \
        if any(off[t + 1] > off[t] for t in terms_q) else -1
    if dmax < dmin:
        return [], []
    acc = np.zeros(dmax - dmin + 1, np.float64)
    hit = np.zeros(dmax - dmin + 1, bool)
    mt = max(int(tf[off[t]:off[t + 1]].max()) for t in terms_q if off[t + 1] > off[t])
    lut = np.array([0.0] + [1.0 + math.log(float(i)) for i in range(1, mt + 1)], np.float64)
    for t in terms_q:
        sd = 1 if idf_mode == 0 else int(df[t])
        idf = math.log10(float(N // sd))
        d = dn[off[t]:off[t + 1]].astype(np.int64) - dmin
        acc[d] += lut[tf[off[t]:off[t + 1]]] * idf
        hit[d] = True
    docs = np.nonzero(hit)[0]
    sc = acc[docs]
    order = np.lexsort((docs, -sc))[:k]
    return (docs[order] + dmin).tolist(), sc[order].tolist()
