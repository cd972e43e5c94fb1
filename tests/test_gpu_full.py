"""The device path at FULL BASELINE configuration size against golden digests.

tests/golden/full_c2.json (and full_c5.json when present) hold digests of the
full-size index and query results computed on the CPU by cpu-opt
(oracle/oracle_cpuopt.cc), which tests/test_cpu_baseline.py holds to the
ref-faithful oracle (TermKGramDocIndexer.java:119-213, rank() of
IntDocVectorsForwardIndex.java:192-222) record for record and score bit for bit;
made by tools/gen_full_golden.py.  Here the device builds the same corpus in HBM
(sme_synth_corpus) and must reproduce:

  * N, V, P, sum tf and the sha256 of the reduce-order CSR (offsets, docnos, tfs:
    tf desc / docno asc per term -- the reducer's output, bit-exact) and of the
    term strings (TermDF order)
  * per query batch -- configs[2]'s full 100,000-query c3 batch (2-8 terms drawn by
    df, top-10), its uniform-vocabulary variant, 2,000 top-100; c5's 1,000,000
    top-100 batch, answered whole, of which the golden holds the first 50,000
    queries' rows and every 20th row (50,000 more, spread over the batch; the CPU
    port needs hours for all of them) -- the sha256 of every
    docno and every fp64 score bit (docno tie-break, reference idf mode).
"""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _terms_sha(ix):
    h = hashlib.sha256()
    for t in range(ix.V):
        b = ix.term(t).encode("utf-16-le", "surrogatepass")
        h.update(len(b).to_bytes(4, "little") + b)
    return h.hexdigest()


def _first_mismatch(group, d, s, terms_of):
    for q, (tl, gd, gs) in enumerate(group["first"]):
        if terms_of(q) != tl or d[q].tolist() != gd or [float(x).hex() for x in s[q]] != gs:
            return q, tl, gd, d[q].tolist()
    return None


@pytest.mark.parametrize("name", ["c2", "c5"])
def test_full_config_digests(sme, synth, name):
    path = os.path.join(GOLD, "full_%s.json" % name)
    if not os.path.exists(path):
        if name == "c2":
            pytest.fail("missing golden fixture %s (run tools/gen_full_golden.py)" % path)
        pytest.skip("no %s (tools/gen_full_golden.py c5full)" % path)
    g = json.load(open(path))
    c = g["config"]
    corpus = sme.DeviceCorpus(c["n"], V=c["V"], seed=c["seed"], len_lo=c["lo"], len_hi=c["hi"])
    ctx = sme.Context(1, 1, 0)
    ctx.load_docno_mapping(synth.mapping_bytes(c["n"]))
    ix = ctx.build_device(corpus.ptr, corpus.nbytes)
    corpus.close()
    assert (ix.N, ix.V, ix.P) == (g["N"], g["V"], g["P"])
    off, dn, tf, _ = ix.csr()
    assert int(tf.astype(np.int64).sum()) == g["sum_tf"]
    assert _sha(off.astype("<i8"), dn.astype("<i4"), tf.astype("<i4")) == g["csr_sha256"]
    del dn, tf
    assert _terms_sha(ix) == g["terms_sha256"]
    df = np.diff(off).astype(np.int32)
    for group in g["queries"]:
        tids, qoff = synth.queries_by_df(df, group["n"], seed=group["seed"], uniform=(group["kind"] == "uniform"))
        assert _sha(tids.astype("<i4"), qoff.astype("<i8")) == group["terms_sha256"]
        d, s = ix.query_topk(tids, qoff, group["k"])
        nc = group.get("checked", group["n"])  # rows the golden scored (c5: 50,000 of the 1 M)
        stride = group.get("stride", 1)  # (c5: the leading 50,000 and every 20th row)
        d, s = d[::stride][:nc], s[::stride][:nc]
        if _sha(d.astype("<i4"), s.astype("<f8")) != group["result_sha256"]:
            bad = _first_mismatch(group, d, s, lambda q: [ix.term(int(t)) for t in
                                                          tids[qoff[q * stride]:qoff[q * stride + 1]]])
            pytest.fail("%s %s batch (%d queries, top-%d) differs from the golden; first listed mismatch: %r"
                        % (name, group["kind"], group["n"], group["k"], bad))
    ix.close()
    ctx.close()
