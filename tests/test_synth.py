import numpy as np
import oracle_lib as O
import pytest


def test_host_generator_format(synth):
    c = synth.gen_corpus(5, V=1000, seed=3, len_lo=10, len_hi=20)
    recs = O.split_records(c)
    assert len(recs) == 5
    assert c.startswith(b"<DOC>\n<DOCNO>D000000000</DOCNO>\n<TEXT>\n")
    assert c.endswith(b"</TEXT>\n</DOC>\n")
    assert synth.gen_corpus(5, V=1000, seed=3, len_lo=10, len_hi=20) == c


def test_vocab_has_no_stopwords(synth):
    blob, offs = synth.make_vocab(5000, 1)
    words = [blob[offs[i]:offs[i + 1]].decode() for i in range(5000)]
    assert len(set(words)) == 5000
    assert not any(O.is_stopword(w) for w in words)
    assert all(3 <= len(w) <= 12 for w in words)


def test_oracle_indexes_synthetic(synth):
    n = 50
    c = synth.gen_corpus(n, V=2000, seed=5, len_lo=30, len_hi=60)
    ix = O.OracleIndex(c, synth.mapping_bytes(n), 1, 1)
    assert ix.N == n
    terms = ix.terms()
    docid_terms = [t for t in terms if t[0][0].startswith("d0000")]
    assert len(docid_terms) == n  # T7: the DOCNO text is itself indexed


@pytest.mark.gpu
def test_device_generator_matches_host(synth, sme):
    import ctypes as C
    n, V, seed = 300, 5000, 9
    blob, offs = synth.make_vocab(V, seed)
    cdf = synth.zipf_cdf(V)
    L = sme.lib()
    L.sme_synth_corpus.argtypes = [C.c_int, C.c_char_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64,
                                   C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.sme_synth_free.argtypes = [C.c_void_p]
    ptr, nb = C.c_void_p(), C.c_size_t()
    rc = L.sme_synth_corpus(0, blob, offs.ctypes.data, V, cdf.ctypes.data, n, 0, seed, 40, 80, C.byref(ptr),
                            C.byref(nb))
    assert rc == 0
    host = np.zeros(nb.value, dtype=np.uint8)
    sme.memcpy(host.ctypes.data, ptr.value, nb.value)
    L.sme_synth_free(ptr)
    assert host.tobytes() == synth.gen_corpus(n, V=V, seed=seed, len_lo=40, len_hi=80)
