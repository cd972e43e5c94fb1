"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

Test infrastructure only: the oracle is the checker, never the product.
"""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(LIB_PATH)
        L.or_process_content_utf8.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_int)]
        L.or_tag_tokenize_utf8.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_int)]
        L.or_stem_utf8.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.or_is_stopword_utf8.argtypes = [C.c_char_p, C.c_size_t]
        L.or_build_index.restype = C.c_void_p
        L.or_build_index.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int, C.c_int,
                                     C.c_void_p, C.c_int]
        L.or_index_free.argtypes = [C.c_void_p]
        L.or_index_nterms.argtypes = [C.c_void_p]
        L.or_index_N.argtypes = [C.c_void_p]
        L.or_index_part_len.argtypes = [C.c_void_p, C.c_int]
        L.or_index_part_len.restype = C.c_size_t
        L.or_index_part_bytes.argtypes = [C.c_void_p, C.c_int]
        L.or_index_part_bytes.restype = C.c_void_p
        for f in ("or_index_term_part", "or_index_term_npost", "or_index_term_df_field", "or_index_term_k"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_int]
        L.or_index_term_gram.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int]
        L.or_index_term_postings.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.or_query_utf8.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_void_p, C.c_void_p]
        L.or_last_error.restype = C.c_char_p
        L.or_lookup_selfcheck.argtypes = [C.c_void_p]
        L.or_set_ref_scan.argtypes = [C.c_int]
        L.or_sort_docscores.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
        L.or_count_distinct_terms.restype = C.c_int64
        L.or_count_distinct_terms.argtypes = [C.c_char_p, C.c_void_p, C.c_int64]
        L.or_split_records.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int]
        L.or_cpuopt_split_records.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int]
        L.or_chargram.restype = C.c_void_p
        L.or_chargram.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int]
        L.or_chargram_ngrams.argtypes = [C.c_void_p]
        L.or_chargram_npairs.argtypes = [C.c_void_p]
        L.or_chargram_npairs.restype = C.c_longlong
        L.or_chargram_part_len.argtypes = [C.c_void_p, C.c_int]
        L.or_chargram_part_len.restype = C.c_size_t
        L.or_chargram_part_bytes.argtypes = [C.c_void_p, C.c_int]
        L.or_chargram_part_bytes.restype = C.c_void_p
        L.or_chargram_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def mutf8_decode(b):
    """DataInput.readUTF body -> str; surrogate pairs are combined like Java strings."""
    units, i = [], 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            units.append(c)
            i += 1
        elif c & 0xE0 == 0xC0:
            units.append(((c & 0x1F) << 6) | (b[i + 1] & 0x3F))
            i += 2
        else:
            units.append(((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F))
            i += 3
    raw = b"".join(u.to_bytes(2, "little") for u in units)
    return raw.decode("utf-16-le", "surrogatepass")


def _decode_toks(buf, n, ntok):
    out, k = [], 0
    for _ in range(ntok):
        ln = (buf[k] << 8) | buf[k + 1]
        out.append(mutf8_decode(bytes(buf[k + 2:k + 2 + ln])))
        k += 2 + ln
    return out


def _tok_call(fn, text):
    b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
    cap = 8 * len(b) + 64
    buf = (C.c_ubyte * cap)()
    nt = C.c_int(0)
    r = fn(b, len(b), buf, cap, C.byref(nt))
    assert r >= 0
    return _decode_toks(buf, r, nt.value)


def process_content(text):
    """GalagoTokenizer.processContent"""
    return _tok_call(lib().or_process_content_utf8, text)


def tag_tokenize(text):
    """TagTokenizer.tokenize(text).terms"""
    return _tok_call(lib().or_tag_tokenize_utf8, text)


def stem(word):
    b = word.encode("utf-8")
    buf = (C.c_ubyte * (4 * len(b) + 16))()
    r = lib().or_stem_utf8(b, len(b), buf, len(buf))
    return mutf8_decode(bytes(buf[:r]))


def is_stopword(word):
    b = word.encode("utf-8")
    return bool(lib().or_is_stopword_utf8(b, len(b)))


def split_records(corpus, cpuopt=False):
    """XMLRecordReader's records: the oracle's serial reader, or (cpuopt) the cpu-opt
    baseline's parallel split that must equal it."""
    cap = corpus.count(b"<DOC>") + 1
    off = (C.c_uint64 * cap)()
    ln = (C.c_uint64 * cap)()
    f = lib().or_cpuopt_split_records if cpuopt else lib().or_split_records
    n = f(corpus, len(corpus), off, ln, cap)
    return [(off[i], ln[i]) for i in range(n)]


class OracleIndex:
    """Result of the ref-faithful index job (terms in (partition, key) order)."""

    def __init__(self, corpus, mapping, K=1, R=1, splits=None):
        L = lib()
        sp = None
        nsp = 0
        if splits is not None:
            arr = (C.c_uint64 * len(splits))(*splits)
            sp, nsp = arr, len(splits) - 1
        self._h = L.or_build_index(corpus, len(corpus), mapping, len(mapping), K, R, sp, nsp)
        if not self._h:
            raise RuntimeError(L.or_last_error().decode())
        self.K, self.R = K, R
        self.N = L.or_index_N(self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_index_free(self._h)
            self._h = None

    def partition_bytes(self, part):
        L = lib()
        n = L.or_index_part_len(self._h, part)
        p = L.or_index_part_bytes(self._h, part)
        return C.string_at(p, n) if n else b""

    def terms(self):
        """list of (gram tuple, part, df_field, [(docno, tf), ...])"""
        L = lib()
        out = []
        buf = (C.c_ubyte * 70000)()
        for t in range(L.or_index_nterms(self._h)):
            k = L.or_index_term_k(self._h, t)
            gram = []
            for g in range(k):
                ln = L.or_index_term_gram(self._h, t, g, buf, len(buf))
                gram.append(mutf8_decode(bytes(buf[:ln])))
            n = L.or_index_term_npost(self._h, t)
            d = (C.c_int32 * max(n, 1))()
            f = (C.c_int32 * max(n, 1))()
            L.or_index_term_postings(self._h, t, d, f)
            out.append((tuple(gram), L.or_index_term_part(self._h, t), L.or_index_term_df_field(self._h, t),
                        [(d[i], f[i]) for i in range(n)]))
        return out

    def lookup_selfcheck(self):
        """disagreements between the forward-index lookup table and the O(V) scan"""
        return lib().or_lookup_selfcheck(self._h)

    def query(self, terms, k=10, idf_mode=0, order=0):
        """rank() over already-processed query terms; order 0 docno tie-break,
        1 Java-6 Collections.sort with DocScore comparator, 2 first-encounter,
        3 Java-7 Collections.sort (ComparableTimSort) with the DocScore comparator
        (None, None where Java 7 throws IllegalArgumentException)."""
        bs = [t.encode("utf-8") for t in terms]
        blob = b"".join(bs)
        offs = [0]
        for b in bs:
            offs.append(offs[-1] + len(b))
        o = (C.c_int * len(offs))(*offs)
        dn = (C.c_int32 * max(k, 1))()
        sc = (C.c_double * max(k, 1))()
        r = lib().or_query_utf8(self._h, blob, o, len(terms), k, idf_mode, order, dn, sc)
        if r < 0:  # order 3: Java 7's TimSort throws IllegalArgumentException here
            return None, None
        return [dn[i] for i in range(r)], [sc[i] for i in range(r)]


class OracleCharGram:
    """CharKGramTermIndexer restated on the CPU (oracle/oracle_chargram.c): the
    TextOutputFormat bytes of every reduce partition."""

    def __init__(self, corpus, k, R):
        self.R = R
        self._h = lib().or_chargram(corpus, len(corpus), k, R)
        if not self._h:
            raise ValueError("bad k/R")
        self.ngrams = lib().or_chargram_ngrams(self._h)
        self.npairs = lib().or_chargram_npairs(self._h)

    def part_bytes(self, p):
        n = lib().or_chargram_part_len(self._h, p)
        return C.string_at(lib().or_chargram_part_bytes(self._h, p), n) if n else b""

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_chargram_free(self._h)
            self._h = None


def write_mapping(docids):
    """TrecDocnoMapping.writeDocnoData format: int32 N, N x writeUTF (sorted docids)."""
    import struct
    out = [struct.pack(">i", len(docids))]
    for d in docids:
        b = d.encode("utf-8")
        out.append(struct.pack(">H", len(b)) + b)
    return b"".join(out)


class CpuOptIndex:
    """The cpu-opt baseline build (oracle/oracle_cpuopt.cc, OpenMP): K = 1, one split."""

    @staticmethod
    def _sigs():
        L = lib()
        L.or_cpuopt_build.restype = C.c_void_p
        L.or_cpuopt_build.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int]
        L.or_cpuopt_free.argtypes = [C.c_void_p]
        L.or_cpuopt_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_int64)] * 3 + [C.POINTER(C.c_double)]
        L.or_cpuopt_csr.argtypes = [C.c_void_p] + [C.c_void_p] * 5
        L.or_cpuopt_query.restype = C.c_double
        L.or_cpuopt_query.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_void_p, C.c_void_p]
        L.or_cpuopt_from_csr.restype = C.c_void_p
        L.or_cpuopt_from_csr.argtypes = [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
        return L

    def __init__(self, corpus, mapping, threads=0):
        import numpy as np
        L = self._sigs()
        self._h = L.or_cpuopt_build(corpus, len(corpus), mapping, len(mapping), threads)
        if not self._h:
            raise RuntimeError("cpu-opt build rejected the corpus")
        n, v, p, s = C.c_int64(), C.c_int64(), C.c_int64(), C.c_double()
        L.or_cpuopt_stats(self._h, C.byref(n), C.byref(v), C.byref(p), C.byref(s))
        self.N, self.V, self.P, self.build_s = n.value, v.value, p.value, s.value
        self.threads = threads

    @classmethod
    def from_csr(cls, N, off, docno, tf):
        """Wrap CSR arrays (reduce order) of an index built elsewhere; no term strings."""
        import numpy as np
        L = cls._sigs()
        self = cls.__new__(cls)
        off = np.ascontiguousarray(off, np.int64)
        docno = np.ascontiguousarray(docno, np.int32)
        tf = np.ascontiguousarray(tf, np.int32)
        self._h = L.or_cpuopt_from_csr(N, len(off) - 1, off.ctypes.data, docno.ctypes.data, tf.ctypes.data)
        self.N, self.V, self.P, self.build_s, self.threads = N, len(off) - 1, int(off[-1]), 0.0, 0
        return self

    def csr(self):
        """(offsets, docno, tf) in reduce order and the term strings (TermDF order)."""
        import numpy as np
        off = np.zeros(self.V + 1, np.int64)
        dn = np.zeros(max(self.P, 1), np.int32)
        tf = np.zeros(max(self.P, 1), np.int32)
        toff = np.zeros(self.V + 1, np.int64)
        lib().or_cpuopt_csr(self._h, off.ctypes.data, dn.ctypes.data, tf.ctypes.data, toff.ctypes.data, None)
        tch = np.zeros(max(int(toff[-1]), 1), np.uint16)
        lib().or_cpuopt_csr(self._h, off.ctypes.data, dn.ctypes.data, tf.ctypes.data, toff.ctypes.data,
                            tch.ctypes.data)
        raw = tch.tobytes()
        terms = [raw[2 * toff[i]:2 * toff[i + 1]].decode("utf-16-le", "surrogatepass") for i in range(self.V)]
        return off, dn[:self.P], tf[:self.P], terms

    def query(self, terms, qoff, k, idf_mode=0, threads=0):
        """Batched rank(); returns (docno [nq, k], score [nq, k], seconds)."""
        import numpy as np
        terms = np.ascontiguousarray(terms, np.int32)
        qoff = np.ascontiguousarray(qoff, np.int64)
        nq = len(qoff) - 1
        dn = np.zeros((max(nq, 1), k), np.int32)
        sc = np.zeros((max(nq, 1), k), np.float64)
        s = lib().or_cpuopt_query(self._h, terms.ctypes.data, qoff.ctypes.data, nq, k, idf_mode, threads,
                                  dn.ctypes.data, sc.ctypes.data)
        return dn[:nq], sc[:nq], s

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_cpuopt_free(self._h)
            self._h = None


def sort_docscores(scores, order):
    """rank()'s Collections.sort alone (oracle or_sort_docscores): candidates in
    list order with these scores -> their list indices in sorted order (order 1
    Java 6 legacy merge sort, 3 Java 7 ComparableTimSort, both over the DocScore
    comparator), or None where Java 7 throws IllegalArgumentException."""
    import numpy as np
    sc = np.ascontiguousarray(scores, dtype=np.float64)
    perm = np.zeros(max(len(sc), 1), np.int32)
    r = lib().or_sort_docscores(sc.ctypes.data, len(sc), order, perm.ctypes.data)
    return None if r < 0 else perm[:len(sc)].tolist()
