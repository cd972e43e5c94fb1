"""sme -- MI355X-native drop-in for the reference's index/TF-IDF/query hot path.

Host-side mirror of the reference operator surface (names follow the Java
classes; see include/sme.h for the C-ABI each call goes through):

  TermKGramDocIndexer    C/sa/edu/kaust/indexing/TermKGramDocIndexer.java:227-283 (run)
  TrecDocnoMapping       C/edu/umd/cloud9/collection/trec/TrecDocnoMapping.java:92-155
  GalagoTokenizer        C/ivory/tokenize/GalagoTokenizer.java:139-183 (processContent)
  IntDocVectorsForwardIndex  C/sa/edu/kaust/fwindex/IntDocVectorsForwardIndex.java:131-223
                         (getValue / rank), batched as Index.query_topk

Everything computes on the GPU through libsme.so.  There is no CPU fallback:
if the HIP library is missing or no GPU is visible, calls raise SmeError.
"""
import ctypes as C
import os
import struct

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SME_LIB_PATH") or os.path.join(_HERE, "libsme.so")

SME_IDF_REFERENCE = 0
SME_TIE_DOCNO = 0      # score desc, docno asc (north star)
SME_TIE_REFERENCE = 1  # score desc, then rank()'s printed order (first encounter; include/sme.h)
SME_TIE_JAVA7 = 2      # rank()'s list as Java 7's Collections.sort (TimSort) leaves it; -2 rows: it throws
SME_IDF_TRUE_DF = 1


class SmeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("sme error %d: %s" % (code, msg))
        self.code = code


class _Config(C.Structure):
    _fields_ = [("k", C.c_int), ("num_partitions", C.c_int), ("idf_mode", C.c_int), ("tiebreak", C.c_int),
                ("device", C.c_int), ("reserved", C.c_int * 11)]


_lib = None

EXPORTS = [
    "sme_last_error", "sme_version", "sme_device_alloc", "sme_device_free", "sme_memcpy", "sme_create", "sme_destroy", "sme_load_docno_mapping", "sme_build_index",
    "sme_build_index_device", "sme_index_free", "sme_index_stats", "sme_index_partition_records", "sme_index_serialize",
    "sme_index_copy_records", "sme_index_csr",
    "sme_index_device_arrays", "sme_index_term", "sme_tokenize", "sme_lookup_terms", "sme_query_topk",
    "sme_query_topk_device", "sme_query_topk_device_tie", "sme_query_topk_tie", "sme_last_build_profile", "sme_index_reweight", "sme_number_documents",
    "sme_build_chargram", "sme_build_chargram_device", "sme_chargram_partition_text", "sme_chargram_stats",
    "sme_split_points", "sme_split_points_device", "sme_index_term_fingerprints", "sme_set_option",
    "sme_index_prepare_queries", "sme_hbm_copy_bench", "sme_index_pack_pieces", "sme_merge_pieces",
    "sme_index_record_docnos", "sme_df_owner_pack", "sme_df_owner_sum", "sme_df_owner_unpack",
    "sme_topk_merge_rows", "sme_count_shared_keys",
]


def lib():
    """Load libsme.so (fails loudly: the product has no CPU path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SmeError(-2, "libsme.so not built (run __graft_entry__.build() or make -C %s)" % _HERE)
    # a process that also drives the device through torch lets torch's HIP runtime
    # open it first (torch's lazy init fails once libsme's runtime holds the device)
    import sys
    t = sys.modules.get("torch")
    if t is not None and t.cuda.is_available():
        t.cuda.init()
    L = C.CDLL(LIB_PATH)
    vp, sz, i64p, i32p = C.c_void_p, C.c_size_t, C.POINTER(C.c_int64), C.POINTER(C.c_int32)
    L.sme_last_error.restype = C.c_char_p
    L.sme_device_alloc.argtypes = [C.c_int, sz, C.POINTER(vp)]
    L.sme_device_free.argtypes = [vp]
    L.sme_device_free.restype = None
    L.sme_memcpy.argtypes = [vp, vp, sz, vp]
    L.sme_version.restype = C.c_char_p
    L.sme_create.argtypes = [C.POINTER(_Config), C.POINTER(vp)]
    L.sme_destroy.argtypes = [vp]
    L.sme_destroy.restype = None
    L.sme_load_docno_mapping.argtypes = [vp, C.c_char_p, sz]
    L.sme_build_index.argtypes = [vp, C.c_char_p, sz, C.POINTER(vp)]
    L.sme_build_index_device.argtypes = [vp, vp, sz, vp, C.POINTER(vp)]
    L.sme_index_free.argtypes = [vp]
    L.sme_index_free.restype = None
    L.sme_index_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.sme_index_partition_records.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(sz)]
    L.sme_index_serialize.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_float)]
    L.sme_index_copy_records.argtypes = [vp, C.c_int, vp, sz, C.POINTER(sz)]
    L.sme_index_csr.argtypes = [vp, C.POINTER(i64p), C.POINTER(i32p), C.POINTER(i32p), C.POINTER(i32p)]
    L.sme_index_device_arrays.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]
    L.sme_index_term.argtypes = [vp, C.c_int64, C.POINTER(vp), C.POINTER(sz)]
    L.sme_tokenize.argtypes = [vp, C.c_char_p, sz, vp, sz, i64p, C.c_int, C.POINTER(C.c_int)]
    L.sme_lookup_terms.argtypes = [vp, C.c_char_p, i64p, C.c_int, i32p]
    L.sme_query_topk.argtypes = [vp, i32p, i64p, C.c_int, C.c_int, i32p, C.POINTER(C.c_double)]
    L.sme_query_topk_device.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, vp]
    L.sme_query_topk_device_tie.argtypes = [vp, vp, vp, C.c_int, C.c_int, vp, vp, vp, vp]
    L.sme_query_topk_tie.argtypes = [vp, i32p, i64p, C.c_int, C.c_int, i32p, C.POINTER(C.c_double),
                                     C.POINTER(C.c_uint32)]
    L.sme_last_build_profile.argtypes = [vp, C.POINTER(C.c_char_p)]
    L.sme_index_reweight.argtypes = [vp, C.c_int64, vp, vp]
    L.sme_number_documents.argtypes = [vp, C.c_char_p, sz, C.POINTER(vp), C.POINTER(sz)]
    L.sme_build_chargram.argtypes = [vp, C.c_char_p, sz, C.POINTER(vp)]
    L.sme_build_chargram_device.argtypes = [vp, vp, sz, vp, C.POINTER(vp)]
    L.sme_chargram_partition_text.argtypes = [vp, C.c_int, C.POINTER(vp), C.POINTER(sz)]
    L.sme_chargram_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.sme_synth_corpus.argtypes = [C.c_int, C.c_char_p, vp, C.c_int64, vp, C.c_int64, C.c_int64, C.c_uint64, C.c_int,
                                   C.c_int, C.POINTER(vp), C.POINTER(sz)]
    L.sme_index_term_fingerprints.argtypes = [vp, vp, vp]
    L.sme_split_points.argtypes = [vp, C.c_char_p, sz, C.c_int, C.POINTER(C.c_uint64)]
    L.sme_split_points_device.argtypes = [vp, vp, sz, C.c_int, vp, C.POINTER(C.c_uint64)]
    L.sme_set_option.argtypes = [vp, C.c_char_p, C.c_int64]
    L.sme_index_prepare_queries.argtypes = [vp, vp, C.POINTER(C.c_float)]
    L.sme_synth_free.argtypes = [vp]
    L.sme_hbm_copy_bench.argtypes = [C.c_int, sz, C.c_int, C.POINTER(C.c_double)]
    L.sme_synth_free.restype = None
    L.sme_index_pack_pieces.argtypes = [vp, C.c_int, vp, C.POINTER(C.c_uint64), vp]
    L.sme_merge_pieces.argtypes = [vp, vp, C.POINTER(C.c_uint64), C.c_int, vp, C.POINTER(vp)]
    L.sme_index_record_docnos.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_int64)]
    L.sme_df_owner_pack.argtypes = [vp, vp, vp, C.c_int64, C.c_int, vp, vp, vp, i64p, vp]
    L.sme_df_owner_sum.argtypes = [vp, vp, vp, C.c_int64, vp, i64p, vp]
    L.sme_df_owner_unpack.argtypes = [vp, vp, vp, C.c_int64, vp, vp]
    L.sme_topk_merge_rows.argtypes = [vp, vp, vp, vp, C.c_int64, C.c_int, C.c_int, vp, vp, vp, vp]
    L.sme_count_shared_keys.argtypes = [vp, vp, C.c_int64, i64p, vp]
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise SmeError(rc, lib().sme_last_error().decode("utf-8", "replace"))


def memcpy(dst, src, nbytes, stream=None):
    """Copy between host and device memory through libsme's HIP runtime
    (sme_memcpy; stream None = synchronous).  Python never loads a HIP runtime
    of its own: torch's bundled one and the library's could disagree."""
    _check(lib().sme_memcpy(C.c_void_p(dst), C.c_void_p(src), nbytes, C.c_void_p(stream or 0)))


def _d2h(arr, dptr, nbytes):
    """device -> host into a numpy array."""
    memcpy(arr.ctypes.data, dptr, nbytes)


def _host_bytes(p, n):
    """Copy n bytes at host address p (ctypes.string_at takes a C int size: < 2 GiB)."""
    if not n:
        return b""
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_ubyte)), shape=(n,)).tobytes()


def _mutf8_decode(b):
    """DataInput.readUTF body -> str (surrogates kept)."""
    out, i = [], 0
    while i < len(b):
        c = b[i]
        if c < 0x80:
            out.append(c)
            i += 1
        elif c & 0xE0 == 0xC0:
            out.append(((c & 0x1F) << 6) | (b[i + 1] & 0x3F))
            i += 2
        else:
            out.append(((c & 0x0F) << 12) | ((b[i + 1] & 0x3F) << 6) | (b[i + 2] & 0x3F))
            i += 3
    raw = b"".join(u.to_bytes(2, "little") for u in out)
    return raw.decode("utf-16-le", "surrogatepass")


# ---------------------------------------------------------------------------
class TrecDocnoMapping:
    """Docno mapping file: int32 N, N x writeUTF(docid), docids sorted (writeDocnoData)."""

    @staticmethod
    def write(docids):
        out = [struct.pack(">i", len(docids))]
        for d in docids:
            b = d.encode("utf-8")
            out.append(struct.pack(">H", len(b)) + b)
        return b"".join(out)


class Context:
    """One device context (sme_ctx): config + docno mapping + reusable HBM workspace."""

    def __init__(self, k=1, num_partitions=1, idf_mode=SME_IDF_REFERENCE, device=0, tiebreak=SME_TIE_DOCNO):
        cfg = _Config(k, num_partitions, idf_mode, tiebreak, device)
        h = C.c_void_p()
        _check(lib().sme_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.k, self.num_partitions, self.idf_mode, self.device = k, num_partitions, idf_mode, device
        self.tiebreak = tiebreak

    def close(self):
        if getattr(self, "_h", None):
            lib().sme_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_option(self, name, value):
        """sme_set_option: a result-preserving path option (include/sme.h)."""
        _check(lib().sme_set_option(self._h, name.encode(), int(value)))

    def load_docno_mapping(self, mapping_bytes):
        _check(lib().sme_load_docno_mapping(self._h, mapping_bytes, len(mapping_bytes)))

    def number_documents(self, corpus):
        """NumberTrecDocuments + writeDocnoData on the device: the mapping file bytes."""
        p, n = C.c_void_p(), C.c_size_t()
        _check(lib().sme_number_documents(self._h, corpus, len(corpus), C.byref(p), C.byref(n)))
        return C.string_at(p, n.value)

    def build(self, corpus):
        """Build from host bytes (copied to HBM)."""
        h = C.c_void_p()
        _check(lib().sme_build_index(self._h, corpus, len(corpus), C.byref(h)))
        return Index(h, self)

    def build_ptr(self, host_ptr, nbytes):
        """Build from nbytes of host memory at address host_ptr (pinned memory is
        copied to HBM at DMA rate)."""
        h = C.c_void_p()
        _check(lib().sme_build_index(self._h, C.cast(C.c_void_p(host_ptr), C.c_char_p), nbytes, C.byref(h)))
        return Index(h, self)

    def build_device(self, d_ptr, nbytes, stream=None):
        """Build from a corpus already in HBM (e.g. a torch uint8 tensor's data_ptr())."""
        h = C.c_void_p()
        _check(lib().sme_build_index_device(self._h, C.c_void_p(d_ptr), nbytes, C.c_void_p(stream or 0),
                                            C.byref(h)))
        return Index(h, self)

    def df_owner_pack(self, d_fp, d_df, n, world, d_send_fp, d_send_df, d_pos, stream=None):
        """sme_df_owner_pack: rows grouped by owner rank (fp word 0 mod world) for
        one all_to_all; returns the rows per owner (list of `world` ints)."""
        counts = (C.c_int64 * max(world, 1))()
        _check(lib().sme_df_owner_pack(self._h, C.c_void_p(d_fp), C.c_void_p(d_df), n, world, C.c_void_p(d_send_fp),
                                       C.c_void_p(d_send_df), C.c_void_p(d_pos), counts, C.c_void_p(stream or 0)))
        return [int(c) for c in counts[:world]]

    def df_owner_sum(self, d_fp, d_df, n, d_out, stream=None):
        """sme_df_owner_sum: per received row, df summed over its fingerprint's
        rows; returns the number of distinct fingerprints."""
        dist = C.c_int64()
        _check(lib().sme_df_owner_sum(self._h, C.c_void_p(d_fp), C.c_void_p(d_df), n, C.c_void_p(d_out),
                                      C.byref(dist), C.c_void_p(stream or 0)))
        return dist.value

    def df_owner_unpack(self, d_ret, d_pos, n, d_out, stream=None):
        """sme_df_owner_unpack: out[i] = ret[pos[i]]."""
        _check(lib().sme_df_owner_unpack(self._h, C.c_void_p(d_ret), C.c_void_p(d_pos), n, C.c_void_p(d_out),
                                         C.c_void_p(stream or 0)))

    def topk_merge_rows(self, d_score, d_docno, d_tie, rows, m, k, d_out_docno, d_out_score, d_out_tie, stream=None):
        """sme_topk_merge_rows: rows x m candidates (device; d_tie may be 0) -> per
        row the best k by (score desc, tie asc, docno asc), docno -1 pads."""
        _check(lib().sme_topk_merge_rows(self._h, C.c_void_p(d_score), C.c_void_p(d_docno), C.c_void_p(d_tie or 0),
                                         rows, m, k, C.c_void_p(d_out_docno), C.c_void_p(d_out_score),
                                         C.c_void_p(d_out_tie or 0), C.c_void_p(stream or 0)))

    def count_shared_keys(self, d_rows, n, stream=None):
        """sme_count_shared_keys: (key, source rank) u64 pairs -> distinct keys
        that arrive from two or more sources."""
        cnt = C.c_int64()
        _check(lib().sme_count_shared_keys(self._h, C.c_void_p(d_rows), n, C.byref(cnt), C.c_void_p(stream or 0)))
        return cnt.value

    def merge_pieces(self, d_blobs, sizes):
        """sme_merge_pieces: the blobs one rank received from every shard (device
        memory at d_blobs, back to back, `sizes` bytes each, shard order) -> a
        records-only Index whose partitions p with p % world == rank are the
        reference's reduce output for those partitions (include/sme.h)."""
        n = len(sizes)
        arr = (C.c_uint64 * max(n, 1))(*[int(x) for x in sizes])
        h = C.c_void_p()
        _check(lib().sme_merge_pieces(self._h, C.c_void_p(d_blobs), arr, n, None, C.byref(h)))
        return Index(h, self)

    def build_chargram(self, corpus):
        """CharKGramTermIndexer over host bytes (k = this context's k, R = num_partitions)."""
        h = C.c_void_p()
        _check(lib().sme_build_chargram(self._h, corpus, len(corpus), C.byref(h)))
        return CharGramOutput(h, self)

    def build_chargram_device(self, d_ptr, nbytes, stream=None):
        h = C.c_void_p()
        _check(lib().sme_build_chargram_device(self._h, C.c_void_p(d_ptr), nbytes, C.c_void_p(stream or 0),
                                               C.byref(h)))
        return CharGramOutput(h, self)

    def last_build_profile(self):
        import json
        p = C.c_char_p()
        _check(lib().sme_last_build_profile(self._h, C.byref(p)))
        return json.loads(p.value.decode())

    def process_content(self, text):
        """GalagoTokenizer.processContent on the device."""
        b = text.encode("utf-8") if isinstance(text, str) else bytes(text)
        cap_tok = len(b) + 4
        buf = (C.c_ubyte * (3 * len(b) + 16))()
        offs = (C.c_int64 * (cap_tok + 1))()
        nt = C.c_int(0)
        _check(lib().sme_tokenize(self._h, b, len(b), buf, len(buf), offs, cap_tok, C.byref(nt)))
        raw = bytes(buf)
        return [_mutf8_decode(raw[offs[i]:offs[i + 1]]) for i in range(nt.value)]


class Index:
    """A built index (sme_index): reduce output + query-side CSR, resident in HBM."""

    def __init__(self, h, ctx):
        self._h, self.ctx = h, ctx
        n, v, p = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().sme_index_stats(h, C.byref(n), C.byref(v), C.byref(p)))
        self.N, self.V, self.P = n.value, v.value, p.value

    def close(self):
        if getattr(self, "_h", None):
            lib().sme_index_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def partition_records(self, part):
        """Record bytes of reduce partition `part`, always as a bytearray (one D2H
        copy into it; large partitions are not copied again into immutable bytes --
        wrap with bytes() where an immutable/hashable object is needed)."""
        offs, _ = self.serialize()
        out = bytearray(int(offs[part + 1] - offs[part]))
        self.copy_records(part, out)
        return out

    def record_docnos_ptr(self):
        """(device pointer, N): the docnos of the index's records in input order."""
        p, n = C.c_void_p(), C.c_int64()
        _check(lib().sme_index_record_docnos(self._h, C.byref(p), C.byref(n)))
        return p.value or 0, n.value

    def pack_pieces(self, world, d_out=None):
        """sme_index_pack_pieces: sizes of this shard's `world` per-owner blobs
        (d_out None), or write them back to back at device address d_out."""
        arr = (C.c_uint64 * world)()
        _check(lib().sme_index_pack_pieces(self._h, int(world), C.c_void_p(d_out or 0), arr, None))
        return [int(x) for x in arr]

    def serialize(self):
        """Device serialization of every partition (once per index):
        (partition byte offsets [R+1] in the concatenated stream, k_ser_* device ms)."""
        R = self.ctx.num_partitions
        offs = (C.c_uint64 * (R + 1))()
        ms = C.c_float()
        _check(lib().sme_index_serialize(self._h, offs, C.byref(ms)))
        return np.array(offs[:], dtype=np.int64), float(ms.value)

    def copy_records(self, part, out):
        """Copy partition `part`'s records (part = -1: all partitions back to back)
        into `out` (a writable buffer: bytearray, numpy uint8 array, pinned torch
        tensor's numpy view ...) straight from HBM; returns the byte count."""
        n = C.c_size_t()
        if hasattr(out, "ctypes"):
            ptr, cap = out.ctypes.data, out.nbytes
        else:
            mv = memoryview(out)
            cap = mv.nbytes
            ptr = C.addressof((C.c_char * max(cap, 1)).from_buffer(out)) if cap else None
        _check(lib().sme_index_copy_records(self._h, part, ptr, cap, C.byref(n)))
        return n.value

    def csr(self):
        """(offsets[V+1], docno[P], tf[P], true_df[V]) in reduce-output order (tf desc, docno asc)."""
        o, d, t, f = C.POINTER(C.c_int64)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)(), C.POINTER(C.c_int32)()
        _check(lib().sme_index_csr(self._h, C.byref(o), C.byref(d), C.byref(t), C.byref(f)))
        V, P = self.V, self.P

        def arr(ptr, n, dt):  # empty host vectors may hand out NULL
            return np.ctypeslib.as_array(ptr, (n,)).copy() if n else np.zeros(0, dt)
        return arr(o, V + 1, np.int64), arr(d, P, np.int32), arr(t, P, np.int32), arr(f, V, np.int32)

    def device_arrays(self):
        o, d, w = C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check(lib().sme_index_device_arrays(self._h, C.byref(o), C.byref(d), C.byref(w)))
        return o.value, d.value, w.value

    def offsets(self):
        """int64 offsets[V+1] of the postings per term (df = np.diff)."""
        o, _, _ = self.device_arrays()
        off = np.zeros(self.V + 1, np.int64)
        _d2h(off, o, 8 * (self.V + 1))
        return off

    def term_fingerprints(self, d_out, stream=None):
        """128-bit fingerprint per term into device memory d_out (uint64 [V, 2])."""
        _check(lib().sme_index_term_fingerprints(self._h, C.c_void_p(d_out), C.c_void_p(stream or 0)))

    def weights(self):
        """Host copies of the query-side CSR and the TF-IDF weight pass's output:
        (offsets[V+1], docno[P] docno-ascending per term, w[P] fp64)."""
        o, d, w = self.device_arrays()
        V, P = self.V, self.P
        off = np.zeros(V + 1, np.int64)
        dn = np.zeros(max(P, 1), np.int32)
        ws = np.zeros(max(P, 1), np.float64)
        _d2h(off, o, 8 * (V + 1))
        if P:
            _d2h(dn, d, 4 * P)
            _d2h(ws, w, 8 * P)
        return off, dn[:P], ws[:P]

    def term(self, t):
        p, n = C.c_void_p(), C.c_size_t()
        _check(lib().sme_index_term(self._h, t, C.byref(p), C.byref(n)))
        return _mutf8_decode(C.string_at(p, n.value))

    def terms(self):
        return [self.term(t) for t in range(self.V)]

    def lookup(self, terms):
        bs = [t.encode("utf-8", "surrogatepass") for t in terms]
        offs = np.zeros(len(bs) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(b) for b in bs]) if bs else []
        ids = np.zeros(max(len(bs), 1), dtype=np.int32)
        _check(lib().sme_lookup_terms(self._h, b"".join(bs), offs.ctypes.data_as(C.POINTER(C.c_int64)), len(bs),
                                      ids.ctypes.data_as(C.POINTER(C.c_int32))))
        return ids[:len(bs)]

    def query_topk(self, term_ids, q_offsets, k=10, with_tie=False):
        """Batched rank(): returns (docno[nq,k], score[nq,k]); docno -1 pads.
        with_tie: also the uint32 tie word of every result (sme_query_topk_tie),
        the key doc-shard merges need under SME_TIE_REFERENCE."""
        term_ids = np.ascontiguousarray(term_ids, dtype=np.int32)
        q_offsets = np.ascontiguousarray(q_offsets, dtype=np.int64)
        nq = len(q_offsets) - 1
        dn = np.zeros((max(nq, 1), k), dtype=np.int32)
        sc = np.zeros((max(nq, 1), k), dtype=np.float64)
        args = [self._h, term_ids.ctypes.data_as(C.POINTER(C.c_int32)), q_offsets.ctypes.data_as(C.POINTER(C.c_int64)),
                nq, k, dn.ctypes.data_as(C.POINTER(C.c_int32)), sc.ctypes.data_as(C.POINTER(C.c_double))]
        if not with_tie:
            _check(lib().sme_query_topk(*args))
            return dn[:nq], sc[:nq]
        tie = np.zeros((max(nq, 1), k), dtype=np.uint32)
        _check(lib().sme_query_topk_tie(*args, tie.ctypes.data_as(C.POINTER(C.c_uint32))))
        return dn[:nq], sc[:nq], tie[:nq]

    def prepare_queries(self, stream=None):
        """Build the query-side heavy rows now (else the first query batch does);
        returns their device build time in ms."""
        ms = C.c_float(0.0)
        _check(lib().sme_index_prepare_queries(self._h, C.c_void_p(stream or 0), C.byref(ms)))
        return ms.value

    def reweight(self, n_global, d_df_global=None, stream=None):
        """TF-IDF weights with all-reduced N (and df) of a doc-sharded index."""
        _check(lib().sme_index_reweight(self._h, n_global, C.c_void_p(d_df_global or 0), C.c_void_p(stream or 0)))

    def query_topk_device(self, d_terms, d_qoff, nq, k, d_out_docno, d_out_score, stream=None, d_out_tie=None):
        if d_out_tie is None:
            _check(lib().sme_query_topk_device(self._h, C.c_void_p(d_terms), C.c_void_p(d_qoff), nq, k,
                                               C.c_void_p(d_out_docno), C.c_void_p(d_out_score),
                                               C.c_void_p(stream or 0)))
        else:
            _check(lib().sme_query_topk_device_tie(self._h, C.c_void_p(d_terms), C.c_void_p(d_qoff), nq, k,
                                                   C.c_void_p(d_out_docno), C.c_void_p(d_out_score),
                                                   C.c_void_p(d_out_tie), C.c_void_p(stream or 0)))


class DeviceCorpus:
    """A synthetic Zipfian TREC corpus generated directly in HBM (sme_synth_corpus;
    the same bytes as synth.gen_corpus): docs d0 .. d0+n_docs-1."""

    def __init__(self, n_docs, V=1 << 20, seed=42, len_lo=400, len_hi=600, d0=0, device=0):
        from . import synth
        blob, voff = synth.make_vocab(V, seed)
        cdf = synth.zipf_cdf(V, 1.0)
        p, n = C.c_void_p(), C.c_size_t()
        _check(lib().sme_synth_corpus(device, blob, voff.ctypes.data, V, cdf.ctypes.data, n_docs, d0, seed, len_lo,
                                      len_hi, C.byref(p), C.byref(n)))
        self.ptr, self.nbytes = p.value, n.value

    def to_host(self):
        """Copy the corpus bytes back (hipMemcpy device -> host)."""
        out = np.zeros(max(self.nbytes, 1), np.uint8)
        _d2h(out, self.ptr, self.nbytes)
        return out[:self.nbytes].tobytes()

    def close(self):
        if getattr(self, "ptr", None):
            lib().sme_synth_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------
class CharGramOutput:
    """Output of the CharKGramTermIndexer job: the text of every reduce partition."""

    def __init__(self, h, ctx):
        self._h, self.ctx = h, ctx
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib().sme_chargram_stats(h, C.byref(a), C.byref(b)))
        self.ngrams, self.npairs = a.value, b.value

    def close(self):
        if getattr(self, "_h", None):
            lib().sme_index_free(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def partition_text(self, part):
        p, n = C.c_void_p(), C.c_size_t()
        _check(lib().sme_chargram_partition_text(self._h, part, C.byref(p), C.byref(n)))
        return _host_bytes(p, n.value)


# reference-shaped facades
class GalagoTokenizer:
    """GalagoTokenizer.processContent, evaluated by the device tokenizer."""

    def __init__(self, ctx=None):
        self.ctx = ctx or Context()

    def processContent(self, text):  # noqa: N802 (reference name)
        return self.ctx.process_content(text)


class NumberTrecDocuments:
    """NumberTrecDocuments.run(input, output, mappingFile, nMappers) as one device
    call: returns (and optionally writes) the docno mapping file."""

    def __init__(self, device=0):
        self.ctx = Context(device=device)

    def run(self, corpus, mapping_file=None):
        corpus = open(corpus, "rb").read() if isinstance(corpus, str) else corpus
        m = self.ctx.number_documents(corpus)
        if mapping_file is not None:
            with open(mapping_file, "wb") as f:
                f.write(m)
        return m


class TermKGramDocIndexer:
    """TermKGramDocIndexer.run(K, input, output, mapping) as one device call.

    run() returns the Index; if output_dir is given, the reduce partitions are
    written as part-NNNNN files (SequenceFile v6 container, see seqfile.py).
    """

    def __init__(self, k=1, num_reduce_tasks=10, idf_mode=SME_IDF_REFERENCE, device=0):
        self.ctx = Context(k, num_reduce_tasks, idf_mode, device)

    def run(self, corpus, mapping, output_dir=None):
        corpus = open(corpus, "rb").read() if isinstance(corpus, str) else corpus
        mapping = open(mapping, "rb").read() if isinstance(mapping, str) else mapping
        self.ctx.load_docno_mapping(mapping)
        ix = self.ctx.build(corpus)
        if output_dir is not None:
            from . import seqfile
            seqfile.write_index_dir(ix, output_dir)
        return ix


class CharKGramTermIndexer:
    """CharKGramTermIndexer.run(K, input, output) as one device call (R = 10 reducers
    as the reference's run() sets); writes part-NNNNN text files if output_dir is given."""

    def __init__(self, k=2, num_reduce_tasks=10, device=0):
        self.ctx = Context(k, num_reduce_tasks, SME_IDF_REFERENCE, device)

    def run(self, corpus, output_dir=None):
        corpus = open(corpus, "rb").read() if isinstance(corpus, str) else corpus
        out = self.ctx.build_chargram(corpus)
        if output_dir is not None:
            os.makedirs(output_dir, exist_ok=True)
            for p in range(self.ctx.num_partitions):
                with open(os.path.join(output_dir, "part-%05d" % p), "wb") as f:
                    f.write(out.partition_text(p))
        return out


class IntDocVectorsForwardIndex:
    """Query side: getValue(terms) then rank() -> up to 10 docnos (score desc,
    docno asc), plus the REPL contract of IntDocVectorsForwardIndex.main
    (C/sa/edu/kaust/fwindex/IntDocVectorsForwardIndex.java:243-322) in query_line."""

    def __init__(self, index, mapping=None):
        self.index = index
        self._terms = []
        self._docids = None
        if mapping is not None:  # TrecDocnoMapping.loadMapping: {"", docids...}
            n = struct.unpack_from(">i", mapping, 0)[0]
            p, ids = 4, [""]
            for _ in range(n):
                ln = struct.unpack_from(">H", mapping, p)[0]
                ids.append(_mutf8_decode(mapping[p + 2:p + 2 + ln]))
                p += 2 + ln
            self._docids = ids

    def getValue(self, terms):  # noqa: N802
        ids = self.index.lookup(list(terms))
        self._terms = [int(t) for t in ids if t >= 0]  # unknown terms are skipped silently

    def rank(self, k=10):
        if not self._terms:
            return []
        dn, _ = self.index.query_topk(np.array(self._terms, np.int32), np.array([0, len(self._terms)], np.int64), k)
        return [int(d) for d in dn[0] if d >= 0]

    def query_line(self, line, tokenizer=None):
        """One REPL turn (:284-320): trim; an empty line, or one that is not 1-2
        raw words (String.split("\\s+")), ends the session (returns None);
        otherwise processContent -> getValue -> rank, printed as main prints it:
        Arrays.toString of the docnos, or the docids each followed by a space
        (mapping given), or "No results ..."."""
        import re
        term = line
        b, e = 0, len(term)
        while b < e and ord(term[b]) <= 0x20:  # String.trim
            b += 1
        while e > b and ord(term[e - 1]) <= 0x20:
            e -= 1
        term = term[b:e]
        if not term:
            return None
        orig = re.split(r"[ \t\n\x0b\f\r]+", term)
        if len(orig) not in (1, 2):
            return None
        ctx = tokenizer or self.index.ctx
        self.getValue(ctx.process_content(term))
        res = self.rank()
        if self._docids is None:
            body = ("[" + ", ".join(str(d) for d in res) + "]") if res else "No results ..."
        else:
            body = "".join(self._docids[d] + " " for d in res) if res else "No results ..."
        return term + ": " + body
