"""Doc-sharded multi-GPU plumbing: one process per GPU, torch.distributed
("nccl" = RCCL over xGMI on the GPU box, "gloo" in the CPU tests).

The index build itself has no data-path collective: every rank builds the index of
its own contiguous <DOC>-aligned shard (a Hadoop map split: each shard's doc-counter
postings start with (0,0), TermKGramDocIndexer.java:84-90,126).  The exchanges are
the small global statistics and the query results:

  split_points     Hadoop split ownership (XMLInputFormat.java:110-143): a record
                   belongs to the split its <DOC> start tag begins in; cuts are
                   record starts of one device reader pass (sme_split_points)
  global_count     N = sum of per-shard record counts        (all_reduce, 8 B)
  global_vocab     term strings of every shard -> global ids in TermDF.compareTo
                   order (all_gather of UTF-16BE bytes, local sort)
  global_df        df per global term = sum of shard postings lengths (all_reduce);
                   returned per LOCAL term for sme_index_reweight
  global_df_index  the same for a libsme shard, keyed by 128-bit device term
                   fingerprints, exchanged by owner rank (df_exchange: all_to_all
                   to the owner, sums of 1/W of the terms, all_to_all back; the
                   local steps are libsme kernels, sme_df_owner_*)
  reference_partitions  the reference's R term-partitioned part files from the
                   shards: all_to_all of per-owner term/postings blobs, per-term
                   reducer merge on the owner (sme_merge_pieces)
  merge_topk_owner per-shard top-k -> global top-k of the queries a rank owns
                   (query-owner all_to_all of Q x k x (4 + 8) B, then the W lists
                   of each owned query merged by score desc, tie word asc, docno
                   asc in libsme, sme_topk_merge_rows); merge_topk also
                   all_gathers the merged slices
  docno_duplicates docids held by two shards (owner all_to_all of (docno, rank)
                   rows grouped by sme_df_owner_pack, counted by
                   sme_count_shared_keys)

No torch sort / unique runs on these product paths: the grouping, sums, merges
and counts are libsme kernels (DeviceDfOps); the CPU tests pass a numpy / torch
restatement of the same local steps (tests/test_dist.py HostDfOps).

Exactness: with docids unique across shards (every synthetic corpus), the sharded
result equals the single-index result bit for bit: a document's score only uses its
own postings, and N / df are the global ones.  A docid duplicated ACROSS shards is
merged by the reference's single reducer: reference_partitions merges it the same
way (tf summed); the per-shard query path cannot (two partial postings), so
shard_docno_duplicates detects it so callers can refuse to score such shards.
"""
import importlib

import numpy as np
import torch
import torch.distributed as dist


def split_points(corpus, world, ctx=None):
    """Byte offsets [0, s1, ..., n] of `world` doc shards (sme_split_points):
    shard g = the records whose <DOC> match begins in [n*g/world, n*(g+1)/world)
    (Hadoop split ownership, XMLInputFormat.java:110-143,173-198), with the record
    starts taken from ONE record-reader pass on the device, so a shard never starts
    inside '<<DOC>' or at a nested <DOC>.  `corpus` is host bytes, or a
    sme.DeviceCorpus / (device pointer, nbytes) pair."""
    import ctypes as C
    import importlib
    sme = importlib.import_module(__package__)
    own = ctx is None
    ctx = ctx or sme.Context()
    try:
        cuts = (C.c_uint64 * (world + 1))()
        L = sme.lib()
        if isinstance(corpus, (bytes, bytearray)):
            rc = L.sme_split_points(ctx._h, bytes(corpus), len(corpus), world, cuts)
        else:
            ptr, n = (corpus.ptr, corpus.nbytes) if hasattr(corpus, "ptr") else corpus
            rc = L.sme_split_points_device(ctx._h, C.c_void_p(ptr), n, world, None, cuts)
        sme._check(rc)
        return [int(c) for c in cuts]
    finally:
        if own:
            ctx.close()


def cuts_from_starts(starts, n, world):
    """The same cut rule over a known list of record start offsets (sorted):
    cuts[g] = first start >= n*g//world, else n."""
    import bisect
    cuts = [0]
    for g in range(1, world):
        i = bisect.bisect_left(starts, n * g // world)
        cuts.append(starts[i] if i < len(starts) else n)
    cuts.append(n)
    return cuts


def _dev(group):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def global_count(n_local, group=None):
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=_dev(group))
    dist.all_reduce(t, group=group)
    return int(t.item())


def _gather_bytes(blob, group=None):
    dev = _dev(group)
    world = dist.get_world_size(group)
    ln = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    lens = [torch.zeros_like(ln) for _ in range(world)]
    dist.all_gather(lens, ln, group=group)
    m = max(int(x.item()) for x in lens)
    buf = torch.zeros(max(m, 1), dtype=torch.uint8, device=dev)
    if blob:
        buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    outs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return [bytes(o[:int(l.item())].cpu().numpy().tobytes()) for o, l in zip(outs, lens)]


def _encode_terms(terms):
    """UTF-16BE strings, each prefixed by its unit count (u32 BE)."""
    out = bytearray()
    for t in terms:
        b = t.encode("utf-16-be", "surrogatepass")
        out += (len(b) // 2).to_bytes(4, "big") + b
    return bytes(out)


def _decode_terms(blob):
    out, i = [], 0
    while i < len(blob):
        n = int.from_bytes(blob[i:i + 4], "big")
        out.append(blob[i + 4:i + 4 + 2 * n])
        i += 4 + 2 * n
    return out


def global_vocab(local_terms, group=None):
    """local_terms: this shard's terms (Python str, local id order).  Returns
    (global term list as UTF-16BE bytes in String.compareTo order, int64 array
    local id -> global id)."""
    parts = _gather_bytes(_encode_terms(local_terms), group)
    allt = sorted(set(t for p in parts for t in _decode_terms(p)))  # UTF-16BE byte order == compareTo
    pos = {t: i for i, t in enumerate(allt)}
    l2g = np.array([pos[t.encode("utf-16-be", "surrogatepass")] for t in local_terms], dtype=np.int64)
    return allt, l2g


def global_df(local_df, l2g, n_global_terms, group=None):
    """All-reduced df over global ids, returned per LOCAL term (int64)."""
    dev = _dev(group)
    g = torch.zeros(n_global_terms, dtype=torch.int64, device=dev)
    if len(l2g):
        g.index_add_(0, torch.from_numpy(l2g).to(dev), torch.from_numpy(np.asarray(local_df, np.int64)).to(dev))
    dist.all_reduce(g, group=group)
    return g[torch.from_numpy(l2g).to(dev)] if len(l2g) else g[:0]


_OWNER_CTX = {}


def _owner_ctx():
    """A libsme context on the current device for the owner-side kernels of
    callers that hold no index (merge_topk_owner, docno_duplicates)."""
    sme = importlib.import_module(__package__)
    d = torch.cuda.current_device()
    if d not in _OWNER_CTX:
        _OWNER_CTX[d] = sme.Context(device=d)
    return _OWNER_CTX[d]


class DeviceDfOps:
    """The multi-GPU path's local steps on the device, in libsme: the df
    exchange's owner grouping (counting scatter), owner sums (fingerprint hash
    table) and return gather (sme_dfx.hip), and the query owner's merge of the
    shards' top-k rows and the shared-docid count (sme_owner.hip).  Tensors are
    CUDA tensors (merge_rows / count_shared move theirs there and back); libsme
    runs them on the context's own stream, synchronized before torch reads the
    results."""

    def __init__(self, ctx=None):
        self.ctx = ctx if ctx is not None else _owner_ctx()

    def pack(self, fp, df, world):
        n = int(fp.shape[0])
        sfp = torch.empty((max(n, 1), 2), dtype=torch.int64, device=fp.device)
        sdf = torch.empty(max(n, 1), dtype=torch.int64, device=fp.device)
        pos = torch.empty(max(n, 1), dtype=torch.int64, device=fp.device)
        fp, df = fp.contiguous(), df.contiguous()
        torch.cuda.synchronize()
        counts = self.ctx.df_owner_pack(fp.data_ptr(), df.data_ptr(), n, world, sfp.data_ptr(), sdf.data_ptr(),
                                        pos.data_ptr())
        return sfp[:n], sdf[:n], pos[:n], counts

    def owner_sum(self, fp, df):
        n = int(fp.shape[0])
        out = torch.empty(max(n, 1), dtype=torch.int64, device=fp.device)
        fp, df = fp.contiguous(), df.contiguous()
        torch.cuda.synchronize()
        distinct = self.ctx.df_owner_sum(fp.data_ptr(), df.data_ptr(), n, out.data_ptr())
        return out[:n], distinct

    def unpack(self, ret, pos):
        n = int(pos.shape[0])
        out = torch.empty(max(n, 1), dtype=torch.int64, device=pos.device)
        ret = ret.contiguous()
        torch.cuda.synchronize()
        if n:
            self.ctx.df_owner_unpack(ret.data_ptr(), pos.data_ptr(), n, out.data_ptr())
        return out[:n]

    def merge_rows(self, s, d, k, t=None):
        """rows of candidates (score f64, docno i32, tie u32 as int64 or None)
        -> (docno int32, score f64, tie int64) [rows, k] (sme_topk_merge_rows),
        on the inputs' device."""
        src = s.device
        dev = torch.device("cuda", torch.cuda.current_device())
        rows, m = int(s.shape[0]), int(s.shape[1])
        s_ = s.to(dev, torch.float64).contiguous()
        d_ = d.to(dev, torch.int32).contiguous()
        t_ = t.to(dev, torch.int64).to(torch.int32).contiguous() if t is not None else None  # (low 32 bits)
        od = torch.empty((max(rows, 1), k), dtype=torch.int32, device=dev)
        os_ = torch.empty((max(rows, 1), k), dtype=torch.float64, device=dev)
        ot = torch.empty((max(rows, 1), k), dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        if rows:
            self.ctx.topk_merge_rows(s_.data_ptr(), d_.data_ptr(), t_.data_ptr() if t_ is not None else 0, rows, m, k,
                                     od.data_ptr(), os_.data_ptr(), ot.data_ptr())
        return od[:rows].to(src), os_[:rows].to(src), (ot[:rows].to(torch.int64) & 0xFFFFFFFF).to(src)

    def count_shared(self, rows):
        """(key, source rank) int64 [n, 2] rows -> distinct keys from two or more
        ranks (sme_count_shared_keys)."""
        dev = torch.device("cuda", torch.cuda.current_device())
        r = rows.to(dev).contiguous()
        torch.cuda.synchronize()
        return self.ctx.count_shared_keys(r.data_ptr(), int(r.shape[0])) if r.shape[0] else 0


def df_exchange(fp, df, group=None, timings=None, ops=None):
    """Global df per local term, keyed by term fingerprints (int64 [V, 2]; df int64
    [V]).  Each fingerprint has ONE owner rank (first word, as u64, mod W): one
    all_to_all sends every local (fingerprint, df) to its owner, each owner sums
    only the ~1/W of the terms it owns, and a second all_to_all returns the summed
    df to the senders.  Per rank that moves 24 B per local term out and 8 B back,
    and groups ~(sum of shard vocabularies) / W rows -- where an all_gather +
    unique on every rank would move and sort all of them (the reducer's view of
    df, TermKGramDocIndexer.java:175-183, is the postings length summed over the
    map outputs).  The local steps are `ops` (pack / owner_sum / unpack):
    DeviceDfOps (libsme kernels, the product) -- there is no host path; the CPU
    tests pass a numpy restatement of the same three steps."""
    import time
    if ops is None:
        raise ValueError("df_exchange needs its local steps (DeviceDfOps(ctx) on a GPU)")
    world = dist.get_world_size(group)
    cdev = _dev(group)
    V = int(fp.shape[0])
    t0 = time.perf_counter()
    send_fp, send_df, pos, cs = ops.pack(fp, df, world)
    counts = torch.tensor(cs, dtype=torch.int64, device=cdev)
    rcounts = torch.empty_like(counts)
    dist.all_to_all_single(rcounts, counts, group=group)
    rc = rcounts.tolist()
    nrecv = int(sum(rc))
    recv_fp = torch.empty((nrecv, 2), dtype=torch.int64, device=cdev)
    recv_df = torch.empty(nrecv, dtype=torch.int64, device=cdev)
    dist.all_to_all_single(recv_fp.view(-1), send_fp.to(cdev).contiguous().view(-1), [2 * c for c in rc],
                           [2 * c for c in cs], group=group)
    dist.all_to_all_single(recv_df, send_df.to(cdev).contiguous(), rc, cs, group=group)
    if cdev.type == "cuda":
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    back, n_owned_local = ops.owner_sum(recv_fp.to(fp.device), recv_df.to(fp.device))
    n_owned = torch.tensor([int(n_owned_local)], dtype=torch.int64, device=cdev)
    t2 = time.perf_counter()
    ret = torch.empty(V, dtype=torch.int64, device=cdev)
    dist.all_to_all_single(ret, back.to(cdev).contiguous(), cs, rc, group=group)
    dist.all_reduce(n_owned, group=group)
    out = ops.unpack(ret.to(fp.device), pos)
    if fp.device.type == "cuda":
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    if timings is not None:
        timings.update(exchange_ms=(t1 - t0) * 1e3, dedup_ms=(t2 - t1) * 1e3, return_ms=(t3 - t2) * 1e3,
                       local_terms=V, owned_rows=nrecv, owned_terms=int(n_owned_local),
                       global_terms=int(n_owned.item()), bytes_out_per_rank=24 * V, bytes_back_per_rank=8 * V)
    return out


def global_df_index(ix, group=None, timings=None):
    """All-reduced df per LOCAL term of a libsme shard index, as a CUDA int64 tensor
    ready for sme_index_reweight: shards agree on terms through their 128-bit device
    fingerprints (sme_index_term_fingerprints), exchanged by owner (df_exchange) --
    no term strings on the host, and the shard's df comes from its device offsets
    (never through host memory).

    The fingerprints and the offsets copy run on libsme's own stream of the index's
    context (sme_index_term_fingerprints / sme_memcpy with a null stream), which is
    synchronized before torch reads them, so no stream handle crosses between
    torch's HIP runtime and libsme's.  `timings` (a dict) receives the wall ms of
    the fingerprint, exchange, dedup and return steps."""
    import time
    sme = importlib.import_module(__package__)
    dev = _dev(group)
    V = int(ix.V)
    t0 = time.perf_counter()
    fp = torch.empty((max(V, 1), 2), dtype=torch.int64, device="cuda")
    offs = torch.empty(V + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # the tensors exist before libsme's stream writes them
    if V:
        ix.term_fingerprints(fp.data_ptr(), None)  # every row written, libsme's stream (synchronized)
        o_ptr, _, _ = ix.device_arrays()
        sme.memcpy(offs.data_ptr(), o_ptr, 8 * (V + 1), None)
    else:
        offs.zero_()
    df = offs[1:] - offs[:-1]
    fp = fp[:V]
    t1 = time.perf_counter()
    out = df_exchange(fp, df, group, timings, ops=DeviceDfOps(ix.ctx))
    out = out.to("cuda").contiguous()
    torch.cuda.current_stream().synchronize()
    if timings is not None:
        timings.update(fingerprints_ms=(t1 - t0) * 1e3)
    return out


def reference_partitions(ix, group=None, timings=None):
    """The reference's R part files from doc shards (last row): this
    shard's terms and reduce-order postings go, per term partition p
    ((Arrays.hashCode & MAX) % R, TermDF.java:79-81), to rank p % W in one
    all_to_all of self-describing blobs (sme_index_pack_pieces); every rank
    merges what it received per term exactly as the single reducer would
    (MyReducer.reduce, TermKGramDocIndexer.java:189-211: docno sort, equal
    docnos -- a docid duplicated across shards -- summed, stable tf-desc sort;
    sme_merge_pieces).  Returns (records-only Index, the partitions this rank
    owns): read them with Index.partition_records(p)."""
    import time
    sme = importlib.import_module(__package__)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = _dev(group)
    t0 = time.perf_counter()
    sizes = ix.pack_pieces(world)
    send = torch.empty(max(sum(sizes), 16), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ix.pack_pieces(world, send.data_ptr())
    t1 = time.perf_counter()
    cnt = torch.tensor(sizes, dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rsizes = rcnt.tolist()
    recv = torch.empty(max(sum(rsizes), 16), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv[:sum(rsizes)], send[:sum(sizes)].to(dev), rsizes, sizes, group=group)
    recv = recv.to("cuda")
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    merged = ix.ctx.merge_pieces(recv.data_ptr(), rsizes)
    del send, recv
    t3 = time.perf_counter()
    R = ix.ctx.num_partitions
    if timings is not None:
        timings.update(pack_ms=(t1 - t0) * 1e3, exchange_ms=(t2 - t1) * 1e3, merge_ms=(t3 - t2) * 1e3,
                       bytes_out=int(sum(sizes)), bytes_in=int(sum(rsizes)))
    return merged, [p for p in range(R) if p % world == rank]


def docno_duplicates(docnos, group=None, ops=None):
    """Number of distinct docnos that more than one shard holds (docnos: this
    shard's record docnos, an int64 tensor).  Disjoint [min, max] ranges answer
    0 at once (all_gather of 16 B); otherwise every (docno, rank) row goes to the
    docno's owner rank (grouped by `ops.pack`, one all_to_all) and each owner
    counts the docnos that arrive from two or more ranks (`ops.count_shared`),
    summed over the owners.  A docid duplicated across shards is one posting
    with summed tf in the reference's single reducer
    (TermKGramDocIndexer.java:202-210); per-shard scoring would keep two.
    `ops`: DeviceDfOps (libsme, the default) or the CPU tests' restatement."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    cdev = _dev(group)
    n = int(docnos.shape[0])
    big = 1 << 62
    mm = torch.tensor([int(docnos.min()) if n else big, int(docnos.max()) if n else -big], dtype=torch.int64, device=cdev)
    alls = [torch.empty_like(mm) for _ in range(world)]
    dist.all_gather(alls, mm, group=group)
    rng = sorted((int(a[0]), int(a[1])) for a in alls if int(a[0]) <= int(a[1]))
    if all(rng[i][1] < rng[i + 1][0] for i in range(len(rng) - 1)):
        return 0
    if ops is None:
        ops = DeviceDfOps()
    # keys: docnos as zero-extended 32-bit values (never the table's empty marker)
    dd = docnos.to(torch.int64) & 0xFFFFFFFF
    rows = torch.stack([dd, torch.full_like(dd, rank)], 1).contiguous()
    if hasattr(ops, "ctx"):
        rows = rows.to("cuda")
    send, _, _, cs = ops.pack(rows, torch.zeros_like(dd).to(rows.device), world)
    counts = torch.tensor(cs, dtype=torch.int64, device=cdev)
    rcounts = torch.empty_like(counts)
    dist.all_to_all_single(rcounts, counts, group=group)
    rc = rcounts.tolist()
    recv = torch.empty((int(sum(rc)), 2), dtype=torch.int64, device=cdev)
    dist.all_to_all_single(recv.view(-1), send.to(cdev).contiguous().view(-1), [2 * c for c in rc],
                           [2 * c for c in cs], group=group)
    dup = torch.tensor([int(ops.count_shared(recv))], dtype=torch.int64, device=cdev)
    dist.all_reduce(dup, group=group)
    return int(dup.item())


def shard_docno_duplicates(ix, group=None):
    """docno_duplicates over a libsme shard index's record docnos."""
    sme = importlib.import_module(__package__)
    ptr, n = ix.record_docnos_ptr()
    d = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    if n:
        sme.memcpy(d.data_ptr(), ptr, 4 * n, None)
    return docno_duplicates(d[:n].to(torch.int64).to(_dev(group)), group)


def owner_bounds(nq, world):
    """Query-owner split: rank r merges queries [b[r], b[r+1])."""
    return [nq * r // world for r in range(world + 1)]


def _merge_rows(s, d, k, t=None, ops=None):
    """rows of candidate (score, docno[, tie]) lists -> the best k per row, (score
    desc, tie asc, docno asc); docno -1 pads.  The tie word (sme_query_topk_tie)
    is 0 under SME_TIE_DOCNO and the first-encounter rank under SME_TIE_REFERENCE,
    a property of the document and the query alone, so shards merge into the
    single index's order.  libsme's merge kernel (sme_topk_merge_rows) unless
    `ops` restates it (CPU tests)."""
    return (ops if ops is not None else DeviceDfOps()).merge_rows(s, d, k, t)


def merge_topk_owner(docno, score, k, group=None, tie=None, ops=None):
    """Query-owner merge: docno int32 [Q, k] (-1 pads), score float64
    [Q, k] of this shard -> (q0, q1, docno [q1-q0, k], score [q1-q0, k]), the global
    top-k of the queries this rank owns.  One all_to_all moves every shard's lists
    of query q to q's owner (Q x k x 12 B per rank in all), and each rank sorts only
    its Q/W queries' W x k candidates."""
    world, r = dist.get_world_size(group), dist.get_rank(group)
    nq = docno.shape[0]
    b = owner_bounds(nq, world)
    my = b[r + 1] - b[r]
    ins = [(b[i + 1] - b[i]) * k for i in range(world)]
    rs = torch.empty(world * my * k, dtype=score.dtype, device=score.device)
    rd = torch.empty(world * my * k, dtype=docno.dtype, device=docno.device)
    dist.all_to_all_single(rs, score.contiguous().reshape(-1), [my * k] * world, ins, group=group)
    dist.all_to_all_single(rd, docno.contiguous().reshape(-1), [my * k] * world, ins, group=group)
    s = rs.reshape(world, my, k).permute(1, 0, 2).reshape(my, world * k)
    d = rd.reshape(world, my, k).permute(1, 0, 2).reshape(my, world * k)
    t = None
    if tie is not None:  # uint32 words travel as int64 (collectives have no uint32)
        rt = torch.empty(world * my * k, dtype=torch.int64, device=docno.device)
        dist.all_to_all_single(rt, tie.to(torch.int64).contiguous().reshape(-1), [my * k] * world, ins, group=group)
        t = rt.reshape(world, my, k).permute(1, 0, 2).reshape(my, world * k)
    md, ms, _ = _merge_rows(s, d, k, t, ops)
    return b[r], b[r + 1], md, ms


def merge_topk(docno, score, k, group=None, tie=None, ops=None):
    """Global (docno, score) [Q, k] on every rank: the query-owner merge, then an
    all_gather of the merged slices (Q x k x 12 B, not W x Q x k)."""
    world = dist.get_world_size(group)
    nq = docno.shape[0]
    q0, q1, md, ms = merge_topk_owner(docno, score, k, group, tie, ops)
    b = owner_bounds(nq, world)
    m = max(b[i + 1] - b[i] for i in range(world))
    pd = torch.full((m, k), -1, dtype=md.dtype, device=md.device)
    ps = torch.zeros((m, k), dtype=ms.dtype, device=ms.device)
    pd[:q1 - q0] = md
    ps[:q1 - q0] = ms
    gd = [torch.empty_like(pd) for _ in range(world)]
    gs = [torch.empty_like(ps) for _ in range(world)]
    dist.all_gather(gd, pd, group=group)
    dist.all_gather(gs, ps, group=group)
    out_d = torch.cat([x[:b[i + 1] - b[i]] for i, x in enumerate(gd)], 0)
    out_s = torch.cat([x[:b[i + 1] - b[i]] for i, x in enumerate(gs)], 0)
    return out_d, out_s
