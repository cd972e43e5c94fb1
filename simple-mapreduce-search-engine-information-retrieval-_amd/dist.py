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
                   fingerprints (all_gather + torch.unique, no host strings)
  merge_topk       per-shard top-k -> global top-k, (score desc, docno asc)
                   (all_gather of Q x k x (4 + 8) B)

Exactness: with docids unique across shards (every synthetic corpus), the sharded
result equals the single-index result bit for bit: a document's score only uses its
own postings, and N / df are the global ones.  A docid duplicated ACROSS shards would
be merged by the reference's single reducer but stays two postings here.
"""
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


def global_df_index(ix, group=None):
    """All-reduced df per LOCAL term of a libsme shard index, as a CUDA int64 tensor
    ready for sme_index_reweight: shards agree on terms through their 128-bit device
    fingerprints (sme_index_term_fingerprints), gathered and deduplicated with
    torch.unique on the collective's device -- no term strings on the host."""
    dev = _dev(group)
    world = dist.get_world_size(group)
    V = int(ix.V)
    fp = torch.zeros((max(V, 1), 2), dtype=torch.int64, device="cuda")
    if V:
        ix.term_fingerprints(fp.data_ptr())
    fp = fp[:V].to(dev)
    n = torch.tensor([V], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    pad = torch.zeros((m, 2), dtype=torch.int64, device=dev)
    pad[:V] = fp
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    allfp = torch.cat([o[:c] for o, c in zip(outs, ns)], 0)
    uniq, inv = torch.unique(allfp, dim=0, return_inverse=True)
    r = dist.get_rank(group)
    mine = inv[sum(ns[:r]):sum(ns[:r]) + V]
    df = torch.from_numpy(np.diff(ix.offsets())).to(dev)
    g = torch.zeros(uniq.shape[0], dtype=torch.int64, device=dev)
    if V:
        g.index_add_(0, mine, df)
    dist.all_reduce(g, group=group)
    return g[mine].to("cuda").contiguous()


def merge_topk(docno, score, k, group=None):
    """docno int32 [Q, k] (-1 pads), score float64 [Q, k] torch tensors of this
    shard -> global (docno, score) [Q, k]: score desc, docno asc."""
    world = dist.get_world_size(group)
    gs = [torch.empty_like(score) for _ in range(world)]
    gd = [torch.empty_like(docno) for _ in range(world)]
    dist.all_gather(gs, score, group=group)
    dist.all_gather(gd, docno, group=group)
    s = torch.cat(gs, 1)
    d = torch.cat(gd, 1).to(torch.int64)
    valid = d >= 0
    s = torch.where(valid, s, torch.full_like(s, -float("inf")))
    d = torch.where(valid, d, torch.full_like(d, 1 << 40))
    # (score desc, docno asc): stable sort by docno, then stable sort by -score
    i1 = torch.argsort(d, dim=1, stable=True)
    s1, d1 = torch.gather(s, 1, i1), torch.gather(d, 1, i1)
    i2 = torch.argsort(-s1, dim=1, stable=True)[:, :k]
    out_d, out_s = torch.gather(d1, 1, i2), torch.gather(s1, 1, i2)
    pad = out_d >= (1 << 40)
    return (torch.where(pad, torch.full_like(out_d, -1), out_d).to(torch.int32),
            torch.where(pad, torch.zeros_like(out_s), out_s))
