"""The N>1 path on CPU: world_size-2 gloo over 127.0.0.1.

Each rank indexes its own Hadoop-style split (the CPU oracle stands in for the
per-GPU index: same records, postings and doc counters as libsme's shard index),
then runs the collectives of dist.py -- global N, global vocabulary and df, and the
per-shard top-k merge -- and must reproduce the single-index result of the whole
corpus bit for bit (docids are unique across shards)."""
import importlib
import math
import os
import socket

import numpy as np
import oracle_lib as O
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

PKG = "simple-mapreduce-search-engine-information-retrieval-_amd"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_scores(terms_q, local, N, df_of, idf_mode, k):
    """rank() over this shard's postings with GLOBAL N / df: per document, fp64
    adds of (1 + ln tf) * log10(N / df) in query-token order (oracle arithmetic)."""
    acc = {}
    for t in terms_q:
        if t not in local:
            continue
        posts = local[t]
        df = 1 if idf_mode == 0 else df_of[t]
        idf = math.log10(float(N // df))
        for d, tf in posts:
            w = (1.0 + math.log(float(tf))) * idf
            acc[d] = acc[d] + w if d in acc else w
    top = sorted(acc.items(), key=lambda x: (-x[1], x[0]))[:k]
    dn = np.full(k, -1, np.int32)
    sc = np.zeros(k, np.float64)
    for i, (d, s) in enumerate(top):
        dn[i], sc[i] = d, s
    return dn, sc


def _worker(rank, world, port, idf_mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D = importlib.import_module(PKG + ".dist")
        synth = importlib.import_module(PKG + ".synth")
        n = 90
        corpus = synth.gen_corpus(n, V=700, seed=5, len_lo=20, len_hi=70)
        mapping = synth.mapping_bytes(n)
        cuts = D.cuts_from_starts([o for o, _ in O.split_records(corpus)], len(corpus), world)
        shard = corpus[cuts[rank]:cuts[rank + 1]]
        ix = O.OracleIndex(shard, mapping, 1, 1)
        terms = [t for t in ix.terms() if t[0] != (" ",)]
        local_terms = [t[0][0] for t in terms]
        local = {t[0][0]: t[3] for t in terms}
        N = D.global_count(ix.N)
        assert N == n
        allt, l2g = D.global_vocab(local_terms)
        gdf = D.global_df([len(t[3]) for t in terms], l2g, len(allt)).numpy()
        df_of = dict(zip(local_terms, gdf.tolist()))
        full = O.OracleIndex(corpus, mapping, 1, 1)
        fterms = [t for t in full.terms() if t[0] != (" ",)]
        assert [t[0][0].encode("utf-16-be", "surrogatepass") for t in fterms] == allt  # same global order
        fdf = {t[0][0]: len(t[3]) for t in fterms}
        assert all(df_of[t] == fdf[t] for t in local_terms)
        rng = np.random.default_rng(3)
        names = [t[0][0] for t in fterms]
        k = 10
        queries = [[names[i] for i in rng.integers(0, len(names), rng.integers(1, 6))] for _ in range(40)]
        dn = np.zeros((len(queries), k), np.int32)
        sc = np.zeros((len(queries), k), np.float64)
        for q, tq in enumerate(queries):
            dn[q], sc[q] = _shard_scores(tq, local, N, df_of, idf_mode, k)
        md, ms = D.merge_topk(torch.from_numpy(dn), torch.from_numpy(sc), k, ops=HostDfOps())
        q0, q1, od, osc = D.merge_topk_owner(torch.from_numpy(dn), torch.from_numpy(sc), k, ops=HostDfOps())
        assert (q0, q1) == tuple(D.owner_bounds(len(queries), world)[rank:rank + 2])
        assert torch.equal(od, md[q0:q1]) and torch.equal(osc, ms[q0:q1])  # the owner's slice
        for q, tq in enumerate(queries):
            rd, rs = full.query(tq, k, idf_mode, 0)
            assert md[q, :len(rd)].tolist() == rd, (q, tq)
            assert ms[q, :len(rs)].numpy().tolist() == rs, q  # bit-exact
            assert (md[q, len(rd):] == -1).all()
        open(os.path.join(out_dir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("where", ["host", pytest.param("device", marks=pytest.mark.gpu)])
def test_merge_rows_tie_words(where):
    """_merge_rows orders by (score desc, tie asc, docno asc): the tie word is the
    reference order's first-encounter rank (sme_query_topk_tie), pads last --
    the libsme kernel (sme_topk_merge_rows, the product) and the CPU tests'
    restatement alike."""
    s = torch.tensor([[2.0, 5.0, 5.0, 5.0, 1.0, 0.0]], dtype=torch.float64)
    d = torch.tensor([[4, 9, 3, 7, 8, -1]], dtype=torch.int32)
    t = torch.tensor([[0, (1 << 24) | 5, (2 << 24) | 1, (1 << 24) | 2, 0, 0xFFFFFFFF]], dtype=torch.int64)
    D = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.dist")
    ops = HostDfOps() if where == "host" else None
    md, ms, mt = D._merge_rows(s, d, 6, t, ops)
    assert md.tolist() == [[7, 9, 3, 4, 8, -1]]
    assert ms.tolist() == [[5.0, 5.0, 5.0, 2.0, 1.0, 0.0]]
    assert mt.tolist() == [[(1 << 24) | 2, (1 << 24) | 5, (2 << 24) | 1, 0, 0, 0xFFFFFFFF]]
    md0, _, _ = D._merge_rows(s, d, 6, None, ops)  # no tie words: docno order among equal scores
    assert md0.tolist() == [[3, 7, 9, 4, 8, -1]]
    neg = torch.tensor([[-5, -2, 3]], dtype=torch.int32)  # unmapped docids (T14, <= -2) sort as signed ints
    mn, _, _ = D._merge_rows(torch.tensor([[1.0, 1.0, 1.0]], dtype=torch.float64), neg, 3, None, ops)
    assert mn.tolist() == [[-5, -2, 3]]
    # k below the candidates per row, and more candidates than one LDS chunk
    # (k = 600: chunks of 1448 in the kernel), rows of random order
    g = np.random.default_rng(4)
    for rows, m, k in ((7, 40, 10), (3, 5000, 600), (2, 3, 5)):
        sc = torch.from_numpy(g.integers(0, 6, size=(rows, m)).astype(np.float64))
        dn = torch.from_numpy(g.permutation(rows * m).reshape(rows, m).astype(np.int32) - 50)
        dn[dn == -1] = -1000000  # (-1 is the pad docno)
        dn[:, ::9] = -1
        tw = torch.from_numpy(g.integers(0, 1 << 32, size=(rows, m), dtype=np.int64))
        for tt in (None, tw):
            a = D._merge_rows(sc, dn, k, tt, ops)
            b = HostDfOps().merge_rows(sc, dn, k, tt)
            assert all(torch.equal(x, y) for x, y in zip(a, b)), (rows, m, k, tt is None)


@pytest.mark.parametrize("idf_mode,world", [(0, 2), (1, 2), (0, 3)])
def test_two_shards_gloo(tmp_path, idf_mode, world):
    mp.spawn(_worker, args=(world, _free_port(), idf_mode, str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / ("ok%d" % r)).exists() for r in range(world))


def test_cuts_own_every_record_and_quirks():
    """The cut rule over one reader pass: every record in exactly one shard, and
    no shard starts at a '<<DOC>' or a nested <DOC> (XMLInputFormat.java:173-198)."""
    import common
    D = importlib.import_module(PKG + ".dist")
    synth = importlib.import_module(PKG + ".synth")
    for corpus in (synth.gen_corpus(50, V=300, seed=2, len_lo=5, len_hi=40), common.fuzz_corpus(9, 60)[0],
                   b"<DOC> a <DOC> b </DOC> <<DOC> c </DOC> <DOC> d </DOC>" * 7):
        recs = O.split_records(corpus)
        starts = [o for o, _ in recs]
        for w in (1, 2, 3, 8, 13):
            cuts = D.cuts_from_starts(starts, len(corpus), w)
            assert cuts[0] == 0 and cuts[-1] == len(corpus) and cuts == sorted(cuts)
            got = []
            for a, b in zip(cuts, cuts[1:]):
                got += [(a + o, ln) for o, ln in O.split_records(corpus[a:b])]
            assert got == recs, w


class HostDfOps:
    """numpy restatement of dist.DeviceDfOps' three local steps (sme_dfx.hip),
    so the CPU tests drive dist.df_exchange's collectives without a GPU: owner =
    fingerprint word 0 as u64 mod world, rows grouped by owner; per received row
    the df summed over its 128-bit fingerprint; the return gather."""

    def pack(self, fp, df, world):
        f = fp.numpy()
        owner = (f[:, 0].view(np.uint64) % np.uint64(world)).astype(np.int64)
        order = np.argsort(owner, kind="stable")
        pos = np.empty(len(order), np.int64)
        pos[order] = np.arange(len(order))
        counts = np.bincount(owner, minlength=world).tolist()
        return (torch.from_numpy(f[order].copy()), torch.from_numpy(df.numpy()[order].copy()),
                torch.from_numpy(pos), counts)

    def owner_sum(self, fp, df):
        f = fp.numpy()
        if len(f) == 0:
            return torch.zeros(0, dtype=torch.int64), 0
        _, inv = np.unique(f, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        sums = np.zeros(int(inv.max()) + 1, np.int64)
        np.add.at(sums, inv, df.numpy())
        return torch.from_numpy(sums[inv]), len(sums)

    def unpack(self, ret, pos):
        return torch.from_numpy(ret.numpy()[pos.numpy()].copy())

    def merge_rows(self, s, d, k, t=None):
        """torch restatement of sme_topk_merge_rows: (score desc, tie asc, docno
        asc), docno -1 pads (score 0, tie ~0); rows of fewer than k candidates padded."""
        if s.shape[1] < k:  # pad columns: docno -1
            e = k - s.shape[1]
            s = torch.cat([s, torch.zeros((s.shape[0], e), dtype=s.dtype)], 1)
            d = torch.cat([d.to(torch.int64), torch.full((d.shape[0], e), -1, dtype=torch.int64)], 1)
            if t is not None:
                t = torch.cat([t.to(torch.int64), torch.zeros((t.shape[0], e), dtype=torch.int64)], 1)
        d = d.to(torch.int64)
        valid = d != -1
        s = torch.where(valid, s, torch.full_like(s, -float("inf")))
        # u64 key tie << 32 | (docno + 2^31), its sign bit flipped so int64 order is
        # the unsigned order (tie words reach 2^32 - 1); pads last
        key = d + (1 << 31)
        if t is not None:
            key = key | ((t.to(torch.int64) & 0xFFFFFFFF) << 32)
        flip = torch.tensor(-(1 << 63), dtype=torch.int64)
        key = torch.bitwise_xor(key, flip)
        key = torch.where(valid, key, torch.full_like(key, (1 << 63) - 1))
        i1 = torch.argsort(key, dim=1, stable=True)
        s1, k1 = torch.gather(s, 1, i1), torch.gather(key, 1, i1)
        i2 = torch.argsort(-s1, dim=1, stable=True)[:, :k]
        out_k, out_s = torch.gather(k1, 1, i2), torch.gather(s1, 1, i2)
        pad = out_k == (1 << 63) - 1
        out_k = torch.bitwise_xor(out_k, flip)
        out_d = (out_k & 0xFFFFFFFF) - (1 << 31)
        out_t = (out_k >> 32) & 0xFFFFFFFF
        return (torch.where(pad, torch.full_like(out_d, -1), out_d).to(torch.int32),
                torch.where(pad, torch.zeros_like(out_s), out_s),
                torch.where(pad, torch.full_like(out_t, 0xFFFFFFFF), out_t))

    def count_shared(self, rows):
        """numpy restatement of sme_count_shared_keys: keys arriving from >= 2 ranks."""
        r = rows.numpy()
        if len(r) == 0:
            return 0
        pairs = np.unique(r, axis=0)  # distinct (key, source)
        _, c = np.unique(pairs[:, 0], return_counts=True)
        return int((c > 1).sum())


def _dfx_worker(rank, world, port, out_dir, collide):
    """df_exchange over random shard vocabularies: every local term's result must be
    the df summed over every shard holding its fingerprint."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D = importlib.import_module(PKG + ".dist")
        g = np.random.default_rng(11)
        universe = g.integers(-(1 << 62), 1 << 62, size=(3000, 2), dtype=np.int64)
        if collide:  # equal first words, different second words: the exact row-wise path
            universe[1::7, 0] = universe[0::7, 0][:universe[1::7].shape[0]]
        shards = []
        for r in range(world):
            gr = np.random.default_rng(100 + r)
            ids = np.sort(gr.choice(3000, size=int(gr.integers(0, 1200)), replace=False))
            shards.append((ids, gr.integers(1, 50, size=ids.shape[0]).astype(np.int64)))
        ids, df = shards[rank]
        t = {}
        out = D.df_exchange(torch.from_numpy(universe[ids].copy()), torch.from_numpy(df), timings=t,
                            ops=HostDfOps()).numpy()
        want = {}
        for i2, d2 in shards:
            for i, d in zip(i2.tolist(), d2.tolist()):
                key = tuple(universe[i].tolist())
                want[key] = want.get(key, 0) + d
        exp = np.array([want[tuple(universe[i].tolist())] for i in ids.tolist()], np.int64)
        assert np.array_equal(out, exp)
        assert t["global_terms"] == len(want)
        open(os.path.join(out_dir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,collide", [(2, False), (3, True), (4, False)])
def test_df_exchange_owner_gloo(tmp_path, world, collide):
    """The owner-partitioned df exchange (all_to_all to the fingerprint's owner,
    dedup there, all_to_all back) equals the brute-force sum over shards."""
    mp.spawn(_dfx_worker, args=(world, _free_port(), str(tmp_path), collide), nprocs=world, join=True)
    assert all((tmp_path / ("ok%d" % r)).exists() for r in range(world))


def _dup_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D = importlib.import_module(PKG + ".dist")
        ops = HostDfOps()
        # disjoint ranges: 0 without the exchange
        d = torch.arange(100 * rank, 100 * rank + 100, dtype=torch.int64)
        assert D.docno_duplicates(d, ops=ops) == 0
        # overlapping ranges, no duplicates (interleaved), one shard empty
        d = torch.arange(rank, 600, world, dtype=torch.int64) if rank != 1 else torch.zeros(0, dtype=torch.int64)
        assert D.docno_duplicates(d, ops=ops) == 0
        # duplicates: 7 and 42 in every shard, -3 (an unmapped docid) in shards 0 and 1,
        # 99 twice inside shard 0 only (not a cross-shard duplicate)
        extra = [7, 42] + ([-3] if rank < 2 else []) + ([99, 99] if rank == 0 else [])
        d = torch.tensor(extra + list(range(1000 + 10 * rank, 1010 + 10 * rank)), dtype=torch.int64)
        assert D.docno_duplicates(d, ops=ops) == (3 if world >= 2 else 0)
        open(os.path.join(out_dir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_docno_duplicates_gloo(tmp_path, world):
    """Docnos held by more than one shard (a docid duplicated across doc shards):
    counted exactly, duplicates inside one shard excluded."""
    mp.spawn(_dup_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / ("ok%d" % r)).exists() for r in range(world))
