"""One rank of the c4 multi-rank test (tests/test_dist_gpu.py::test_c4_four_shards):
a fresh process that touches the GPU only after it starts.

The corpus is 60,000 docs of the BASELINE c4 distribution (V_w = 2^22, 200-360
tokens, Zipf s = 1, seed 44), generated in HBM by sme_synth_corpus.  Rank r builds
the records a Hadoop split [n r/W, n (r+1)/W) owns (cuts from sme_split_points,
XMLInputFormat.java:110-143,195) with libsme; N and P are all-reduced, df goes
through the fingerprint exchange (dist.global_df_index) into sme_index_reweight,
and every rank scores the golden queries on its shard.  The query-owner merge
(dist.merge_topk_owner) must give, for the queries this rank owns, exactly the
docnos and fp64 score bits the single-index CPU oracle produced for the whole
corpus (tests/golden/scale_c4multi.json, tools/gen_scale_golden.py) -- the
reference's one global reduce (TermKGramDocIndexer.java:175-183,246).  The
shards' reference_partitions (term-partition all_to_all + per-term reducer merge)
must reproduce the oracle's R = 10 part files for the same 4 map tasks
(scale_c4multi.json split_parts, tools/gen_scale_golden.py c4multi-parts), and
the K = 3 job's part files likewise (split_parts_k3, c4multi-parts-k3).
usage: dist_c4_worker.py RANK WORLD PORT OUT_DIR"""
import importlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PKG = "simple-mapreduce-search-engine-information-retrieval-_amd"


def check_group(ix, D, group, k_out, world, rank):
    names = [q[0] for q in group["q"]]
    flat = sorted({t for tl in names for t in tl})
    ids = dict(zip(flat, ix.lookup(flat).tolist()))  # -1: not in this shard (skipped like an unknown term)
    terms = np.array([ids[t] for tl in names for t in tl], np.int32)
    qoff = np.zeros(len(names) + 1, np.int64)
    qoff[1:] = np.cumsum([len(tl) for tl in names])
    k = group["k"]
    dn, sc = ix.query_topk(terms, qoff, k)
    q0, q1, md, ms = D.merge_topk_owner(torch.from_numpy(dn), torch.from_numpy(sc), k)
    assert (q0, q1) == tuple(D.owner_bounds(len(names), world)[rank:rank + 2])
    for i, q in enumerate(range(q0, q1)):
        tl, d, s = group["q"][q]
        assert md[i, :len(d)].tolist() == d, (group["kind"], q, tl)
        assert [float(x).hex() for x in ms[i, :len(d)].tolist()] == s, (group["kind"], q)
        assert (md[i, len(d):] == -1).all()
    k_out.append(q1 - q0)


def main():
    rank, world, port, out_dir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sme = importlib.import_module(PKG)
        D = importlib.import_module(PKG + ".dist")
        synth = importlib.import_module(PKG + ".synth")
        torch.cuda.set_device(0)
        g = json.load(open(os.path.join(HERE, "golden", "scale_c4multi.json")))
        c = g["config"]
        corpus = sme.DeviceCorpus(c["n"], V=c["V"], seed=c["seed"], len_lo=c["lo"], len_hi=c["hi"])
        mapping = synth.mapping_bytes(c["n"])
        timing = {"rank": rank}
        checked = []
        sp = g["split_parts"]  # the oracle's R = 10 part files for these 4 map tasks
        for idf_mode in (0, 1):
            ctx = sme.Context(1, sp["R"], idf_mode)
            cuts = D.split_points(corpus, world, ctx)
            ctx.load_docno_mapping(mapping)
            ix = ctx.build_device(corpus.ptr + cuts[rank], cuts[rank + 1] - cuts[rank])
            N = D.global_count(ix.N)
            assert N == g["N"]
            assert D.global_count(ix.P) == g["P"]  # postings partition over the shards
            t = {}
            t0 = time.perf_counter()
            gdf = D.global_df_index(ix, timings=t)
            t["total_ms"] = (time.perf_counter() - t0) * 1e3
            assert t["global_terms"] == g["V"]  # the union of the shard vocabularies
            timing["df_exchange_mode%d" % idf_mode] = t
            if idf_mode == 0:
                # reference-layout output: the shards' postings merged per term on
                # the partition owners equal the single reducer's R part files
                assert cuts == sp["cuts"] and world == sp["world"]
                assert D.shard_docno_duplicates(ix) == 0
                tp = {}
                t0 = time.perf_counter()
                merged, owned = D.reference_partitions(ix, timings=tp)
                tp["total_ms"] = (time.perf_counter() - t0) * 1e3
                import common
                for p in owned:
                    assert common.canon_digest(merged.partition_records(p)) == sp["parts"][p], p
                timing["reference_partitions"] = tp
                merged.close()
            ix.reweight(N, gdf.data_ptr() if idf_mode == 1 else None)
            for group in g["queries"]:
                if group["idf_mode"] == idf_mode:
                    check_group(ix, D, group, checked, world, rank)
            ix.close()
            ctx.close()
        # the K = 3 job (TermKGramDocIndexer.java:138-159) over the same 4 map
        # tasks: the shards' 3-gram postings merged on the partition owners equal
        # the oracle's R part files (scale_c4multi.json split_parts_k3)
        sp3 = g.get("split_parts_k3")
        if sp3 is not None:
            import common
            ctx = sme.Context(3, sp3["R"], 0)
            cuts = D.split_points(corpus, world, ctx)
            assert cuts == sp3["cuts"]
            ctx.load_docno_mapping(mapping)
            ix = ctx.build_device(corpus.ptr + cuts[rank], cuts[rank + 1] - cuts[rank])
            merged, owned = D.reference_partitions(ix)
            for p in owned:
                assert common.canon_digest(merged.partition_records(p)) == sp3["parts"][p], ("K=3", p)
            timing["k3_partitions_checked"] = len(owned)
            merged.close()
            ix.close()
            ctx.close()
        timing["queries_checked"] = int(sum(checked))
        json.dump(timing, open(os.path.join(out_dir, "timing%d.json" % rank), "w"))
        open(os.path.join(out_dir, "ok%d" % rank), "w").write("ok")
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
