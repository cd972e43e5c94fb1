"""df exchange (dist.global_df_index) at c4 vocabulary size, on one GPU.

c4 is 50 M docs doc-sharded over 8 GPUs: one shard is 6.25 M docs of
the c4 distribution (V_w = 2^22, 200-360 tokens, Zipf s = 1, seed 44) with about
6.8 M local terms (the words it holds + its 6.25 M docid terms).  This builds
such a shard in HBM, runs the real global_df_index on a world-1 RCCL group
(fingerprints + offsets, owner pack, all_to_all, owner sums, return), and then
times the part that grows with the world on the device: the owner's sums
(sme_df_owner_sum, a fingerprint hash table) over the
8-shard set, emulated from this shard's own fingerprints (rows with df > 1 --
the words -- shared by all 8 shards, the df = 1 rows -- docid terms and rare
words -- made shard-private by xoring the shard number into the fingerprint):
dist.df_exchange sends each row to the owner rank of its fingerprint, so one
owner deduplicates and sums 1/8 of all shards' rows.  The all_to_alls need 8
GPUs; their volume is reported.  Writes gpurun_out/dfx_c4.json (kept as profiles/r04_dfx_c4.json).
    python tools/dfx_c4.py [--docs 6250000] [--world 8]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "simple-mapreduce-search-engine-information-retrieval-_amd"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--docs", type=int, default=6_250_000)
    p.add_argument("--world", type=int, default=8)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    sme = importlib.import_module(PKG)
    D = importlib.import_module(PKG + ".dist")
    synth = importlib.import_module(PKG + ".synth")
    t0 = time.perf_counter()
    corpus = sme.DeviceCorpus(a.docs, V=1 << 22, seed=44, len_lo=200, len_hi=360)
    ctx = sme.Context(1, 1, 1)
    ctx.load_docno_mapping(synth.mapping_bytes(a.docs))
    ix = ctx.build_device(corpus.ptr, corpus.nbytes)
    torch.cuda.synchronize()
    print("shard built: N=%d V=%d P=%d (%.1f s)" % (ix.N, ix.V, ix.P, time.perf_counter() - t0), flush=True)
    out = {"shard_docs": a.docs, "text_bytes": int(corpus.nbytes), "local_terms": int(ix.V), "postings": int(ix.P)}
    runs = []
    for _ in range(3):
        t = {}
        ts = time.perf_counter()
        gdf = D.global_df_index(ix, timings=t)
        t["total_ms"] = (time.perf_counter() - ts) * 1e3
        runs.append(t)
    out["world1_global_df_index"] = runs[-1]
    # emulated world-W owner exchange (dist.df_exchange): rank r receives, from
    # each of the W shards, the rows whose fingerprint's first word is r mod W;
    # it deduplicates and sums only those, then returns each sender its rows
    V = int(ix.V)
    fp = torch.empty((V, 2), dtype=torch.int64, device="cuda")
    ix.term_fingerprints(fp.data_ptr(), torch.cuda.current_stream().cuda_stream)
    o_ptr, _, _ = ix.device_arrays()
    offs = torch.empty(V + 1, dtype=torch.int64, device="cuda")
    sme.memcpy(offs.data_ptr(), o_ptr, 8 * (V + 1), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    df = offs[1:] - offs[:-1]
    private = df == 1
    parts, dfs = [], []
    for s in range(a.world):
        f = fp.clone()
        f[private, 1] ^= (s + 1) << 40
        f[private, 0] ^= (s + 1) << 40  # shard-private terms: owners spread like any term's
        parts.append(f)
        dfs.append(df)
    allfp = torch.cat(parts, 0)
    alldf = torch.cat(dfs, 0)
    del parts, dfs
    # the owner of a row: word 0 as u64 mod W (sme_df_owner_pack's rule)
    w0 = allfp[:, 0]
    u_mod = (torch.remainder(w0, a.world) + torch.where(w0 < 0, (1 << 64) % a.world, 0)) % a.world
    mine = u_mod == 0
    recv_fp = allfp[mine].contiguous()
    recv_df = alldf[mine].contiguous()
    del allfp, alldf, w0, u_mod
    ops = D.DeviceDfOps(ctx)
    send_t, owner_t = [], []
    for _ in range(3):
        torch.cuda.synchronize()
        ts = time.perf_counter()
        send_fp, send_df, pos, counts = ops.pack(fp, df, a.world)  # libsme sme_df_owner_pack
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        back, n_owned = ops.owner_sum(recv_fp, recv_df)  # libsme sme_df_owner_sum
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        send_t.append((t1 - ts) * 1e3)
        owner_t.append((t2 - t1) * 1e3)
    out["emulated_world"] = a.world
    out["emulated_rows_received_by_owner"] = int(recv_fp.shape[0])
    out["emulated_terms_owned"] = int(n_owned)
    out["emulated_send_prep_ms"] = round(min(send_t), 3)
    out["emulated_owner_dedup_reduce_ms"] = round(min(owner_t), 3)
    out["all_to_all_bytes_out_per_rank"] = int(24 * V)
    out["all_to_all_bytes_back_per_rank"] = int(8 * V)
    out["private_terms"] = int(private.sum().item())
    out["what"] = ("world-1 global_df_index at c4 shard size (real path), then the owner side of dist.df_exchange "
                   "for an emulated %d-shard set (df>1 rows shared, df=1 rows shard-private): one owner's received "
                   "rows (1/%d of every shard's) summed per fingerprint (sme_df_owner_sum), and the sender's owner pack (sme_df_owner_pack); the two "
                   "all_to_alls need %d GPUs and are reported as bytes" % (a.world, a.world, a.world))
    res = back
    del res, gdf
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "dfx_c4.json"), "w"), indent=1)
    ix.close()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
