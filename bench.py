"""bench.py -- index build GB/s (+ top-k QPS) on MI355X, BASELINE.json configs.

Default workload (N=1): configs[1] "Synthetic Zipfian corpus 1M docs x ~500
tokens, 1 MI355X: index build + TF-IDF" (N=1e6, doc length
U[400,600], V_w=2^20, Zipf s=1, seed 42).  One step = one full index build +
TF-IDF weight pass over the HBM-resident corpus (sme_build_index_device): record
split, docno lookup, tokenize/stop/stem, per-record tf aggregation, term sort,
weights, and the reduce-order (tf desc, docno asc) postings.  The corpus is
generated on the device before the timed region.  After the timed build steps,
the c3 query batch (100k queries, 2-8 terms drawn by df, top-10) is timed the
same way and reported in "query".

--config c5: MS MARCO-shaped c5 (8,841,823 passages, V_w=30,000, 40-72 tokens,
seed 9, strong scaling: the passages are split over the ranks) + 1M-query top-100;
--config c4shard: one GPU's shard of c4 (6.25M docs of ~280 tokens, V_w=2^22,
seed 44, weak scaling).  These are profiling lines (profiles/), not the driver's.

Beside `value`, timed the same way: value_with_records (+ the I9 serialization),
value_query_ready (+ the once-per-index query preparation) and value_true_df
(build in true-df idf mode + the global df exchange by owner rank over RCCL and
the re-weight: the north star's "global df is an RCCL all-reduce" step).

After the timed regions (untimed): full-size property checks of the built index
(sum tf = tokens + docid tokens, V = distinct terms of the vocabulary + N, CSR
offsets monotone, docnos ascending per term), a cross-kernel check of a query
sample (tiled default == postings-only == streaming kernel, bit for bit), and the
I9 serialization of the partition records as its own stage.

Multi-GPU (one rank per GPU, RCCL): `--gpus N` under torchrun (WORLD_SIZE set)
runs as one rank of N; `--gpus N` without WORLD_SIZE starts the N rank processes
itself before anything touches the GPU (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1), and exits with rank 0's status.  The world size the
ranks agree on must equal --gpus (and the node must have that many GPUs unless
SME_BENCH_REHEARSE=1), so an N-GPU line cannot silently measure one GPU.  Every
rank owns a contiguous shard of docs (docids offset by rank), builds its local
index, and the global document count is all-reduced in every step
(reference-mode idf = log10(N_global)).  The query batch is broadcast as one
UTF-8 term blob + offsets (tensors); every shard scores it, and the per-shard
top-k lists go to the queries' owner ranks (one all_to_all) and are merged there
(dist.merge_topk_owner).

Prints ONE JSON line on rank 0.
"""
import argparse
import gc
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "simple-mapreduce-search-engine-information-retrieval-_amd"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CONFIGS = {
    "c2": dict(docs=1_000_000, vocab=1 << 20, seed=42, lo=400, hi=600, queries=100_000, k=10, qseed=7,
               scaling="weak", name="c2: %d docs/GPU x U[400,600] tokens, V_w=%d, Zipf s=1, K=1 index + TF-IDF; "
                                    "c3: %d queries top-%d"),
    "c5": dict(docs=8_841_823, vocab=30_000, seed=9, lo=40, hi=72, queries=1_000_000, k=100, qseed=9,
               scaling="strong", name="c5: %d passages (split over the GPUs) x U[40,72] tokens, V_w=%d, Zipf s=1; "
                                      "%d queries top-%d"),
    "c4shard": dict(docs=6_250_000, vocab=1 << 22, seed=44, lo=200, hi=360, queries=100_000, k=10, qseed=7,
                    scaling="weak", name="c4 shard: %d docs/GPU x U[200,360] tokens, V_w=%d, Zipf s=1; "
                                         "%d queries top-%d"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    p.add_argument("--docs", type=int, default=None, help="docs per GPU (weak) / in total (strong)")
    p.add_argument("--vocab", type=int, default=None)
    p.add_argument("--queries", type=int, default=None)
    p.add_argument("--no-checks", action="store_true", help="skip the untimed post-run checks")
    p.add_argument("--cpu-docs", type=int, default=8000, help="docs in the ref-faithful CPU sample (0 = skip CPU)")
    p.add_argument("--cpu-opt-docs", type=int, default=50000, help="docs in the cpu-opt CPU sample")
    p.add_argument("--cpu-ref-queries", type=int, default=50, help="queries timed with the ref-faithful rank()")
    p.add_argument("--cpu-opt-queries", type=int, default=20000, help="queries timed with the cpu-opt rank()")
    p.add_argument("--no-query", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the untimed host-to-host end-to-end stage")
    p.add_argument("--true-df-steps", type=int, default=None,
                   help="timed steps of the true-df leg (build + global df exchange + reweight; default --steps, "
                        "0 = skip)")
    a = p.parse_args()
    cfg = dict(CONFIGS[a.config])
    for key in ("docs", "vocab", "queries"):
        if getattr(a, key) is not None:
            cfg[key] = getattr(a, key)
    a.cfg = cfg
    a.docs, a.vocab, a.queries = cfg["docs"], cfg["vocab"], cfg["queries"]
    if a.true_df_steps is None:
        a.true_df_steps = a.steps
    return a


def spawn_ranks(n):
    """--gpus N > 1 without a launcher: start N rank processes of this script
    (one per GPU) and return rank 0's exit status (any failing rank fails the
    run).  The children are polled together: when one exits non-zero the others
    (which would wait in a collective until the backend timeout) are terminated
    at once and its status returned.  Nothing here touches the GPU: the children
    initialise their own."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        for p in procs:
            c = p.poll()
            if c is not None and c != 0:
                failed = c
                break
        else:
            time.sleep(0.2)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        return failed
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return codes[0] if codes[0] != 0 else (bad[0] if bad else 0)


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus is not None and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    world = int(env_world or "1")
    if a.gpus is None:
        a.gpus = world
    if a.gpus != world:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # SME_BENCH_REHEARSE=1: the N > 1 code path rehearsed on fewer GPUs than
    # ranks (ranks share devices round-robin, collectives over gloo) -- a check
    # of the multi-rank bench logic, never a scaling measurement
    rehearse = os.environ.get("SME_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    elif world > torch.cuda.device_count():
        raise SystemExit("bench.py: %d ranks but %d visible GPUs (SME_BENCH_REHEARSE=1 rehearses on fewer)"
                         % (world, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # every rank must see the same world: the line's n_gpus is the agreed one
        wt = torch.tensor([1], dtype=torch.int64, device="cpu" if rehearse else "cuda")
        dist.all_reduce(wt)
        if int(wt.item()) != a.gpus:
            raise SystemExit("bench.py: %d ranks joined, --gpus %d" % (int(wt.item()), a.gpus))
    sme = importlib.import_module(PKG)
    synth = importlib.import_module(PKG + ".synth")
    L = sme.lib()

    # ---- corpus shard in HBM (untimed) ----
    cfg = a.cfg
    seed = cfg["seed"]
    blob, voff = synth.make_vocab(a.vocab, seed)
    cdf = synth.zipf_cdf(a.vocab, 1.0)
    L.sme_synth_corpus.argtypes = [C.c_int, C.c_char_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int64,
                                   C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.sme_synth_free.argtypes = [C.c_void_p]
    d_corpus, nbytes = C.c_void_p(), C.c_size_t()
    if cfg["scaling"] == "weak":
        n_local, d0, n_total = a.docs, rank * a.docs, a.docs * world
    else:  # strong: the configured document count is split over the ranks
        n_local = a.docs // world + (1 if rank < a.docs % world else 0)
        d0 = rank * (a.docs // world) + min(rank, a.docs % world)
        n_total = a.docs
    rc = L.sme_synth_corpus(local, blob, voff.ctypes.data, a.vocab, cdf.ctypes.data, n_local, d0, seed, cfg["lo"],
                            cfg["hi"], C.byref(d_corpus), C.byref(nbytes))
    assert rc == 0, rc
    nbytes = nbytes.value
    # every rank loads the global mapping (all docids), so docnos are global
    mapping = synth.mapping_bytes(n_total)
    ctx = sme.Context(k=1, num_partitions=1, device=local)
    # SME_BENCH_OPTS="name=value,...": result-preserving path options (sme_set_option) for A/B runs
    for kv in filter(None, os.environ.get("SME_BENCH_OPTS", "").split(",")):
        ctx.set_option(kv.split("=")[0], int(kv.split("=")[1]))
    ctx.load_docno_mapping(mapping)
    stream = torch.cuda.current_stream().cuda_stream

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    D = importlib.import_module(PKG + ".dist") if dist is not None else None

    def step():
        ix = ctx.build_device(d_corpus.value, nbytes, stream)
        if D is not None:
            ix.reweight(D.global_count(ix.N), None, stream)  # idf = log10(N_global): RCCL all-reduce of N
        return ix

    ix = None
    for _ in range(a.warmup):
        if ix is not None:
            ix.close()
        ix = step()
    barrier()
    profs = []
    gc.collect()
    gc.disable()  # no cyclic-GC pause inside the timed steps (re-enabled after)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if ix is not None:
            ix.close()
        ix = step()
    barrier()
    dt = (time.perf_counter() - t0) / a.steps
    gc.enable()
    # per-stage device-event times of the last step (read after the timed region;
    # every step does identical work)
    profs.append(ctx.last_build_profile())
    prof = {k: round(sum(p.get(k, 0.0) for p in profs) / len(profs), 4) for k in profs[-1]}
    N, V, P = ix.N, ix.V, ix.P
    # the drop-in's product is the part files' records (TermKGramDocIndexer.java:
    # 269-275): the same steps again with the I9 device serialization inside the
    # clock (sme_index_serialize), reported as value_with_records beside value
    barrier()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ix.close()
        ix = step()
        ix.serialize()
    barrier()
    dt_rec = (time.perf_counter() - t0) / a.steps
    gc.enable()
    # a drop-in that serves queries right after its build also pays the
    # once-per-index query preparation (the reference's own post-build step is
    # the forward-index job, BuildIntDocVectorsForwardIndex.java:84-158): the same
    # steps with sme_index_prepare_queries inside the clock -> value_query_ready
    barrier()
    gc.disable()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ix.close()
        ix = step()
        ix.prepare_queries(stream)
    barrier()
    dt_qr = (time.perf_counter() - t0) / a.steps
    gc.enable()
    t_max = dt
    tot_bytes = nbytes
    if dist is not None:
        tt = torch.tensor([dt, float(nbytes), float(N), float(V), float(P), dt_rec, dt_qr], dtype=torch.float64,
                          device="cpu" if rehearse else "cuda")
        ts = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(ts, tt)
        ts = torch.stack(ts).cpu().numpy()
        t_max = float(ts[:, 0].max())
        tot_bytes = float(ts[:, 1].sum())
        dt_rec = float(ts[:, 5].max())
        dt_qr = float(ts[:, 6].max())
    gbs = tot_bytes / t_max / 1e9
    alg_bytes = nbytes + 8 * P + 8 * (V + 1)  # A_build = B + 8P + 8(V+1) per GPU
    # dominant kernel: the stream tokenizer (k_tok_fast).  Algorithmic bytes per
    # launch = the text it tokenizes, read once (B); its duration is the mean of
    # the HIP events bracketing the launch on its stream over the timed steps.
    achieved_build = alg_bytes / dt / 1e9
    tok_ms = prof.get("tok_kernel")
    tok_gbs = nbytes / (tok_ms * 1e-3) / 1e9 if tok_ms else None
    traffic, t_fetch_raw, t_write = pmc_traffic("k_tok_fast", a, detail=True)

    # ---- queries (c3) ----
    query = None
    if not a.no_query and a.queries > 0:
        query = run_queries(a, sme, synth, ix, torch, dist, world, rank, barrier)

    result = {
        "metric": "index build GB/s of text (top-%d queries/sec in 'query')" % cfg["k"],
        "value": round(gbs, 4),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(t_max * 1e3, 3),
        "higher_is_better": True,
        "scaling": cfg["scaling"],
        "vs_baseline": None,
        "dtype": "u8 text / int32 postings / f64 weights",
        "data": "synthetic (device-generated Zipfian TREC corpus, seed %d)" % seed,
        "config": {"workload": cfg["name"] % (a.docs, a.vocab, a.queries, cfg["k"]), "docs_this_gpu": n_local,
                   "text_bytes_per_gpu": nbytes, "N": N, "V": V, "P": P, "parallelism": "doc-sharded x%d" % world},
        "roofline": {"bound": "hbm", "kernel": "k_tok_fast", "achieved": round(tok_gbs, 2) if tok_gbs else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(tok_gbs / HBM_PEAK_GBS, 5) if tok_gbs else None,
                     "traffic": traffic, "traffic_fetch_raw": t_fetch_raw, "traffic_write": t_write,
                     "kernel_ms": tok_ms,
                     "what": "dominant kernel k_tok_fast: algorithmic bytes = text bytes B read once per launch, / "
                             "mean launch time (HIP events on its stream); traffic = PMC HBM bytes per launch "
                             "(profiles/pmc_traffic.json: 2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction)"},
        "value_with_records": {"value": round(tot_bytes / dt_rec / 1e9, 4), "unit": "GB/s",
                               "ms_per_step": round(dt_rec * 1e3, 3),
                               "what": "build + TF-IDF + I9 serialization of the partition records in HBM "
                                       "(sme_index_serialize) per step, max over ranks; the records stay in HBM"
                                       + ("" if world == 1 else "; per-shard records (the reference layout "
                                          "needs dist.reference_partitions' exchange, not timed)")},
        "value_query_ready": {"value": round(tot_bytes / dt_qr / 1e9, 4), "unit": "GB/s",
                              "ms_per_step": round(dt_qr * 1e3, 3),
                              "what": "build + TF-IDF + the once-per-index query preparation "
                                      "(sme_index_prepare_queries: heavy tf / impact rows and their block "
                                      "bounds, sparse posting words) per step, max over ranks: the index "
                                      "ready to answer queries"},
        "build_roofline": {"achieved": round(achieved_build, 2), "unit": "GB/s",
                           "frac": round(achieved_build / HBM_PEAK_GBS, 5),
                           "what": "whole build step: A_build = B + 8P + 8(V+1) per GPU / step time"},
        "stage_ms": prof,
    }
    if rehearse and world > 1:
        result["rehearsal"] = "SME_BENCH_REHEARSE: %d ranks on %d GPU(s), gloo -- not a scaling measurement" % (
            world, torch.cuda.device_count())
    if query is not None:
        result["query"] = query
    # calibration: the achievable HBM rate of a streaming copy on this device,
    # reported beside the 8 TB/s spec every frac above is priced against
    cal = C.c_double()
    if L.sme_hbm_copy_bench(local, 4 << 30, 10, C.byref(cal)) == 0:
        result["roofline"]["peak_measured_copy"] = round(cal.value, 1)
        result["roofline"]["frac_of_measured"] = (round(tok_gbs / cal.value, 5) if tok_gbs else None)
        result["hbm_copy_GBps"] = {"value": round(cal.value, 1), "what": "sme_hbm_copy_bench: 4 GiB device copy, "
                                   "16-byte nontemporal loads/stores, read + write bytes / kernel time (x10)"}
    qinternal = None
    if query is not None:
        qinternal = (query.pop("_terms"), query.pop("_qoff"), query.pop("_out"))
    if not a.no_checks:
        result["checks"] = post_checks(a, sme, synth, ix, n_local, d0, qinternal, rank,
                                       n_global=D.global_count(ix.N) if D is not None else None)
        result["stage_ms"]["serialize_records_untimed"] = serialize_stage(ix, torch)
    cpu_full = None
    if rank == 0 and a.cpu_docs > 0 and a.config == "c2" and qinternal is not None:
        cpu_full = cpu_query_full(ix, qinternal, a)
    if not a.no_e2e and world == 1:
        ix.close()
        ix = None
        gc.collect()
        result["end_to_end_ms"] = end_to_end_stage(sme, ctx, d_corpus.value, nbytes, torch)
    if ix is not None:
        ix.close()
        ix = None
    ctx.close()
    if a.true_df_steps > 0:
        result["value_true_df"] = true_df_leg(a, sme, ctx_args=dict(k=1, num_partitions=1, device=local),
                                              mapping=mapping, d_corpus=d_corpus.value, nbytes=nbytes,
                                              stream=stream, D=D, barrier=barrier, world=world, torch=torch,
                                              rehearse=rehearse)
    if rank == 0 and a.cpu_docs > 0:
        result["cpu_baseline"] = cpu_baseline(synth, a)
        if a.config == "c2":
            result["c1_sample"] = c1_sample(sme, a)
        if cpu_full is not None:
            result["cpu_baseline"]["cpu_opt"].update(cpu_full)
    if rank == 0:
        print(json.dumps(result), flush=True)
    L.sme_synth_free(d_corpus)
    if dist is not None:
        dist.destroy_process_group()


def true_df_leg(a, sme, ctx_args, mapping, d_corpus, nbytes, stream, D, barrier, world, torch, rehearse):
    """The north star's collective in a timed leg: "global df is an RCCL
    all-reduce over xGMI".  Each step builds the shard in true-df idf mode
    (log10(N / df)) and, on N > 1 ranks, exchanges the df of every local term
    with its owner rank (dist.global_df_index: device fingerprints, owner
    all_to_all, owner sums in libsme, all_to_all back) plus the all-reduce of N,
    then re-weights the shard with the global statistics (sme_index_reweight) --
    the reducer's df over all map outputs, TermKGramDocIndexer.java:175-183.
    Timed like `value` (barrier + synchronize on both sides, max over ranks).
    Runs after the main legs with their context closed (one build workspace in
    HBM at a time)."""
    ctx = sme.Context(idf_mode=sme.SME_IDF_TRUE_DF, **ctx_args)
    ctx.load_docno_mapping(mapping)
    ex = {}

    def step(timings=None):
        ix = ctx.build_device(d_corpus, nbytes, stream)
        if D is not None:
            gdf = D.global_df_index(ix, timings=timings)
            ix.reweight(D.global_count(ix.N), gdf.data_ptr(), stream)
        return ix

    ix = None
    for _ in range(max(1, a.warmup)):
        if ix is not None:
            ix.close()
        ix = step()
    barrier()
    gc.disable()
    t0 = time.perf_counter()
    for i in range(a.true_df_steps):
        ix.close()
        ix = step(ex if i == a.true_df_steps - 1 else None)
    barrier()
    dt = (time.perf_counter() - t0) / a.true_df_steps
    gc.enable()
    tot = float(nbytes)
    if D is not None:
        import torch.distributed as tdist
        tt = torch.tensor([dt, float(nbytes)], dtype=torch.float64, device="cpu" if rehearse else "cuda")
        ts = [torch.zeros_like(tt) for _ in range(world)]
        tdist.all_gather(ts, tt)
        ts = torch.stack(ts).cpu().numpy()
        dt, tot = float(ts[:, 0].max()), float(ts[:, 1].sum())
    prof = ctx.last_build_profile()
    ix.close()
    ctx.close()
    out = {"value": round(tot / dt / 1e9, 4), "unit": "GB/s", "ms_per_step": round(dt * 1e3, 3),
           "steps": a.true_df_steps, "build_ms_last_step": prof.get("total"),
           "what": "build in true-df idf mode + (N > 1) the global df exchange by owner rank and the all-reduce of N "
                   "over %s + sme_index_reweight with the global N / df, per step, max over ranks"
                   % ("RCCL" if D is not None and not rehearse else "gloo" if D is not None else "no collective "
                      "(one rank: the local df is the global df)")}
    if ex:
        out["df_exchange_ms_last_step"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in ex.items()}
    return out


def run_queries(a, sme, synth, ix, torch, dist, world, rank, barrier):
    k = a.cfg["k"]
    _, _, _, df = ix.csr()
    terms, qoff = synth.queries_by_df(df, a.queries, seed=a.cfg["qseed"])
    if dist is not None:
        # queries are defined by term strings (rank 0's draw); every shard maps them
        # to its own ids.  The batch travels as tensors: one UTF-8 blob of the
        # distinct terms + their offsets, and per query term its index among them
        terms, qoff = broadcast_queries(ix, terms, qoff, dist, rank, torch)
    d_terms = torch.from_numpy(terms).cuda()
    d_qoff = torch.from_numpy(qoff).cuda()
    out_d = torch.empty((a.queries, k), dtype=torch.int32, device="cuda")
    out_s = torch.empty((a.queries, k), dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    # query-side heavy rows of the index: built once per index (like the
    # reference's forward-index job), outside the per-batch timing, reported
    qidx_ms = ix.prepare_queries(stream)

    def qstep():
        ix.query_topk_device(d_terms.data_ptr(), d_qoff.data_ptr(), a.queries, k, out_d.data_ptr(), out_s.data_ptr(),
                             stream)
        if dist is not None:
            # per-shard top-k lists -> global top-k of the queries this rank owns
            # (RCCL query-owner all_to_all + merge, dist.merge_topk_owner)
            return importlib.import_module(PKG + ".dist").merge_topk_owner(out_d, out_s, k)
        return out_d

    qstep()
    barrier()
    gc.collect()
    gc.disable()  # no cyclic-GC pause inside the timed batches (re-enabled after)
    # batches: at least 10 and enough for ~1.5 s of query work, at most 50;
    # every rank runs the same count
    ts1 = time.perf_counter()
    qstep()
    torch.cuda.synchronize()
    t_one = time.perf_counter() - ts1
    if dist is not None:
        tt1 = torch.tensor([t_one], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt1, op=dist.ReduceOp.MAX)
        t_one = float(tt1.item())
    barrier()
    steps = max(a.steps, min(50, max(10, int(1.5 / max(t_one, 1e-6)))))
    kms, pms, kname = [], [], "k_query"

    def _cg():
        try:
            return {l.split()[0]: int(l.split()[1]) for l in open("/sys/fs/cgroup/cpu.stat")}
        except (OSError, ValueError, IndexError):
            return {}
    cg0 = _cg() if os.environ.get("SME_BENCH_VERBOSE") else None
    # the per-batch records are allocated before the clock starts (a ~50 ms
    # host stall was measured at the first allocation after it on the GPU box)
    walls = [0.0] * steps
    starts = [0.0] * steps
    t0 = time.perf_counter()
    for i in range(steps):
        tq = time.perf_counter()
        starts[i] = tq
        qstep()
        walls[i] = (time.perf_counter() - tq) * 1e3
    tb = time.perf_counter()
    barrier()
    dt = (time.perf_counter() - t0) / steps
    gc.enable()
    if os.environ.get("SME_BENCH_VERBOSE"):
        cg1 = _cg()
        print("query step walls %s ms, loop %.3f ms, closing barrier %.3f ms, cgroup cpu.stat delta %s" % (
              ["%.3f" % w for w in walls], (tb - t0) * 1e3, (time.perf_counter() - tb) * 1e3,
              {k: cg1[k] - cg0.get(k, 0) for k in cg1}), file=sys.stderr)
        print("query step gaps (start - previous end) %s ms" % ["%.3f" % ((starts[i] - (starts[i - 1] if i else t0)) * 1e3 -
              (walls[i - 1] if i else 0.0)) for i in range(len(starts))], file=sys.stderr)
    # device-event timings of the last batch (read after the timed region: the
    # profile call is measurement overhead, not query work; every batch is identical)
    qp = ix.ctx.last_build_profile()
    kms.append(qp.get("query_kernel"))
    pms.append(qp.get("query_prep"))
    kname = qp.get("query_kernel_name", kname)
    qextra = {key: qp[key] for key in ("query_seed", "query_final", "query_total", "query_overflow") if key in qp}
    kms = [x for x in kms if x is not None]
    qk_ms = sum(kms) / len(kms) if kms else None
    pms = [x for x in pms if x is not None]
    qp_ms = sum(pms) / len(pms) if pms else None
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    qps = a.queries / dt
    nt = np.diff(qoff)
    # algorithmic bytes: postings of distinct batch terms read once (docno + weight = 12 B here)
    tv = terms[terms >= 0]
    uniq = np.unique(tv)
    # SURVEY 8d A_q with this layout's 8 B per posting (int32 docno + int32 tf)
    alg = 8 * int(df[uniq].sum()) + 4 * int(nt.sum()) + 12 * k * a.queries
    touched = 8 * int(df[tv].sum())
    t_k = (qk_ms * 1e-3) if qk_ms else dt
    qtr = pmc_traffic(kname, a, detail=True)
    uni = None
    if dist is None:
        try:
            # c3's uniform-over-vocabulary variant (seed 8): same batch
            # size and k, terms drawn uniformly over the index's term ids; timed
            # after the headline batches, not part of `value`
            tu, qu = synth.queries_by_df(df, a.queries, seed=8, uniform=True)
            du, dq = torch.from_numpy(tu).cuda(), torch.from_numpy(qu).cuda()
            ud, us = torch.empty_like(out_d), torch.empty_like(out_s)  # the headline batch's results stay for post_checks

            def ustep():
                ix.query_topk_device(du.data_ptr(), dq.data_ptr(), a.queries, k, ud.data_ptr(), us.data_ptr(), stream)
            ustep()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(5):
                ustep()
            torch.cuda.synchronize()
            du_ms = (time.perf_counter() - t1) / 5 * 1e3
            up = ix.ctx.last_build_profile()
            uni = {"value": round(a.queries / (du_ms * 1e-3), 1), "unit": "queries/s", "ms_per_batch": round(du_ms, 3),
                   "kernel_ms": up.get("query_kernel"), "terms_per_query": "U{2..8} uniform over the %d term ids (seed 8)"
                   % len(df), "what": "c3 uniform-vocabulary variant, 5 batches after the timed ones (not in value)"}
            del du, dq, ud, us
        except Exception as e:  # an extra measurement: never fails the bench line
            uni = {"error": repr(e)[:200]}

    return {"metric": "top-%d queries/sec" % k, "uniform_vocab": uni, "value": round(qps, 1), "unit": "queries/s", "queries": a.queries, "batches": steps,
            "terms_per_query": "U{2..8} drawn by df (seed %d)" % a.cfg["qseed"], "ms_per_batch": round(dt * 1e3, 3),
            "prep_ms": qp_ms, "query_index_build_ms": round(qidx_ms, 3),
            "query_index_what": "once per index, not per batch: tf byte rows + 16/1024-doc block maxima of the "
                                "terms with df >= span/128 (sme_index_prepare_queries)",
            "_terms": terms, "_qoff": qoff, "_out": (out_d, out_s),
            "prep_what": "per batch, inside ms_per_batch: skip table (distinct batch terms x 1024-doc tiles), "
                         "impact tables of the batch terms, heaviest-term query order",
            "roofline": {"bound": "hbm", "kernel": kname, "kernel_ms": qk_ms,
                         "achieved": round(alg / t_k / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / t_k / 1e9 / HBM_PEAK_GBS, 6), "traffic": qtr[0],
                         "traffic_fetch_raw": qtr[1], "traffic_write": qtr[2],
                         "what": "A_q = 8*sum(df of distinct batch terms) + 4*sum|q| + 12*k*Q per launch / "
                                 "mean launch time (HIP events)"},
            "kernel_split_ms": qextra,
            "kernel_split_what": "k_query_win path: seed (k_query_seed), final selection + overflow re-runs "
                                 "(k_query_final, k_query_bm), their total; query_overflow = queries re-run",
            "postings_touched_GBps": round(touched / t_k / 1e9, 2),
            "postings_touched_what": "8 B x postings of every query term (re-reads across queries included)"}


def broadcast_queries(ix, terms, qoff, dist, rank, torch):
    """Rank 0's query batch (its own term ids) -> every rank's local term ids of
    the same term strings.  Broadcasts: sizes (int64 [3]), the distinct terms as
    one UTF-8 blob (uint8) + offsets (int64), the per-term index into them (int32)
    and the query offsets (int64); each rank resolves the strings with
    sme_lookup_terms (Index.lookup)."""
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    if rank == 0:
        uniq, pos = np.unique(terms, return_inverse=True)
        bs = [ix.term(int(t)).encode("utf-8", "surrogatepass") for t in uniq]
        blob = np.frombuffer(b"".join(bs), dtype=np.uint8)
        boff = np.zeros(len(bs) + 1, np.int64)
        boff[1:] = np.cumsum([len(b) for b in bs])
        hdr = torch.tensor([len(blob), len(bs), len(terms)], dtype=torch.int64, device=dev)
    else:
        hdr = torch.zeros(3, dtype=torch.int64, device=dev)
    dist.broadcast(hdr, 0)
    nb, nu, nt = (int(x) for x in hdr.tolist())
    nq1 = len(qoff) if rank == 0 else 0
    t_nq = torch.tensor([nq1], dtype=torch.int64, device=dev)
    dist.broadcast(t_nq, 0)
    nq1 = int(t_nq.item())
    if rank == 0:
        tb = torch.from_numpy(blob.copy() if nb else np.zeros(1, np.uint8)).to(dev)
        to = torch.from_numpy(boff).to(dev)
        tp = torch.from_numpy(pos.astype(np.int32)).to(dev)
        tq = torch.from_numpy(np.asarray(qoff, np.int64)).to(dev)
    else:
        tb = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
        to = torch.empty(nu + 1, dtype=torch.int64, device=dev)
        tp = torch.empty(nt, dtype=torch.int32, device=dev)
        tq = torch.empty(nq1, dtype=torch.int64, device=dev)
    for t in (tb, to, tp, tq):
        dist.broadcast(t, 0)
    blob, boff = tb.cpu().numpy()[:nb].tobytes(), to.cpu().numpy()
    strs = [blob[boff[i]:boff[i + 1]].decode("utf-8", "surrogatepass") for i in range(nu)]
    loc = ix.lookup(strs)
    return loc[tp.cpu().numpy()].astype(np.int32), tq.cpu().numpy()


def post_checks(a, sme, synth, ix, n_local, d0, qinternal, rank, n_global=None):
    """Untimed, size-independent checks of the full-size build and query batch."""
    out = {}
    off, dn, tf, df = ix.csr()
    lens = synth.doc_lengths(d0, d0 + n_local, a.cfg["seed"], a.cfg["lo"], a.cfg["hi"])
    # every synthetic token is one term, plus the docid token of <DOCNO> (T7)
    out["sum_tf_eq_tokens"] = bool(int(tf.astype(np.int64).sum()) == int(lens.sum()) + n_local)
    out["offsets_monotone"] = bool((np.diff(off) >= 1).all() and off[0] == 0 and off[-1] == ix.P)
    # reduce order inside every term: tf desc, then docno asc
    newt = np.zeros(max(ix.P, 1), bool)  # position p starts a term
    newt[off[:-1][off[:-1] < ix.P]] = True
    same = ~newt[1:ix.P]
    out["reduce_order"] = bool((((tf[1:] <= tf[:-1]) | ~same).all()) and
                               (((tf[1:] != tf[:-1]) | (dn[1:] > dn[:-1]) | ~same).all()))
    # query-side CSR: docnos strictly ascending per term
    o2, dd, _ = ix.weights()
    out["docno_order"] = bool(np.array_equal(o2, off) and ((dd[1:] > dd[:-1]) | ~same).all())
    del dd, same, newt
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    if rank == 0:
        import oracle_lib as O
        blob, voff = synth.make_vocab(a.vocab, a.cfg["seed"])
        nv = int(O.lib().or_count_distinct_terms(blob, voff.ctypes.data, a.vocab))
        # every vocabulary word occurs at c2 sizes (rank 2^20 has ~34 expected occurrences)
        full = a.config == "c2" and a.docs == CONFIGS["c2"]["docs"] and a.vocab == CONFIGS["c2"]["vocab"]
        out["V_eq_distinct_terms_plus_docids"] = bool(ix.V == nv + n_local) if full else None
        out["V_expected"] = nv + n_local
    if qinternal is not None:
        terms, qoff, (out_d, out_s) = qinternal
        nq = min(2000, len(qoff) - 1)
        t_s, q_s = terms[:qoff[nq]], qoff[:nq + 1]
        k = a.cfg["k"]
        base = (out_d[:nq].cpu().numpy(), out_s[:nq].cpu().numpy()) if hasattr(out_d, "cpu") else None
        d1, s1 = ix.query_topk(t_s, q_s, k)
        ok = base is None or (np.array_equal(base[0], d1) and np.array_equal(base[1], s1))
        for opts in ({"heavy_div": 0}, {"query_kernel": 2}, {"query_kernel": 1}):
            if "query_kernel" in opts and k > 32:
                continue
            try:
                for n, v in opts.items():
                    ix.ctx.set_option(n, v)
                d2, s2 = ix.query_topk(t_s, q_s, k)
            finally:
                ix.ctx.set_option("heavy_div", 128)
                ix.ctx.set_option("query_kernel", 0)
            ok = ok and np.array_equal(d1, d2) and np.array_equal(s1, s2)
        out["query_sample_kernels_agree"] = bool(ok)
        out["query_sample"] = nq
        # the batch's first queries against a numpy restatement of rank() over the
        # index's own postings (tests/common.np_rank; docnos + fp64 score bits),
        # with the N the index is weighted by (all-reduced over the ranks if N > 1)
        import common
        nr = min(100, nq)
        good = True
        n_idf = ix.N if n_global is None else int(n_global)
        for q in range(nr):
            rd, rs = common.np_rank(off, dn, tf, terms[qoff[q]:qoff[q + 1]].tolist(), n_idf, k)
            good = good and d1[q, :len(rd)].tolist() == rd and s1[q, :len(rd)].tolist() == rs
        out["query_sample_vs_np_rank"] = bool(good)
        out["query_sample_np_rank"] = nr
    return out


def serialize_stage(ix, torch):
    """I9: the partition records, untimed, as its own stage: the device serializer
    (k_ser_*, HIP events) and the copy of the concatenated record stream to host
    memory -- pinned (the drop-in's direct ByteBuffer case: one DMA) and pageable
    (through the library's pinned staging)."""
    offs, dev_ms = ix.serialize()
    total = int(offs[-1])
    host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    t0 = time.perf_counter()
    n = ix.copy_records(-1, hv)
    pin_ms = (time.perf_counter() - t0) * 1e3
    del host, hv
    page = np.empty(max(total, 1), np.uint8)
    page[::4096] = 0  # pages touched once (first-touch faults are not the copy)
    t0 = time.perf_counter()
    ix.copy_records(-1, page)
    page_ms = (time.perf_counter() - t0) * 1e3
    del page
    return {"device_ms": round(dev_ms, 3), "d2h_pinned_ms": round(pin_ms, 2), "d2h_pageable_ms": round(page_ms, 2),
            "ms": round(dev_ms + pin_ms, 2), "bytes": n, "d2h_pinned_GBps": round(n / pin_ms / 1e6, 2),
            "d2h_pageable_GBps": round(n / page_ms / 1e6, 2),
            "what": "sme_index_serialize (device k_ser_* time) + sme_index_copy_records(-1) of every partition's "
                    "records into pinned host memory; 'ms' = device + pinned copy, after the timed steps"}


def end_to_end_stage(sme, ctx, d_corpus, nbytes, torch, reps=2):
    """Host corpus -> part-file records on the host, untimed in the step: the
    corpus sits in pinned host memory (the drop-in's direct ByteBuffer), then
    sme_build_index (H2D + build) + sme_index_serialize + sme_index_copy_records
    into pinned host memory.  Best of `reps` after one warm-up call."""
    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    _hip_copy(host.data_ptr(), d_corpus, nbytes, 2)
    out = None
    best = None
    for i in range(reps + 1):
        t0 = time.perf_counter()
        ix = ctx.build_ptr(host.data_ptr(), nbytes)
        t1 = time.perf_counter()
        offs, dev_ms = ix.serialize()
        if out is None:
            out = torch.empty(max(int(offs[-1]), 1), dtype=torch.uint8, pin_memory=True)
        n = ix.copy_records(-1, out.numpy())
        t2 = time.perf_counter()
        prof = ctx.last_build_profile()
        ix.close()
        if i > 0 and (best is None or t2 - t0 < best["ms"] / 1e3):
            best = {"ms": round((t2 - t0) * 1e3, 2), "build_from_host_ms": round((t1 - t0) * 1e3, 2),
                    "build_device_ms": prof.get("total"), "serialize_device_ms": round(dev_ms, 3),
                    "serialize_and_d2h_ms": round((t2 - t1) * 1e3, 2), "record_bytes": n}
    best["h2d_ms_est"] = round(best["build_from_host_ms"] - (best["build_device_ms"] or 0.0), 2)
    best["GBps_text"] = round(nbytes / best["ms"] / 1e6, 2)
    best["what"] = ("pinned host corpus -> sme_build_index (H2D + build + TF-IDF) -> sme_index_serialize -> "
                    "sme_index_copy_records into pinned host memory; best of %d after a warm-up" % reps)
    del host, out
    return best


def _hip_copy(dst, src, n, kind):
    importlib.import_module(PKG).memcpy(dst, src, n)


def pmc_traffic(kernel, a, detail=False):
    """HBM bytes per launch of `kernel` from the committed PMC passes
    (profiles/pmc_traffic[_CONFIG].json, written by tools/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench config), or None.
    detail=True: (corrected total, raw FETCH_SIZE bytes, WRITE_SIZE bytes)."""
    name = "pmc_traffic.json" if a.config == "c2" else "pmc_traffic_%s.json" % a.config
    path = os.path.join(ROOT, "profiles", name)
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return (None, None, None) if detail else None
    if d.get("docs") != a.docs or d.get("vocab") != a.vocab:
        return (None, None, None) if detail else None
    k = d.get("kernels", {}).get(kernel)
    if k is None:
        return (None, None, None) if detail else None
    if detail:
        return k.get("hbm_bytes_per_launch"), k.get("fetch_bytes_raw"), k.get("write_bytes")
    return k.get("hbm_bytes_per_launch")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_threads():
    """Threads the CPU legs use: OMP_NUM_THREADS when set (the GPU box sets it to
    the CPU share it grants one GPU's job, 16), else every CPU this process may
    run on (sched_getaffinity)."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return env or aff, aff


def cpu_query_full(ix, qinternal, a):
    """cpu-opt rank() over the SAME full-size index as the GPU query batch: the
    device-built CSR (held equal to the oracle's by the parity tests) wrapped as a
    cpu-opt index, the first queries of the same c3 batch, all granted threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    terms, qoff, _ = qinternal
    threads, _ = cpu_threads()
    off, dn, tf, _ = ix.csr()
    cix = O.CpuOptIndex.from_csr(ix.N, off, dn, tf)
    nq = min(a.cpu_opt_queries, len(qoff) - 1)
    _, _, dt = cix.query(terms[:qoff[nq]], qoff[:nq + 1], a.cfg["k"], 0, threads)
    del cix, off, dn, tf
    return {"query_qps_full_index": round(nq / dt, 1), "query_full_index_docs": ix.N,
            "query_full_index_sample": "first %d queries of the GPU's c3 batch over the full %d-doc c2 index "
                                       "(device-built CSR), %d threads, %.2f s" % (nq, ix.N, threads, dt)}


def cpu_baseline(synth, a):
    """BASELINE.md section 2, on this box's host cores, bounded samples of the c2 / c3
    distributions (the oracle is the checker and the timed CPU port; the tests hold
    both modes to identical outputs):
      ref-faithful  oracle_index.c, 1 thread: per-token emit, string-key merge sort,
                    the reducer's list sorts; rank() with the reference's indexOf scan
      cpu-opt       oracle_cpuopt.cc, OpenMP over documents / queries: hash
                    aggregation, counting sorts, dense accumulators, partial-sort top-k
    `value` is the cpu-opt build rate (the honest CPU comparison)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    threads, aff = cpu_threads()
    out = {"unit": "GB/s", "cores": threads, "kind": "port", "nproc": os.cpu_count(), "affinity_cpus": aff,
           "cpu_model": _cpu_model(),
           "cores_what": "threads used = OMP_NUM_THREADS (the GPU box's CPU share for one GPU's job; nproc "
                         "shows the whole host) or the affinity set"}
    # ref-faithful build + rank() (indexOf scan) on a small sample of this config's distribution
    cfg = a.cfg
    n_ref = a.cpu_docs
    corpus = synth.gen_corpus(n_ref, V=a.vocab, seed=cfg["seed"], len_lo=cfg["lo"], len_hi=cfg["hi"])
    mapping = synth.mapping_bytes(n_ref)
    t0 = time.perf_counter()
    ref = O.OracleIndex(corpus, mapping, 1, 1)
    dt_ref = time.perf_counter() - t0
    # cpu-opt build of the same sample (threads), then a larger sample
    cpu_small = O.CpuOptIndex(corpus, mapping, threads)
    off, _, _, terms = cpu_small.csr()
    df = np.diff(off).astype(np.int32)
    tq, qo = synth.queries_by_df(df, a.cpu_ref_queries, seed=cfg["qseed"])
    O.lib().or_set_ref_scan(1)
    t0 = time.perf_counter()
    for q in range(len(qo) - 1):
        ref.query([terms[t] for t in tq[qo[q]:qo[q + 1]]], cfg["k"], 0, 0)
    dt_rq = time.perf_counter() - t0
    O.lib().or_set_ref_scan(0)
    del ref, cpu_small
    out["ref_faithful"] = {
        "build_GBps": round(len(corpus) / dt_ref / 1e9, 6), "cores": 1,
        "build_sample": "%d docs (%d bytes) of %s, %.1f s" % (n_ref, len(corpus), a.config, dt_ref),
        "query_qps": round(a.cpu_ref_queries / dt_rq, 2),
        "query_sample": "%d c3-style top-%d queries over that %d-doc index (indexOf accumulator), %.1f s"
                        % (a.cpu_ref_queries, cfg["k"], n_ref, dt_rq)}
    n_opt = a.cpu_opt_docs
    corpus = synth.gen_corpus(n_opt, V=a.vocab, seed=cfg["seed"], len_lo=cfg["lo"], len_hi=cfg["hi"])
    mapping = synth.mapping_bytes(n_opt)
    t0 = time.perf_counter()
    cpu = O.CpuOptIndex(corpus, mapping, threads)
    dt_opt = time.perf_counter() - t0
    off, _, _, _ = cpu.csr()
    df = np.diff(off).astype(np.int32)
    tq, qo = synth.queries_by_df(df, a.cpu_opt_queries, seed=cfg["qseed"])
    _, _, dt_q = cpu.query(tq, qo, cfg["k"], 0, threads)
    out["value"] = round(len(corpus) / dt_opt / 1e9, 6)
    out["sample"] = ("cpu-opt (%d threads): build of %d docs (%d bytes) of %s in %.1f s; %d c3-style top-%d queries "
                     "over that index in %.2f s" % (threads, n_opt, len(corpus), a.config, dt_opt, a.cpu_opt_queries,
                                                    cfg["k"], dt_q))
    out["cpu_opt"] = {"build_GBps": out["value"], "build_GBps_per_thread": round(out["value"] / threads, 6),
                      "query_qps": round(a.cpu_opt_queries / dt_q, 1), "query_index_docs": n_opt,
                      "query_what": "query_qps: over the %d-doc sample index; query_qps_full_index: over the "
                                    "GPU's full-size index" % n_opt}
    return out


def c1_sample(sme, a):
    """c1: the committed 1,000-document seed-1 sample
    (tests/golden/c1_sample_trec.xml + its mapping), built by libsme from device
    memory (best of 5 after a warm-up) and by both CPU legs."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    g = os.path.join(ROOT, "tests", "golden")
    corpus = open(os.path.join(g, "c1_sample_trec.xml"), "rb").read()
    mapping = open(os.path.join(g, "c1_sample_mapping.bin"), "rb").read()
    threads, _ = cpu_threads()
    ctx = sme.Context(1, 1)
    ctx.load_docno_mapping(mapping)
    d = torch.frombuffer(bytearray(corpus), dtype=torch.uint8).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    ms = []
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ix = ctx.build_device(d.data_ptr(), len(corpus), stream)
        torch.cuda.synchronize()
        if i:
            ms.append((time.perf_counter() - t0) * 1e3)
        N, V, P = ix.N, ix.V, ix.P
        ix.close()
    ctx.close()
    t0 = time.perf_counter()
    ref = O.OracleIndex(corpus, mapping, 1, 1)
    dt_ref = time.perf_counter() - t0
    del ref
    t0 = time.perf_counter()
    cpu = O.CpuOptIndex(corpus, mapping, threads)
    dt_opt = time.perf_counter() - t0
    del cpu
    return {"docs": N, "terms": V, "postings": P, "bytes": len(corpus), "gpu_build_ms": round(min(ms), 3),
            "gpu_build_GBps": round(len(corpus) / min(ms) / 1e6, 3),
            "cpu_ref_faithful_ms": round(dt_ref * 1e3, 1), "cpu_opt_ms": round(dt_opt * 1e3, 1),
            "cpu_opt_threads": threads,
            "what": "tests/golden/c1_sample_trec.xml (1,000 docs, seed 1): libsme build from device memory (best of "
                    "5, wall clock incl. launch latency), oracle ref-faithful (1 thread), cpu-opt; parity of this "
                    "sample is tests/test_gpu_parity.py::test_c1_sample_on_device"}


if __name__ == "__main__":
    main()
