"""Build-path A/B on the GPU (timing; parity is the tests' job): the device corpus
of a BASELINE config built under several sme_set_option settings, per setting the
median stage times (ms) of `--reps` builds after a warm-up and a sha256 of the
CSR + term strings (must agree across settings).
    python tools/buildexp.py [--config c2|c5|c4shard] [--opts "docid_terms=0;docid_terms=1"]
"""
import argparse
import hashlib
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "simple-mapreduce-search-engine-information-retrieval-_amd"
CFG = dict(c2=dict(n=1_000_000, V=1 << 20, seed=42, lo=400, hi=600),
           c5=dict(n=8_841_823, V=30_000, seed=9, lo=40, hi=72),
           c4shard=dict(n=6_250_000, V=1 << 22, seed=44, lo=200, hi=360))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--opts", default="")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--digest", type=int, default=1)
    a = p.parse_args()
    import torch
    torch.cuda.init()
    sme = importlib.import_module(PKG)
    synth = importlib.import_module(PKG + ".synth")
    c = CFG[a.config]
    dc = sme.DeviceCorpus(c["n"], V=c["V"], seed=c["seed"], len_lo=c["lo"], len_hi=c["hi"])
    ctx = sme.Context(k=1, num_partitions=1, device=0)
    ctx.load_docno_mapping(synth.mapping_bytes(c["n"]))
    st = torch.cuda.current_stream().cuda_stream
    for s in [x for x in a.opts.split(";")] or [""]:
        opts = dict(kv.split("=") for kv in s.split(",") if kv.strip())
        for k, v in opts.items():
            ctx.set_option(k.strip(), int(v))
        profs = []
        ix = None
        for r in range(a.reps + 1):
            if ix is not None:
                ix.close()
            ix = ctx.build_device(dc.ptr, dc.nbytes, st)
            torch.cuda.synchronize()
            if r:
                profs.append(ctx.last_build_profile())
        med = {k: round(float(np.median([pp.get(k, 0.0) for pp in profs])), 3) for k in profs[-1]
               if isinstance(profs[-1][k], (int, float))}
        dig = None
        if a.digest:
            off, dn, tf, _ = ix.csr()
            h = hashlib.sha256(off.tobytes() + dn.tobytes() + tf.tobytes())
            tot = ix.term_blob() if hasattr(ix, "term_blob") else None
            if tot is None:
                for t in range(0, ix.V, max(1, ix.V // 20000)):
                    h.update(ix.term(t).encode("utf-16-le", "surrogatepass"))
            else:
                h.update(tot)
            dig = h.hexdigest()[:16]
        print(json.dumps({"config": a.config, "opts": s or "default", "N": ix.N, "V": ix.V, "P": ix.P,
                          "digest": dig, "stage_ms": med}), flush=True)
        ix.close()


if __name__ == "__main__":
    main()
