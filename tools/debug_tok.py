"""Debug aid (GPU): build the test_build_synthetic corpus, list (term, docno)
pairs whose tf differs from the oracle and print where the term occurs in that
record (byte offset in the corpus, offset mod 64 / mod 16 KiB, context)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402

sme = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd")
synth = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.synth")

n = 400
c = synth.gen_corpus(n, V=5000, seed=1, len_lo=50, len_hi=150)
mb = O.write_mapping(synth.docids(n))
ref = O.OracleIndex(c, mb, 1, 1)
ctx = sme.Context(1, 1, 0)
ctx.load_docno_mapping(mb)
ix = ctx.build(c)
off, dn, tf, df = ix.csr()
got = {}
for i in range(ix.V):
    for d, f in zip(dn[off[i]:off[i + 1]].tolist(), tf[off[i]:off[i + 1]].tolist()):
        got[(ix.term(i), d)] = f
want = {}
for t in ref.terms():
    if t[0] == (" ",):
        continue
    for d, f in t[3]:
        want[(t[0][0], d)] = f
starts = []
p = 0
while True:
    p = c.find(b"<DOC>", p)
    if p < 0:
        break
    starts.append(p)
    p += 1
bad = [k for k in set(got) | set(want) if got.get(k) != want.get(k)]
print("mismatches", len(bad))
for term, d in sorted(bad)[:20]:
    rs = starts[d - 1]
    re_ = c.find(b"</DOC>", rs) + 6
    rec = c[rs:re_]
    occ = [rs + i for i in range(len(rec)) if rec[i:i + len(term)] == term.encode()]
    print(term, d, "got", got.get((term, d)), "want", want.get((term, d)), "rec", rs, re_)
    for o in occ:
        print("   at", o, "mod64", (o - rs) % 64, "rel", o - rs, repr(c[max(rs, o - 40):o + 20]))

# per-doc token totals: GPU sum tf vs oracle, and which occurrence positions are lost
from collections import Counter
gsum, wsum = Counter(), Counter()
for (term, d), f in got.items():
    gsum[d] += f
for (term, d), f in want.items():
    wsum[d] += f
diff = {d: wsum[d] - gsum[d] for d in wsum if wsum[d] != gsum[d]}
print("docs with token deficit", len(diff), "total", sum(diff.values()), "extra docs", sum(1 for d in gsum if gsum[d] > wsum[d]))
for d in sorted(diff)[:12]:
    rs = starts[d - 1]
    re_ = c.find(b"</DOC>", rs) + 6
    lost = sorted({o for (term, dd) in bad if dd == d for o in
                   [rs + i for i in range(re_ - rs) if c[rs + i:rs + i + len(term)] == term.encode()]})
    print("doc", d, "deficit", diff[d], "len", re_ - rs, "rs%16", rs % 16, "lost rel-to-end", [o - re_ for o in lost])
