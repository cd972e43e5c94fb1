"""c1: the reference's bundled sample ./data/sample-trec-small.xml
(TermKGramDocIndexer.java:61) is absent, so the plumbing config uses a committed
1,000-document synthetic TREC file, seed 1: the c2 document shape at the
published run's length (247.7 indexed tokens per document, J2 job 0196),
Zipf s = 1 over 2^14 words.  Writes tests/golden/c1_sample_trec.xml and its
docno mapping file (TrecDocnoMapping format) c1_sample_mapping.bin.
    python tools/gen_c1_sample.py"""
import hashlib
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
synth = importlib.import_module("simple-mapreduce-search-engine-information-retrieval-_amd.synth")


def main():
    n = 1000
    corpus = synth.gen_corpus(n, V=1 << 14, seed=1, len_lo=200, len_hi=300)
    out = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(out, "c1_sample_trec.xml"), "wb") as f:
        f.write(corpus)
    with open(os.path.join(out, "c1_sample_mapping.bin"), "wb") as f:
        f.write(synth.mapping_bytes(n))
    print("c1: %d docs, %d bytes, sha256 %s" % (n, len(corpus), hashlib.sha256(corpus).hexdigest()))


if __name__ == "__main__":
    main()
