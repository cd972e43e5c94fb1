"""Independent pure-Python restatement of CharKGramTermIndexer's output
(C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:88-129, one map task) used to
cross-check the C oracle (oracle/oracle_chargram.c).  Test infrastructure only.

Tokens come from the oracle's processContent (pinned separately by the KATs); what
is restated here is the job itself: '$'+token+'$' k-unit substrings, one set per gram
with JDK 6 HashMap iteration order (simulated), Text byte order, HashPartitioner,
TextOutputFormat lines."""
import oracle_lib as O


def java_hash(units):
    h = 0
    for u in units:
        h = (31 * h + u) & 0xFFFFFFFF
    return h


def spread6(h):
    h &= 0xFFFFFFFF
    h ^= (h >> 20) ^ (h >> 12)
    return (h ^ (h >> 7) ^ (h >> 4)) & 0xFFFFFFFF


class HashSet6:
    """java.util.HashSet on JDK 6: head insertion, resize when size++ >= threshold."""

    def __init__(self):
        self.table = [[] for _ in range(16)]
        self.size, self.thr = 0, 12

    def add(self, key, h):
        hh = spread6(h)
        ch = self.table[hh & (len(self.table) - 1)]
        if any(k == key for k, _ in ch):
            return
        ch.insert(0, (key, hh))
        self.size += 1
        if self.size - 1 >= self.thr:
            nt = [[] for _ in range(2 * len(self.table))]
            for c in self.table:
                for k, v in c:
                    nt[v & (len(nt) - 1)].insert(0, (k, v))
            self.table, self.thr = nt, int(len(nt) * 0.75)

    def __iter__(self):
        for c in self.table:
            for k, _ in c:
                yield k


def units(s):
    b = s.encode("utf-16-le", "surrogatepass")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def from_units(u):
    return b"".join(x.to_bytes(2, "little") for x in u).decode("utf-16-le", "surrogatepass")


def java_utf8(s):
    """String.getBytes("UTF-8"): an unpaired surrogate becomes '?'."""
    out, u, i = [], units(s), 0
    while i < len(u):
        c = u[i]
        if 0xD800 <= c <= 0xDBFF and i + 1 < len(u) and 0xDC00 <= u[i + 1] <= 0xDFFF:
            out.append(from_units(u[i:i + 2]).encode("utf-8"))
            i += 2
            continue
        out.append(b"?" if 0xD800 <= c <= 0xDFFF else chr(c).encode("utf-8"))
        i += 1
    return b"".join(out)


def chargram_parts(corpus, k, R):
    sets = {}
    for off, ln in O.split_records(corpus):
        for tok in O.process_content(corpus[off:off + ln]):
            t = units("$" + tok + "$")
            for i in range(len(t) - k + 1):
                g = java_utf8(from_units(t[i:i + k]))  # the Text key
                if g not in sets:
                    sets[g] = HashSet6()
                sets[g].add(tok, java_hash(units(tok)))
    parts = [[] for _ in range(R)]
    for g, hs in sets.items():
        key = g
        h = 1
        for b in key:
            h = (31 * h + (b - 256 if b > 127 else b)) & 0xFFFFFFFF
        p = (h & 0x7FFFFFFF) % R
        line = key + b"\t[" + b", ".join(java_utf8(t) for t in hs) + b"]\n"
        parts[p].append((key, line))
    return [b"".join(l for _, l in sorted(ps)) for ps in parts]
