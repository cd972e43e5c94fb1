/*
 * oracle_cpuopt.cc -- "cpu-opt" CPU baseline of the index build and rank()
 * (BASELINE.md section 2): all host cores (OpenMP), hash aggregation, counting
 * sorts, dense per-thread score accumulators, partial-sort top-k.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): the GPU product never
 * links this.  Same semantics as the ref-faithful restatement in
 * oracle_index.c, which the tests hold it against:
 *
 *   records     XMLRecordReader (XMLInputFormat.java:110-143,173-198), one split
 *   docno       TrecDocument.getDocid + Arrays.binarySearch over the mapping
 *               (TrecDocument.java:76-89, TrecDocnoMapping.java:67-69)
 *   tokens      GalagoTokenizer.processContent (GalagoTokenizer.java:139-183): a
 *               byte-level TagTokenizer for records of simple markup (the device's
 *               fast path: raw tokens = runs of non-split bytes outside tag /
 *               entity spans), each DISTINCT raw token normalized, stop-filtered
 *               and stemmed once per thread (T13); other records through the
 *               oracle's TagTokenizer
 *   postings    MyReducer.reduce (TermKGramDocIndexer.java:168-213): per term
 *               docno asc with duplicate docnos merged, then stable tf desc
 *   terms       TermDF.compareTo order (String.compareTo on UTF-16 units), K = 1
 *   rank()      IntDocVectorsForwardIndex.java:192-223: score += (1 + ln tf) * idf
 *               in query-token order, postings in stored order; score desc,
 *               docno asc
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <parallel/algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "oracle.h"

extern "C" int or_split_records(const uint8_t *b, size_t n, uint64_t *off, uint64_t *len, int cap);
extern "C" int or_stopword_count(void);
extern "C" const char *or_stopword(int i);

namespace {

using u16s = std::u16string;

struct U16Hash {
  size_t operator()(const u16s &s) const {
    uint64_t h = 1469598103934665603ull;
    for (char16_t c : s) h = (h ^ (uint64_t)c) * 1099511628211ull;
    return (size_t)h;
  }
};

struct CpuIndex {
  int64_t N = 0, V = 0, P = 0;
  std::vector<int64_t> toff;         // term strings, TermDF order: units [toff[t], toff[t + 1])
  std::vector<char16_t> tchars;
  std::vector<int64_t> off;          // V + 1
  std::vector<int32_t> docno, tf;    // reduce order: tf desc, docno asc
  double build_s = 0;
};

// readUntilMatch over one split (XMLRecordReader, XMLInputFormat.java:173-198),
// in parallel.  Its matcher is naive: on a mismatch the match index resets to 0
// WITHOUT re-testing the byte ("<<DOC>" holds no start tag), so its state at any
// byte depends on the bytes since the last state-0 point.  A byte outside the
// tags' alphabet {< / D O C >} resets both matchers (start "<DOC>", end
// "</DOC>"), so chunks cut just after such a byte start from state 0; every
// thread records where each matcher, run from its chunk start, completes a tag
// (both tags leave the other matcher at state 0 too, so at every mode switch the
// whole-file reader and these independent scans agree), and one serial pass
// alternates start / end detections exactly as the reader does.  Bytes between
// '<'s are skipped by memchr: a state > 0 needs a '<' since the last reset.
// (or_cpuopt_split_records exports it; the tests hold it to or_split_records.)
struct TagHits {
  std::vector<uint64_t> st, en;  // start-tag first bytes; end-tag byte after '>'
};
static inline bool tag_byte(uint8_t c) {
  return c == '<' || c == '/' || c == 'D' || c == 'O' || c == 'C' || c == '>';
}
static void scan_tags(const uint8_t *b, size_t n, size_t a, size_t e, TagHits *h) {
  static const char S[] = "<DOC>", E[] = "</DOC>";
  size_t p = a;
  while (p < n) {
    const uint8_t *q = (const uint8_t *)memchr(b + p, '<', n - p);
    if (!q) break;
    p = (size_t)(q - b);
    if (p >= e) break;  // a tag starting at or past e belongs to the next chunk
    // both matchers from state 0 at this '<' until both are back at 0
    int is = 0, ie = 0;
    size_t x = p;
    do {
      const uint8_t c = b[x];
      if (c == (uint8_t)S[is]) {
        if (++is == 5) {
          h->st.push_back(x + 1 - 5);
          is = 0;
        }
      } else {
        is = 0;
      }
      if (c == (uint8_t)E[ie]) {
        if (++ie == 6) {
          h->en.push_back(x + 1);
          ie = 0;
        }
      } else {
        ie = 0;
      }
      x++;
    } while (x < n && (is | ie));
    p = x;
  }
}
std::vector<std::pair<uint64_t, uint64_t>> records(const uint8_t *b, size_t n) {
  const int T = std::max(1, std::min(omp_get_max_threads(), (int)(n >> 20) + 1));
  std::vector<size_t> cut((size_t)T + 1, n);
  cut[0] = 0;
  for (int t = 1; t < T; t++) {
    size_t c = n / (size_t)T * (size_t)t;
    while (c < n && (c == 0 || tag_byte(b[c - 1]))) c++;  // just after a byte that resets both matchers
    cut[(size_t)t] = std::max(c, cut[(size_t)t - 1]);
  }
  std::vector<TagHits> hits((size_t)T);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < T; t++) scan_tags(b, n, cut[(size_t)t], cut[(size_t)t + 1], &hits[(size_t)t]);
  // the reader: a start tag, then the first end tag completed after it, ...
  std::vector<std::pair<uint64_t, uint64_t>> out;
  size_t ti = 0, si = 0, tj = 0, ej = 0;
  uint64_t pos = 0;
  for (;;) {
    // first start tag beginning at or after pos
    uint64_t rs = UINT64_MAX;
    while (ti < (size_t)T) {
      if (si < hits[ti].st.size()) {
        if (hits[ti].st[si] >= pos) {
          rs = hits[ti].st[si];
          break;
        }
        si++;
      } else {
        ti++;
        si = 0;
      }
    }
    if (rs == UINT64_MAX) break;
    // first end tag whose first byte follows the start tag
    uint64_t re = UINT64_MAX;
    while (tj < (size_t)T) {
      if (ej < hits[tj].en.size()) {
        if (hits[tj].en[ej] - 6 >= rs + 5) {
          re = hits[tj].en[ej];
          break;
        }
        ej++;
      } else {
        tj++;
        ej = 0;
      }
    }
    if (re == UINT64_MAX) break;  // unterminated: the reader drops it
    out.emplace_back(rs, re - rs);
    pos = re;
  }
  return out;
}

int jcmp(const u16s &a, const u16s &b) {
  const size_t m = std::min(a.size(), b.size());
  for (size_t i = 0; i < m; i++)
    if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  return (int)a.size() - (int)b.size();
}

// TagTokenizer split bytes (TagTokenizer.java:73-95): 0..32 and ;"&/:!#?$%()@^*+-,=><[]{}|`~_
struct SplitTab {
  bool t[256];
  SplitTab() {
    for (int c = 0; c < 256; c++) t[c] = c <= 32 || (c < 128 && strchr(";\"&/:!#?$%()@^*+-,=><[]{}|`~_", c) != nullptr);
  }
};
const SplitTab kSplit;
inline bool split_byte(uint8_t c) { return kSplit.t[c]; }
// span end (inclusive) of the markup at '<' p of a simple record (sme_build.hip lt_span_end)
int64_t lt_end(const uint8_t *t, int64_t n, int64_t p) {
  if (p + 1 >= n) return n;
  const uint8_t c = t[p + 1];
  if (c == '!' && p + 3 < n && t[p + 2] == '-' && t[p + 3] == '-') {
    for (int64_t i = p + 1; i + 2 < n; i++)
      if (t[i] == '-' && t[i + 1] == '-' && t[i + 2] == '>') return i + 2;
    return n;
  }
  if (c == '?') {
    for (int64_t i = p + 1; i + 1 < n; i++)
      if (t[i] == '?' && t[i + 1] == '>') return i + 1;
    return n;
  }
  for (int64_t i = p + (c == '/' ? 2 : 1); i < n; i++)
    if (t[i] == '>') return i;
  return n;
}
// entity span end: '&' [a-z0-9#]* ';' (TagTokenizer.onAmpersand 644-662); p if none
int64_t amp_end(const uint8_t *t, int64_t n, int64_t p) {
  for (int64_t i = p + 1; i < n; i++) {
    const uint8_t d = t[i];
    if ((d >= 'a' && d <= 'z') || (d >= '0' && d <= '9') || d == '#') continue;
    return d == ';' ? i : p;
  }
  return p;
}
// every '<' of the record is markup the byte-level path reproduces exactly
// (sme_build.hip lt_simple: terminated, no '<' inside, begin tags without space /
// non-ASCII before '>', not script / style)
bool simple_record(const uint8_t *t, int64_t n) {
  for (const uint8_t *q = (const uint8_t *)memchr(t, '<', (size_t)n); q;
       q = (const uint8_t *)memchr(q + 1, '<', (size_t)(t + n - q - 1))) {
    const int64_t p = q - t;
    if (p + 1 >= n) return false;
    const uint8_t c = t[p + 1];
    if (c == '/' || c == '!' || c == '?') {
      int64_t e;
      if (c == '/') {
        e = n;
        for (int64_t i = p + 2; i < n; i++)
          if (t[i] == '>') {
            e = i;
            break;
          }
      } else if (c == '!' && !(p + 3 < n && t[p + 2] == '-' && t[p + 3] == '-')) {
        e = n;
        for (int64_t i = p + 1; i < n; i++)
          if (t[i] == '>') {
            e = i;
            break;
          }
      } else {
        e = lt_end(t, n, p);
      }
      if (e >= n) return false;
      for (int64_t i = p + 1; i <= e; i++)
        if (t[i] == '<') return false;
      continue;
    }
    int64_t i = p + 1;
    for (; i < n; i++) {
      const uint8_t x = t[i];
      if (x == '>') break;
      if (x == ' ' || x >= 0x80 || x == '<') return false;
    }
    if (i >= n) return false;
    const int64_t l = i - (p + 1);
    auto lc = [&](int64_t k) { const uint8_t x = t[p + 1 + k]; return (x >= 'A' && x <= 'Z') ? x + 32 : x; };
    if (l == 6 && lc(0) == 's' && lc(1) == 'c' && lc(2) == 'r' && lc(3) == 'i' && lc(4) == 'p' && lc(5) == 't')
      return false;
    if (l == 5 && lc(0) == 's' && lc(1) == 't' && lc(2) == 'y' && lc(3) == 'l' && lc(4) == 'e') return false;
  }
  return true;
}

// open-addressing table of distinct raw tokens (byte strings): lookup returns the
// token's id (insertion order); lp / ll hold each id's bytes.  Entries carry the
// first 16 bytes inline (no token byte is 0, so zero padding is unambiguous):
// tokens of <= 16 bytes compare without touching the text
struct RawTab {
  struct E {
    uint64_t h;  // hash | 1; 0 = empty
    uint64_t w0, w1;
    int32_t len, id;  // (a long token's bytes: lp[id])
  };
  std::vector<E> e;
  std::vector<const uint8_t *> lp;
  std::vector<int32_t> ll;
  std::vector<uint64_t> lh;  // each id's hash (the parallel merge's shard key)
  uint64_t mask = 0;
  RawTab() { rehash(1 << 14); }
  static inline void head(const uint8_t *s, int64_t l, uint64_t *w0, uint64_t *w1) {
    uint64_t a = 0, b = 0;
    if (l >= 16) {
      memcpy(&a, s, 8);
      memcpy(&b, s + 8, 8);
    } else if (l >= 8) {
      memcpy(&a, s, 8);
      memcpy(&b, s + 8, (size_t)(l - 8));
    } else {
      memcpy(&a, s, (size_t)l);
    }
    *w0 = a;
    *w1 = b;
  }
  static inline uint64_t hash(const uint8_t *s, int64_t l, uint64_t w0, uint64_t w1) {
    uint64_t x = (0x9E3779B97F4A7C15ull ^ (uint64_t)l ^ w0) * 0xFF51AFD7ED558CCDull;
    x = (x ^ (x >> 32) ^ w1) * 0xC4CEB9FE1A85EC53ull;
    for (int64_t i = 16; i < l; i += 8) {
      uint64_t w = 0;
      memcpy(&w, s + i, (size_t)std::min<int64_t>(8, l - i));
      x = (x ^ (x >> 29) ^ w) * 0xFF51AFD7ED558CCDull;
    }
    x ^= x >> 29;
    return x | 1ull;
  }
  void rehash(uint64_t cap) {
    std::vector<E> o(cap, E{0, 0, 0, 0, 0});
    for (const E &x : e) {
      if (!x.h) continue;
      uint64_t s = x.h & (cap - 1);
      while (o[s].h) s = (s + 1) & (cap - 1);
      o[s] = x;
    }
    e.swap(o);
    mask = cap - 1;
  }
  inline int32_t find_or_add(const uint8_t *s, int64_t l, uint64_t x, uint64_t w0, uint64_t w1) {
    uint64_t i = x & mask;
    while (e[i].h) {
      const E &q = e[i];
      if (q.h == x && q.len == l && q.w0 == w0 && q.w1 == w1 &&
          (l <= 16 || memcmp(lp[(size_t)q.id] + 16, s + 16, (size_t)(l - 16)) == 0))
        return q.id;
      i = (i + 1) & mask;
    }
    const int32_t id = (int32_t)lp.size();
    lp.push_back(s);
    ll.push_back((int32_t)l);
    lh.push_back(x);
    e[i] = E{x, w0, w1, (int32_t)l, id};
    if (2 * lp.size() > mask + 1) rehash(2 * (mask + 1));
    return id;
  }
  int32_t lookup(const uint8_t *s, int64_t l) {
    uint64_t w0, w1;
    head(s, l, &w0, &w1);
    return find_or_add(s, l, hash(s, l, w0, w1), w0, w1);
  }
};

// raw-token bytes of the normalize fast path: ASCII letters, digits, apostrophe
struct AlnumApoTab {
  bool t[256];
  AlnumApoTab() {
    for (int c = 0; c < 256; c++)
      t[c] = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '\'';
  }
};
const AlnumApoTab kAlnumApo;

// the stopword list (GalagoTokenizer's, oracle_tok.c) as an open-addressing set
// of ASCII words of <= 16 units keyed by their bytes (every stopword is ASCII
// and shorter; checked when the table is built)
struct StopTab {
  struct E {
    uint64_t w0, w1;
    int32_t len;
  };
  std::vector<E> e;
  uint64_t mask = 0;
  static uint64_t h(uint64_t w0, uint64_t w1, int32_t n) {
    uint64_t x = (w0 ^ 0x9E3779B97F4A7C15ull ^ (uint64_t)n) * 0xFF51AFD7ED558CCDull;
    x = (x ^ (x >> 31) ^ w1) * 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 29);
  }
  static void pack(const uint16_t *w, int32_t n, uint64_t *w0, uint64_t *w1) {
    uint64_t a = 0, b = 0;
    for (int32_t i = 0; i < n && i < 8; i++) a |= (uint64_t)(uint8_t)w[i] << (8 * i);
    for (int32_t i = 8; i < n; i++) b |= (uint64_t)(uint8_t)w[i] << (8 * (i - 8));
    *w0 = a;
    *w1 = b;
  }
  StopTab() {
    const int cnt = or_stopword_count();
    e.assign(1024, E{0, 0, 0});
    while (e.size() < (size_t)cnt * 4) e.resize(e.size() * 2);
    mask = e.size() - 1;
    for (int i = 0; i < cnt; i++) {
      const char *s = or_stopword(i);
      const int32_t n = (int32_t)strlen(s);
      uint16_t w[16];
      if (n > 16 || n == 0) abort();  // (never: the list is short ASCII words)
      for (int32_t k = 0; k < n; k++) {
        if ((unsigned char)s[k] >= 0x80) abort();
        w[k] = (uint8_t)s[k];
      }
      uint64_t w0, w1;
      pack(w, n, &w0, &w1);
      uint64_t j = h(w0, w1, n) & mask;
      while (e[j].len) j = (j + 1) & mask;
      e[j] = E{w0, w1, n};
    }
  }
  // w: ASCII units
  bool has(const uint16_t *w, int32_t n) const {
    if (n > 16) return false;
    uint64_t w0, w1;
    pack(w, n, &w0, &w1);
    for (uint64_t j = h(w0, w1, n) & mask; e[j].len; j = (j + 1) & mask)
      if (e[j].len == n && e[j].w0 == w0 && e[j].w1 == w1) return true;
    return false;
  }
};
const StopTab &stop_tab() {
  static const StopTab t;
  return t;
}

// bump allocator of UTF-16 units (pointers stay valid until it is destroyed)
struct Arena {
  std::vector<std::unique_ptr<char16_t[]>> blk;
  size_t used = 0, cap = 0;
  char16_t *take(size_t n) {
    if (used + n > cap) {
      cap = std::max<size_t>(n, (size_t)1 << 20);
      blk.emplace_back(new char16_t[cap]);
      used = 0;
    }
    char16_t *p = blk.back().get() + used;
    used += n;
    return p;
  }
};

}  // namespace

extern "C" {

/* The parallel record split (tests: equal to or_split_records). */
int or_cpuopt_split_records(const uint8_t *b, size_t n, uint64_t *off, uint64_t *len, int cap) {
  const auto r = records(b, n);
  for (size_t i = 0; i < r.size() && i < (size_t)cap; i++) {
    off[i] = r[i].first;
    len[i] = r[i].second;
  }
  return (int)r.size();
}

/* Build from a host corpus; mapping = TrecDocnoMapping file bytes.  threads <= 0:
 * omp default.  Returns NULL on a record the reference rejects (no </DOCNO>). */
void *or_cpuopt_build(const uint8_t *corpus, size_t n, const uint8_t *map, size_t map_len, int threads) {
  if (threads > 0) omp_set_num_threads(threads);
  const double t0 = omp_get_wtime();
  // mapping {"", docids...} as UTF-16 (modified UTF-8 in the file; ASCII docids are the same bytes)
  std::vector<u16s> ids(1);
  {
    if (map_len < 4) return nullptr;
    const int32_t cnt = (int32_t)(((uint32_t)map[0] << 24) | ((uint32_t)map[1] << 16) | ((uint32_t)map[2] << 8) | map[3]);
    size_t p = 4;
    for (int32_t i = 0; i < cnt; i++) {
      const size_t l = ((size_t)map[p] << 8) | map[p + 1];
      p += 2;
      u16s s;
      size_t q = p;
      while (q < p + l) {  // DataInput.readUTF
        const unsigned c = map[q];
        if (c < 0x80) {
          s.push_back((char16_t)c);
          q++;
        } else if ((c & 0xE0) == 0xC0) {
          s.push_back((char16_t)(((c & 0x1F) << 6) | (map[q + 1] & 0x3F)));
          q += 2;
        } else {
          s.push_back((char16_t)(((c & 0x0F) << 12) | ((map[q + 1] & 0x3F) << 6) | (map[q + 2] & 0x3F)));
          q += 3;
        }
      }
      ids.push_back(std::move(s));
      p += l;
    }
  }
  std::unordered_set<u16s, U16Hash> stop;
  for (int i = 0; i < or_stopword_count(); i++) {
    const char *w = or_stopword(i);
    stop.insert(u16s(w, w + strlen(w)));
  }
  const auto recs = records(corpus, n);
  const int64_t nR = (int64_t)recs.size();
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "records", omp_get_wtime() - t0);
  // Three phases, no locks; every DISTINCT raw token is normalized, stop-filtered
  // and stemmed once (T13):
  //  1. per record (threads): docno; raw tokens by the byte-level TagTokenizer
  //     into the thread's table of distinct raw tokens (local ids per record);
  //     records of complex markup through the oracle's TagTokenizer (terms)
  //  2. the threads' distinct raw tokens merged into one table, each normalized
  //     once (in parallel); the vocabulary = the sorted distinct outputs
  //  3. per record (threads): local raw ids -> term ids -> tf
  const int nthr = omp_get_max_threads();
  std::vector<int32_t> rdocno((size_t)nR);
  // a simple record's local raw ids: [rbeg[r], rbeg[r] + rcnt[r]) of its thread's
  // buffer (one flat buffer per thread, no allocation per record)
  std::vector<int64_t> rbeg((size_t)nR, 0);
  std::vector<int32_t> rcnt((size_t)nR, 0);
  std::vector<std::vector<int32_t>> tokb((size_t)nthr);
  std::vector<std::vector<u16s>> rterm((size_t)nR);     // terms (complex records)
  std::vector<int16_t> rthr((size_t)nR);
  std::vector<RawTab> tabs((size_t)nthr);
  int fail = 0;
#pragma omp parallel reduction(| : fail)
  {
    const int me = omp_get_thread_num();
    RawTab &raw = tabs[(size_t)me];
    std::vector<int32_t> &tb = tokb[(size_t)me];
    tb.reserve((size_t)(n / (size_t)nthr / 6 + 1024));
    struct Pend {
      const uint8_t *s;
      int64_t l;
      uint64_t w0, w1, h;
    };
    std::vector<Pend> pend;
    jstr text, st;
    js_init(&text);
    js_init(&st);
    jstr_list toks;
    jl_init(&toks);
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = 0; r < nR; r++) {
      const uint8_t *b = corpus + recs[(size_t)r].first;
      const int64_t len = (int64_t)recs[(size_t)r].second;
      // getDocid: trim(substring(indexOf("<DOCNO>") + 7, indexOf("</DOCNO>", start)));
      // the tags are ASCII, so byte offsets locate the same characters
      u16s docid;
      const uint8_t *a = (const uint8_t *)memmem(b, (size_t)len, "<DOCNO>", 7);
      if (a) {
        const uint8_t *e = (const uint8_t *)memmem(a + 7, (size_t)(b + len - (a + 7)), "</DOCNO>", 8);
        if (!e) {
          fail |= 1;
          continue;
        }
        const uint8_t *b0 = a + 7, *e0 = e;
        while (b0 < e0 && *b0 <= 0x20) b0++;
        while (e0 > b0 && e0[-1] <= 0x20) e0--;
        utf8_to_utf16(b0, (size_t)(e0 - b0), &text);
        docid.assign((const char16_t *)text.p, (size_t)text.n);
      }
      int lo = 0, hi = (int)ids.size() - 1, dn = 0;  // Arrays.binarySearch
      bool found = false;
      while (lo <= hi) {
        const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
        const int c = jcmp(ids[(size_t)mid], docid);
        if (c < 0) lo = mid + 1;
        else if (c > 0) hi = mid - 1;
        else {
          dn = mid;
          found = true;
          break;
        }
      }
      rdocno[(size_t)r] = found ? dn : -(lo + 1);
      rthr[(size_t)r] = (int16_t)me;
      if (simple_record(b, len)) {
        // byte-level TagTokenizer (the device's fast path, sme_build.hip k_tok_fast):
        // raw tokens = maximal runs of non-split bytes starting outside every
        // tag / comment / PI / entity span
        // two passes over the record's tokens: bounds, head words and hashes with
        // the home slots prefetched, then the table lookups (the slots of the
        // record's tail tokens are in flight together instead of one miss each)
        pend.clear();
        int64_t i = 0;
        while (i < len) {
          const uint8_t c = b[i];
          if (c == '<') {
            i = lt_end(b, len, i) + 1;
            continue;
          }
          if (c == '&') {
            i = amp_end(b, len, i) + 1;
            continue;
          }
          if (split_byte(c)) {
            i++;
            continue;
          }
          int64_t j = i + 1;
          while (j < len && !split_byte(b[j])) j++;
          Pend q;
          q.s = b + i;
          q.l = j - i;
          RawTab::head(q.s, q.l, &q.w0, &q.w1);
          q.h = RawTab::hash(q.s, q.l, q.w0, q.w1);
          __builtin_prefetch(&raw.e[q.h & raw.mask]);
          pend.push_back(q);
          i = j;
        }
        rbeg[(size_t)r] = (int64_t)tb.size();
        rcnt[(size_t)r] = (int32_t)pend.size();
        for (size_t k = 0; k < pend.size(); k++)
          tb.push_back(raw.find_or_add(pend[k].s, pend[k].l, pend[k].h, pend[k].w0, pend[k].w1));
      } else {
        // complex markup: the oracle's TagTokenizer over the decoded record
        utf8_to_utf16(b, (size_t)len, &text);
        for (int i = 0; i < toks.n; i++) js_free(&toks.v[i]);
        toks.n = 0;
        or_tag_tokenize(text.p, text.n, &toks);
        for (int i = 0; i < toks.n; i++) {
          u16s w((const char16_t *)toks.v[i].p, (size_t)toks.v[i].n);
          if (stop.count(w)) continue;
          or_stem_js(toks.v[i].p, toks.v[i].n, &st);
          rterm[(size_t)r].emplace_back((const char16_t *)st.p, (size_t)st.n);
        }
      }
    }
    jl_free(&toks);
    js_free(&text);
    js_free(&st);
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "tokens", omp_get_wtime() - t0);
  if (fail) return nullptr;
  // 2. one table of the distinct raw tokens (local id -> global id per thread):
  // the threads' tables merged in parallel, shard s (hash bits) by one thread,
  // global id = shard base + id inside the shard
  constexpr int kShards = 256;
  std::vector<RawTab> shard((size_t)kShards);
  std::vector<std::vector<int32_t>> lmap((size_t)nthr);
  for (int t = 0; t < nthr; t++) lmap[(size_t)t].resize(tabs[(size_t)t].lp.size());
  // every thread's ids bucketed by shard (one pass per table), so a shard visits
  // only its own entries
  std::vector<std::vector<std::vector<int32_t>>> bucket((size_t)nthr);
#pragma omp parallel for schedule(dynamic, 1)
  for (int t = 0; t < nthr; t++) {
    const RawTab &tb = tabs[(size_t)t];
    auto &b = bucket[(size_t)t];
    b.assign((size_t)kShards, {});
    for (size_t i = 0; i < tb.lp.size(); i++) b[(size_t)((tb.lh[i] >> 56) % kShards)].push_back((int32_t)i);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int sh = 0; sh < kShards; sh++) {
    RawTab &g = shard[(size_t)sh];
    for (int t = 0; t < nthr; t++) {
      const RawTab &tb = tabs[(size_t)t];
      for (const int32_t i : bucket[(size_t)t][(size_t)sh]) {
        uint64_t w0, w1;
        RawTab::head(tb.lp[i], tb.ll[i], &w0, &w1);
        lmap[(size_t)t][i] = g.find_or_add(tb.lp[i], tb.ll[i], tb.lh[i], w0, w1);
      }
    }
  }
  std::vector<int64_t> sbase((size_t)kShards + 1, 0);
  for (int sh = 0; sh < kShards; sh++) sbase[(size_t)sh + 1] = sbase[(size_t)sh] + (int64_t)shard[(size_t)sh].lp.size();
  const int64_t G = sbase[(size_t)kShards];
  struct GTok {
    std::vector<const uint8_t *> lp;
    std::vector<int32_t> ll;
  } glob;
  glob.lp.resize((size_t)G);
  glob.ll.resize((size_t)G);
#pragma omp parallel for schedule(dynamic, 1)
  for (int sh = 0; sh < kShards; sh++)
    for (size_t i = 0; i < shard[(size_t)sh].lp.size(); i++) {
      glob.lp[(size_t)sbase[(size_t)sh] + i] = shard[(size_t)sh].lp[i];
      glob.ll[(size_t)sbase[(size_t)sh] + i] = shard[(size_t)sh].ll[i];
    }
#pragma omp parallel for schedule(dynamic, 1)
  for (int t = 0; t < nthr; t++) {
    const RawTab &tb = tabs[(size_t)t];
    for (size_t i = 0; i < tb.lp.size(); i++) lmap[(size_t)t][i] += (int32_t)sbase[(size_t)((tb.lh[i] >> 56) % kShards)];
  }
  std::vector<RawTab>().swap(shard);
  std::vector<RawTab>().swap(tabs);
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f (%lld distinct raw tokens)\n", "merge", omp_get_wtime() - t0, (long long)G);
  // processContent of each distinct raw token, once (parallel).  A raw token of
  // ASCII letters, digits and apostrophes is one TagTokenizer token whose fix
  // (simpleFix; complexFix = simpleFix + toLowerCase on ASCII) lowercases it and
  // drops the apostrophes (TagTokenizer.java:403-476); other raw tokens go through
  // the oracle's TagTokenizer.  Outputs land in per-thread arenas as runs of
  // (length, units): token g has gn[g] outputs starting at gp[g].
  const StopTab &stab = stop_tab();
  std::vector<int32_t> gn((size_t)G, 0);
  std::vector<const char16_t *> gp((size_t)G, nullptr);
  std::vector<Arena> arena((size_t)nthr);
#pragma omp parallel
  {
    Arena &ar = arena[(size_t)omp_get_thread_num()];
    jstr text, st;
    js_init(&text);
    js_init(&st);
    jstr_list toks;
    jl_init(&toks);
    std::vector<u16s> outs;
    uint16_t w16[128];
#pragma omp for schedule(dynamic, 1024)
    for (int64_t g = 0; g < G; g++) {
      const uint8_t *s = glob.lp[(size_t)g];
      const int32_t l = glob.ll[(size_t)g];
      bool fast = l < 100;
      for (int32_t i = 0; fast && i < l; i++) fast = kAlnumApo.t[s[i]];
      if (fast) {
        int32_t m = 0;
        for (int32_t i = 0; i < l; i++) {
          const uint8_t c = s[i];
          if (c == '\'') continue;
          w16[m++] = (uint16_t)((c >= 'A' && c <= 'Z') ? c + 32 : c);
        }
        if (m == 0 || stab.has(w16, m)) continue;  // (add_token drops an empty token)
        or_stem_js(w16, m, &st);
        char16_t *o = ar.take((size_t)st.n + 1);
        o[0] = (char16_t)st.n;
        memcpy(o + 1, st.p, (size_t)st.n * sizeof(uint16_t));
        gn[(size_t)g] = 1;
        gp[(size_t)g] = o;
        continue;
      }
      utf8_to_utf16(s, (size_t)l, &text);
      for (int i = 0; i < toks.n; i++) js_free(&toks.v[i]);
      toks.n = 0;
      or_tag_tokenize(text.p, text.n, &toks);
      outs.clear();
      size_t tot = 0;
      for (int i = 0; i < toks.n; i++) {
        u16s w((const char16_t *)toks.v[i].p, (size_t)toks.v[i].n);
        if (stop.count(w)) continue;
        or_stem_js(toks.v[i].p, toks.v[i].n, &st);
        outs.emplace_back((const char16_t *)st.p, (size_t)st.n);
        tot += (size_t)st.n + 1;
      }
      if (outs.empty()) continue;
      char16_t *o = ar.take(tot);
      gp[(size_t)g] = o;
      gn[(size_t)g] = (int32_t)outs.size();
      for (const u16s &w : outs) {
        o[0] = (char16_t)w.size();  // (a token is < 100 units: add_token)
        memcpy(o + 1, w.data(), w.size() * sizeof(char16_t));
        o += w.size() + 1;
      }
    }
    jl_free(&toks);
    js_free(&text);
    js_free(&st);
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "normalize", omp_get_wtime() - t0);
  // vocabulary in String.compareTo order (UTF-16 unit order): the sorted distinct
  // outputs.  Keys: units 0-3 and 4-7 (zero padded; no term unit is 0, a split
  // character), so strings of <= 8 units compare by key alone
  struct TK {
    uint64_t k0, k1;
    const char16_t *p;
    int32_t len;
    int32_t slot;  // the output's place in gterm (-1: a complex record's term)
  };
  auto tkey = [](const char16_t *p, int32_t n) {
    TK t{0, 0, p, n, -1};
    for (int32_t i = 0; i < 8; i++) {
      const uint64_t u = i < n ? (uint64_t)(uint16_t)p[i] : 0ull;
      if (i < 4) t.k0 = (t.k0 << 16) | u;
      else t.k1 = (t.k1 << 16) | u;
    }
    return t;
  };
  auto tless = [](const TK &x, const TK &y) {
    if (x.k0 != y.k0) return x.k0 < y.k0;
    if (x.k1 != y.k1) return x.k1 < y.k1;
    if (x.len <= 8 && y.len <= 8) return x.len < y.len;
    return std::lexicographical_compare(x.p + 8, x.p + x.len, y.p + 8, y.p + y.len);  // (equal keys: both >= 8 units)
  };
  auto teq = [](const TK &x, const TK &y) {
    return x.k0 == y.k0 && x.k1 == y.k1 && x.len == y.len &&
           (x.len <= 8 || memcmp(x.p + 8, y.p + 8, (size_t)(x.len - 8) * sizeof(char16_t)) == 0);
  };
  // every distinct raw token's outputs keyed in parallel (slot = its place in
  // gterm), the complex records' terms after them; after the sort each output's
  // term id is its run's rank (no search per output)
  std::vector<int32_t> go0((size_t)G + 1, 0);
  for (int64_t g = 0; g < G; g++) go0[(size_t)g + 1] = go0[(size_t)g] + gn[(size_t)g];
  const size_t nout = (size_t)go0[(size_t)G];
  size_t nrt = 0;
  for (auto &v : rterm) nrt += v.size();
  std::vector<TK> keyed(nout + nrt);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t g = 0; g < G; g++) {
    const char16_t *o = gp[(size_t)g];
    for (int32_t k = 0; k < gn[(size_t)g]; k++) {
      TK t = tkey(o + 1, (int32_t)o[0]);
      t.slot = go0[(size_t)g] + k;
      keyed[(size_t)t.slot] = t;
      o += (size_t)o[0] + 1;
    }
  }
  {
    size_t i = nout;
    for (auto &v : rterm)
      for (auto &w : v) keyed[i++] = tkey(w.data(), (int32_t)w.size());
  }
  __gnu_parallel::sort(keyed.begin(), keyed.end(), tless);
  std::vector<int32_t> gterm(nout);
  std::vector<size_t> first;  // first sorted entry of each distinct term
  for (size_t i = 0; i < keyed.size(); i++) {
    if (i == 0 || !teq(keyed[i], keyed[i - 1])) first.push_back(i);
    if (keyed[i].slot >= 0) gterm[(size_t)keyed[i].slot] = (int32_t)(first.size() - 1);
  }
  const int64_t V = (int64_t)first.size();
  std::vector<TK> vk((size_t)V);
  std::vector<int64_t> toff((size_t)V + 1, 0);
  for (int64_t i = 0; i < V; i++) {
    vk[(size_t)i] = keyed[first[(size_t)i]];
    toff[(size_t)i + 1] = toff[(size_t)i] + vk[(size_t)i].len;
  }
  std::vector<char16_t> tchars((size_t)toff[(size_t)V]);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < V; i++)
    memcpy(tchars.data() + toff[(size_t)i], vk[(size_t)i].p, (size_t)vk[(size_t)i].len * sizeof(char16_t));
  std::vector<TK>().swap(keyed);
  auto term_of = [&](const u16s &w) {  // (complex records' terms)
    const TK k = tkey(w.data(), (int32_t)w.size());
    return (int32_t)(std::lower_bound(vk.begin(), vk.end(), k, tless) - vk.begin());
  };
  // per thread: local raw id -> its single term id (>= 0), no term (-1) or the
  // first of several at gterm[-v - 2] (one random access per token below)
  std::vector<std::vector<int32_t>> ltm((size_t)nthr);
#pragma omp parallel for schedule(dynamic, 1)
  for (int t = 0; t < nthr; t++) {
    const std::vector<int32_t> &lm = lmap[(size_t)t];
    std::vector<int32_t> &o = ltm[(size_t)t];
    o.resize(lm.size());
    for (size_t i = 0; i < lm.size(); i++) {
      const int32_t g = lm[i], a = go0[(size_t)g], b = go0[(size_t)g + 1];
      o[i] = b - a == 1 ? gterm[(size_t)a] : (b == a ? -1 : -2 - g);
    }
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "vocab_sort", omp_get_wtime() - t0);
  // 3. per record: term ids -> tf
  std::vector<std::vector<std::pair<int32_t, int32_t>>> rid((size_t)nR);
#pragma omp parallel
  {
    std::vector<int32_t> tfc((size_t)V, 0), touched;
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = 0; r < nR; r++) {
      touched.clear();
      auto count = [&](int32_t id) {
        if (tfc[(size_t)id]++ == 0) touched.push_back(id);
      };
      const std::vector<int32_t> &lm = ltm[(size_t)rthr[(size_t)r]];
      const int32_t *rt = tokb[(size_t)rthr[(size_t)r]].data() + rbeg[(size_t)r];
      for (int32_t i = 0; i < rcnt[(size_t)r]; i++) {
        const int32_t x = rt[i];
        const int32_t v = lm[(size_t)x];
        if (v >= 0) {
          count(v);
        } else if (v <= -2) {
          const int32_t g = -v - 2;
          for (int32_t k = go0[(size_t)g]; k < go0[(size_t)g + 1]; k++) count(gterm[(size_t)k]);
        }
      }
      for (const u16s &w : rterm[(size_t)r]) count(term_of(w));
      auto &out = rid[(size_t)r];
      out.reserve(touched.size());
      for (int32_t id : touched) {
        out.emplace_back(id, tfc[(size_t)id]);
        tfc[(size_t)id] = 0;
      }
    }
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "lmap", omp_get_wtime() - t0);
  // records in docno order (the reducer sorts postings by docno; stable, so equal
  // docnos keep input order before they merge)
  std::vector<int64_t> order((size_t)nR);
  for (int64_t r = 0; r < nR; r++) order[(size_t)r] = r;
  if (!std::is_sorted(rdocno.begin(), rdocno.end()))  // (file order is usually docno order already)
    std::stable_sort(order.begin(), order.end(),
                     [&](int64_t a, int64_t b) { return rdocno[(size_t)a] < rdocno[(size_t)b]; });
  // counting sort by term, in docno order: the docno-ordered records cut into one
  // contiguous chunk per thread; per-thread term counts, a prefix over (term,
  // thread), then every thread scatters its chunk (the chunks' order is docno order)
  std::vector<int64_t> start((size_t)V + 1, 0);
  std::vector<std::vector<int64_t>> tcnt((size_t)nthr);
  auto chunk_of = [&](int t) { return std::make_pair(nR * t / nthr, nR * (t + 1) / nthr); };
#pragma omp parallel num_threads(nthr)
  {
    const int t = omp_get_thread_num();
    std::vector<int64_t> &c = tcnt[(size_t)t];
    c.assign((size_t)V, 0);
    const auto ch = chunk_of(t);
    for (int64_t i = ch.first; i < ch.second; i++)
      for (auto &p : rid[(size_t)order[(size_t)i]]) c[(size_t)p.first]++;
  }
  {
    int64_t acc = 0;
    for (int64_t v = 0; v < V; v++) {
      start[(size_t)v] = acc;
      for (int t = 0; t < nthr; t++) {
        const int64_t n_ = tcnt[(size_t)t][(size_t)v];
        tcnt[(size_t)t][(size_t)v] = acc;  // this thread's first slot of term v
        acc += n_;
      }
    }
    start[(size_t)V] = acc;
  }
  const int64_t Pm = start[(size_t)V];
  std::vector<int32_t> pd((size_t)Pm), pf((size_t)Pm);
#pragma omp parallel num_threads(nthr)
  {
    const int t = omp_get_thread_num();
    std::vector<int64_t> &cur = tcnt[(size_t)t];
    const auto ch = chunk_of(t);
    for (int64_t i = ch.first; i < ch.second; i++) {
      const int64_t r = order[(size_t)i];
      for (auto &p : rid[(size_t)r]) {
        const int64_t x = cur[(size_t)p.first]++;
        pd[(size_t)x] = rdocno[(size_t)r];
        pf[(size_t)x] = p.second;
      }
    }
  }
  std::vector<std::vector<int64_t>>().swap(tcnt);
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "scatter", omp_get_wtime() - t0);
  rid.clear();
  rid.shrink_to_fit();
  // per term: merge equal docnos (sum tf), then stable sort by tf desc
  CpuIndex *ix = new CpuIndex();
  ix->N = nR;
  ix->V = V;
  ix->toff = std::move(toff);
  ix->tchars = std::move(tchars);
  std::vector<int64_t> merged((size_t)V, 0);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t t = 0; t < V; t++) {
    const int64_t b = start[(size_t)t], e = start[(size_t)t + 1];
    int64_t w = b;
    for (int64_t i = b; i < e; i++) {
      if (w > b && pd[(size_t)w - 1] == pd[(size_t)i]) {
        pf[(size_t)w - 1] += pf[(size_t)i];
      } else {
        pd[(size_t)w] = pd[(size_t)i];
        pf[(size_t)w] = pf[(size_t)i];
        w++;
      }
    }
    merged[(size_t)t] = w - b;
    std::vector<std::pair<int32_t, int32_t>> tmp;
    tmp.reserve((size_t)(w - b));
    for (int64_t i = b; i < w; i++) tmp.emplace_back(pf[(size_t)i], pd[(size_t)i]);
    std::stable_sort(tmp.begin(), tmp.end(), [](const std::pair<int32_t, int32_t> &x, const std::pair<int32_t, int32_t> &y) {
      return x.first > y.first;
    });
    for (int64_t i = b; i < w; i++) {
      pf[(size_t)i] = tmp[(size_t)(i - b)].first;
      pd[(size_t)i] = tmp[(size_t)(i - b)].second;
    }
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "reduce", omp_get_wtime() - t0);
  ix->off.assign((size_t)V + 1, 0);
  for (int64_t t = 0; t < V; t++) ix->off[(size_t)t + 1] = ix->off[(size_t)t] + merged[(size_t)t];
  ix->P = ix->off[(size_t)V];
  if (ix->P == Pm) {  // no duplicate docnos merged: the lists are in place
    ix->docno = std::move(pd);
    ix->tf = std::move(pf);
    if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "finish", omp_get_wtime() - t0);
    ix->build_s = omp_get_wtime() - t0;
    return ix;
  }
  ix->docno.resize((size_t)ix->P);
  ix->tf.resize((size_t)ix->P);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t t = 0; t < V; t++) {
    const int64_t s = start[(size_t)t];
    for (int64_t i = 0; i < merged[(size_t)t]; i++) {
      ix->docno[(size_t)(ix->off[(size_t)t] + i)] = pd[(size_t)(s + i)];
      ix->tf[(size_t)(ix->off[(size_t)t] + i)] = pf[(size_t)(s + i)];
    }
  }
  if (getenv("SME_CPU_PROF")) fprintf(stderr, "cpuopt %s %.3f\n", "finish", omp_get_wtime() - t0);
  ix->build_s = omp_get_wtime() - t0;
  return ix;
}

void or_cpuopt_free(void *h) { delete (CpuIndex *)h; }

/* An index over given CSR arrays (reduce order, no term strings), so the cpu-opt
 * rank() can be timed over an index too large to build on the CPU inside a bench
 * (bench.py: the GPU-built full-size c2 index, held equal to the oracle's by the
 * parity tests). */
void *or_cpuopt_from_csr(int64_t N, int64_t V, const int64_t *off, const int32_t *docno, const int32_t *tf) {
  CpuIndex *ix = new CpuIndex();
  ix->N = N;
  ix->V = V;
  ix->off.assign(off, off + V + 1);
  ix->P = ix->off[(size_t)V];
  ix->docno.assign(docno, docno + ix->P);
  ix->tf.assign(tf, tf + ix->P);
  return ix;
}

void or_cpuopt_stats(const void *h, int64_t *N, int64_t *V, int64_t *P, double *build_s) {
  const CpuIndex *ix = (const CpuIndex *)h;
  *N = ix->N;
  *V = ix->V;
  *P = ix->P;
  *build_s = ix->build_s;
}

/* CSR (reduce order) and the term strings as UTF-16 units (toff: V + 1) */
void or_cpuopt_csr(const void *h, int64_t *off, int32_t *docno, int32_t *tf, int64_t *toff, uint16_t *tchars) {
  const CpuIndex *ix = (const CpuIndex *)h;
  memcpy(off, ix->off.data(), ix->off.size() * sizeof(int64_t));
  memcpy(docno, ix->docno.data(), ix->docno.size() * sizeof(int32_t));
  memcpy(tf, ix->tf.data(), ix->tf.size() * sizeof(int32_t));
  if (ix->toff.empty()) {  // (an index over given CSR arrays: no term strings)
    for (int64_t t = 0; t <= ix->V; t++) toff[t] = 0;
    return;
  }
  memcpy(toff, ix->toff.data(), ix->toff.size() * sizeof(int64_t));
  if (tchars) memcpy(tchars, ix->tchars.data(), ix->tchars.size() * sizeof(uint16_t));
}

/* Batched rank(): term ids (-1 skipped) per query, k results per query (docno
 * -1 / score 0 padding).  idf_mode 0: log10(N / 1), 1: log10(N / df) (int
 * division).  Returns wall seconds. */
double or_cpuopt_query(const void *h, const int32_t *terms, const int64_t *qoff, int nq, int k, int idf_mode,
                       int threads, int32_t *out_d, double *out_s) {
  if (threads > 0) omp_set_num_threads(threads);
  const CpuIndex *ix = (const CpuIndex *)h;
  const double t0 = omp_get_wtime();
  int32_t dmin = INT32_MAX, dmax = INT32_MIN;
  for (int32_t d : ix->docno) {
    dmin = std::min(dmin, d);
    dmax = std::max(dmax, d);
  }
  const int64_t span = ix->P ? (int64_t)dmax - dmin + 1 : 1;
#pragma omp parallel
  {
    std::vector<double> acc((size_t)span, 0.0);
    std::vector<uint8_t> hit((size_t)span, 0);
    std::vector<int32_t> touched;
    std::vector<std::pair<double, int32_t>> cand;
#pragma omp for schedule(dynamic, 16)
    for (int q = 0; q < nq; q++) {
      touched.clear();
      for (int64_t i = qoff[q]; i < qoff[q + 1]; i++) {
        const int32_t t = terms[i];
        if (t < 0 || t >= ix->V) continue;
        const int64_t b = ix->off[(size_t)t], e = ix->off[(size_t)t + 1];
        const int64_t df = idf_mode == 0 ? 1 : e - b;
        const double idf = log10((double)(ix->N / df));
        for (int64_t p = b; p < e; p++) {
          const int64_t x = (int64_t)ix->docno[(size_t)p] - dmin;
          const double w = (1.0 + log((double)ix->tf[(size_t)p])) * idf;
          if (hit[(size_t)x]) {
            acc[(size_t)x] += w;
          } else {
            hit[(size_t)x] = 1;
            acc[(size_t)x] = 0.0 + w;
            touched.push_back((int32_t)x);
          }
        }
      }
      cand.clear();
      for (int32_t x : touched) {
        cand.emplace_back(acc[(size_t)x], x + dmin);
        hit[(size_t)x] = 0;
      }
      const size_t kk = std::min((size_t)k, cand.size());
      std::partial_sort(cand.begin(), cand.begin() + (ptrdiff_t)kk, cand.end(),
                        [](const std::pair<double, int32_t> &a, const std::pair<double, int32_t> &b) {
                          return a.first > b.first || (a.first == b.first && a.second < b.second);
                        });
      for (int r = 0; r < k; r++) {
        out_d[(int64_t)q * k + r] = (size_t)r < kk ? cand[(size_t)r].second : -1;
        out_s[(int64_t)q * k + r] = (size_t)r < kk ? cand[(size_t)r].first : 0.0;
      }
    }
  }
  return omp_get_wtime() - t0;
}

}  // extern "C"
