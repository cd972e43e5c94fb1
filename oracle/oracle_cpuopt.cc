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
 *   tokens      GalagoTokenizer.processContent (GalagoTokenizer.java:139-183):
 *               the oracle's TagTokenizer, stopword hash set, per-thread stem cache
 *   postings    MyReducer.reduce (TermKGramDocIndexer.java:168-213): per term
 *               docno asc with duplicate docnos merged, then stable tf desc
 *   terms       TermDF.compareTo order (String.compareTo on UTF-16 units), K = 1
 *   rank()      IntDocVectorsForwardIndex.java:192-223: score += (1 + ln tf) * idf
 *               in query-token order, postings in stored order; score desc,
 *               docno asc
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
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
  std::vector<u16s> terms;           // TermDF order
  std::vector<int64_t> off;          // V + 1
  std::vector<int32_t> docno, tf;    // reduce order: tf desc, docno asc
  double build_s = 0;
};

// readUntilMatch over one split (the oracle's record reader, exported)
std::vector<std::pair<uint64_t, uint64_t>> records(const uint8_t *b, size_t n) {
  int cap = 1024;
  for (;;) {
    std::vector<uint64_t> off((size_t)cap), len((size_t)cap);
    int r = or_split_records(b, n, off.data(), len.data(), cap);
    if (r <= cap) {
      std::vector<std::pair<uint64_t, uint64_t>> out((size_t)r);
      for (int i = 0; i < r; i++) out[(size_t)i] = {off[(size_t)i], len[(size_t)i]};
      return out;
    }
    cap = r;
  }
}

int jcmp(const u16s &a, const u16s &b) {
  const size_t m = std::min(a.size(), b.size());
  for (size_t i = 0; i < m; i++)
    if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  return (int)a.size() - (int)b.size();
}

}  // namespace

extern "C" {

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
  // per record: docno and its (term, tf) pairs (term as string, aggregated)
  std::vector<int32_t> rdocno((size_t)nR);
  std::vector<std::vector<std::pair<u16s, int32_t>>> rterms((size_t)nR);
  int fail = 0;
#pragma omp parallel reduction(| : fail)
  {
    std::unordered_map<u16s, u16s, U16Hash> stem_cache;
    jstr text, st;
    js_init(&text);
    js_init(&st);
    jstr_list toks;
    jl_init(&toks);
    std::unordered_map<u16s, int32_t, U16Hash> tfm;
#pragma omp for schedule(dynamic, 64)
    for (int64_t r = 0; r < nR; r++) {
      utf8_to_utf16(corpus + recs[(size_t)r].first, recs[(size_t)r].second, &text);
      // getDocid: trim(substring(indexOf("<DOCNO>") + 7, indexOf("</DOCNO>", start)))
      static const char16_t O[] = u"<DOCNO>", Cl[] = u"</DOCNO>";
      const u16s doc((const char16_t *)text.p, (size_t)text.n);
      u16s docid;
      const size_t a = doc.find(O);
      if (a != u16s::npos) {
        const size_t e = doc.find(Cl, a);
        if (e == u16s::npos || e < a + 7) {
          fail |= 1;
          continue;
        }
        size_t b0 = a + 7, e0 = e;
        while (b0 < e0 && doc[b0] <= 0x20) b0++;
        while (e0 > b0 && doc[e0 - 1] <= 0x20) e0--;
        docid = doc.substr(b0, e0 - b0);
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
      for (int i = 0; i < toks.n; i++) js_free(&toks.v[i]);
      toks.n = 0;
      or_tag_tokenize(text.p, text.n, &toks);
      tfm.clear();
      for (int i = 0; i < toks.n; i++) {
        u16s w((const char16_t *)toks.v[i].p, (size_t)toks.v[i].n);
        if (stop.count(w)) continue;
        auto it = stem_cache.find(w);
        if (it == stem_cache.end()) {
          or_stem_js(toks.v[i].p, toks.v[i].n, &st);
          it = stem_cache.emplace(w, u16s((const char16_t *)st.p, (size_t)st.n)).first;
        }
        tfm[it->second]++;
      }
      auto &out = rterms[(size_t)r];
      out.reserve(tfm.size());
      for (auto &kv : tfm) out.emplace_back(kv.first, kv.second);
    }
    jl_free(&toks);
    js_free(&text);
    js_free(&st);
  }
  if (fail) return nullptr;
  // vocabulary in String.compareTo order (UTF-16 unit order = u16string operator<)
  std::vector<u16s> vocab;
  {
    const int nt = omp_get_max_threads();
    std::vector<std::unordered_set<u16s, U16Hash>> loc((size_t)nt);
#pragma omp parallel
    {
      auto &s = loc[(size_t)omp_get_thread_num()];
#pragma omp for schedule(static)
      for (int64_t r = 0; r < nR; r++)
        for (auto &p : rterms[(size_t)r]) s.insert(p.first);
    }
    std::unordered_set<u16s, U16Hash> all;
    for (auto &s : loc) all.insert(s.begin(), s.end());
    vocab.assign(all.begin(), all.end());
    std::sort(vocab.begin(), vocab.end());
  }
  const int64_t V = (int64_t)vocab.size();
  std::unordered_map<u16s, int32_t, U16Hash> tid;
  tid.reserve((size_t)V * 2);
  for (int64_t t = 0; t < V; t++) tid.emplace(vocab[(size_t)t], (int32_t)t);
  // pairs by record, records in docno order (the reducer sorts postings by docno;
  // stable, so equal docnos keep input order before they merge)
  std::vector<int64_t> order((size_t)nR);
  for (int64_t r = 0; r < nR; r++) order[(size_t)r] = r;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return rdocno[(size_t)a] < rdocno[(size_t)b]; });
  std::vector<std::vector<std::pair<int32_t, int32_t>>> rid((size_t)nR);  // (term id, tf)
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t r = 0; r < nR; r++) {
    auto &o = rid[(size_t)r];
    o.reserve(rterms[(size_t)r].size());
    for (auto &p : rterms[(size_t)r]) o.emplace_back(tid.at(p.first), p.second);
    rterms[(size_t)r].clear();
    rterms[(size_t)r].shrink_to_fit();
  }
  // counting sort by term: counts, prefix, scatter in docno order
  std::vector<int64_t> cnt((size_t)V + 1, 0);
  for (int64_t r = 0; r < nR; r++)
    for (auto &p : rid[(size_t)r]) cnt[(size_t)p.first]++;
  std::vector<int64_t> start((size_t)V + 1, 0);
  for (int64_t t = 0; t < V; t++) start[(size_t)t + 1] = start[(size_t)t] + cnt[(size_t)t];
  const int64_t Pm = start[(size_t)V];
  std::vector<int32_t> pd((size_t)Pm), pf((size_t)Pm);
  {
    std::vector<int64_t> cur(start.begin(), start.end());
    for (int64_t i = 0; i < nR; i++) {
      const int64_t r = order[(size_t)i];
      for (auto &p : rid[(size_t)r]) {
        const int64_t x = cur[(size_t)p.first]++;
        pd[(size_t)x] = rdocno[(size_t)r];
        pf[(size_t)x] = p.second;
      }
    }
  }
  rid.clear();
  rid.shrink_to_fit();
  // per term: merge equal docnos (sum tf), then stable sort by tf desc
  CpuIndex *ix = new CpuIndex();
  ix->N = nR;
  ix->V = V;
  ix->terms = std::move(vocab);
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
  ix->off.assign((size_t)V + 1, 0);
  for (int64_t t = 0; t < V; t++) ix->off[(size_t)t + 1] = ix->off[(size_t)t] + merged[(size_t)t];
  ix->P = ix->off[(size_t)V];
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
  int64_t o = 0;
  toff[0] = 0;
  for (int64_t t = 0; t < ix->V; t++) {
    const u16s &s = ix->terms[(size_t)t];
    if (tchars) memcpy(tchars + o, s.data(), s.size() * sizeof(uint16_t));
    o += (int64_t)s.size();
    toff[t + 1] = o;
  }
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
