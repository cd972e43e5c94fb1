// sme_build.hip -- device pipeline for the index build (TermKGramDocIndexer job, K = 1)
// and the TF-IDF weight pass.
//
// Reference stages replaced (C/ = ABDURRAHMAN-PA2-3-code/src/):
//   record split      XMLRecordReader.next/readUntilMatch  C/edu/umd/cloud9/collection/XMLInputFormat.java:110-143,173-198
//   docid -> docno    TrecDocument.getDocid (trec/TrecDocument.java:76-89), TrecDocnoMapping.getDocno (:67-69)
//   map               MyMapper.map: processContent + emit  C/sa/edu/kaust/indexing/TermKGramDocIndexer.java:119-160
//   shuffle/sort      [Hadoop] sort by TermDF.compareTo    C/sa/edu/kaust/io/TermDF.java:64-70
//   combine/reduce    MyReducer.reduce                     TermKGramDocIndexer.java:168-213
//   TF-IDF weights    (1 + ln tf) * log10(N / df)          C/sa/edu/kaust/fwindex/IntDocVectorsForwardIndex.java:211
//
// Pipeline (one split = the whole device-resident corpus):
//   K1 k_scan_tags      one pass over the bytes: <DOC>/</DOC> candidates (with the naive
//                       matcher's reset quirk), and every '<' whose tag is not "simple"
//   K1b k_chain/records record spans exactly as the XMLRecordReader alternation yields them
//   K2 k_docno          per record docid -> docno (binary search over the mapping)
//   K3 k_tok_fast       per record, 256 lanes x 16 B: byte-parallel split classes, tag/entity
//                       masking by a block max-scan, raw-token hashing, raw-vocab insert
//      k_tok_slow       records with complex markup: the sequential TagTokenizer, 1 lane/record
//   K4 vocabulary       once per DISTINCT raw token: normalize, stop, stem (T13); dedup the
//                       final terms, rank them in String.compareTo order -> term ids
//   K5 k_agg            per record (docno order): raw slot -> term ids, tf aggregation in an
//                       LDS hash (the combiner), emit (term, docno, tf)
//   K6 sort by term     stable -> postings in docno order per term (+ duplicate-docno merge)
//   K7 weights          w = LUT[tf] * idf(term)  (fp64, no contraction)
//   K8 sort by (term, tf desc)  stable -> MyReducer.reduce's output order
#include <hip/hip_runtime.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <chrono>

#include "sme_internal.hpp"
#include "sme_text.hpp"
#include "sme_trec.hpp"

namespace sme {

// ============================================================================
// K1: tag scan
// ============================================================================

// State of XMLRecordReader.readUntilMatch just before byte p is 0 (so a match
// of `tag` may start at p) iff the chain of partial prefixes ending right
// before p has even length (each active partial prefix makes the next '<'
// a consumed mismatch; XMLInputFormat.java:188-193 resets without re-testing).
template <typename B>
__device__ bool doc_tag_valid(const B &t, int64_t p, const char *tag, int tl) {
  int chain = 0;
  int64_t x = p;
  for (;;) {
    int64_t q = -1;
    for (int j = 1; j < tl; j++) {
      if (x - j < 0) break;
      if (t(x - j) == '<') {
        q = x - j;
        break;
      }
    }
    if (q < 0) break;
    bool pre = true;
    for (int64_t k = 1; k < x - q; k++) pre &= (t(q + k) == (uint8_t)tag[k]);
    if (!pre) break;
    chain++;
    x = q;
  }
  return (chain & 1) == 0;
}

// Span end (inclusive) of the markup starting at '<' p for a record known to be
// "simple" (see lt_simple); -1 if none.
template <typename B>
__device__ __forceinline__ int64_t lt_span_end(const B &t, int64_t n, int64_t p) {
  if (p + 1 >= n) return n;
  uint8_t c = t(p + 1);
  if (c == '/') {
    for (int64_t i = p + 2; i < n; i++)
      if (t(i) == '>') return i;
    return n;
  }
  if (c == '!') {
    if (p + 3 < n && t(p + 2) == '-' && t(p + 3) == '-') {
      for (int64_t i = p + 1; i + 2 < n; i++)
        if (t(i) == '-' && t(i + 1) == '-' && t(i + 2) == '>') return i + 2;
      return n;
    }
    for (int64_t i = p + 1; i < n; i++)
      if (t(i) == '>') return i;
    return n;
  }
  if (c == '?') {
    for (int64_t i = p + 1; i + 1 < n; i++)
      if (t(i) == '?' && t(i + 1) == '>') return i + 1;
    return n;
  }
  for (int64_t i = p + 1; i < n; i++)
    if (t(i) == '>') return i;
  return n;
}

// Is the markup at '<' p one the byte-parallel path reproduces exactly?
// Simple = terminated, no other '<' inside its span, and for begin tags no
// space / non-ASCII byte before the first '>' (no attribute parsing, no Zs
// name end) and a name other than script/style (no ignore mode).
// TagTokenizer.java:179-202 (end), 155-177 (comment, PI), 291-393 (begin).
template <typename B>
__device__ bool lt_simple(const B &t, int64_t n, int64_t p) {
  if (p + 1 >= n) return false;
  uint8_t c = t(p + 1);
  int64_t q;
  if (c == '/' || c == '!' || c == '?') {
    q = lt_span_end(t, n, p);
    if (q >= n) return false;
    for (int64_t i = p + 1; i <= q; i++)
      if (t(i) == '<') return false;
    return true;
  }
  int64_t i = p + 1;
  for (; i < n; i++) {
    uint8_t b = t(i);
    if (b == '>') break;
    if (b == ' ' || b >= 0x80 || b == '<') return false;
  }
  if (i >= n) return false;
  int64_t len = i - (p + 1);
  auto lc = [&](int64_t k) { uint8_t b = t(p + 1 + k); return (b >= 'A' && b <= 'Z') ? b + 32 : b; };
  if (len == 6 && lc(0) == 's' && lc(1) == 'c' && lc(2) == 'r' && lc(3) == 'i' && lc(4) == 'p' && lc(5) == 't')
    return false;
  if (len == 5 && lc(0) == 's' && lc(1) == 't' && lc(2) == 'y' && lc(3) == 'l' && lc(4) == 'e') return false;
  return true;
}

// byte accessors for the markup tests: plain global text, or an LDS stage of it
struct GlobalBytes {
  const uint8_t *t;
  __device__ __forceinline__ uint8_t operator()(int64_t p) const { return t[p]; }
};
struct StagedBytes {
  const uint8_t *stg;  // stage: text [base, base + len)
  const uint8_t *t;
  int64_t base, len;
  __device__ __forceinline__ uint8_t operator()(int64_t p) const {
    const int64_t o = p - base;
    return (o >= 0 && o < len) ? stg[o] : t[p];
  }
};

struct ScanOut {
  uint64_t *S, *E, *C;
  uint32_t capS, capE, capC;
  unsigned long long *cnt;  // [3]
};

// Candidates are collected per workgroup in LDS and flushed with ONE global
// atomic per list per flush: a same-address global atomic per tag (one lane per
// wave, ~6 tags per record) serialises at the memory side (~14 ns each).
constexpr int kScanNT = 256;
constexpr int kScanBuf = 1024;  // per list; overflow beyond it falls back to one global atomic per tag

struct ScanLds {
  uint64_t buf[3][kScanBuf];
  unsigned cnt[3];
  unsigned long long base[3];
};

__device__ __forceinline__ void scan_push(ScanLds &L, const ScanOut &o, int list, uint64_t p) {
  unsigned i = atomicAdd(&L.cnt[list], 1u);
  if (i < (unsigned)kScanBuf) {
    L.buf[list][i] = p;
  } else {  // rare: more '<' in one step than the buffer holds
    uint64_t *dst = list == 0 ? o.S : list == 1 ? o.E : o.C;
    const uint32_t cap = list == 0 ? o.capS : list == 1 ? o.capE : o.capC;
    unsigned long long g = atomicAdd(&o.cnt[list], 1ull);
    if (g < cap) dst[g] = p;
  }
}

template <typename B>
__device__ __forceinline__ void scan_lt(const B &t, int64_t n, int64_t p, const ScanOut &o,
                                        ScanLds &L) {
  if (p + 5 <= n && t(p + 1) == 'D' && t(p + 2) == 'O' && t(p + 3) == 'C' && t(p + 4) == '>') {
    if (doc_tag_valid(t, p, "<DOC>", 5)) scan_push(L, o, 0, (uint64_t)p);
  } else if (p + 6 <= n && t(p + 1) == '/' && t(p + 2) == 'D' && t(p + 3) == 'O' && t(p + 4) == 'C' &&
             t(p + 5) == '>') {
    if (doc_tag_valid(t, p, "</DOC>", 6)) scan_push(L, o, 1, (uint64_t)p);
  }
  if (!lt_simple(t, n, p)) scan_push(L, o, 2, (uint64_t)p);
}

// flush the LDS lists (all threads of the block call this)
__device__ void scan_flush(ScanLds &L, const ScanOut &o) {
  __syncthreads();
  if (threadIdx.x < 3) {
    const unsigned c = min(L.cnt[threadIdx.x], (unsigned)kScanBuf);
    L.base[threadIdx.x] = c ? atomicAdd(&o.cnt[threadIdx.x], (unsigned long long)c) : 0ull;
  }
  __syncthreads();
#pragma unroll
  for (int list = 0; list < 3; list++) {
    const unsigned c = min(L.cnt[list], (unsigned)kScanBuf);
    uint64_t *dst = list == 0 ? o.S : list == 1 ? o.E : o.C;
    const uint64_t cap = list == 0 ? o.capS : list == 1 ? o.capE : o.capC;
    for (unsigned i = threadIdx.x; i < c; i += blockDim.x)
      if (L.base[list] + i < cap) dst[L.base[list] + i] = L.buf[list][i];
  }
  __syncthreads();
  if (threadIdx.x < 3) L.cnt[threadIdx.x] = 0;
  __syncthreads();
}

__device__ __forceinline__ uint32_t has_lt(uint32_t w) {  // bytes equal to '<' (0x3C)
  uint32_t x = w ^ 0x3C3C3C3Cu;
  return (x - 0x01010101u) & ~x & 0x80808080u;
}

// K1a: one streaming pass over the text collects the position of every '<'
// (coalesced 16-byte loads, 4 words per lane per step; positions buffered in LDS
// and flushed with one global atomic per flush).
constexpr int kLtBuf = 2048;
struct LtLds {
  uint64_t buf[kLtBuf];
  unsigned cnt;
  unsigned long long base;
};

__global__ __launch_bounds__(kScanNT) void k_scan_lt(const uint8_t *__restrict__ t, int64_t n, uint64_t *lt,
                                                     uint64_t cap, unsigned long long *nlt) {
  __shared__ LtLds L;
  if (threadIdx.x == 0) L.cnt = 0;
  __syncthreads();
  const int64_t mis = (int64_t)((uintptr_t)t & 15);
  const uint4 *a = reinterpret_cast<const uint4 *>(t - mis);
  const int64_t nv = (n + mis + 15) >> 4;
  constexpr int kU = 4;
  auto flush = [&]() {
    __syncthreads();
    const unsigned c = min(L.cnt, (unsigned)kLtBuf);
    if (threadIdx.x == 0) L.base = c ? atomicAdd(nlt, (unsigned long long)c) : 0ull;
    __syncthreads();
    for (unsigned i = threadIdx.x; i < c; i += kScanNT)
      if (L.base + i < cap) lt[L.base + i] = L.buf[i];
    __syncthreads();
    if (threadIdx.x == 0) L.cnt = 0;
    __syncthreads();
  };
  const int64_t stride = (int64_t)gridDim.x * kScanNT * kU;
  for (int64_t v0 = blockIdx.x * (int64_t)kScanNT * kU; v0 < nv; v0 += stride) {
    uint4 qs[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int64_t v = v0 + u * kScanNT + threadIdx.x;
      qs[u] = v < nv ? a[v] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int64_t v = v0 + u * kScanNT + threadIdx.x;
      const uint32_t w[4] = {qs[u].x, qs[u].y, qs[u].z, qs[u].w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!has_lt(w[k])) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (((w[k] >> (8 * j)) & 0xFF) != '<') continue;
          const int64_t p = 16 * v + 4 * k + j - mis;
          if (p < 0 || p >= n) continue;
          const unsigned i = atomicAdd(&L.cnt, 1u);
          if (i < (unsigned)kLtBuf) {
            L.buf[i] = (uint64_t)p;
          } else {  // more '<' in one step than the buffer holds
            const unsigned long long g = atomicAdd(nlt, 1ull);
            if (g < cap) lt[g] = (uint64_t)p;
          }
        }
      }
    }
    __syncthreads();
    if (L.cnt >= kLtBuf / 2) flush();  // block-uniform (read after the barrier)
  }
  flush();
}

// K1b: one lane per '<': <DOC> / </DOC> with the reader's reset quirk, and the
// "simple markup" test, into the S / E / C lists
__global__ __launch_bounds__(kScanNT) void k_tag_classify(const uint8_t *__restrict__ t, int64_t n,
                                                          const uint64_t *lt, int64_t nlt, ScanOut o) {
  __shared__ ScanLds L;
  if (threadIdx.x < 3) L.cnt[threadIdx.x] = 0;
  __syncthreads();
  const GlobalBytes gb{t};
  for (int64_t i0 = blockIdx.x * (int64_t)kScanNT; i0 < nlt; i0 += (int64_t)gridDim.x * kScanNT) {
    const int64_t i = i0 + threadIdx.x;
    if (i < nlt) scan_lt(gb, n, (int64_t)lt[i], o, L);
    __syncthreads();
    const bool full = L.cnt[0] >= kScanBuf / 2 || L.cnt[1] >= kScanBuf / 2 || L.cnt[2] >= kScanBuf / 2;
    if (full) scan_flush(L, o);
  }
  scan_flush(L, o);
}

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t m = (lo + hi) >> 1;
    if (a[m] < v)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

// next pointers of the start/end alternation (XMLRecordReader.next)
__global__ __launch_bounds__(256) void k_chain(const uint64_t *S, int64_t nS, const uint64_t *E, int64_t nE,
                                               int64_t *e_of, int64_t *next_s, unsigned long long *bad) {
  // the two counts: per thread over its records, then one atomic per block (even
  // one atomic per wave on one address serialised: 137 k of them took 1.7 ms on c5)
  unsigned long long n_end = 0, n_broken = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nS; i += (int64_t)gridDim.x * blockDim.x) {
    // well-formed input alternates start and end tags: end tag i and start tag
    // i + 1 are the answers whenever the neighbours confirm them (two binary
    // searches of 23 dependent steps each per record otherwise: 1.7 ms on c5)
    const uint64_t si = S[i];
    int64_t e;
    if (i < nE && E[i] >= si + 5 && (i == 0 || E[i - 1] < si + 5)) e = i;
    else e = lower_bound_u64(E, nE, si + 5);
    const bool has_end = e < nE;
    bool broken = false;
    if (!has_end) {
      e_of[i] = -1;
      next_s[i] = nS;
    } else {
      e_of[i] = e;
      const uint64_t ve = E[e] + 6;
      int64_t ns;
      if (i + 1 >= nS || S[i + 1] >= ve) ns = i + 1;  // S[i] < ve always (E[e] >= S[i] + 5)
      else ns = lower_bound_u64(S, nS, ve);
      next_s[i] = ns;
      // a start tag inside record i (nested <DOC>) or past the last end tag breaks
      // "records = the start tags that have an end tag": walk the chain instead
      broken = ns != i + 1 && i + 1 < nS;
    }
    n_end += has_end ? 1ull : 0ull;
    n_broken += broken ? 1ull : 0ull;
  }
  __shared__ unsigned long long s_c[2];
  if (threadIdx.x < 2) s_c[threadIdx.x] = 0;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    n_end += __shfl_xor(n_end, o, 64);
    n_broken += __shfl_xor(n_broken, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (n_end) atomicAdd(&s_c[0], n_end);
    if (n_broken) atomicAdd(&s_c[1], n_broken);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_c[0]) atomicAdd(bad + 2, s_c[0]);
    if (s_c[1]) atomicAdd(bad, s_c[1]);
  }
}

// well-formed case: records are S[i] for every i that has an end tag
__global__ void k_records_direct(const uint64_t *S, const uint64_t *E, const int64_t *e_of, int64_t nR,
                                 uint64_t *rs, uint64_t *re) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x) {
    rs[i] = S[i];
    re[i] = E[e_of[i]] + 6;
  }
}

// general case (nested <DOC> inside records): walk the chain
__global__ void k_records_walk(const uint64_t *S, int64_t nS, const uint64_t *E, const int64_t *e_of,
                               const int64_t *next_s, uint64_t *rs, uint64_t *re, unsigned long long *nrec) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t i = 0, r = 0;
  while (i < nS) {
    if (e_of[i] < 0) break;  // no </DOC>: readUntilMatch hits EOF, the reader stops
    rs[r] = S[i];
    re[r] = E[e_of[i]] + 6;
    r++;
    i = next_s[i];
  }
  *nrec = (unsigned long long)r;
}

// ============================================================================
// K2: docid -> docno
// ============================================================================
// Compare mapping entry m (UTF-16) with the UTF-8 byte range b[0..n) decoded
// with replacement (String.compareTo on the decoded docid).
__device__ int cmp_u16_utf8(const uint16_t *m, int64_t mn, const uint8_t *b, int64_t n) {
  int64_t i = 0, k = 0;
  uint16_t u[2];
  while (i < n && k < mn) {
    int nu;
    int used = utf8_step(b, i, n, u, &nu);
    for (int x = 0; x < nu; x++) {
      if (k >= mn) return -1;  // m shorter
      if (m[k] != u[x]) return (int)m[k] - (int)u[x];
      k++;
    }
    i += used;
  }
  if (i < n) return -1;  // m is a proper prefix
  return k < mn ? 1 : 0;
}

// Docid hash table over the mapping (built once when the mapping is loaded, as
// MyMapper.configure loads it once per task): slots hold entry index + 1; a record
// whose docid hashes to an equal entry takes that index, and only a miss (docid not
// in the mapping: the negative insertion point of Arrays.binarySearch) or a mapping
// with duplicate docids falls back to the binary search.
__device__ __forceinline__ uint64_t docid_hash_step(uint64_t h, uint16_t u) { return (h ^ u) * 0x100000001B3ull; }
__device__ __forceinline__ uint64_t docid_hash_fin(uint64_t h) { return fmix64(h) | 1ull; }

__global__ void k_map_hash(const uint16_t *mchars, const int64_t *moff, int64_t mn, uint32_t *slots, uint64_t mask,
                           unsigned int *ovf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < mn; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (int64_t x = moff[i]; x < moff[i + 1]; x++) h = docid_hash_step(h, mchars[x]);
    uint64_t sl = docid_hash_fin(h) & mask;
    for (uint64_t probe = 0;; probe++) {
      if (probe > mask) {
        atomicOr(ovf, 1u);
        break;
      }
      if (atomicCAS(&slots[sl], 0u, (uint32_t)(i + 1)) == 0u) break;
      sl = (sl + 1) & mask;
    }
  }
}

// One thread per record.  The record's first kDocWin bytes are staged into a
// private LDS window with six independent 16-byte loads, and <DOCNO>..</DOCNO>
// is located and the docid hashed from there (one load latency instead of a
// dependent byte walk through global memory); a docid not inside the window
// takes the byte walk over the text (docid_span).
constexpr int kDocWin = 96;
__global__ __launch_bounds__(256) void k_docno(const uint8_t *t, int64_t n, const uint64_t *rs, const uint64_t *re,
                                               int64_t nR, const uint16_t *mchars, const int64_t *moff, int64_t mn,
                                               const uint32_t *mslots, uint64_t mmask, int32_t *docno,
                                               unsigned long long *err, uint64_t *dspan) {
  __shared__ uint4 win[256][kDocWin / 16];
  uint8_t *w = reinterpret_cast<uint8_t *>(win[threadIdx.x]);
  const int64_t mis = (int64_t)((uintptr_t)t & 15);
  const uint4 *a4 = reinterpret_cast<const uint4 *>(t - mis);
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = (int64_t)rs[r], e = (int64_t)re[r];
    const int64_t Q = (s + mis) & ~(int64_t)15;  // window byte j = text position Q - mis + j
    const int64_t w0 = Q - mis;
#pragma unroll
    for (int c = 0; c < kDocWin / 16; c++)
      win[threadIdx.x][c] = Q + 16 * c < n + mis ? a4[(Q >> 4) + c] : make_uint4(0, 0, 0, 0);
    const int js = (int)(s - w0), je = (int)min<int64_t>(kDocWin, e - w0);
    int a = -1, z = -1;
    for (int j = js; j + 7 <= je; j++)
      if (w[j] == '<' && w[j + 1] == 'D' && w[j + 2] == 'O' && w[j + 3] == 'C' && w[j + 4] == 'N' &&
          w[j + 5] == 'O' && w[j + 6] == '>') {
        a = j;
        break;
      }
    if (a >= 0)
      for (int j = a; j + 8 <= je; j++)
        if (w[j] == '<' && w[j + 1] == '/' && w[j + 2] == 'D' && w[j + 3] == 'O' && w[j + 4] == 'C' &&
            w[j + 5] == 'N' && w[j + 6] == 'O' && w[j + 7] == '>') {
          z = j;
          break;
        }
    int64_t ib, ie;
    const uint8_t *db;  // the docid's bytes (window or text)
    if (a >= 0 && z >= 0) {
      int b = a + 7, f = z;
      while (b < f && w[b] <= 0x20) b++;
      while (f > b && w[f - 1] <= 0x20) f--;
      ib = w0 + b;
      ie = w0 + f;
      db = w + b;
    } else {
      if (!docid_span(t, s, e, &ib, &ie)) {  // getDocid throws: the map task fails
        atomicAdd(err, 1ull);
        docno[r] = 0;
        dspan[r] = 0;
        continue;
      }
      db = t + ib;
    }
    const int64_t dl = ie - ib;
    dspan[r] = dl <= 255 ? (((uint64_t)ib << 8) | (uint64_t)dl) : 0;  // the docid's bytes (K4b)
    if (mslots) {
      uint64_t h = 0xCBF29CE484222325ull;
      for (int64_t p = 0; p < dl;) {
        uint16_t u[2];
        int nu;
        p += utf8_step(db, p, dl, u, &nu);
        for (int x = 0; x < nu; x++) h = docid_hash_step(h, u[x]);
      }
      uint64_t sl = docid_hash_fin(h) & mmask;
      int64_t found = -1;
      for (uint32_t v; (v = mslots[sl]) != 0u; sl = (sl + 1) & mmask) {
        const int64_t m = (int64_t)v - 1;
        if (cmp_u16_utf8(mchars + moff[m], moff[m + 1] - moff[m], db, dl) == 0) {
          found = m;
          break;
        }
      }
      if (found >= 0) {
        docno[r] = (int32_t)found;
        continue;
      }
    }
    // Arrays.binarySearch over {"", docids...}
    int64_t lo = 0, hi = mn - 1;
    int64_t res = INT64_MIN;
    while (lo <= hi) {
      int64_t mid = (int64_t)(((uint64_t)lo + (uint64_t)hi) >> 1);
      int c = cmp_u16_utf8(mchars + moff[mid], moff[mid + 1] - moff[mid], db, dl);
      if (c < 0)
        lo = mid + 1;
      else if (c > 0)
        hi = mid - 1;
      else {
        res = mid;
        break;
      }
    }
    if (res == INT64_MIN) res = -(lo + 1);
    docno[r] = (int32_t)res;
  }
}

// mark records that contain a complex '<' (sorted complex list)
#ifndef SME_MINFASTREC
#define SME_MINFASTREC 48
#endif
constexpr int64_t kMinFastRec = SME_MINFASTREC;

__global__ void k_mark_slow(const uint64_t *rs, const uint64_t *re, int64_t nR, const uint64_t *C, int64_t nC,
                            uint8_t *slow, unsigned long long *nslow) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t i = lower_bound_u64(C, nC, rs[r]);
    // complex markup, or a record too short for the stream tokenizer's window
    // (at most kChunk / kMinFastRec + 2 records overlap one chunk)
    bool s = (i < nC && C[i] < re[r]) || re[r] - rs[r] < kMinFastRec;
    slow[r] = s;
    if (s) atomicAdd(nslow, 1ull);
  }
}

// ============================================================================
// raw-token vocabulary (open addressing, exact)
// ============================================================================
// One 32-byte slot per distinct raw token: hash, (byte offset << 24 | length) of
// a representative occurrence, and the first 16 bytes of the token inline, so a
// lookup of a token of <= 16 bytes is decided from the slot's cache line alone.
// Slots are written once (0 -> value).  A plain read may return a stale 0 from
// another XCD's L2; "found" is only concluded from non-zero final values, and a
// mismatch is re-checked with coherent (RMW) reads before probing on.
// The slot's words live in three arrays: the 16 token bytes (w0, w1) that the
// tokenizer's fast probe reads -- 16 bytes a slot, so the probed array is half
// the size of a 32-byte slot table (c2: 128 MB at 8 M slots) -- and the key and
// rep words that only inserts and the vocabulary pass read.
struct RawTable {
  ulonglong2 *tok;           // (w0, w1)
  unsigned long long *key;   // hash (0: empty)
  unsigned long long *rep;   // (byte offset << 24 | length), written last
  uint64_t mask;
  const uint8_t *text;
  unsigned int *overflow;
};
constexpr size_t kRawSlotBytes = sizeof(ulonglong2) + 2 * sizeof(unsigned long long);

// Raw-token signature: w0/w1 = the first 16 bytes (little-endian, zero padded),
// h = a hash of them (+ the length and further 8-byte words for tokens longer
// than 16 bytes).  No token byte is 0 (0 is a split byte), so (w0, w1) alone
// identify a token of <= 16 bytes; longer ones are compared byte-wise.
// The hash is multilinear in the four 32-bit words (two v_mad_u64_u32) and ends
// in a 32-bit finaliser: low word of h = table hash, high word = the product's
// low word | 1 (h != 0 marks a used slot).  Every multiply is 32-bit: 64-bit
// multiplies are four quarter-rate VALU ops each on CDNA.
struct TokSig {
  uint64_t h, w0, w1;
};
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint64_t sig_head(uint64_t w0, uint64_t w1) {
  const uint64_t p = (uint64_t)((uint32_t)w0 + 0x9E3779B9u) * (uint64_t)((uint32_t)(w0 >> 32) + 0x85EBCA6Bu) +
                     (uint64_t)((uint32_t)w1 + 0xC2B2AE35u) * (uint64_t)((uint32_t)(w1 >> 32) + 0x27D4EB2Fu);
  const uint32_t x = fmix32((uint32_t)(p >> 32) ^ ((uint32_t)p >> 13));
  return ((uint64_t)((uint32_t)p | 1u) << 32) | x;
}
__device__ __forceinline__ uint64_t sig_mix(uint64_t h, uint64_t w) {  // long tokens: length and words 16..
  const uint64_t p = (uint64_t)((uint32_t)w + 0x165667B1u) * (uint64_t)((uint32_t)(w >> 32) + 0xD3A2646Cu);
  const uint32_t x = fmix32((uint32_t)h ^ (uint32_t)(p >> 32) ^ ((uint32_t)p >> 11));
  return ((uint64_t)(((uint32_t)(h >> 32) ^ (uint32_t)p) | 1u) << 32) | x;
}
__device__ __forceinline__ uint64_t load_word_bytes(const uint8_t *p, int64_t n) {  // n in [0, 8]
  uint64_t w = 0;
  for (int64_t i = 0; i < n; i++) w |= (uint64_t)p[i] << (8 * i);
  return w;
}
__device__ __forceinline__ TokSig sig_bytes(const uint8_t *p, int64_t len) {
  TokSig g;
  g.w0 = load_word_bytes(p, len < 8 ? len : 8);
  g.w1 = len > 8 ? load_word_bytes(p + 8, len < 16 ? len - 8 : 8) : 0;
  uint64_t h = sig_head(g.w0, g.w1);
  if (len > 16) h = sig_mix(h, (uint64_t)len);
  for (int64_t o = 16; o < len; o += 8) h = sig_mix(h, load_word_bytes(p + o, len - o < 8 ? len - o : 8));
  g.h = h;
  return g;
}

constexpr uint64_t kMaxProbe = 4096;  // longer runs mean the table is too full: retry with 4x slots

// Slot words are read with agent-scope relaxed loads (global_load ... sc1): a
// plain load may hit a line this XCD's L2 cached before another XCD filled the
// slot, and would then see a stale 0 on every later lookup of that token.
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The four words of a slot, as independent loads (one round trip).  Slots are
// written once, so a plain (L2-cacheable) read is either current or shows the
// slot (partly) empty; only then are the words re-read agent-coherently.
struct SlotVal {
  unsigned long long key, rep, w0, w1;
};
__device__ __forceinline__ SlotVal ld_slot(const RawTable &tb, uint64_t s) {
  SlotVal v;
  v.key = ld_agent(&tb.key[s]);
  v.rep = ld_agent(&tb.rep[s]);
  v.w0 = ld_agent(&tb.tok[s].x);
  v.w1 = ld_agent(&tb.tok[s].y);
  return v;
}
__device__ __forceinline__ SlotVal ld_slot_plain(const RawTable &tb, uint64_t s) {
  SlotVal v;
  v.key = tb.key[s];
  v.rep = tb.rep[s];
  const ulonglong2 t = tb.tok[s];
  v.w0 = t.x;
  v.w1 = t.y;
  return v;
}

// Find-or-insert the raw token (signature gh/gw0/gw1, text[off, off+len)); v holds
// the plainly loaded words of its home slot (gh & mask).  Returns the slot index.
// Scalar arguments only: a struct passed by reference to a non-inlined call
// lives in scratch memory, and the token loop would spill every signature.
__device__ __noinline__ uint32_t raw_insert_s(ulonglong2 *tok, unsigned long long *key, unsigned long long *rep,
                                              uint64_t mask, const uint8_t *text, unsigned int *overflow, uint64_t gh,
                                              uint64_t gw0, uint64_t gw1, uint64_t off, uint64_t len,
                                              unsigned long long vkey, unsigned long long vrep,
                                              unsigned long long vw0, unsigned long long vw1) {
  const RawTable tb{tok, key, rep, mask, text, overflow};
  const TokSig g{gh, gw0, gw1};
  SlotVal v{vkey, vrep, vw0, vw1};
  if (len >= (1ull << 24)) {
    atomicOr(tb.overflow, 2u);
    return 0xFFFFFFFFu;
  }
  const uint64_t rep_me = (off << 24) | len;
  uint64_t slot = g.h & tb.mask;
  const uint64_t max_probe = tb.mask < kMaxProbe ? tb.mask : kMaxProbe;
  for (uint64_t probe = 0; probe <= max_probe; probe++) {
    if (probe > 0) v = ld_slot_plain(tb, slot);
    if (v.key == 0 || (v.key == g.h && v.rep == 0)) v = ld_slot(tb, slot);  // maybe stale: re-read coherently
    unsigned long long k = v.key;
    if (k == 0) {
      unsigned long long old = atomicCAS(&tb.key[slot], 0ull, (unsigned long long)g.h);
      if (old == 0) {
        // w0/w1 must be performed before rep (readers trust w0/w1 once rep != 0).
        // The atomics execute at the memory side; waiting for their completion
        // orders them without __threadfence(), whose agent-scope release is an
        // L2 writeback + invalidate (buffer_wbl2 / buffer_inv sc1) per insert.
        atomicExch(&tb.tok[slot].x, (unsigned long long)g.w0);
        atomicExch(&tb.tok[slot].y, (unsigned long long)g.w1);
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
        atomicExch(&tb.rep[slot], (unsigned long long)rep_me);
        return (uint32_t)slot;
      }
      k = old;
      v.rep = 0;  // written after key: reload below
    }
    if (k == g.h) {
      unsigned long long r = v.rep;
      if (r == 0) {  // slot being filled by another lane: wait for rep (written last, after w0/w1)
        for (int spin = 0; r == 0 && spin < (1 << 22); spin++) r = ld_agent(&tb.rep[slot]);
        if (r == 0) {
          atomicOr(tb.overflow, 4u);
          return 0xFFFFFFFFu;
        }
        v.w0 = ld_agent(&tb.tok[slot].x);
        v.w1 = ld_agent(&tb.tok[slot].y);
      }
      if ((r & 0xFFFFFFull) == len) {
        bool eq = v.w0 == g.w0 && v.w1 == g.w1;
        if (!eq) {  // w0/w1 may have been read before rep: re-read them after it
          eq = ld_agent(&tb.tok[slot].x) == g.w0 && ld_agent(&tb.tok[slot].y) == g.w1;
        }
        if (eq && len > 16) {
          const uint64_t ro = r >> 24;
          for (uint64_t i = 16; i < len && eq; i++) eq = tb.text[ro + i] == tb.text[off + i];
        }
        if (eq) return (uint32_t)slot;
      }
    }
    slot = (slot + 1) & tb.mask;
  }
  atomicOr(tb.overflow, 1u);
  return 0xFFFFFFFFu;
}
__device__ __forceinline__ uint32_t raw_insert(const RawTable &tb, const TokSig &g, uint64_t off, uint64_t len,
                                               const SlotVal &v) {
  return raw_insert_s(tb.tok, tb.key, tb.rep, tb.mask, tb.text, tb.overflow, g.h, g.w0, g.w1, off, len, v.key, v.rep,
                      v.w0, v.w1);
}
__device__ __forceinline__ uint32_t raw_insert(const RawTable &tb, const TokSig &g, uint64_t off, uint64_t len) {
  return raw_insert(tb, g, off, len, ld_slot_plain(tb, g.h & tb.mask));
}

// ============================================================================
// K3: tokenization (raw tokens -> raw-vocab slots)
// ============================================================================
// Byte-parallel TagTokenizer for records whose markup is simple: a raw token is
// a maximal run of non-split bytes whose first byte lies outside every tag /
// comment / PI / entity span (spans begin and end on split characters, so a run
// is either wholly inside a span or wholly outside).
//
// A workgroup owns a contiguous range of records and walks their bytes as ONE
// stream of 16 KiB chunks (records are ~4 KiB: a chunk-per-record walk would
// leave most of every second chunk idle).  Per chunk:
//   1. coalesced 16-byte loads into LDS (+1 KiB lookahead), the overlapping
//      records' spans into LDS;
//   2. byte classes of every lane's 64 bytes from a 1 KiB LDS class table (one
//      ds_read_b32 + one v_lshl_or per byte builds the split and span-starter
//      bit masks together), span coverage by a block max-scan, token ranks by a
//      block sum-scan, each lane's token-end mask into LDS;
//   3. the chunk's token start positions listed in LDS by rank, then dealt
//      round-robin to the 256 lanes (no lane idles behind a lane with more
//      tokens): token end from the end masks, 16 bytes from LDS dwords by
//      v_alignbyte, a 32-bit-multiply signature, and the raw-vocabulary home
//      slots of two tokens loaded together;
//   4. the raw slots stored coalesced per record.
// Token i of record r goes to tokstream[(rs[r] >> 1) + i]; ntok[r] is written by
// the lane holding r's last byte.
// Streams read or written once (the text, the token stream, the pairs) bypass
// the L2 with nontemporal loads / stores (SME_NT = 1), so the hot raw-vocabulary
// slots and raw_term entries the probes and gathers reuse stay cached.
#ifndef SME_NT
#define SME_NT 1
#endif
template <typename T>
__device__ __forceinline__ T ld_stream(const T *p) {
#if SME_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#if SME_NT
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
#else
  const u32x4 v = *reinterpret_cast<const u32x4 *>(p);
#endif
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <typename T>
__device__ __forceinline__ void st_stream(T *p, T v) {
#if SME_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
#ifndef SME_TOKNT
#define SME_TOKNT 256
#endif
constexpr int kTokNT = SME_TOKNT;  // lanes per workgroup (one 64-byte lane slice each)
constexpr int kTokWords = 4;                      // 16-byte words per lane
constexpr int kTokBytes = 16 * kTokWords;         // 64 bytes per lane
constexpr int kChunk = kTokNT * kTokBytes;        // 16 KiB of text per block step
#ifndef SME_TOKLA
#define SME_TOKLA 64
#endif
constexpr int kStageV = kTokNT * kTokWords + SME_TOKLA;  // staged 16-byte words: chunk + lookahead (1 KiB)
constexpr int kRecWin = (SME_MINFASTREC >= 72 ? 256 : 384) * (kTokNT / 256);  // records overlapping one chunk: fast-path records are >= kMinFastRec bytes
static_assert(16384 / SME_MINFASTREC + 2 <= 384, "kRecWin");
#ifndef SME_TOKCAP
#define SME_TOKCAP 2560
#endif
constexpr int kTokCap = SME_TOKCAP * (kTokNT / 256);  // chunk tokens per round (a c2 16 KiB chunk holds ~1950; more take further rounds)
#ifndef SME_TOKMISS
#define SME_TOKMISS 256
#endif
constexpr int kTokMiss = SME_TOKMISS;  // deferred raw-vocabulary inserts per round (more: inserted in place)
// SME_TOK_V2 (default 1): every probe lane stores its token's raw slot straight to
// the token stream (the lanes of a wave hold consecutive chunk ranks, so the
// stores stay coalesced), so tl keeps only the 16-bit start positions, the
// record ids are read from frec where a record ends, and the store pass and its
// barrier are gone: 37.9 -> 31.3 KB of LDS, five workgroups per CU instead of four
#ifndef SME_TOK_V2
#define SME_TOK_V2 1
#endif
// SME_TOK_V3: one-barrier block scans and per-wave deferred inserts (no block
// barrier between the probe pass and the inserts): c2 k_tok_fast 7.12 -> 6.88 ms
#ifndef SME_D2H_PINNED
#define SME_D2H_PINNED 1
#endif
#ifndef SME_TOK_V3
#define SME_TOK_V3 1
#endif
#ifndef SME_TOK_WIN
#define SME_TOK_WIN 1
#endif
// V2: five workgroups per CU (its 31.3 KB of LDS) with one token per lane step in
// the probe pass (96 VGPRs, no spills; two tokens per step spill at five):
// c2 k_tok_fast 8.46 -> 7.87 ms
#ifndef SME_TOKOCC
#define SME_TOKOCC (SME_TOK_V2 ? 1280 / SME_TOKNT : 1024 / SME_TOKNT)
#endif
#ifndef SME_TOKG
#define SME_TOKG (SME_TOK_V2 ? 1 : 2)
#endif
constexpr int kTokG = SME_TOKG;  // tokens per lane step in the probe pass
#ifndef SME_FASTPROBES
#define SME_FASTPROBES 4
#endif
constexpr int kFastProbes = SME_FASTPROBES;  // slots a probe checks with plain loads before raw_insert

// entity span end: '&' [a-z0-9#]* ';'  (TagTokenizer.onAmpersand 644-662); p if none
template <typename B>
__device__ __forceinline__ int64_t amp_span_end_f(B &&byte, int64_t e, int64_t p) {
  for (int64_t i = p + 1; i < e; i++) {
    uint8_t d = byte(i);
    if ((d >= 'a' && d <= 'z') || (d >= '0' && d <= '9') || d == '#') continue;
    return d == ';' ? i : p;
  }
  return p;
}
// markup span end for '<' at p in a simple record (see lt_simple)
template <typename B>
__device__ __forceinline__ int64_t lt_span_end_f(B &&byte, int64_t n, int64_t p) {
  if (p + 1 >= n) return n;
  uint8_t c = byte(p + 1);
  if (c == '!' && p + 3 < n && byte(p + 2) == '-' && byte(p + 3) == '-') {
    for (int64_t i = p + 1; i + 2 < n; i++)
      if (byte(i) == '-' && byte(i + 1) == '-' && byte(i + 2) == '>') return i + 2;
    return n;
  }
  if (c == '?') {
    for (int64_t i = p + 1; i + 1 < n; i++)
      if (byte(i) == '?' && byte(i + 1) == '>') return i + 1;
    return n;
  }
  for (int64_t i = p + (c == '/' ? 2 : 1); i < n; i++)
    if (byte(i) == '>') return i;
  return n;
}

// Chunk-relative positions: position c_lo + p of the text is stage byte p
// (the stage starts at the chunk's first aligned word), so the per-lane state
// is 32-bit.  Record bounds in the window are clamped to [-1, kFar].
constexpr int32_t kFar = 1 << 30;

struct TokLds {
  uint4 st4[kStageV];
  int32_t rs[kRecWin], re[kRecWin];  // chunk-relative, clamped
  int64_t tbase0;                    // tokstream offset (rs >> 1) of window record 0 (others: from rs)
  int32_t c0[kRecWin];
#if !SME_TOK_V2
  int32_t rid[kRecWin];               // record index
#endif
  uint64_t emask[kTokNT];             // token-end bytes of every lane's 64: split, outside a fast record, record start
  int32_t sc32[kTokNT / 64 + 1];
#if SME_TOK_V3
  int32_t sm32[kTokNT / 64];          // the max scan's wave totals (sc32: the sum scan's)
  int32_t nmissw[kTokNT / 64];        // per-wave deferred inserts (miss[64 w ..])
#endif
  uint32_t cls[256];                  // byte class: bit 0 split byte, bit 16 span starter ('<' or '&')
#if SME_TOK_V2
  uint16_t tl[kTokCap];               // round's chunk tokens by rank: start position (< 2^15)
#else
  uint32_t tl[kTokCap];               // round's chunk tokens by rank: start position, then raw slot
#endif
  int32_t miss[kTokMiss];             // round's tokens whose probe found no slot: inserted together
  int32_t nmiss;
};

// byte at chunk-relative position p (stage, or global beyond the lookahead)
__device__ __forceinline__ uint8_t tok_byte(const uint8_t *stg, const uint8_t *t, int64_t c_lo, int32_t p) {
  return (p >= 0 && p < kStageV * 16) ? stg[p] : t[c_lo + p];
}
__device__ __noinline__ int32_t lt_span_rel(const uint8_t *stg, const uint8_t *t, int64_t c_lo, int32_t e, int32_t p) {
  if (p + 1 >= e) return e;
  const uint8_t c = tok_byte(stg, t, c_lo, p + 1);
  if (c == '!' && p + 3 < e && tok_byte(stg, t, c_lo, p + 2) == '-' && tok_byte(stg, t, c_lo, p + 3) == '-') {
    for (int32_t i = p + 1; i + 2 < e; i++)
      if (tok_byte(stg, t, c_lo, i) == '-' && tok_byte(stg, t, c_lo, i + 1) == '-' && tok_byte(stg, t, c_lo, i + 2) == '>')
        return i + 2;
    return e;
  }
  if (c == '?') {
    for (int32_t i = p + 1; i + 1 < e; i++)
      if (tok_byte(stg, t, c_lo, i) == '?' && tok_byte(stg, t, c_lo, i + 1) == '>') return i + 1;
    return e;
  }
  for (int32_t i = p + (c == '/' ? 2 : 1); i < e; i++)
    if (tok_byte(stg, t, c_lo, i) == '>') return i;
  return e;
}
__device__ __noinline__ int32_t amp_span_rel(const uint8_t *stg, const uint8_t *t, int64_t c_lo, int32_t e, int32_t p) {
  for (int32_t i = p + 1; i < e; i++) {
    const uint8_t d = tok_byte(stg, t, c_lo, i);
    if ((d >= 'a' && d <= 'z') || (d >= '0' && d <= '9') || d == '#') continue;
    return d == ';' ? i : p;
  }
  return p;
}

// first split byte at or after byte k of the 16-byte window (lo, hi); 16 if none
__device__ __forceinline__ int first_split16(uint64_t lo, uint64_t hi, int k) {
  for (int i = k; i < 16; i++) {
    const uint8_t b = (uint8_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xFF);
    if (is_split_byte(b)) return i;
  }
  return 16;
}

// signature of the token starting at chunk-relative x (its first byte is a word
// char); e bounds it (the record end).  Long tokens continue byte-wise.
struct TokSigLen {
  uint64_t h, w0, w1;
  int32_t len;
};
__device__ __noinline__ TokSigLen tok_sig_long(const uint8_t *stg, const uint8_t *t, int64_t c_lo, int32_t x,
                                               int32_t e) {
  int32_t y = x;
  while (y < e && !is_split_byte(tok_byte(stg, t, c_lo, y))) y++;
  const TokSig g = sig_bytes(t + c_lo + x, y - x);
  return TokSigLen{g.h, g.w0, g.w1, y - x};
}

// Signature and length of the token starting at chunk-relative x.  The end is
// the first token-end byte after x in this lane's or the next lane's mask;
// tokens running further (> 16 bytes, or past the chunk) take the byte path.
__device__ __forceinline__ void tok_sig_at(const TokLds &L, const uint8_t *t, int64_t c_lo, int32_t x, TokSig *g,
                                           int32_t *len_o) {
  const int ln = x >> 6, bi = x & 63;
  const uint64_t rest = L.emask[ln] >> bi >> 1;  // bytes x+1 .. end of lane
  int32_t len = 99;
  if (rest) {
    len = __ffsll((unsigned long long)rest);
  } else if (ln + 1 < kTokNT) {
    const uint64_t m = L.emask[ln + 1];
    if (m) len = 64 - bi + __ffsll((unsigned long long)m) - 1;
  }
  if (len <= 16) {
    const uint32_t *st32 = reinterpret_cast<const uint32_t *>(L.st4);
    const int a = x >> 2, r = x & 3;
    const uint32_t d0 = st32[a], d1 = st32[a + 1], d2 = st32[a + 2], d3 = st32[a + 3], d4 = st32[a + 4];
    const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, r) |
                        ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, r) << 32);
    const uint64_t hi = (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, r) |
                        ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, r) << 32);
    g->w0 = len >= 8 ? lo : (lo & ((1ull << (8 * len)) - 1ull));
    g->w1 = len <= 8 ? 0ull : (len >= 16 ? hi : (hi & ((1ull << (8 * (len - 8))) - 1ull)));
    g->h = sig_head(g->w0, g->w1);
  } else {
    // record end bounds the byte walk
    int lo_k = 0, hi_k = kRecWin;
    while (lo_k < hi_k) {
      const int m = (lo_k + hi_k) >> 1;
      if (L.rs[m] <= x)
        lo_k = m + 1;
      else
        hi_k = m;
    }
    const int32_t e = L.re[lo_k > 0 ? lo_k - 1 : 0];
    const TokSigLen s = tok_sig_long(reinterpret_cast<const uint8_t *>(L.st4), t, c_lo, x, e);
    g->h = s.h;
    g->w0 = s.w0;
    g->w1 = s.w1;
    len = s.len;
  }
  *len_o = len;
}

// The probe's fast path loads only the slot's 16 token bytes (w0, w1; one
// 16-byte load).  A token of < 16 bytes is its zero-padded (w0, w1) (no token
// byte is 0), and a slot's (w0, w1) of a token of >= 16 bytes has no zero byte,
// so equal words mean the same token, whether or not the slot's rep is
// published yet.  Tokens of >= 16 bytes, and every mismatch, take raw_insert
// (which re-reads the whole slot coherently).
__device__ __forceinline__ bool slot_hit16(const ulonglong2 &v, const TokSig &g, int32_t len) {
  return len < 16 && v.x == g.w0 && v.y == g.w1;
}

#if SME_TOK_V3
// one-barrier block scans: every thread reads the NT/64 wave totals itself (no
// serial step, no trailing barrier: a scratch array is next written a chunk later,
// after further barriers)
template <int NT, typename T>
__device__ __forceinline__ T tok_block_excl_sum(T v, T *scratch, T *total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  const T inc = wave_incl_sum(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const T t = scratch[i];
    pre += i < w ? t : (T)0;
    tot += t;
  }
  *total = tot;
  return pre + inc - v;
}
template <int NT>
__device__ __forceinline__ int32_t tok_block_excl_max(int32_t v, int32_t lo, int32_t *scratch, int32_t *total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  const int32_t inc = wave_incl_max(v);
  const int32_t exc = __builtin_amdgcn_update_dpp(lo, inc, 0x138, 0xF, 0xF, false);  // wave_shr:1 (lane 0: lo)
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  int32_t pre = lo, tot = lo;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    const int32_t t = scratch[i];
    pre = i < w ? max(pre, t) : pre;
    tot = max(tot, t);
  }
  *total = tot;
  return max(pre, exc);
}
#endif

// rs_g / re_g: record bounds of the fast records in frec order (rsF[f] = rs[frec[f]])
__global__ __launch_bounds__(kTokNT, SME_TOKOCC) void k_tok_fast(const uint8_t *__restrict__ t, int64_t n,
                                                     const uint64_t *__restrict__ rs_g,
                                                     const uint64_t *__restrict__ re_g,
                                                     const int32_t *__restrict__ frec, int64_t nF, int64_t rpb,
                                                     uint32_t *__restrict__ tokstream, int32_t *__restrict__ ntok,
                                                     RawTable tb, int texp) {
  __shared__ TokLds L;
  __shared__ int32_t s_adv;
  const int64_t f0 = blockIdx.x * rpb;
  if (f0 >= nF) return;
  const int64_t f1 = min(nF, f0 + rpb);
  const int64_t mis = (int64_t)((uintptr_t)t & 15);
  const uint4 *a4 = reinterpret_cast<const uint4 *>(t - mis);
  const int64_t nq = n + mis;
  const uint8_t *stg = reinterpret_cast<const uint8_t *>(L.st4);
  const int tid = threadIdx.x;
  if (tid < 256) L.cls[tid] = (is_split_byte((uint32_t)tid) ? 1u : 0u) | ((tid == '<' || tid == '&') ? 0x10000u : 0u);
  const int64_t end_all = (int64_t)re_g[f1 - 1];
  int64_t fcur = f0;        // first fast record not wholly before the current chunk
  int64_t mask_carry = -1;  // absolute end of the furthest span begun in earlier chunks
  int32_t tok_carry = 0;    // tokens of the record continuing from the previous chunk
  int64_t Q = ((int64_t)rs_g[f0] + mis) & ~(int64_t)15;
  uint8_t prev_chunk_byte = Q - mis > 0 ? t[Q - mis - 1] : (uint8_t)' ';
  for (; Q < end_all + mis; Q += kChunk) {
    const int64_t c_lo = Q - mis;  // chunk = positions c_lo + [0, kChunk)
    for (int i = tid; i < kRecWin; i += kTokNT) {
      const int64_t f = fcur + i;
#if SME_TOK_V2 && SME_TOK_WIN
      // (the record id is read only where a record ends: both bounds load
      // independently, no rs -> re chain)
      const bool in = f < f1;
      const int64_t a = in ? (int64_t)rs_g[f] : INT64_MAX;
      const int64_t b0 = in ? (int64_t)re_g[f] : INT64_MAX;
      const bool ok = a < c_lo + kChunk;
      const int64_t b = ok ? b0 : INT64_MAX;
#else
      const int32_t r = f < f1 ? frec[f] : -1;
      const int64_t a = r >= 0 ? (int64_t)rs_g[f] : INT64_MAX;  // (independent loads: no frec -> rs chain)
      const bool ok = a < c_lo + kChunk;
      const int64_t b = ok ? (int64_t)re_g[f] : INT64_MAX;
#endif
      L.rs[i] = ok ? (int32_t)max<int64_t>(a - c_lo, -1) : kFar;
      L.re[i] = ok ? (int32_t)min<int64_t>(b - c_lo, kFar) : kFar;
      if (i == 0) L.tbase0 = ok ? (a >> 1) : 0;
#if !SME_TOK_V2
      L.rid[i] = ok ? r : -1;
#endif
      L.c0[i] = 0;
    }
    for (int i = tid; i < kStageV; i += kTokNT) {
      const int64_t q = Q + 16 * (int64_t)i;
      L.st4[i] = q < nq ? ld_stream(a4 + (q >> 4)) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int32_t p0 = kTokBytes * tid;
    int j;  // window record holding p0 (or -1)
    {
      int lo = 0, hi = kRecWin;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (L.rs[m] <= p0)
          lo = m + 1;
        else
          hi = m;
      }
      j = lo - 1;
    }
    const int32_t mc = (int32_t)max<int64_t>(min<int64_t>(mask_carry - c_lo, kFar), -1);
    // pass 1: byte classes of this lane's 64 bytes as bit masks (bit i = byte p0 + i)
    uint64_t S = 0, SPN = 0;  // split bytes; '<' / '&' bytes (span starters)
#pragma unroll
    for (int w = 0; w < kTokWords; w++) {
      if (texp & 32) break;  // (timing experiment: no byte classes)
      const uint4 q = L.st4[kTokWords * tid + w];
      uint32_t acc = 0;  // bits 0-15 split, 16-31 span starter
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint32_t dw = i < 4 ? q.x : (i < 8 ? q.y : (i < 12 ? q.z : q.w));
        acc |= L.cls[(dw >> (8 * (i & 3))) & 0xFFu] << i;
      }
      S |= (uint64_t)(acc & 0xFFFFu) << (16 * w);
      SPN |= (uint64_t)(acc >> 16) << (16 * w);
    }
    // bytes inside a (fast-path) record: all of them unless a record boundary
    // falls in this lane; record-start bytes end a token too
    uint64_t IN, RS = 0;
    const bool whole = j >= 0 && L.re[j] >= p0 + kTokBytes;
    if (whole) {
      IN = ~0ull;
      RS = L.rs[j] == p0 ? 1ull : 0ull;
    } else {
      IN = 0;
      for (int k = j < 0 ? 0 : j; k < kRecWin && L.rs[k] < p0 + kTokBytes; k++) {
        const int32_t a = max(L.rs[k] - p0, 0), b = min(L.re[k] - p0, kTokBytes);
        if (b > a) IN |= (b >= 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((1ull << a) - 1ull);
        if (L.rs[k] >= p0) RS |= 1ull << (L.rs[k] - p0);
      }
    }
    L.emask[tid] = S | ~IN | RS;
    const uint64_t prev_split = is_split_byte(tid > 0 ? stg[p0 - 1] : prev_chunk_byte) ? 1ull : 0ull;
    uint64_t cand = IN & ~S & ((S << 1) | prev_split);
    int32_t lane_max = -1;
    uint64_t sp = SPN & IN;
    if (sp) {  // rare: markup / entities in this lane
      // '>' bytes of the lane: a '<' followed by neither '!' nor '?' spans to the
      // first '>' after it (lt_span_end), found here from the mask when it lies
      // in this lane and before the record end
      uint64_t GT = 0;
#pragma unroll
      for (int w = 0; w < kTokWords * 4; w++) {
        const uint32_t d = reinterpret_cast<const uint32_t *>(L.st4)[kTokWords * 4 * tid + w] ^ 0x3E3E3E3Eu;
        const uint32_t z = ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;  // 0x80 where byte == '>'
        GT |= (uint64_t)(((z >> 7) * 0x10204080u) >> 28) << (4 * w);
      }
      int jj = j;
      while (sp) {
        const int i = __ffsll((unsigned long long)sp) - 1;
        sp &= sp - 1;
        const int32_t p = p0 + i;
        while (jj + 1 < kRecWin && L.rs[jj + 1] <= p) jj++;
        const int32_t e = L.re[jj];
        int32_t q;
        const uint8_t c1 = i < kTokBytes - 1 ? stg[p + 1] : 0;
        const uint64_t gt_after = i < 63 ? (GT >> i >> 1) : 0ull;
        if (stg[p] == '<' && i < kTokBytes - 1 && c1 != '!' && c1 != '?' && gt_after &&
            p + __ffsll((unsigned long long)gt_after) < e)
          q = p + __ffsll((unsigned long long)gt_after);
        else
          q = stg[p] == '<' ? lt_span_rel(stg, t, c_lo, e, p) : amp_span_rel(stg, t, c_lo, e, p);
        lane_max = q > lane_max ? q : lane_max;
        // tokens may not start inside the span (p, q]
        const int32_t hi_bit = q - p0;
        if (hi_bit > i) {
          const uint64_t upto = hi_bit >= 63 ? ~0ull : ((1ull << (hi_bit + 1)) - 1ull);
          cand &= ~(upto & (i >= 63 ? 0ull : (~0ull << (i + 1))));  // bits (i, hi_bit]; no shift by 64
        }
      }
    }
    int32_t blk_max;
#if SME_TOK_V3
    int32_t before = tok_block_excl_max<kTokNT>(lane_max, -1, L.sm32, &blk_max);
#else
    int32_t before = block_excl_max<kTokNT, int32_t>(lane_max, -1, L.sc32, &blk_max);
#endif
    before = before > mc ? before : mc;
    // candidates at or below `before` lie inside a span begun in an earlier lane
    const int32_t cut = before - p0 + 1;  // bits [0, cut) are covered
    const uint64_t keep_all =
        cut <= 0 ? cand : (cut >= kTokBytes ? 0ull : cand & ~((1ull << cut) - 1ull));
    int32_t blk_cnt;
#if SME_TOK_V3
    const int32_t base = tok_block_excl_sum<kTokNT, int32_t>(__popcll(keep_all), L.sc32, &blk_cnt);
#else
    const int32_t base = block_excl_sum<kTokNT, int32_t>(__popcll(keep_all), L.sc32, &blk_cnt);
#endif
    // c0: chunk rank of the first token of every record that starts in this lane
    for (int k = (j < 0 ? 0 : j); k < kRecWin && L.rs[k] < p0 + kTokBytes; k++)
      if (L.rs[k] >= p0) L.c0[k] = base + __popcll(keep_all & ((1ull << (L.rs[k] - p0)) - 1ull));
    __syncthreads();
    const int32_t carry0 = L.rs[0] < 0 ? tok_carry : 0;  // window record 0 began in an earlier chunk
    // ntok of every record whose last byte is in this lane (no token starts at its '>')
    for (int k = (j < 0 ? 0 : j); k < kRecWin && L.rs[k] < p0 + kTokBytes; k++) {
      const int32_t last = L.re[k] - 1;
      if (last >= p0 && last < p0 + kTokBytes) {
        const int32_t r0k = k == 0 ? L.c0[0] - carry0 : L.c0[k];
#if SME_TOK_V2
        ntok[frec[fcur + k]] = base + __popcll(keep_all & ((1ull << (last - p0)) - 1ull)) - r0k;
#else
        ntok[L.rid[k]] = base + __popcll(keep_all & ((1ull << (last - p0)) - 1ull)) - r0k;
#endif
      }
    }
    // next chunk: records wholly before it are dropped from the window; the one
    // running into it carries its token count
    if (tid == 0) {
      int adv = 0, kl = -1;
      for (int k = 0; k < kRecWin && L.rs[k] < kChunk; k++) {
        kl = k;
        if (L.re[k] <= kChunk) adv = k + 1;
      }
      s_adv = adv;
      L.sc32[0] = (kl >= 0 && L.re[kl] > kChunk) ? blk_cnt - (kl == 0 ? L.c0[0] - carry0 : L.c0[kl]) : 0;
    }
    if (blk_max >= 0) mask_carry = max<int64_t>(mask_carry, c_lo + blk_max);
    prev_chunk_byte = stg[kChunk - 1];
    int nk;  // window records starting before the chunk end
    {
      int lo = 0, hi = kRecWin;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (L.rs[m] < kChunk) lo = m + 1;
        else hi = m;
      }
      nk = lo;
    }
    auto fr = [&](int k) { return (k == 0 && L.rs[0] < 0) ? 0 : L.c0[k]; };
#if SME_TOK_V2
    // token stream index of chunk token i of window record k
    auto dest_of = [&](int k, int32_t i) -> int64_t {
      const int32_t r0k = k == 0 ? L.c0[0] - carry0 : L.c0[k];
      const int64_t tbse = k == 0 ? L.tbase0 : ((c_lo + L.rs[k]) >> 1);
      return tbse + (i - r0k);
    };
    // last window record k < nk with fr(k) <= i
    auto rec_of = [&](int32_t i) -> int {
      int lo = 0, hi = nk;
      while (hi - lo > 1) {
        const int m = (lo + hi) >> 1;
        if (fr(m) <= i) lo = m;
        else hi = m;
      }
      return lo;
    };
#endif
    for (int32_t rlo = 0; rlo < ((texp & 16) ? 0 : blk_cnt); rlo += kTokCap) {  // (16: no token passes)
      const int32_t nr = min(kTokCap, blk_cnt - rlo);
      // pass 2: start positions of the round's tokens by chunk rank
#if SME_TOK_V3
      if (tid < kTokNT / 64) L.nmissw[tid] = 0;
#else
      if (tid == 0) L.nmiss = 0;
#endif
      {
        uint64_t keep = keep_all;
        int32_t idx = base - rlo;
        if (idx < nr && idx + __popcll(keep) > 0) {
          while (keep) {
            const int i0 = __ffsll((unsigned long long)keep) - 1;
            keep &= keep - 1;
            if (idx >= 0 && idx < nr) L.tl[idx] = (std::remove_reference_t<decltype(L.tl[0])>)(p0 + i0);
            idx++;
          }
        }
      }
      __syncthreads();
      // pass 3: signature + raw-vocabulary slot, kTokG tokens per lane step (their
      // home-slot loads in flight together)
#if SME_TOK_V2
      int kc = tid < nr ? rec_of(rlo + tid) : 0;  // record of the lane's next token (ranks ascend)
#endif
      for (int32_t r0 = (texp & 1) ? nr : tid; r0 < nr; r0 += kTokG * kTokNT) {
        TokSig g[kTokG];
        int32_t len[kTokG], x[kTokG];
        ulonglong2 v[kTokG];
#pragma unroll
        for (int u = 0; u < kTokG; u++) {
          const int32_t r = r0 + u * kTokNT;
          x[u] = (int32_t)L.tl[r < nr ? r : r0];
          tok_sig_at(L, t, c_lo, x[u], &g[u], &len[u]);
        }
#pragma unroll
        for (int u = 0; u < kTokG; u++)
          v[u] = tb.tok[g[u].h & tb.mask];
#pragma unroll
        for (int u = 0; u < kTokG; u++) {
          const int32_t r = r0 + u * kTokNT;
          if (r < nr) {
#if SME_TOK_V2
            const int32_t ci = rlo + r;
            while (kc + 1 < nk && fr(kc + 1) <= ci) kc++;
            uint32_t *const dst = tokstream + dest_of(kc, ci);
#endif
            // linear probing over occupied slots of other tokens with plain
            // loads (a slot, once filled, never changes); an empty-looking slot,
            // a token of >= 16 bytes or a long probe run take raw_insert
            uint64_t sl = g[u].h & tb.mask;
            bool hit = slot_hit16(v[u], g[u], len[u]);
            if (!hit && len[u] < 16 && v[u].x != 0 && !(texp & 8)) {
              for (int pr = 1; pr < kFastProbes; pr++) {
                const uint64_t s2 = (sl + pr) & tb.mask;
                const ulonglong2 w = tb.tok[s2];
                if (slot_hit16(w, g[u], len[u])) {
                  hit = true;
                  sl = s2;
                  break;
                }
                if (w.x == 0) break;
              }
            }
            if (hit || (texp & 12)) {  // (timing experiments 4 / 8: no insert / no probe walk)
#if SME_TOK_V2
              if (!(texp & 2)) st_stream(dst, (uint32_t)sl);
#else
              L.tl[r] = (uint32_t)sl;
#endif
            } else {
              // a new raw token (or a long / contended probe): inserted after the
              // probe pass, with the round's other inserts, so a wave waits on one
              // insert chain rather than on one per lane step
#if SME_TOK_V3
              const int k = atomicAdd(&L.nmissw[tid >> 6], 1);
              if (k < kTokMiss / (kTokNT / 64))
                L.miss[(tid >> 6) * (kTokMiss / (kTokNT / 64)) + k] = r;
#else
              const int k = atomicAdd(&L.nmiss, 1);
              if (k < kTokMiss)
                L.miss[k] = r;
#endif
              else
#if SME_TOK_V2
                *dst = raw_insert(tb, g[u], (uint64_t)(c_lo + x[u]), (uint64_t)len[u], SlotVal{0, 0, 0, 0});
#else
                L.tl[r] = raw_insert(tb, g[u], (uint64_t)(c_lo + x[u]), (uint64_t)len[u], SlotVal{0, 0, 0, 0});
#endif
            }
          }
        }
      }
#if SME_TOK_V3
      // pass 3b per wave (its own deferred inserts, right after its probes: no
      // block barrier; the noinline raw_insert re-reads the home slot coherently,
      // concurrent inserts of one token resolve there)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      constexpr int kMissW = kTokMiss / (kTokNT / 64);
      for (int i = tid & 63; i < min(L.nmissw[tid >> 6], kMissW); i += 64) {
        const int32_t r = L.miss[(tid >> 6) * kMissW + i];
#else
      __syncthreads();
      // pass 3b: the deferred inserts (the noinline raw_insert re-reads the home
      // slot coherently; concurrent inserts of one token resolve there)
      for (int i = tid; i < min(L.nmiss, kTokMiss); i += kTokNT) {
        const int32_t r = L.miss[i];
#endif
        const int32_t x = (int32_t)L.tl[r];
        TokSig g;
        int32_t len;
        tok_sig_at(L, t, c_lo, x, &g, &len);
#if SME_TOK_V2
        tokstream[dest_of(rec_of(rlo + r), rlo + r)] =
            raw_insert(tb, g, (uint64_t)(c_lo + x), (uint64_t)len, SlotVal{0, 0, 0, 0});
#else
        L.tl[r] = raw_insert(tb, g, (uint64_t)(c_lo + x), (uint64_t)len, SlotVal{0, 0, 0, 0});
#endif
      }
#if SME_TOK_V2
      if (rlo + kTokCap < blk_cnt) __syncthreads();  // the next round rewrites tl / miss
    }
#else
      __syncthreads();
      // pass 4: coalesced stores: chunk token i belongs to the last window record
      // whose first chunk token is <= i (records without tokens share that rank
      // with their successor, so they are skipped)
      {
        const int32_t i0 = rlo + tid;
        int k = 0;
        if (i0 < rlo + nr) {
          int lo = 0, hi = nk;  // last k with fr(k) <= i0
          while (hi - lo > 1) {
            const int m = (lo + hi) >> 1;
            if (fr(m) <= i0) lo = m;
            else hi = m;
          }
          k = lo;
        }
        for (int32_t i = (texp & 2) ? rlo + nr : i0; i < rlo + nr; i += kTokNT) {
          while (k + 1 < nk && fr(k + 1) <= i) k++;
          const int32_t r0k = k == 0 ? L.c0[0] - carry0 : L.c0[k];
          const int64_t tbse = k == 0 ? L.tbase0 : ((c_lo + L.rs[k]) >> 1);
          st_stream(tokstream + tbse + (i - r0k), L.tl[i - rlo]);
        }
      }
      if (rlo + kTokCap < blk_cnt) __syncthreads();  // the next round rewrites tl
    }
#endif
    __syncthreads();  // LDS is overwritten by the next chunk (s_adv / sc32[0] are rewritten only after
                      // the next chunk's staging barrier)
    fcur += s_adv;
    tok_carry = L.sc32[0];
  }
}

__global__ void k_gather_bounds(const int32_t *frec, int64_t nF, const uint64_t *rs, const uint64_t *re, uint64_t *rsF,
                                uint64_t *reF) {
  for (int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; f < nF; f += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = frec[f];
    rsF[f] = rs[r];
    reF[f] = re[r];
  }
}

// slow path: sequential TagTokenizer on the decoded record, one thread per record
__global__ void k_tok_slow(const uint8_t *__restrict__ t, const uint64_t *rs, const uint64_t *re,
                           const int64_t *slow_list, int64_t nslow, const int64_t *scratch_off, uint16_t *u16s,
                           uint32_t *boffs, uint32_t *tokstream, int32_t *ntok, RawTable tb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nslow; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = slow_list[i];
    const int64_t s = (int64_t)rs[r], e = (int64_t)re[r];
    uint16_t *u = u16s + scratch_off[i];
    uint32_t *bo = boffs + scratch_off[i];
    int64_t nu = 0;
    for (int64_t p = s; p < e;) {
      uint16_t tmp[2];
      int k;
      int used = utf8_step(t, p, e, tmp, &k);
      for (int x = 0; x < k; x++) {
        u[nu] = tmp[x];
        bo[nu] = (uint32_t)(p - s);
        nu++;
      }
      p += used;
    }
    bo[nu] = (uint32_t)(e - s);
    uint32_t *out = tokstream + (s >> 1);
    int32_t cnt = 0;
    TagScan sc;
    sc.t = u;
    sc.n = (int)nu;
    sc.run([&](int u0, int u1) {
      uint64_t x = (uint64_t)s + bo[u0], len = bo[u1] - bo[u0];
      out[cnt++] = raw_insert(tb, sig_bytes(t + x, (int64_t)len), x, len);
    });
    ntok[r] = cnt;
  }
}

// ============================================================================
// K4: vocabulary
// ============================================================================
// The distinct raw tokens are first compacted into rlist (ascending slot order),
// so one lane per listed token does real work (a sweep over the hash slots left
// most lanes of a wave idle).  Every output of raw token i lives in its own pool
// region [poff[i], poff[i] + len_bytes) -- outputs never exceed the raw token's
// UTF-8 length (stems only shrink; acronym pieces are disjoint substrings; the
// one lowercase expansion, U+0130, is 2 units for 2 bytes) -- so no shared
// allocation counter is touched.  Output 0 is candidate i; further outputs
// (acronym splits, rare) and, for those tokens, a copy of output 0 go to an
// overflow list keyed (slot << 32 | ordinal).
constexpr uint64_t kNoCand = ~0ull;

struct CandOut {
  uint16_t *pool;
  const int64_t *poff;  // per list index, units
  uint64_t *cand_str;   // (pool offset << 16) | len, [0, nraw) primary, [nraw, nraw + ovf_cap) overflow
  int64_t nraw;
  uint64_t *ovf_key;    // (raw slot << 32) | ordinal
  unsigned long long *novf;
  uint64_t ovf_cap;
  int32_t *raw_nout;
  int32_t *max_nout;
  unsigned int *err;  // bit 1: an output overran its token's pool region (cannot happen; checked)
  unsigned int *pres; // 128-bit presence of the code units (& 127) of every output (the one-word term sort)
};
// a stem's code units into the lane's 128-bit presence mask
__device__ __forceinline__ void unit_bits(const uint16_t *b, int l, uint64_t &lo, uint64_t &hi) {
  for (int k = 0; k < l; k++) {
    const uint32_t c = b[k] & 127u;
    if (c < 64) lo |= 1ull << c;
    else hi |= 1ull << (c - 64);
  }
}
// one atomic per wave and mask word
__device__ __forceinline__ void flush_unit_bits(unsigned int *pres, uint64_t lo, uint64_t hi) {
  const unsigned int m[4] = {(unsigned int)lo, (unsigned int)(lo >> 32), (unsigned int)hi, (unsigned int)(hi >> 32)};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    unsigned int v = m[k];
    for (int o = 32; o > 0; o >>= 1) v |= (unsigned int)__shfl_xor((int)v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicOr(&pres[k], v);
  }
}

__device__ __forceinline__ void ovf_push(const CandOut &co, uint32_t slot, uint32_t ord, uint64_t cs) {
  unsigned long long j = atomicAdd(co.novf, 1ull);
  if (j < co.ovf_cap) {
    co.ovf_key[j] = ((uint64_t)slot << 32) | ord;
    co.cand_str[co.nraw + j] = cs;
  }
}

__device__ __forceinline__ void vocab_finish(const CandOut &co, int64_t i, uint32_t slot, uint32_t nout) {
  co.raw_nout[slot] = (int32_t)nout;
  if (nout == 0) co.cand_str[i] = kNoCand;
  if (nout > 1) {
    ovf_push(co, slot, 0, co.cand_str[i]);
    atomicMax(co.max_nout, (int32_t)nout);
  }
}

// normalize + stop + stem one decoded raw token (units) of list index i
__device__ void vocab_one(const CandOut &co, int64_t i, uint32_t slot, const uint16_t *units, int nu,
                          uint16_t *work, int work_cap, uint64_t &plo, uint64_t &phi) {
  uint32_t ord = 0;
  uint64_t used = 0;
  Stemmer st;
  normalize_raw(units, nu, work, work_cap, [&](const uint16_t *p, int l) {
    if (is_stopword(p, l)) return;
    for (int k = 0; k < l; k++) st.b[k] = p[k];
    st.len = l;
    st.run();
    unit_bits(st.b, st.len, plo, phi);
    const uint64_t po = (uint64_t)co.poff[i] + used;
    if (po + (uint64_t)st.len > (uint64_t)co.poff[i + 1]) {
      atomicOr(co.err, 1u);
      return;
    }
    for (int k = 0; k < st.len; k++) co.pool[po + k] = st.b[k];
    used += (uint64_t)st.len;
    const uint64_t cs = (po << 16) | (uint64_t)st.len;
    if (ord == 0)
      co.cand_str[i] = cs;
    else
      ovf_push(co, slot, ord, cs);
    ord++;
  });
  vocab_finish(co, i, slot, ord);
}

// Fast path for the common raw token: only [a-z0-9] (checkTokenStatus == Clean), so
// normalization is the identity and the token goes straight to stop list + stemmer.
__device__ bool vocab_clean(const CandOut &co, int64_t i, uint32_t slot, const uint8_t *p, uint64_t len,
                            uint16_t *lds_buf, uint64_t &plo, uint64_t &phi) {
  if (len > 48) return false;
  StemmerT<64> st(lds_buf);  // the word in the lane's LDS slice (a scratch array was the kernel's bottleneck)
  for (uint64_t k = 0; k < len; k++) {
    uint8_t c = p[k];
    if (!((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'))) return false;
    st.b[k] = c;
  }
  uint32_t ord = 0;
  if (!is_stopword(st.b, (int)len)) {  // <= 48 ASCII bytes: addToken's >= 100-byte rule cannot apply
    st.len = (int)len;
    st.run();
    unit_bits(st.b, st.len, plo, phi);
    const uint64_t po = (uint64_t)co.poff[i];
    for (int k = 0; k < st.len; k++) co.pool[po + k] = st.b[k];
    co.cand_str[i] = (po << 16) | (uint64_t)st.len;
    ord = 1;
  }
  vocab_finish(co, i, slot, ord);
  return true;
}

constexpr int kShortRaw = 200;

__global__ void k_not_flags(const uint8_t *a, int64_t n, uint8_t *f) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = !a[i];
}
__global__ void k_raw_flags(const unsigned long long *key, uint64_t n, uint8_t *flag) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x)
    flag[s] = key[s] != 0;
}
__global__ void k_raw_lens(const unsigned long long *rep, const int32_t *rlist, int64_t nraw, int64_t *lens) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= nraw; i += (int64_t)gridDim.x * blockDim.x)
    lens[i] = i < nraw ? (int64_t)(rep[rlist[i]] & 0xFFFFFFull) : 0;
}

constexpr int kVocabNT = 256;
__global__ __launch_bounds__(kVocabNT, 4) void k_vocab(const RawTable tb, const int32_t *rlist, int64_t nraw, CandOut co,
                                                   int64_t *long_list, unsigned long long *nlong, uint64_t long_cap) {
  __shared__ uint16_t sbuf[kVocabNT][66];  // 64 units + 2 of padding: lanes' slices start on different banks
  uint64_t plo = 0, phi = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nraw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t slot = (uint32_t)rlist[i];
    uint64_t r = tb.rep[slot];
    uint64_t off = r >> 24, len = r & 0xFFFFFFull;
    if (vocab_clean(co, i, slot, tb.text + off, len, sbuf[threadIdx.x], plo, phi)) continue;
    if (len > kShortRaw) {
      unsigned long long j = atomicAdd(nlong, 1ull);
      if (j < long_cap) long_list[j] = i;
      continue;
    }
    uint16_t units[kShortRaw + 2];
    uint16_t work[4 * kShortRaw + 16];
    int nu = 0;
    for (uint64_t p = 0; p < len;) {
      uint16_t tmp[2];
      int k;
      int used = utf8_step(tb.text + off, (int64_t)p, (int64_t)len, tmp, &k);
      for (int x = 0; x < k; x++) units[nu++] = tmp[x];
      p += used;
    }
    vocab_one(co, i, slot, units, nu, work, 4 * kShortRaw + 16, plo, phi);
  }
  flush_unit_bits(co.pres, plo, phi);
}

__global__ void k_vocab_long(const RawTable tb, const int32_t *rlist, CandOut co, const int64_t *long_list,
                             int64_t nlong, const int64_t *scr_off, uint16_t *scr) {
  uint64_t plo = 0, phi = 0;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nlong; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = long_list[j];
    const uint32_t slot = (uint32_t)rlist[i];
    uint64_t r = tb.rep[slot];
    uint64_t off = r >> 24, len = r & 0xFFFFFFull;
    uint16_t *units = scr + scr_off[j];
    int nu = 0;
    for (uint64_t p = 0; p < len;) {
      uint16_t tmp[2];
      int k;
      int used = utf8_step(tb.text + off, (int64_t)p, (int64_t)len, tmp, &k);
      for (int x = 0; x < k; x++) units[nu++] = tmp[x];
      p += used;
    }
    uint16_t *work = units + len + 8;
    vocab_one(co, i, slot, units, nu, work, (int)(4 * len + 16), plo, phi);
  }
  flush_unit_bits(co.pres, plo, phi);
}

// final-term dedup table over pool strings
__device__ __forceinline__ uint64_t hash_u16(const uint16_t *p, int l) {
  uint64_t h = 0x84222325cbf29ce4ull;
  for (int i = 0; i < l; i++) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  h = fmix64(h ^ (uint64_t)l);
  return h ? h : 1;
}

__global__ void k_final_insert(const uint16_t *pool, const uint64_t *cand_str, int64_t ncand,
                               unsigned long long *fkeys, unsigned long long *freps, uint64_t fmask,
                               uint32_t *cand_final, unsigned int *overflow, int32_t *maxlen) {
  int32_t ml = 0;
  uint32_t orv = 0;  // OR of every unit: a term with a unit >= 128 (no 7-bit packing of the sort keys)
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncand; c += (int64_t)gridDim.x * blockDim.x) {
    uint64_t cs = cand_str[c];
    if (cs == kNoCand) {  // raw token with no output (stopword / dropped)
      cand_final[c] = 0xFFFFFFFFu;
      continue;
    }
    const uint16_t *w = pool + (cs >> 16);
    int l = (int)(cs & 0xFFFF);
    ml = max(ml, l);
    for (int i = 0; i < l; i++) orv |= w[i];
    uint64_t h = hash_u16(w, l);
    uint64_t slot = h & fmask;
    uint32_t res = 0xFFFFFFFFu;
    for (uint64_t probe = 0; probe <= fmask; probe++) {
      unsigned long long k = ld_agent(&fkeys[slot]);
      if (k == 0) {
        unsigned long long old = atomicCAS(&fkeys[slot], 0ull, (unsigned long long)h);
        if (old == 0) {
          atomicExch(&freps[slot], (unsigned long long)(c + 1));
          res = (uint32_t)slot;
          break;
        }
        k = old;
      }
      if (k == h) {
        unsigned long long rr = ld_agent(&freps[slot]);
        for (int spin = 0; rr == 0 && spin < (1 << 22); spin++) rr = ld_agent(&freps[slot]);
        if (rr != 0) {
          uint64_t os = cand_str[rr - 1];
          const uint16_t *o = pool + (os >> 16);
          int ol = (int)(os & 0xFFFF);
          bool eq = ol == l;
          for (int i = 0; i < l && eq; i++) eq = o[i] == w[i];
          if (eq) {
            res = (uint32_t)slot;
            break;
          }
        }
      }
      slot = (slot + 1) & fmask;
    }
    if (res == 0xFFFFFFFFu) atomicOr(overflow, 1u);
    cand_final[c] = res;
  }
  // longest term and the wide flag: one atomic each per block (the candidates
  // are exactly the final terms' strings, duplicates included)
  __shared__ int32_t s_ml[4];
  __shared__ uint32_t s_or[4];
  for (int o = 32; o > 0; o >>= 1) {
    ml = max(ml, __shfl_xor(ml, o, 64));
    orv |= (uint32_t)__shfl_xor((int)orv, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_ml[threadIdx.x >> 6] = ml;
    s_or[threadIdx.x >> 6] = orv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int x = 1; x < (int)(blockDim.x >> 6); x++) {
      ml = max(ml, s_ml[x]);
      orv |= s_or[x];
    }
    if (ml > 0) atomicMax(maxlen, ml);
    if (orv >= 128u) atomicOr(maxlen + 1, 1);
  }
}

// compact occupied final slots; longest term (in units) for the LSD sort depth
// One counter atomic per block: block b owns the slot range [b R, (b + 1) R);
// it counts its used slots, reserves their output range with one atomicAdd and
// writes them (entries come out in any block order: the term sort that follows
// fixes the order).  The longest term by block max.  (A counter atomic per wave
// still serialised 131 k atomics on one address: 0.84 ms on c2.)
__global__ __launch_bounds__(256) void k_final_compact(const unsigned long long *fkeys,
                                                       const unsigned long long *freps, uint64_t fmask,
                                                       const uint64_t *cand_str, const uint16_t *pool,
                                                       unsigned long long *nV, uint32_t *vslot, uint32_t *vidx,
                                                       uint64_t *vcs) {
  __shared__ uint32_t s_w[4];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t n = fmask + 1, R = (n + gridDim.x - 1) / gridDim.x;
  const uint64_t a = blockIdx.x * R, b = min(n, a + R);
  uint32_t c = 0;
  for (uint64_t s = a + threadIdx.x; s < b; s += 256) c += fkeys[s] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) s_w[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    s_base = tot ? atomicAdd(nV, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  unsigned long long base = s_base;
  for (uint64_t s0 = a; s0 < b; s0 += 256) {
    const uint64_t s = s0 + threadIdx.x;
    const bool used = s < b && fkeys[s] != 0;
    const uint64_t m = (uint64_t)__ballot(used);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int x = 0; x < 4; x++) {
      before += x < w ? s_w[x] : 0u;
      tot += s_w[x];
    }
    if (used) {
      const unsigned long long i = base + before + __popcll(m & ((1ull << lane) - 1ull));
      vslot[i] = (uint32_t)s;
      vidx[i] = (uint32_t)i;
      vcs[i] = cand_str[freps[s] - 1];  // the term's pool string, so later passes skip two gathers
    }
    base += tot;
    __syncthreads();
  }
}

// key word w (units 4w..4w+3, big-endian, zero padded) of the term at each order position
// (cpw units of ub bits per word: 4 x 16 in general, 9 x 7 when every unit is
// ASCII -- unit order is code order either way, so fewer words to sort)
__global__ void k_term_word(const uint32_t *order, int64_t V, const uint64_t *vcs, const uint16_t *pool, int w,
                            int cpw, int ub, uint64_t *key) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t cs = vcs[order[i]];
    const uint16_t *u = pool + (cs >> 16);
    int l = (int)(cs & 0xFFFF);
    uint64_t k = 0;
    for (int j = cpw * w; j < cpw * w + cpw; j++) k = (k << ub) | (j < l ? u[j] : 0);
    key[i] = k;
  }
}

__device__ int cmp_pool(const uint16_t *pool, uint64_t a, uint64_t b) {
  const uint16_t *x = pool + (a >> 16), *y = pool + (b >> 16);
  int xl = (int)(a & 0xFFFF), yl = (int)(b & 0xFFFF);
  int m = xl < yl ? xl : yl;
  for (int i = 0; i < m; i++)
    if (x[i] != y[i]) return (int)x[i] - (int)y[i];
  return xl - yl;
}

__device__ bool same_prefix32(const uint16_t *pool, uint64_t a, uint64_t b) {
  const uint16_t *x = pool + (a >> 16), *y = pool + (b >> 16);
  int xl = (int)(a & 0xFFFF), yl = (int)(b & 0xFFFF);
  for (int i = 0; i < 32; i++) {
    uint16_t cx = i < xl ? x[i] : 0, cy = i < yl ? y[i] : 0;
    if (cx != cy) return false;
  }
  return true;
}

// order[] is sorted by the 32-unit prefix; runs of equal prefixes (terms longer than
// 32 units) are finished by full String.compareTo comparison
__global__ void k_final_fixup(uint32_t *order, int64_t V, const uint32_t *vslot, const unsigned long long *freps,
                              const uint64_t *cand_str, const uint16_t *pool) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    auto str = [&](int64_t pos) { return cand_str[freps[vslot[order[pos]]] - 1]; };
    bool start = i == 0 || !same_prefix32(pool, str(i), str(i - 1));
    if (!start) continue;
    int64_t j = i + 1;
    while (j < V && same_prefix32(pool, str(j), str(i))) j++;
    if (j - i < 2) continue;
    for (int64_t a = i + 1; a < j; a++) {  // insertion sort (runs are tiny)
      uint32_t v = order[a];
      uint64_t vs = cand_str[freps[vslot[v]] - 1];
      int64_t b = a - 1;
      while (b >= i && cmp_pool(pool, cand_str[freps[vslot[order[b]]] - 1], vs) > 0) {
        order[b + 1] = order[b];
        b--;
      }
      order[b + 1] = v;
    }
  }
}

// ASCII vocabularies: the code units in use (128-bit presence map), so a sort
// key packs ceil(log2(units + 1)) bits per unit (6 for letters and digits: 10
// units per 64-bit word instead of 9 x 7 bits)
// key of term order[i]: its first cpw units as codes (code[u] = rank of u among
// the units in use + 1; 0 pads), most significant first -- String.compareTo
// order of the first cpw units
// (the units are loaded eight at a time, all in flight together, and coded from an
// LDS copy of the table: a unit-by-unit loop waited on each load in turn)
__global__ __launch_bounds__(256) void k_term_code(const uint32_t *__restrict__ order, int64_t V,
                                                   const uint64_t *__restrict__ vcs,
                                                   const uint16_t *__restrict__ pool,
                                                   const uint8_t *__restrict__ code, int cpw, int ub,
                                                   uint64_t *__restrict__ key) {
  __shared__ uint8_t s_code[128];
  if (threadIdx.x < 128) s_code[threadIdx.x] = code[threadIdx.x];
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t cs = vcs[order[i]];
    const uint16_t *u = pool + (cs >> 16);
    const int l = min((int)(cs & 0xFFFF), cpw);
    uint64_t k = 0;
    for (int j0 = 0; j0 < cpw; j0 += 8) {
      uint16_t v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = j0 + j < l ? u[j0 + j] : (uint16_t)0;
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (j0 + j < cpw) k = (k << ub) | (j0 + j < l ? s_code[v[j] & 127] : 0u);
    }
    key[i] = k;
  }
}
// runs of equal keys (terms sharing their first cpw units): longest run
__global__ void k_key_runs(const uint64_t *key, int64_t V, unsigned int *maxrun) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    if (i > 0 && key[i] == key[i - 1]) continue;
    int64_t j = i + 1;
    while (j < V && key[j] == key[i] && j - i < 4096) j++;
    if (j - i > 1) atomicMax(maxrun, (unsigned int)(j - i));
  }
}
// order each run of equal keys by the whole string (insertion sort: runs are short)
__global__ void k_key_fixup(const uint64_t *key, int64_t V, uint32_t *order, const uint64_t *vcs,
                            const uint16_t *pool) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    if ((i > 0 && key[i] == key[i - 1]) || i + 1 >= V || key[i + 1] != key[i]) continue;
    int64_t j = i + 1;
    while (j < V && key[j] == key[i]) j++;
    for (int64_t a = i + 1; a < j; a++) {
      const uint32_t v = order[a];
      int64_t b = a - 1;
      while (b >= i && cmp_pool(pool, vcs[order[b]], vcs[v]) > 0) {
        order[b + 1] = order[b];
        b--;
      }
      order[b + 1] = v;
    }
  }
}

// rank of every final slot; term lengths in rank order
__global__ void k_final_rank(const uint32_t *order, int64_t V, const uint32_t *vslot, const uint64_t *vcs,
                             int32_t *rank_of_slot, int64_t *term_len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t o = order[i];
    rank_of_slot[vslot[o]] = (int32_t)i;
    term_len[i] = (int64_t)(vcs[o] & 0xFFFF);
  }
}

// (eight units loaded together before they are stored: with possibly aliasing
// pointers a unit-by-unit copy waited on each load in turn)
__global__ __launch_bounds__(256) void k_final_gather(const uint32_t *__restrict__ order, int64_t V,
                                                      const uint64_t *__restrict__ vcs,
                                                      const uint16_t *__restrict__ pool,
                                                      const int64_t *__restrict__ term_off,
                                                      uint16_t *__restrict__ term_chars) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t cs = vcs[order[i]];
    const uint16_t *w = pool + (cs >> 16);
    const int l = (int)(cs & 0xFFFF);
    uint16_t *d = term_chars + term_off[i];
    for (int k0 = 0; k0 < l; k0 += 8) {
      uint16_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = k0 + k < l ? w[k0 + k] : (uint16_t)0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (k0 + k < l) d[k0 + k] = v[k];
    }
  }
}

// raw slot -> term ids.  Primary candidate i (list index) gives raw_term[rlist[i]]
// for single-output tokens; multi-output tokens are resolved from the overflow
// list sorted by (slot, ordinal): multi_term[j..j+nout) and raw_term = -(2 + j).
__global__ void k_raw_term(const int32_t *rlist, int64_t nraw, const uint32_t *cand_final, const int32_t *rank_of_slot,
                           const int32_t *raw_nout, int32_t *raw_term) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nraw; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t slot = rlist[i];
    if (raw_nout[slot] == 1 && cand_final[i] != 0xFFFFFFFFu) raw_term[slot] = rank_of_slot[cand_final[i]];
  }
}
__global__ void k_raw_multi(const uint64_t *okey_s, const uint32_t *oidx_s, int64_t novf, int64_t nraw,
                            const uint32_t *cand_final, const int32_t *rank_of_slot, int32_t *raw_term,
                            int32_t *multi_term) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < novf; j += (int64_t)gridDim.x * blockDim.x) {
    multi_term[j] = rank_of_slot[cand_final[nraw + oidx_s[j]]];
    if ((uint32_t)okey_s[j] == 0) raw_term[(uint32_t)(okey_s[j] >> 32)] = -(int32_t)(2 + j);
  }
}

// ============================================================================
// K5: per-record aggregation (combiner) and emission
// ============================================================================
// K4b: docid terms (T7) beside the word vocabulary
// ============================================================================
// Every record's DOCNO text is indexed like the rest of the record
// (TrecDocument.getContent is the whole record, TrecDocument.java:94-96;
// TermKGramDocIndexer.java:129): on c5 / the c4 shard most of the vocabulary
// is docid terms, one document each.  A raw token that is a record's whole
// trimmed <DOCNO> span and whose term is provably its own lowercase form --
// ASCII letters and digits ending in a digit, at most kDocTermMax bytes, no
// stopword, and Porter2 leaves it unchanged (the stemmer is run to check) --
// skips the per-distinct normalize / dedup / sort of the word vocabulary: in
// file order such docid terms are usually ascending already (checked), so
// their ranks come from a merge with the sorted word terms.  A failed check
// (unsorted or equal docid terms, a docid term equal to a word term) keeps
// the build on the general path; the result is the same either way.
constexpr int kDocTermMax = 48;
constexpr int32_t kDocCode = 0x40000000;  // K6b: a docid term's code in raw_term (| its docid index)
constexpr uint32_t kNoRec = 0xFFFFFFFFu;

__device__ __forceinline__ uint8_t lower_ascii(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

// per record: the raw slot of its docid token when it qualifies, else -1; such
// slots marked in dmark (0; kNoRec: no docid term's).
// The docid's bytes come from k_docno (getDocid's trimmed span).  No stopword
// ends in a digit, and every rule of the 2010 Porter2 (englishStemmer.java:
// Step_0 .. Step_5, exception1 / exception2) matches a letter suffix or a whole
// letter word, so a word of [a-z0-9] ending in a digit stems to itself -- pinned
// by tests/test_docid_terms.py against the oracle's stemmer and stopword list.
// the <= 16 bytes of text[ib, ib + len) as little-endian words, by two aligned
// 16-byte loads (false: not inside the buffer, take the bytes one by one)
__device__ __forceinline__ bool span16(const uint8_t *t, int64_t n, int64_t ib, int64_t len, uint64_t &w0,
                                       uint64_t &w1) {
  const int64_t a0 = (int64_t)(((uintptr_t)(t + ib)) & 15);
  if (len > 16 || ib < a0 || ib - a0 + 32 > n) return false;
  const uint4 *q = reinterpret_cast<const uint4 *>(t + ib - a0);
  const uint4 x = q[0], y = q[1];
  const uint32_t wd[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  w0 = w1 = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int p = (int)a0 + k;
    const uint64_t c = k < len ? (wd[p >> 2] >> (8 * (p & 3))) & 0xFFu : 0u;
    if (k < 8) w0 |= c << (8 * k);
    else w1 |= c << (8 * (k - 8));
  }
  return true;
}
__device__ __forceinline__ bool alnum_byte(uint32_t c) {
  const uint32_t l = c | 0x20u;
  return (c >= '0' && c <= '9') || (l >= 'a' && l <= 'z');
}
__global__ __launch_bounds__(256) void k_docid_slots(const uint8_t *t, int64_t n, const uint64_t *dspan, int64_t nR,
                                                     const RawTable tb, int32_t *dslot, uint32_t *dmark) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x) {
    int32_t out = -1;
    const uint64_t sp = dspan[r];
    const int64_t ib = (int64_t)(sp >> 8), len = (int64_t)(sp & 0xFF);
    bool ok = len >= 2 && len <= kDocTermMax;
    TokSig g{0, 0, 0};
    uint64_t w0, w1;
    if (ok && span16(t, n, ib, len, w0, w1)) {  // the span's bytes as the signature's words, checked in registers
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k < len) ok = ok && alnum_byte((uint32_t)((k < 8 ? w0 >> (8 * k) : w1 >> (8 * (k - 8))) & 0xFFu));
      const uint32_t last = (uint32_t)((len <= 8 ? w0 >> (8 * (len - 1)) : w1 >> (8 * (len - 9))) & 0xFFu);
      ok = ok && last >= '0' && last <= '9';
      g = TokSig{sig_head(w0, w1), w0, w1};
    } else if (ok) {
      ok = t[ib + len - 1] >= '0' && t[ib + len - 1] <= '9';
      for (int64_t k = 0; k < len && ok; k++) ok = alnum_byte(t[ib + k]);
      if (ok) g = sig_bytes(t + ib, len);
    }
    if (ok) {  // its raw slot (the table is complete: plain loads)
      uint64_t s = g.h & tb.mask;
      for (uint64_t probe = 0; probe <= tb.mask && probe <= kMaxProbe; probe++, s = (s + 1) & tb.mask) {
        const unsigned long long key = tb.key[s];
        if (key == 0) break;
        if (key != g.h) continue;
        const ulonglong2 tw = tb.tok[s];
        if (tw.x != g.w0 || tw.y != g.w1) continue;
        bool eq = true;  // (<= 16 bytes: no token byte is 0, so w0 / w1 decide)
        if (len > 16) {
          const uint64_t rp = tb.rep[s];
          eq = (int64_t)(rp & 0xFFFFFFull) == len;
          for (int64_t k = 16; k < len && eq; k++) eq = tb.text[(rp >> 24) + k] == t[ib + k];
        }
        if (eq) {
          out = (int32_t)s;
          break;
        }
      }
      if (out >= 0) dmark[out] = 0u;  // a docid term's slot (a docid in two records: the ascending check fails)
    }
    dslot[r] = out;
  }
}

// the word vocabulary's raw tokens: every used slot that is no docid term's
__global__ void k_raw_flags_words(const unsigned long long *key, const uint32_t *dmark, uint64_t n, uint8_t *flag) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < n; s += (uint64_t)gridDim.x * blockDim.x)
    flag[s] = key[s] != 0 && dmark[s] == kNoRec;
}

__global__ void k_docid_flags(const int32_t *dslot, int64_t nR, uint8_t *flag) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x)
    flag[r] = dslot[r] >= 0;
}

// big-endian 16-byte key of a term's first 16 units (all < 256; zero padded: no
// unit is 0, so a shorter string sorts first) -- exact String.compareTo order for
// terms of <= 16 such units
struct Key16 {
  uint64_t hi, lo;
};
__device__ __forceinline__ int cmp_key16(const Key16 &a, const Key16 &b) {
  if (a.hi != b.hi) return a.hi < b.hi ? -1 : 1;
  if (a.lo != b.lo) return a.lo < b.lo ? -1 : 1;
  return 0;
}
__device__ __forceinline__ Key16 key16_bytes(const uint8_t *p, int len) {  // lowercase ASCII docid bytes
  Key16 k{0, 0};
  for (int i = 0; i < 16; i++) {
    const uint64_t c = i < len ? lower_ascii(p[i]) : 0;
    if (i < 8) k.hi |= c << (56 - 8 * i);
    else k.lo |= c << (56 - 8 * (i - 8));
  }
  return k;
}
// docid term j: (text offset << 8 | length) of its docid span (the bytes of its
// raw slot) and its key
// byte k of a Key16 (k < 16)
__device__ __forceinline__ uint32_t key16_byte(const Key16 &k, int i) {
  return (uint32_t)((i < 8 ? k.hi >> (56 - 8 * i) : k.lo >> (56 - 8 * (i - 8))) & 0xFFu);
}
__global__ void k_docid_keys(const int32_t *dl, int64_t Vd, const uint64_t *dspan, const uint8_t *text, int64_t n,
                             uint64_t *dsrc, Key16 *dkey) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t sp = dspan[dl[j]];  // (the docid span's bytes: those of its raw slot)
    const int64_t ib = (int64_t)(sp >> 8), len = (int64_t)(sp & 0xFF);
    dsrc[j] = sp;
    uint64_t w0, w1;
    if (span16(text, n, ib, len, w0, w1)) {
      // letters and digits: lowercase = | 0x20 on every byte of the term (digits have the bit)
      const uint64_t m0 = len >= 8 ? ~0ull : ((1ull << (8 * len)) - 1), m1 = len >= 16 ? ~0ull : len <= 8 ? 0ull
                                                                                       : ((1ull << (8 * (len - 8))) - 1);
      dkey[j] = Key16{__builtin_bswap64((w0 | 0x2020202020202020ull) & m0), __builtin_bswap64((w1 | 0x2020202020202020ull) & m1)};
    } else {
      dkey[j] = key16_bytes(text + ib, (int)len);
    }
  }
}
// String.compareTo of two docid terms (lowercase ASCII bytes)
__device__ int cmp_docid(const uint8_t *text, uint64_t a, uint64_t b) {
  const uint8_t *x = text + (a >> 8), *y = text + (b >> 8);
  const int xl = (int)(a & 0xFF), yl = (int)(b & 0xFF), m = xl < yl ? xl : yl;
  for (int i = 0; i < m; i++) {
    const int d = (int)lower_ascii(x[i]) - (int)lower_ascii(y[i]);
    if (d) return d;
  }
  return xl - yl;
}
// in file order the docid terms must be strictly ascending (else: general path)
__global__ void k_docid_ascending(const Key16 *dkey, const uint64_t *dsrc, int64_t Vd, const uint8_t *text,
                                  unsigned long long *bad) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x + 1; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    int c = cmp_key16(dkey[j - 1], dkey[j]);
    if (c == 0 && ((dsrc[j - 1] & 0xFF) > 16 || (dsrc[j] & 0xFF) > 16)) c = cmp_docid(text, dsrc[j - 1], dsrc[j]);
    if (c >= 0) atomicAdd(bad, 1ull);
  }
}
// a docid term equal to a word term (final dedup table of the word candidates)
__global__ void k_docid_collide(const uint64_t *dsrc, const Key16 *dkey, int64_t Vd, const uint8_t *text,
                                const uint16_t *pool, const uint64_t *cand_str, const unsigned long long *fkeys,
                                const unsigned long long *freps, uint64_t fmask, unsigned long long *bad) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t *p = text + (dsrc[j] >> 8);
    const int l = (int)(dsrc[j] & 0xFF);
    const Key16 kj = dkey[j];
    auto unit = [&](int i) -> uint32_t { return l <= 16 ? key16_byte(kj, i) : lower_ascii(p[i]); };
    uint64_t h = 0x84222325cbf29ce4ull;  // hash_u16 of the lowercase units
    for (int i = 0; i < l; i++) {
      h ^= unit(i);
      h *= 0x100000001b3ull;
    }
    h = fmix64(h ^ (uint64_t)l);
    h = h ? h : 1;
    for (uint64_t s = h & fmask, probe = 0; probe <= fmask; probe++, s = (s + 1) & fmask) {
      const unsigned long long k = fkeys[s];
      if (k == 0) break;
      if (k != h) continue;
      const uint64_t os = cand_str[freps[s] - 1];
      const uint16_t *o = pool + (os >> 16);
      bool eq = (int)(os & 0xFFFF) == l;
      for (int i = 0; i < l && eq; i++) eq = o[i] == unit(i);
      if (eq) {
        atomicAdd(bad, 1ull);
        break;
      }
    }
  }
}
// sorted word term i: its key (exact when it has <= 16 units, all < 256)
__global__ void k_word_keys(const uint32_t *order, int64_t Vw, const uint64_t *vcs, const uint16_t *pool, Key16 *wkey,
                            uint8_t *wexact) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < Vw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t cs = vcs[order[i]];
    const uint16_t *u = pool + (cs >> 16);
    const int l = (int)(cs & 0xFFFF);
    Key16 k{0, 0};
    bool ex = l <= 16;
    for (int x = 0; x < 16; x++) {
      const uint32_t c = x < l ? u[x] : 0u;
      ex = ex && c < 256u;
      const uint64_t b = c < 256u ? c : 255u;  // (saturated: the key then only bounds, compare the strings)
      if (x < 8) k.hi |= b << (56 - 8 * x);
      else k.lo |= b << (56 - 8 * (x - 8));
    }
    wkey[i] = k;
    wexact[i] = ex;
  }
}
// String.compareTo(word term, docid term)
__device__ int cmp_word_docid(const uint16_t *pool, uint64_t cs, const uint8_t *text, uint64_t ds) {
  const uint16_t *w = pool + (cs >> 16);
  const uint8_t *p = text + (ds >> 8);
  const int wl = (int)(cs & 0xFFFF), dl = (int)(ds & 0xFF), m = wl < dl ? wl : dl;
  for (int i = 0; i < m; i++) {
    const int d = (int)w[i] - (int)lower_ascii(p[i]);
    if (d) return d;
  }
  return wl - dl;
}
__device__ __forceinline__ int cmp_wd(const Key16 &wk, bool wex, const uint16_t *pool, uint64_t cs, const Key16 &dk,
                                      const uint8_t *text, uint64_t ds) {
  if (wex && (ds & 0xFF) <= 16) return cmp_key16(wk, dk);
  return cmp_word_docid(pool, cs, text, ds);
}
// merged ranks: word i -> i + (docid terms below it); docid j -> j + (words below it)
__global__ void k_word_rank(const uint32_t *order, int64_t Vw, const uint32_t *vslot, const uint64_t *vcs,
                            const uint16_t *pool, const Key16 *wkey, const uint8_t *wexact, const Key16 *dkey,
                            const uint64_t *dsrc, int64_t Vd, const uint8_t *text, int32_t *rank_of_slot,
                            int64_t *term_len, int64_t *wrank, int split) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < Vw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t o = order[i];
    const uint64_t cs = vcs[o];
    const Key16 wk = wkey[i];
    const bool wex = wexact[i];
    int64_t lo = 0, hi = Vd;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (cmp_wd(wk, wex, pool, cs, dkey[mid], text, dsrc[mid]) > 0) lo = mid + 1;
      else hi = mid;
    }
    const int64_t rk = i + lo;
    rank_of_slot[vslot[o]] = (int32_t)(split ? i : rk);  // (split: the word's own rank, see kDocCode)
    term_len[rk] = (int64_t)(cs & 0xFFFF);
    wrank[i] = rk;
  }
}
__global__ void k_docid_rank(const Key16 *dkey, const uint64_t *dsrc, int64_t Vd, const uint32_t *order, int64_t Vw,
                             const uint64_t *vcs, const uint16_t *pool, const Key16 *wkey, const uint8_t *wexact,
                             const uint8_t *text, int64_t *term_len, int64_t *drank) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    const Key16 dk = dkey[j];
    const uint64_t ds = dsrc[j];
    int64_t lo = 0, hi = Vw;  // words below docid term j
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (cmp_wd(wkey[mid], wexact[mid], pool, vcs[order[mid]], dk, text, ds) < 0) lo = mid + 1;
      else hi = mid;
    }
    const int64_t rk = j + lo;
    term_len[rk] = (int64_t)(ds & 0xFF);
    drank[j] = rk;
  }
}
// term chars in rank order: the word terms' from the pool, the docid terms'
// lowercase bytes from the text
__global__ __launch_bounds__(256) void k_word_gather(const uint32_t *__restrict__ order, int64_t Vw,
                                                     const uint64_t *__restrict__ vcs,
                                                     const uint16_t *__restrict__ pool,
                                                     const int64_t *__restrict__ wrank,
                                                     const int64_t *__restrict__ term_off,
                                                     uint16_t *__restrict__ term_chars) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < Vw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t cs = vcs[order[i]];
    const uint16_t *w = pool + (cs >> 16);
    const int l = (int)(cs & 0xFFFF);
    uint16_t *d = term_chars + term_off[wrank[i]];
    for (int k0 = 0; k0 < l; k0 += 8) {
      uint16_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = k0 + k < l ? w[k0 + k] : (uint16_t)0;
#pragma unroll
      for (int k = 0; k < 8; k++)
        if (k0 + k < l) d[k0 + k] = v[k];
    }
  }
}
__global__ void k_docid_gather(const uint64_t *dsrc, const Key16 *dkey, int64_t Vd, const int64_t *drank,
                               const uint8_t *text, const int64_t *term_off, uint16_t *term_chars) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t *p = text + (dsrc[j] >> 8);
    const int l = (int)(dsrc[j] & 0xFF);
    uint16_t *d = term_chars + term_off[drank[j]];
    if (l <= 16) {
      const Key16 kj = dkey[j];
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k < l) d[k] = (uint16_t)key16_byte(kj, k);
    } else {
      for (int k = 0; k < l; k++) d[k] = lower_ascii(p[k]);
    }
  }
}
// raw slot -> term id of the docid terms (one term each)
__global__ void k_docid_raw(const int32_t *dl, int64_t Vd, const int32_t *dslot, const int64_t *drank,
                            int32_t *raw_term, int32_t *raw_nout, int split) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = dslot[dl[j]];
    raw_term[s] = split ? (kDocCode | (int32_t)j) : (int32_t)drank[j];
    raw_nout[s] = 1;
  }
}

// ---------------------------------------------------------------------------
// K6b: docid pairs beside the term sort.  On c5 / the c4 shard the docid terms
// push the term ids past 22 bits (three LSD passes), while the word terms alone
// fit two.  With the split, the raw slots carry term CODES -- a word's rank among
// the words, kDocCode | j for docid term j -- and the aggregation writes each
// record's one docid pair (its own docid) beside its word pairs instead of into
// its region.  The word pairs are sorted by word rank; the last pass shifts word
// i's postings by the docid pairs whose terms sort below it (wshift.x) and writes
// its merged id (wshift.y); the docid pairs (one per record, docno order, sorted
// by j when they are not already) then fill the remaining slots: pair q of
// docid term j lands after the word pairs below j.  The CSR is the one the
// single sort builds; a record with two docid-term pairs (a docid in another
// record's text) sends the aggregation back to merged ids.
__global__ void k_code_to_merged(int32_t *raw_term, uint64_t rcap, int32_t *multi, int64_t nmulti,
                                 const int64_t *wrank, const int64_t *drank) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < rcap + (uint64_t)nmulti; s += gs) {
    int32_t *p = s < rcap ? raw_term + s : multi + (s - rcap);
    const int32_t v = *p;
    if (v >= 0) *p = (int32_t)((v & kDocCode) ? drank[v & ~kDocCode] : wrank[v]);
  }
}
__global__ void k_dsplit_flags(const int32_t *dk_rec, int64_t nR, uint8_t *flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x)
    flag[i] = dk_rec[i] >= 0;
}
__global__ void k_dsplit_gather(const int32_t *idx, const unsigned long long *nd, const int32_t *dk_rec,
                                const uint32_t *dv_rec, uint32_t *dk, uint32_t *dv, unsigned long long *desc) {
  const int64_t n = (int64_t)*nd;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    dk[q] = (uint32_t)dk_rec[idx[q]];
    dv[q] = dv_rec[idx[q]];
    if (q > 0 && dk_rec[idx[q - 1]] > dk_rec[idx[q]]) atomicAdd(desc, 1ull);
  }
}
// word i: (docid pairs of terms below it, its merged id)
__global__ void k_word_shift(const int64_t *wrank, int64_t Vw, const uint32_t *dk, int64_t Nd, uint2 *ws) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < Vw; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t below = (uint32_t)(wrank[i] - i);  // docid terms below word i
    int64_t lo = 0, hi = Nd;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (dk[m] < below) lo = m + 1;
      else hi = m;
    }
    ws[i] = make_uint2((uint32_t)lo, (uint32_t)wrank[i]);
  }
}
// word pairs below docid term j: where word x = (words below j) starts, less its shift
__device__ __forceinline__ int64_t words_below(int64_t j, const int64_t *drank, const int64_t *wrank, int64_t Vw,
                                               const uint2 *ws, const int64_t *off, int64_t Pw) {
  const int64_t x = drank[j] - j;
  return x < Vw ? off[wrank[x]] - (int64_t)ws[x].x : Pw;
}
// docid pair q -> its CSR slot (docno / tf / weight / key)
__global__ void k_docid_place(const uint32_t *dk, const uint32_t *dv, int64_t Nd, const int64_t *drank,
                              const int64_t *wrank, int64_t Vw, const uint2 *ws, const int64_t *off, int64_t Pw,
                              int64_t dmin, uint32_t F, int32_t *docno, int32_t *tf, uint32_t *key, const double *lut,
                              double idf, double *w) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < Nd; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = dk[q];
    const int64_t p = q + words_below(j, drank, wrank, Vw, ws, off, Pw);
    const uint32_t v = dv[q];
    docno[p] = (int32_t)((int64_t)(v / F) + dmin);
    tf[p] = (int32_t)(v % F);
    key[p] = (uint32_t)drank[j];
    if (w) w[p] = __dmul_rn(lut[v % F], idf);
  }
}
// docid term j's first posting (its df may be 0 or > 1)
__global__ void k_docid_off(const uint32_t *dk, int64_t Nd, int64_t Vd, const int64_t *drank, const int64_t *wrank,
                            int64_t Vw, const uint2 *ws, int64_t Pw, int64_t *off) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vd; j += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = Nd;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if ((int64_t)dk[m] < j) lo = m + 1;
      else hi = m;
    }
    off[drank[j]] = lo + words_below(j, drank, wrank, Vw, ws, off, Pw);
  }
}

// ============================================================================
constexpr int kAggNT = 256;
constexpr int kAggCap = 4096;    // LDS table entries
constexpr int kAggLimit = 3072;  // beyond this many distinct terms: global-table path

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// insert term into an open-addressing table (keys -1 = empty); returns false on overflow
__device__ __forceinline__ bool agg_insert(int32_t *keys, int32_t *cnt, uint32_t cap_mask, int32_t term,
                                           int32_t *distinct, int32_t limit) {
  uint32_t h = hash32((uint32_t)term) & cap_mask;
  for (uint32_t probe = 0; probe <= cap_mask; probe++) {
    int32_t old = atomicCAS(&keys[h], -1, term);
    if (old == -1) {
      int32_t d = atomicAdd(distinct, 1);
      atomicAdd(&cnt[h], 1);
      return d < limit;
    }
    if (old == term) {
      atomicAdd(&cnt[h], 1);
      return true;
    }
    h = (h + 1) & cap_mask;
  }
  return false;
}

struct AggIn {
  const uint64_t *rs;
  const uint32_t *tokstream;
  const int32_t *ntok;
  const int32_t *raw_term;
  const int32_t *raw_nout;
  const int32_t *multi_term;
  const int32_t *max_nout = nullptr;  // largest number of terms one raw token yields
  const int64_t *perm;   // records in docno order
  const int32_t *docno;  // per record
  // emit form: v32 != nullptr writes the sort's packed u32 value (docno - dmin) * F + tf
  // directly (K = 1, distinct docnos); otherwise p_val = docno << 32 | tf
  uint32_t *v32 = nullptr;
  int64_t dmin = 0;
  uint32_t F = 0;
  unsigned int *max_tf = nullptr;  // count pass: largest tf of any pair (atomicMax)
  // single-pass form (reg_off != nullptr): record i's pairs go to the start of its
  // region [reg_off[i], reg_off[i + 1]) (sized by its token count times max_nout,
  // an upper bound of its distinct terms) and their number to dcnt[i]; the term
  // sort's first pass reads pair x of the docno order from the region of the
  // record holding it (exclusive scan of dcnt), so no count pass and no
  // compaction.  Big records are listed for k_agg_big.
  const int64_t *reg_off = nullptr;
  int64_t *dcnt = nullptr;
  int64_t *big_out = nullptr;
  unsigned long long *nbig = nullptr;
  // K6b split (single-pass form only): a pair whose term code has kDocCode goes to
  // dk_rec[i] / dv_rec[i] (record i in docno order) instead of the region; a
  // second one in the same record sets *dbad
  int32_t *dk_rec = nullptr;
  uint32_t *dv_rec = nullptr;
  unsigned long long *dbad = nullptr;
};
// a record's docid pair beside its region (K6b): the first claims the record's slot
__device__ __forceinline__ void put_docid_pair(const AggIn &in, int64_t i, int32_t code, uint32_t v) {
  if (atomicCAS(&in.dk_rec[i], -1, code & ~kDocCode) == -1) in.dv_rec[i] = v;
  else atomicAdd(in.dbad, 1ull);
}

// Aggregate record r into table (keys/cnt, capacity mask). Returns distinct count or -1 on overflow.
__device__ int32_t agg_record(const AggIn &in, int64_t r, int32_t *keys, int32_t *cnt, uint32_t cap_mask,
                              int32_t limit, int32_t *s_distinct, int32_t *s_ovf) {
  for (uint32_t i = threadIdx.x; i <= cap_mask; i += blockDim.x) {
    keys[i] = -1;
    cnt[i] = 0;
  }
  if (threadIdx.x == 0) {
    *s_distinct = 0;
    *s_ovf = 0;
  }
  __syncthreads();
  const uint32_t *ts = in.tokstream + (in.rs[r] >> 1);
  const int32_t nt = in.ntok[r];
  for (int32_t i = threadIdx.x; i < nt; i += blockDim.x) {
    uint32_t slot = ts[i];
    int32_t rt = in.raw_term[slot];
    if (rt >= 0) {
      if (!agg_insert(keys, cnt, cap_mask, rt, s_distinct, limit)) *s_ovf = 1;
    } else if (rt <= -2) {
      int32_t m0 = -rt - 2, mn = in.raw_nout[slot];
      for (int32_t m = 0; m < mn; m++)
        if (!agg_insert(keys, cnt, cap_mask, in.multi_term[m0 + m], s_distinct, limit)) *s_ovf = 1;
    }
  }
  __syncthreads();
  int32_t d = *s_ovf ? -1 : *s_distinct;
  __syncthreads();
  return d;
}

template <bool EMIT>
__global__ __launch_bounds__(kAggNT) void k_agg(AggIn in, int64_t nR, int32_t *prec, const int64_t *pair_off,
                                                uint32_t *p_term, uint64_t *p_val) {
  __shared__ int32_t keys[kAggCap];
  __shared__ int32_t cnt[kAggCap];
  __shared__ int32_t s_distinct, s_ovf;
  __shared__ int32_t sc32[kAggNT / 64 + 1];
  for (int64_t i = blockIdx.x; i < nR; i += gridDim.x) {
    const int64_t r = in.perm[i];
    if (EMIT && prec[i] < 0) continue;  // big record, handled by k_agg_big
    int32_t d = agg_record(in, r, keys, cnt, kAggCap - 1, kAggLimit, &s_distinct, &s_ovf);
    if (!EMIT) {
      if (threadIdx.x == 0) prec[i] = d;
      continue;
    }
    // compact table -> (term, docno, tf) at pair_off[i]
    const int per = kAggCap / kAggNT;
    int32_t c = 0;
    for (int k = 0; k < per; k++) c += keys[threadIdx.x * per + k] >= 0;
    int32_t tot;
    int32_t o = block_excl_sum<kAggNT, int32_t>(c, sc32, &tot);
    int64_t base = pair_off[i] + o;
    const uint64_t dn = (uint64_t)(uint32_t)in.docno[r] << 32;
    for (int k = 0; k < per; k++) {
      int32_t key = keys[threadIdx.x * per + k];
      if (key >= 0) {
        p_term[base] = (uint32_t)key;
        p_val[base] = dn | (uint32_t)cnt[threadIdx.x * per + k];
        base++;
      }
    }
    __syncthreads();
  }
}

// Wave-per-record aggregation (the common case): each wave owns a 1024-entry
// LDS table, so records proceed independently with no workgroup barriers.
// Records with more than kWLimit distinct terms are flagged (-1) and handled by
// the block-wide k_agg / global-table path.  Pairs of record i (docno order)
// are written at pair_off[i] in 16 coalesced rounds of 64 table entries.
constexpr int kWCap = 1024;
constexpr int kWLimit = 768;
#ifndef SME_AGGU
#define SME_AGGU 8
#endif
constexpr int kAggU = SME_AGGU;

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// insert into the record's table of cap slots (a power of two <= kWCap); the
// counts are u16 pairs (slot h in the low / high half of word h / 2: a record
// of < 2^16 tokens cannot carry one into the other), 6 KB of LDS per wave
__device__ __forceinline__ bool aggw_insert(int32_t *keys, uint32_t *cnt2, int32_t term, uint32_t cap) {
  uint32_t h = hash32((uint32_t)term) & (cap - 1);
  for (uint32_t probe = 0; probe < cap; probe++) {
    const int32_t old = atomicCAS(&keys[h], -1, term);
    if (old == -1 || old == term) {
      atomicAdd(&cnt2[h >> 1], 1u << ((h & 1u) << 4));
      return true;
    }
    h = (h + 1) & (cap - 1);
  }
  return false;
}

// aggregation workgroups: one wave per record in turn, at most 8192 workgroups
// ("agg_grid" overrides)
static unsigned agg_grid_for(const sme_ctx *cx, int64_t nR) {
  const int64_t g = cx->opt_agg_grid > 0 ? cx->opt_agg_grid : 8192;
  return (unsigned)std::min<int64_t>(std::max<int64_t>((nR + 3) / 4, 1), g);
}

template <bool EMIT>
__global__ __launch_bounds__(kAggNT) void k_agg_w(AggIn in, int64_t nR, int32_t *prec, const int64_t *pair_off,
                                                  uint32_t *p_term, uint64_t *p_val) {
  __shared__ int32_t keys_all[kAggNT / 64][kWCap];
  __shared__ uint32_t cnt_all[kAggNT / 64][kWCap / 2];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int32_t *keys = keys_all[wv];
  uint32_t *cnt2 = cnt_all[wv];
  auto cnt_at = [&](uint32_t k) { return (int32_t)((cnt2[k >> 1] >> ((k & 1u) << 4)) & 0xFFFFu); };
  const int64_t nwaves = (int64_t)gridDim.x * (kAggNT / 64);
  uint32_t wmax = 0;  // count pass / single pass: largest tf over this wave's records
  const bool fused = EMIT && in.reg_off != nullptr;
  const int32_t max_nout = max(in.max_nout ? *in.max_nout : 1, 1);
  // software pipeline over the wave's records: the next record's metadata (its
  // record index, token-stream offset, token count, docno, pair base) loads while
  // this one runs, and the record index after it -- a short record (c5: ~56
  // tokens) otherwise waits on three dependent global loads before its first
  // token load
  struct Meta {
    int64_t r, base;
    uint64_t rs;
    int32_t nt, dn, pr;
  };
  auto load_meta = [&](int64_t j, int64_t r) {
    Meta m{r, 0, 0, 0, 0, 0};
    if (j < nR) {
      m.rs = in.rs[r];
      m.nt = in.ntok[r];
      if (EMIT) {
        m.dn = in.docno[r];
        m.base = fused ? in.reg_off[j] : pair_off[j];
        if (!fused) m.pr = prec[j];
      }
    }
    return m;
  };
  const int64_t i0 = (int64_t)blockIdx.x * (kAggNT / 64) + wv;
  Meta cur = load_meta(i0, i0 < nR ? in.perm[i0] : 0);
  int64_t rn = i0 + nwaves < nR ? in.perm[i0 + nwaves] : 0;
  for (int64_t i = i0; i < nR; i += nwaves) {
    const Meta nxt = load_meta(i + nwaves, rn);
    rn = i + 2 * nwaves < nR ? in.perm[i + 2 * nwaves] : 0;
    const Meta m = cur;
    cur = nxt;
    if (EMIT && !fused && m.pr < 0) continue;  // big record: block path
    const uint32_t *ts = in.tokstream + (m.rs >> 1);
    const int32_t nt = m.nt;
    // table of cap slots, a power of two (load <= 2/3 when every token has one
    // term), so short records clear and scan little; a record whose terms do not
    // fit goes to the big-record path
    uint32_t cap = 64;
    // (>= 1.5 x the tokens: load <= 2/3; c4's 200-341-token records take 512
    // slots instead of 1024, halving their clear / count / emit scans: c4 shard
    // aggregate 19.1 -> 18.2 ms; c2's 400-600-token records keep 1024)
    while (cap < kWCap && (int64_t)cap < (3 * (int64_t)nt + 1) / 2) cap <<= 1;
    for (uint32_t k = lane; k < cap; k += 64) {
      keys[k] = -1;
      if (k < cap / 2) cnt2[k] = 0;
    }
    wave_sync_lds();
    // the u16 counts hold up to 65535: bound the record's TERM count (a raw token
    // can yield up to max_nout terms, e.g. a dotted split), not its token count;
    // beyond it the record takes the big-record path
    bool ok = (int64_t)nt * (int64_t)max_nout < 65536;
    // kAggU tokens per lane step: their stream loads, then their raw_term
    // gathers, are in flight together (one step was two dependent latencies)
    for (int32_t t0 = lane; t0 < nt; t0 += kAggU * 64) {
      uint32_t slot[kAggU];
      int32_t rt[kAggU];
#pragma unroll
      for (int u = 0; u < kAggU; u++) slot[u] = t0 + u * 64 < nt ? ld_stream(ts + t0 + u * 64) : 0u;
#pragma unroll
      for (int u = 0; u < kAggU; u++) rt[u] = t0 + u * 64 < nt ? in.raw_term[slot[u]] : -1;
#pragma unroll
      for (int u = 0; u < kAggU; u++) {
        if (rt[u] >= 0) {
          ok &= aggw_insert(keys, cnt2, rt[u], cap);
        } else if (rt[u] <= -2) {
          const int32_t m0 = -rt[u] - 2, mn = in.raw_nout[slot[u]];
          for (int32_t m = 0; m < mn; m++) ok &= aggw_insert(keys, cnt2, in.multi_term[m0 + m], cap);
        }
      }
    }
    wave_sync_lds();
    int32_t d = 0;
    for (uint32_t k = 0; k < cap; k += 64) d += __popcll((uint64_t)__ballot(keys[k + lane] >= 0));
    const bool big = __any(!ok) || d > kWLimit;
    if (!EMIT) {
      if (lane == 0) prec[i] = big ? -1 : d;
      if (!big && in.max_tf) {
#pragma unroll 4
        for (uint32_t k = 0; k < cap; k += 64) wmax = max(wmax, (uint32_t)cnt_at(k + lane));
      }
      wave_sync_lds();
      continue;
    }
    if (fused && big) {
      if (lane == 0) in.big_out[atomicAdd(in.nbig, 1ull)] = i;
      wave_sync_lds();
      continue;
    }
    int64_t base = m.base;
    const uint64_t dn = (uint64_t)(uint32_t)m.dn << 32;
    const uint32_t vdoc = (uint32_t)(((int64_t)m.dn - in.dmin) * (int64_t)in.F);
    int32_t nd = 0;  // K6b: docid pairs kept beside the region
    for (uint32_t k = 0; k < cap; k += 64) {
      const int32_t key = keys[k + lane];
      const bool isd = fused && in.dk_rec && key >= 0 && (key & kDocCode);
      const uint64_t m = __ballot(key >= 0 && !isd);
      if (key >= 0) {
        const int32_t c = cnt_at(k + lane);
        if (isd) {  // (plain stores: a second docid pair in the record is caught by nd below)
          in.dk_rec[i] = key & ~kDocCode;
          in.dv_rec[i] = vdoc + (uint32_t)c;
        } else {
          const int64_t o = base + __popcll(m & ((1ull << lane) - 1ull));
          st_stream(p_term + o, (uint32_t)key);
          if (in.v32)
            st_stream(in.v32 + o, vdoc + (uint32_t)c);
          else
            p_val[o] = dn | (uint32_t)c;
        }
        if (fused) wmax = max(wmax, (uint32_t)c);
      }
      if (in.dk_rec) nd += __popcll((uint64_t)__ballot(isd));
      base += __popcll(m);
    }
    if (fused && lane == 0) in.dcnt[i] = d - nd;
    if (nd > 1 && lane == 0) *in.dbad = 1ull;  // two docid terms' pairs: merged ids (K6b fallback)
    wave_sync_lds();
  }
  if (fused || (!EMIT && in.max_tf)) {  // largest tf: one atomic per block (single-address atomics serialise)
    __shared__ uint32_t s_wmax[kAggNT / 64];
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
    if (lane == 0) s_wmax[wv] = wmax;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int x = 1; x < kAggNT / 64; x++) wmax = max(wmax, s_wmax[x]);
      if (wmax) atomicMax(in.max_tf, wmax);
    }
  }
}

// records with more than kAggLimit distinct terms: table in global scratch
__global__ __launch_bounds__(kAggNT) void k_agg_big(AggIn in, const int64_t *big_list, int64_t nbig,
                                                    const int64_t *tab_off, const int64_t *tab_cap, int32_t *gkeys,
                                                    int32_t *gcnt, int32_t *prec_count, const int64_t *pair_off,
                                                    uint32_t *p_term, uint64_t *p_val, int pass) {
  __shared__ int32_t s_distinct, s_ovf;
  __shared__ int32_t sc32[kAggNT / 64 + 1];
  for (int64_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    const int64_t i = big_list[b];
    const int64_t r = in.perm[i];
    int32_t *keys = gkeys + tab_off[b], *cnt = gcnt + tab_off[b];
    uint32_t cap = (uint32_t)tab_cap[b];
    int32_t d = agg_record(in, r, keys, cnt, cap - 1, (int32_t)cap, &s_distinct, &s_ovf);
    if (pass == 0) {
      if (threadIdx.x == 0) prec_count[i] = d;
      if (in.max_tf) {
        uint32_t m = 0;
        for (uint32_t k = threadIdx.x; k < cap; k += kAggNT) m = max(m, keys[k] >= 0 ? (uint32_t)cnt[k] : 0u);
        for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
        if ((threadIdx.x & 63) == 0 && m) atomicMax(in.max_tf, m);
      }
      __syncthreads();
      continue;
    }
    // emit: chunked compaction over the table (pass 2: into the record's region,
    // whose rest gets gap keys; pair count and largest tf to the counters)
    int64_t base = pair_off[i];
    if (pass == 2 && in.max_tf) {
      uint32_t m = 0;
      for (uint32_t k = threadIdx.x; k < cap; k += kAggNT) m = max(m, keys[k] >= 0 ? (uint32_t)cnt[k] : 0u);
      for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
      if ((threadIdx.x & 63) == 0 && m) atomicMax(in.max_tf, m);
    }
    for (uint32_t c0 = 0; c0 < cap; c0 += kAggNT) {
      uint32_t k = c0 + threadIdx.x;
      int32_t key = k < cap ? keys[k] : -1;
      if (pass == 2 && in.dk_rec && key >= 0 && (key & kDocCode)) {  // K6b: beside the region
        put_docid_pair(in, i, key, (uint32_t)(((int64_t)in.docno[r] - in.dmin) * (int64_t)in.F + cnt[k]));
        key = -1;
      }
      int32_t tot;
      int32_t o = block_excl_sum<kAggNT, int32_t>(key >= 0 ? 1 : 0, sc32, &tot);
      if (key >= 0) {
        p_term[base + o] = (uint32_t)key;
        if (in.v32)
          in.v32[base + o] = (uint32_t)(((int64_t)in.docno[r] - in.dmin) * (int64_t)in.F + cnt[k]);
        else
          p_val[base + o] = ((uint64_t)(uint32_t)in.docno[r] << 32) | (uint32_t)cnt[k];
      }
      base += tot;
    }
    if (pass == 2 && threadIdx.x == 0) in.dcnt[i] = base - pair_off[i];
    __syncthreads();
  }
}

// ============================================================================
// K6-K8: CSR assembly
// ============================================================================
// first posting of every term (key sorted); four keys per 16-byte load
// (HOLES: slots keyed 0xFFFFFFFF -- the docid pairs' places in the K6b split --
// are skipped; the docid terms' offsets are set by k_docid_off)
template <bool HOLES>
__global__ void k_term_offsets(const uint32_t *key, int64_t P, int64_t *off, int64_t V) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = P >> 2;
  constexpr uint32_t H = 0xFFFFFFFFu;
  for (int64_t q = gid; q < n4; q += gs) {
    const uint4 k = reinterpret_cast<const uint4 *>(key)[q];
    const int64_t i = q << 2;
    const uint32_t prev = i == 0 ? ~k.x : key[i - 1];
    if (k.x != prev && (!HOLES || k.x != H)) off[k.x] = i;
    if (k.y != k.x && (!HOLES || k.y != H)) off[k.y] = i + 1;
    if (k.z != k.y && (!HOLES || k.z != H)) off[k.z] = i + 2;
    if (k.w != k.z && (!HOLES || k.w != H)) off[k.w] = i + 3;
  }
  for (int64_t i = (n4 << 2) + gid; i < P; i += gs)
    if ((i == 0 || key[i] != key[i - 1]) && (!HOLES || key[i] != H)) off[key[i]] = i;
  if (gid == 0) off[V] = P;
}

__global__ void k_unpack_vals(const uint64_t *val, int64_t P, int32_t *docno, int32_t *tf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t v = val[i];
    docno[i] = (int32_t)(uint32_t)(v >> 32);
    tf[i] = (int32_t)(uint32_t)v;
  }
}

// duplicate docno handling: composite key (term, docno) for reduce-by-key
__global__ void k_dup_keys(const uint32_t *key, const uint64_t *val, int64_t P, uint64_t *ck, int32_t *tf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    ck[i] = ((uint64_t)key[i] << 32) | (uint32_t)(val[i] >> 32);
    tf[i] = (int32_t)(uint32_t)val[i];
  }
}
__global__ void k_dup_unpack(const uint64_t *ck, const int32_t *tf, int64_t P, uint32_t *key, uint64_t *val) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    key[i] = (uint32_t)(ck[i] >> 32);
    val[i] = (ck[i] << 32) | (uint32_t)tf[i];
  }
}

__device__ __forceinline__ double weight_at(uint32_t t, int32_t tf, const double *lut, double idf_ref,
                                            const int64_t *off, int64_t N, const double *idf_by_df, int64_t sdf,
                                            const double *idf_by_q, int mode) {
  double idf;
  if (mode == SME_IDF_REFERENCE) {
    idf = idf_ref;
  } else {
    const int64_t df = off[t + 1] - off[t];
    idf = df <= sdf ? idf_by_df[df] : idf_by_q[N / df];
  }
  return __dmul_rn(lut[tf], idf);
}
// w = LUT[tf] * idf per posting; four postings per thread step (16-byte tf
// loads, two 16-byte weight stores); the key is read only in the df modes
__global__ void k_weights(const uint32_t *key, const int32_t *tf, int64_t P, const double *lut, double idf_ref,
                          const int64_t *off, int64_t N, const double *idf_by_df, int64_t sdf,
                          const double *idf_by_q, int mode, double *w) {
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, gs = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = P >> 2;
  const bool ref = mode == SME_IDF_REFERENCE;
  for (int64_t q = gid; q < n4; q += gs) {
    const int4 f = reinterpret_cast<const int4 *>(tf)[q];
    const uint4 k = ref ? make_uint4(0, 0, 0, 0) : reinterpret_cast<const uint4 *>(key)[q];
    double2 a, b;
    a.x = weight_at(k.x, f.x, lut, idf_ref, off, N, idf_by_df, sdf, idf_by_q, mode);
    a.y = weight_at(k.y, f.y, lut, idf_ref, off, N, idf_by_df, sdf, idf_by_q, mode);
    b.x = weight_at(k.z, f.z, lut, idf_ref, off, N, idf_by_df, sdf, idf_by_q, mode);
    b.y = weight_at(k.w, f.w, lut, idf_ref, off, N, idf_by_df, sdf, idf_by_q, mode);
    reinterpret_cast<double2 *>(w)[2 * q] = a;
    reinterpret_cast<double2 *>(w)[2 * q + 1] = b;
  }
  for (int64_t i = (n4 << 2) + gid; i < P; i += gs)
    w[i] = weight_at(ref ? 0u : key[i], tf[i], lut, idf_ref, off, N, idf_by_df, sdf, idf_by_q, mode);
}

// Packed 32-bit sort path (the common case): a posting's (docno, tf) fits one
// u32 as (docno - dmin) * F + tf when (dmax - dmin + 1) * F < 2^32, F = max_tf + 1.
__global__ void k_pair_stats(const uint64_t *val, int64_t P, unsigned int *max_tf) {
  unsigned int m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, (unsigned int)(uint32_t)val[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(max_tf, m);
}
__global__ __launch_bounds__(256) void k_docno_range(const int32_t *docno, int64_t n, int *mn, int *mx) {
  __shared__ int s_a[4], s_b[4];
  int a = INT_MAX, b = INT_MIN;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    a = min(a, docno[i]);
    b = max(b, docno[i]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    a = min(a, __shfl_xor(a, o, 64));
    b = max(b, __shfl_xor(b, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    s_a[threadIdx.x >> 6] = a;
    s_b[threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // one atomic pair per block (single-address atomics serialise)
    for (int x = 1; x < 4; x++) {
      a = min(a, s_a[x]);
      b = max(b, s_b[x]);
    }
    atomicMin(mn, a);
    atomicMax(mx, b);
  }
}
__global__ void k_pack_pairs(const uint64_t *val, int64_t P, int64_t dmin, uint32_t F, uint32_t *v32) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t v = val[i];
    v32[i] = (uint32_t)(((int64_t)(int32_t)(uint32_t)(v >> 32) - dmin) * (int64_t)F + (int64_t)(uint32_t)v);
  }
}
__global__ void k_unpack_packed(const uint32_t *v32, int64_t P, int64_t dmin, uint32_t F, int32_t *docno, int32_t *tf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t v = v32[i];
    docno[i] = (int32_t)((int64_t)(v / F) + dmin);
    tf[i] = (int32_t)(v % F);
  }
}
__global__ void k_composite32(const uint32_t *key, const int32_t *tf, int64_t P, int tfbits, uint32_t tfmask,
                              uint32_t *ck) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    ck[i] = (key[i] << tfbits) | (tfmask - (uint32_t)tf[i]);
}
__global__ void k_composite32_tf(const uint32_t *ck, int64_t P, uint32_t tfmask, int32_t *tf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    tf[i] = (int32_t)(tfmask - (ck[i] & tfmask));
}

// idf of every term (the same expression k_weights evaluates per posting)
__global__ void k_term_idf(const int64_t *off, int64_t V, double idf_ref, int64_t N, const int64_t *gdf,
                           const double *idf_by_df, int64_t sdf, const double *idf_by_q, int mode, double *idf) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    if (mode == SME_IDF_REFERENCE) {
      idf[t] = idf_ref;
    } else {
      const int64_t df = gdf ? gdf[t] : off[t + 1] - off[t];
      idf[t] = df <= sdf ? idf_by_df[df] : idf_by_q[N / df];
    }
  }
}

__global__ void k_composite(const uint32_t *key, const int32_t *tf, int64_t P, int tfbits, uint64_t tfmask,
                            uint64_t *ck) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    ck[i] = ((uint64_t)key[i] << tfbits) | (tfmask - (uint64_t)tf[i]);
}
__global__ void k_composite_tf(const uint64_t *ck, int64_t P, uint64_t tfmask, int32_t *tf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    tf[i] = (int32_t)(tfmask - (ck[i] & tfmask));
}

__global__ void k_docno_keys(const int32_t *docno, int64_t nR, uint32_t *k, uint32_t *v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x) {
    k[i] = (uint32_t)docno[i] ^ 0x80000000u;  // signed order
    v[i] = (uint32_t)i;
  }
}
__global__ void k_widen_u32(const uint32_t *a, int64_t n, int64_t *b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = (int64_t)a[i];
}
__global__ void k_not_ascending(const int32_t *d, int64_t n, unsigned long long *cnt) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x + 1; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= d[i] <= d[i - 1];
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(cnt, 1ull);
}
__global__ void k_iota_i64(int64_t *a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) a[i] = i;
}
__global__ void k_adjacent_equal(const uint32_t *k, int64_t n, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x + 1; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (k[i] == k[i - 1]) atomicAdd(cnt, 1ull);
}
__global__ void k_gather_i64(const int64_t *idx, int64_t n, const int32_t *src, int32_t *dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}
__global__ void k_fill_slow_lens(const int64_t *list, int64_t n, const uint64_t *rs, const uint64_t *re,
                                 int64_t *lens) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lens[i] = (int64_t)(re[list[i]] - rs[list[i]]) + 1;
}
__global__ void k_compact_flags(const uint8_t *flag, int64_t n, int64_t *list, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (flag[i]) list[atomicAdd(cnt, 1ull)] = i;
}
__global__ void k_long_lens(const int64_t *list, int64_t n, const int32_t *rlist, const unsigned long long *rep,
                            int64_t *lens) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lens[i] = 5 * (int64_t)(rep[rlist[list[i]]] & 0xFFFFFFull) + 32;
}
__global__ void k_big_list(const int32_t *prec, int64_t n, int64_t *list, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (prec[i] < 0) list[atomicAdd(cnt, 1ull)] = i;
}
// single-pass aggregation: region of record i (docno order) = ntok * max_nout,
// which bounds both its distinct terms and any of its tf (the largest region
// bounds tf for the packed values)
__global__ void k_agg_regions(const int64_t *perm, const int32_t *ntok, int64_t nR, const int32_t *max_nout,
                              int64_t *reg, unsigned long long *mx) {
  unsigned long long m = 0;
  const int64_t mn = max(*max_nout, 1);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = (int64_t)ntok[perm[i]] * mn;
    reg[i] = c;
    m = max(m, (unsigned long long)c);
  }
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}
__global__ void k_big_caps(const int64_t *list, int64_t nbig, const int64_t *perm, const int32_t *ntok,
                           const int32_t *max_nout, int64_t *caps) {
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbig; b += (int64_t)gridDim.x * blockDim.x) {
    int64_t need = (int64_t)ntok[perm[list[b]]] * (int64_t)max(*max_nout, 1) * 2 + 64;
    int64_t c = 1;
    while (c < need) c <<= 1;
    caps[b] = c;
  }
}

__global__ void k_gather_u64(const uint64_t *src, const uint32_t *idx, int64_t nn, uint64_t *dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nn; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}
__global__ void k_iota_u32(uint32_t *a, int64_t nn) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nn; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}
__global__ void k_pair_counts(const int32_t *prec, const int32_t *bcount, int64_t n, int64_t *out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = prec[i] >= 0 ? prec[i] : bcount[i];
}

// ============================================================================
// K >= 2: term k-grams (TermKGramDocIndexer.java:138-159)
// ============================================================================
// A record's term stream is its raw tokens expanded to term ids in order (a raw
// token gives 0..n terms, T13).  Every window of K consecutive terms is a
// k-gram; packed MSB-first with tb bits per term id into a u64, numeric key
// order IS TermDF.compareTo order (element-wise String.compareTo on equal-length
// arrays; term ids are ranks in that order).  Requires K * tb <= 63.
constexpr int kGCap = 1024;
constexpr int kGLimit = 768;

__device__ __forceinline__ int32_t nterms_of(const AggIn &in, uint32_t slot) {
  const int32_t rt = in.raw_term[slot];
  return rt >= 0 ? 1 : (rt <= -2 ? in.raw_nout[slot] : 0);
}

// term-stream length of every record (docno order i)
__global__ __launch_bounds__(kAggNT) void k_tcount(AggIn in, int64_t nR, int64_t *tcnt) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kAggNT / 64);
  for (int64_t i = (int64_t)blockIdx.x * (kAggNT / 64) + wv; i < nR; i += nwaves) {
    const int64_t r = in.perm[i];
    const uint32_t *ts = in.tokstream + (in.rs[r] >> 1);
    const int32_t nt = in.ntok[r];
    int64_t c = 0;
    for (int32_t t = lane; t < nt; t += 64) c += nterms_of(in, ts[t]);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) tcnt[i] = c;
  }
}

// the term stream itself, in token order
__global__ __launch_bounds__(kAggNT) void k_twrite(AggIn in, int64_t nR, const int64_t *toff, int32_t *tstream) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kAggNT / 64);
  for (int64_t i = (int64_t)blockIdx.x * (kAggNT / 64) + wv; i < nR; i += nwaves) {
    const int64_t r = in.perm[i];
    const uint32_t *ts = in.tokstream + (in.rs[r] >> 1);
    const int32_t nt = in.ntok[r];
    int64_t o = toff[i];
    for (int32_t t0 = 0; t0 < nt; t0 += 64) {
      const int32_t t = t0 + lane;
      const uint32_t slot = t < nt ? ts[t] : 0u;
      const int32_t c = t < nt ? nterms_of(in, slot) : 0;
      const int32_t inc = wave_incl_sum(c);
      const int64_t at = o + inc - c;
      if (c == 1 && in.raw_term[slot] >= 0) {
        tstream[at] = in.raw_term[slot];
      } else if (c > 0) {
        const int32_t m0 = -in.raw_term[slot] - 2;
        for (int32_t m = 0; m < c; m++) tstream[at + m] = in.multi_term[m0 + m];
      }
      o += __shfl(inc, 63, 64);
    }
  }
}

__device__ __forceinline__ uint64_t gram_key(const int32_t *ts, int K, int tb) {
  uint64_t k = 0;
  for (int j = 0; j < K; j++) k = (k << tb) | (uint64_t)(uint32_t)ts[j];
  return k;
}

__device__ __forceinline__ bool gram_insert(uint64_t *keys, int32_t *cnt, uint64_t key, int32_t *distinct) {
  uint32_t h = (uint32_t)fmix64(key) & (kGCap - 1);
  for (int probe = 0; probe < kGCap; probe++) {
    const unsigned long long old = atomicCAS((unsigned long long *)&keys[h], ~0ull, (unsigned long long)key);
    if (old == ~0ull) {
      atomicAdd(distinct, 1);
      atomicAdd(&cnt[h], 1);
      return true;
    }
    if (old == key) {
      atomicAdd(&cnt[h], 1);
      return true;
    }
    h = (h + 1) & (kGCap - 1);
  }
  return false;
}

// per record (wave): k-gram tf in an LDS table.  Records with more than kGLimit
// distinct grams emit one (gram, docno, 1) pair per occurrence instead (flag
// big[i]); the reducer-style merge of equal (gram, docno) sums them afterwards.
// pos_key != nullptr: the gram at term-stream position p is pos_key[p] (its rank,
// k_gram_rank_round) instead of the packed term ids (K * tb > 63)
template <bool EMIT>
__global__ __launch_bounds__(kAggNT) void k_gram_agg(const int32_t *tstream, const int64_t *toff, int64_t nR,
                                                     const int64_t *perm, const int32_t *docno_r, int K, int tb,
                                                     int64_t *pcount, uint8_t *big, const int64_t *pair_off,
                                                     uint64_t *pkey, uint64_t *pval, const uint32_t *pos_key) {
  __shared__ uint64_t keys_all[kAggNT / 64][kGCap];
  __shared__ int32_t cnt_all[kAggNT / 64][kGCap];
  __shared__ int32_t dist_all[kAggNT / 64];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint64_t *keys = keys_all[wv];
  int32_t *cnt = cnt_all[wv];
  int32_t *distinct = &dist_all[wv];
  const int64_t nwaves = (int64_t)gridDim.x * (kAggNT / 64);
  for (int64_t i = (int64_t)blockIdx.x * (kAggNT / 64) + wv; i < nR; i += nwaves) {
    const int32_t *ts = tstream + toff[i];
    const int64_t m = toff[i + 1] - toff[i];
    const int64_t ng = m >= K ? m - K + 1 : 0;
    const uint64_t dn = (uint64_t)(uint32_t)docno_r[perm[i]] << 32;
    if (EMIT && big[i]) {
      for (int64_t j = lane; j < ng; j += 64) {
        pkey[pair_off[i] + j] = pos_key ? (uint64_t)pos_key[toff[i] + j] : gram_key(ts + j, K, tb);
        pval[pair_off[i] + j] = dn | 1u;
      }
      continue;
    }
    for (int k = lane; k < kGCap; k += 64) {
      keys[k] = ~0ull;
      cnt[k] = 0;
    }
    if (lane == 0) *distinct = 0;
    wave_sync_lds();
    bool ok = true;
    for (int64_t j = lane; j < ng; j += 64)
      ok &= gram_insert(keys, cnt, pos_key ? (uint64_t)pos_key[toff[i] + j] : gram_key(ts + j, K, tb), distinct);
    wave_sync_lds();
    const int32_t d = *distinct;
    const bool isbig = __any(!ok) || d > kGLimit;
    if (!EMIT) {
      if (lane == 0) {
        pcount[i] = isbig ? ng : d;
        big[i] = isbig;
      }
      wave_sync_lds();
      continue;
    }
    int64_t base = pair_off[i];
    for (int k = 0; k < kGCap / 64; k++) {
      const uint64_t key = keys[k * 64 + lane];
      const uint64_t mb = __ballot(key != ~0ull);
      if (key != ~0ull) {
        const int64_t o = base + __popcll(mb & ((1ull << lane) - 1ull));
        pkey[o] = key;
        pval[o] = dn | (uint32_t)cnt[k * 64 + lane];
      }
      base += __popcll(mb);
    }
    wave_sync_lds();
  }
}

__global__ void k_gram_flags(const uint64_t *k, int64_t P, uint32_t *f) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}
// gram id per pair (inclusive scan - 1) and the components of every gram
__global__ void k_gram_ids(const uint64_t *k, const uint32_t *incl, int64_t P, int K, int tb, uint32_t *gid,
                           int32_t *gcomp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = incl[i] - 1;
    gid[i] = g;
    if (i == 0 || k[i] != k[i - 1])
      for (int j = 0; j < K; j++) gcomp[(int64_t)g * K + j] = (int32_t)((k[i] >> (tb * (K - 1 - j))) & ((1ull << tb) - 1));
  }
}

// K * ceil(log2 V) > 63 (k-grams of a large vocabulary): gram keys by iterated
// ranking.  The 1-gram at position p is its term id t_p; the j-gram at p is the
// pair (rank of the (j-1)-gram at p, t_{p+j-1}), and its rank among the distinct
// j-grams of the corpus, ordered by that pair, is the key of the next round.
// Ranks preserve the lexicographic order of the id tuples, which is
// TermDF.compareTo's order (TermDF.java:64-70: element-wise String.compareTo,
// term ids being ranks in that order), so the last round's rank IS the gram id
// in TermDF order, held in 32 bits whatever K is.  Positions whose j-gram leaves
// the record get the all-ones key and sort last.
__global__ __launch_bounds__(kAggNT) void k_gram_round_keys(const int32_t *tstream, const int64_t *toff, int64_t nR,
                                                            int j, int tb, const uint32_t *rprev, uint64_t *key,
                                                            uint32_t *pos) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t nwaves = (int64_t)gridDim.x * (kAggNT / 64);
  for (int64_t i = (int64_t)blockIdx.x * (kAggNT / 64) + wv; i < nR; i += nwaves) {
    const int64_t a = toff[i], e = toff[i + 1];
    for (int64_t p = a + lane; p < e; p += 64) {
      const bool valid = p + j - 1 < e;
      const uint64_t prev = rprev ? (uint64_t)rprev[p] : (uint64_t)(uint32_t)tstream[p];
      key[p] = valid ? (prev << tb) | (uint64_t)(uint32_t)tstream[p + j - 1] : ~0ull;
      pos[p] = (uint32_t)p;
    }
  }
}
__global__ void k_gram_round_heads(const uint64_t *ks, int64_t M, uint32_t *head) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < M; s += (int64_t)gridDim.x * blockDim.x)
    head[s] = (ks[s] != ~0ull && (s == 0 || ks[s] != ks[s - 1])) ? 1u : 0u;
}
// rank of sorted item s = (inclusive head count) - 1, scattered to its position;
// rep[rank] = one position holding the gram (last round: its components)
__global__ void k_gram_round_scatter(const uint64_t *ks, const uint32_t *ps, const uint32_t *head,
                                     const uint32_t *excl, int64_t M, uint32_t *rnew, uint32_t *rep) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < M; s += (int64_t)gridDim.x * blockDim.x) {
    if (ks[s] == ~0ull) continue;
    const uint32_t r = excl[s] + head[s] - 1u;
    rnew[ps[s]] = r;
    if (rep && head[s]) rep[r] = ps[s];
  }
}
__global__ void k_gram_comp_rep(const uint32_t *rep, int64_t Vg, int K, const int32_t *tstream, int32_t *gcomp) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < Vg; g += (int64_t)gridDim.x * blockDim.x)
    for (int c = 0; c < K; c++) gcomp[g * K + c] = tstream[(int64_t)rep[g] + c];
}

// ============================================================================
// K8: reducer output order -- per term, a STABLE sort by tf descending of the
// docno-ascending postings (MyReducer.reduce's Collections.sort over
// PostingWritable.compareTo, TermKGramDocIndexer.java:211, PostingWritable.java:57-59).
// Segmented counting sort: the term CSR already delimits the segments and tf is a
// small integer, so one read + one write per posting replaces a full radix sort.
// ============================================================================
constexpr int kTfTiny = 8;      // segments up to this: one thread each (insertion sort in registers)
constexpr int kTfSmall = 64;    // segments up to one wave chunk: rank by lane compares
constexpr int kTfWave = 512;    // up to this: one-wave blocks (no cross-wave barriers)
constexpr int kTfMedium = 8192; // up to this: 4-wave blocks; beyond: tiles
constexpr int kTfSortMaxTf = 1023;  // LDS counters (max_tf + 1) x 16 x 4 B <= 64 KiB; above: radix sort

// segments of length <= kTfTiny (every docid term, most rare words): one thread
// each, a stable insertion sort by tf desc in registers
__global__ __launch_bounds__(256) void k_tfsort_tiny(const int64_t *__restrict__ off, int64_t V,
                                                     const int32_t *__restrict__ docno_d,
                                                     const int32_t *__restrict__ tf_d, int32_t *docno_o,
                                                     int32_t *tf_o) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = off[s];
    const int n = (int)(off[s + 1] - b);
    if (n > kTfTiny || n == 0) continue;
    int32_t t[kTfTiny], d[kTfTiny];
#pragma unroll
    for (int j = 0; j < kTfTiny; j++) {
      t[j] = j < n ? tf_d[b + j] : INT_MIN;  // INT_MIN: padding sinks to the end
      d[j] = j < n ? docno_d[b + j] : 0;
    }
#pragma unroll
    for (int j = 1; j < kTfTiny; j++) {  // stable: an item passes only strictly smaller tfs
#pragma unroll
      for (int k = j; k > 0; k--) {
        if (t[k - 1] < t[k]) {
          const int32_t x = t[k - 1], y = d[k - 1];
          t[k - 1] = t[k];
          d[k - 1] = d[k];
          t[k] = x;
          d[k] = y;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kTfTiny; j++)
      if (j < n) {
        docno_o[b + j] = d[j];
        tf_o[b + j] = t[j];
      }
  }
}

// segments of length in (kTfTiny, kTfSmall] (from a class list): one wave each;
// output rank of lane i = #{j : tf_j > tf_i} + #{j < i : tf_j == tf_i}
__global__ __launch_bounds__(256) void k_tfsort_small(const int64_t *__restrict__ off,
                                                      const int32_t *__restrict__ seg,
                                                      const unsigned long long *__restrict__ nseg,
                                                      const int32_t *__restrict__ docno_d,
                                                      const int32_t *__restrict__ tf_d, int32_t *docno_o,
                                                      int32_t *tf_o) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6), ns = (int64_t)*nseg;
  for (int64_t q = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); q < ns; q += nw) {
    const int64_t s = seg[q];
    const int64_t b = off[s];
    const int n = (int)(off[s + 1] - b);
    const bool v = lane < n;
    const int32_t t = v ? tf_d[b + lane] : 0, d = v ? docno_d[b + lane] : 0;
    int r = 0;
    for (int j = 0; j < n; j++) {
      const int32_t tj = __shfl(t, j, 64);
      r += (tj > t) || (tj == t && j < lane);
    }
    if (v) {
      docno_o[b + r] = d;
      tf_o[b + r] = t;
    }
  }
}

// one NW-wave block per segment (length in (lo, hi]): wave w owns a contiguous run
// of 64-posting chunks.  Pass 1 counts tf per wave, a block scan orders the
// counters as (tf desc, wave asc), pass 2 places every posting at its counter +
// its rank among equal-tf lanes of the chunk (ballot), which keeps docno order.
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_tfsort_block(const int64_t *__restrict__ off, int64_t V,
                                                          const int32_t *__restrict__ docno_d,
                                                          const int32_t *__restrict__ tf_d, int32_t *docno_o,
                                                          int32_t *tf_o, const int32_t *__restrict__ seg,
                                                          const unsigned long long *__restrict__ nseg, int max_tf) {
  extern __shared__ int32_t cnt[];  // [(max_tf - tf) * NW + w]
  __shared__ int32_t wsum[NW];
  constexpr int NT = NW * 64;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int L = (max_tf + 1) * NW;
  const uint64_t lt_mask = (1ull << lane) - 1;
  const int64_t ns = (int64_t)*nseg;
  for (int64_t q = blockIdx.x; q < ns; q += gridDim.x) {
    const int64_t s = seg[q];
    const int64_t b = off[s], n = off[s + 1] - b;
    for (int j = tid; j < L; j += NT) cnt[j] = 0;
    __syncthreads();
    const int64_t nch = (n + 63) >> 6, cpw = (nch + NW - 1) / NW;
    const int64_t c0 = (int64_t)w * cpw, c1 = c0 + cpw < nch ? c0 + cpw : nch;
    int32_t tn = c0 < c1 && (c0 << 6) + lane < n ? tf_d[b + (c0 << 6) + lane] : -1;  // one chunk ahead
    for (int64_t c = c0; c < c1; c++) {
      const int64_t i = (c << 6) + lane;
      const bool v = i < n;
      const int32_t t = tn;
      tn = c + 1 < c1 && i + 64 < n ? tf_d[b + i + 64] : -1;
      uint64_t pend = __ballot(v);
      while (pend) {
        const int32_t tv = __shfl(t, __ffsll((unsigned long long)pend) - 1, 64);
        const uint64_t m = __ballot(t == tv);
        if (lane == 0) cnt[(max_tf - tv) * NW + w] += __popcll(m);
        pend &= ~m;
      }
    }
    __syncthreads();
    // exclusive scan of cnt[0..L) (each thread a contiguous run, then across threads)
    const int per = (L + NT - 1) / NT, j0 = tid * per, j1 = j0 + per < L ? j0 + per : L;
    int run = 0;
    for (int j = j0; j < j1; j++) run += cnt[j];
    int inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int base = inc - run;
    for (int k = 0; k < w; k++) base += wsum[k];
    for (int j = j0; j < j1; j++) {
      const int c = cnt[j];
      cnt[j] = base;
      base += c;
    }
    __syncthreads();
    int32_t tn2 = -1, dn2 = 0;  // one chunk ahead
    if (c0 < c1 && (c0 << 6) + lane < n) {
      tn2 = tf_d[b + (c0 << 6) + lane];
      dn2 = docno_d[b + (c0 << 6) + lane];
    }
    for (int64_t c = c0; c < c1; c++) {
      const int64_t i = (c << 6) + lane;
      const bool v = i < n;
      const int32_t t = tn2, d = dn2;
      if (c + 1 < c1 && i + 64 < n) {
        tn2 = tf_d[b + i + 64];
        dn2 = docno_d[b + i + 64];
      } else {
        tn2 = -1;
      }
      uint64_t pend = __ballot(v);
      while (pend) {
        const int32_t tv = __shfl(t, __ffsll((unsigned long long)pend) - 1, 64);
        const uint64_t m = __ballot(t == tv);
        const int slot = (max_tf - tv) * NW + w;
        const int cb = cnt[slot];
        if (t == tv) {
          const int64_t p = b + cb + __popcll(m & lt_mask);
          docno_o[p] = d;
          tf_o[p] = t;
        }
        if (lane == 0) cnt[slot] = cb + __popcll(m);
        pend &= ~m;
      }
    }
    __syncthreads();
  }
}

// Segments longer than kTfMedium are cut into tiles of kTfTile postings so that a
// 1M-posting term spreads over many CUs: (1) per tile tf counts, (2) per segment
// an exclusive scan of the counts in (tf desc, tile asc) order, (3) per tile the
// ballot placement of k_tfsort_block from the tile's scanned counters.
constexpr int kTfTile = 4096;

// segment lists by class (medium: 4-wave blocks, large: tiles), appended with
// one global atomic per block and list; list order is free (segments are
// independent and their output ranges fixed)
__global__ __launch_bounds__(256) void k_tf_classify(const int64_t *__restrict__ off, int64_t V, int32_t *med,
                                                     int32_t *large, int32_t *small, int32_t *wave,
                                                     unsigned long long *ctr) {
  __shared__ unsigned int s_n[4];
  __shared__ unsigned long long s_b[4];
  for (int64_t s0 = (int64_t)blockIdx.x * 256; s0 < V; s0 += (int64_t)gridDim.x * 256) {  // block-uniform
    const int64_t s = s0 + threadIdx.x;
    const int64_t n = s < V ? off[s + 1] - off[s] : 0;
    const int cls = n > kTfMedium ? 1 : n > kTfWave ? 0 : n > kTfSmall ? 3 : n > kTfTiny ? 2 : -1;  // ctr index
    if (threadIdx.x < 4) s_n[threadIdx.x] = 0;
    __syncthreads();
    unsigned int pos = 0;
    if (cls >= 0) pos = atomicAdd(&s_n[cls], 1u);
    __syncthreads();
    if (threadIdx.x < 4)
      s_b[threadIdx.x] = s_n[threadIdx.x] ? atomicAdd(&ctr[threadIdx.x], (unsigned long long)s_n[threadIdx.x]) : 0ull;
    __syncthreads();
    if (cls == 0) med[s_b[0] + pos] = (int32_t)s;
    if (cls == 1) large[s_b[1] + pos] = (int32_t)s;
    if (cls == 2) small[s_b[2] + pos] = (int32_t)s;
    if (cls == 3) wave[s_b[3] + pos] = (int32_t)s;
    __syncthreads();
  }
}
// tiles of large segment q (0 beyond the list: the scan covers V + 1 entries)
__global__ void k_tf_ntiles(const int64_t *off, const int32_t *large, const unsigned long long *nlarge, int64_t V,
                            int64_t *nt) {
  const int64_t nl = (int64_t)*nlarge;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q <= V; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = q < nl ? off[large[q] + 1] - off[large[q]] : 0;
    nt[q] = (n + kTfTile - 1) / kTfTile;
  }
}

// segment of tile tau: the s with toff[s] <= tau < toff[s + 1]
__device__ __forceinline__ int64_t tile_segment(const int64_t *toff, int64_t V, int64_t tau) {
  int64_t lo = 0, hi = V;  // toff[lo] <= tau < toff[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (toff[mid] <= tau) lo = mid;
    else hi = mid;
  }
  return lo;
}

// (1) one wave per tile: LDS counts (order-free), written as tcnt[tau][max_tf - tf]
__global__ __launch_bounds__(256) void k_tf_tile_count(const int64_t *__restrict__ off,
                                                       const int32_t *__restrict__ large,
                                                       const unsigned long long *__restrict__ nlarge,
                                                       const int64_t *__restrict__ toff, int64_t ntiles,
                                                       const int32_t *__restrict__ tf_d, int max_tf,
                                                       int32_t *tcnt) {
  extern __shared__ int32_t h[];  // 4 waves x (max_tf + 1)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, F = max_tf + 1;
  int32_t *hw = h + w * F;
  const int64_t nwv = (int64_t)gridDim.x * 4;
  const int64_t nl = (int64_t)*nlarge;
  for (int64_t tau = (int64_t)blockIdx.x * 4 + w; tau < ntiles; tau += nwv) {  // wave-uniform
    const int64_t q = tile_segment(toff, nl, tau), s = large[q];
    const int64_t b = off[s] + (tau - toff[q]) * kTfTile, e = min(off[s + 1], b + (int64_t)kTfTile);
    for (int j = lane; j < F; j += 64) hw[j] = 0;
    __builtin_amdgcn_wave_barrier();
    // per 64-posting chunk: one LDS add per distinct tf (ballot groups) -- most
    // postings have tf 1, and per-lane atomics on that one counter serialise
    int32_t tn = b + lane < e ? tf_d[b + lane] : -1;  // the next chunk loads before this one is counted
    for (int64_t c = b; c < e; c += 64) {
      const bool v = c + lane < e;
      const int32_t t = tn;
      tn = c + 64 + lane < e ? tf_d[c + 64 + lane] : -1;
      uint64_t pend = __ballot(v);
      while (pend) {
        const int32_t tv = __shfl(t, __ffsll((unsigned long long)pend) - 1, 64);
        const uint64_t m = __ballot(t == tv);
        if (lane == 0) hw[max_tf - tv] += __popcll(m);
        pend &= ~m;
      }
    }
    __builtin_amdgcn_wave_barrier();
    for (int j = lane; j < F; j += 64) tcnt[tau * F + j] = hw[j];
    __builtin_amdgcn_wave_barrier();
  }
}

// (2) one block per large segment: counters -> segment-relative start positions,
// in (tf desc, tile asc) order.  Thread f owns counter column f (= max_tf - tf,
// up to 4 per thread): its total over the segment's tiles, one block scan of the
// totals, then a walk down its column (coalesced across threads at every tile).
__global__ __launch_bounds__(256) void k_tf_tile_scan(const unsigned long long *__restrict__ nlarge,
                                                      const int64_t *__restrict__ toff, int max_tf, int32_t *tcnt) {
  __shared__ int32_t sc[256 / 64 + 1];
  const int tid = threadIdx.x, F = max_tf + 1;
  const int64_t nl = (int64_t)*nlarge;
  for (int64_t q = blockIdx.x; q < nl; q += gridDim.x) {
    const int64_t t0 = toff[q], T = toff[q + 1] - t0;
    int32_t *c = tcnt + t0 * F;
    int32_t carry = 0;
    for (int f0 = 0; f0 < F; f0 += 256) {  // block-uniform
      const int f = f0 + tid;
      int32_t tot = 0;
      if (f < F) {
#pragma unroll 8
        for (int64_t j = 0; j < T; j++) tot += c[j * F + f];
      }
      int32_t all;
      int32_t run = carry + block_excl_sum<256, int32_t>(tot, sc, &all);
      carry += all;
      if (f < F) {
#pragma unroll 8
        for (int64_t j = 0; j < T; j++) {
          const int32_t x = c[j * F + f];
          c[j * F + f] = run;
          run += x;
        }
      }
    }
  }
}

// (3) one wave per tile: stable placement from the tile's counters
__global__ __launch_bounds__(256) void k_tf_tile_place(const int64_t *__restrict__ off,
                                                       const int32_t *__restrict__ large,
                                                       const unsigned long long *__restrict__ nlarge,
                                                       const int64_t *__restrict__ toff, int64_t ntiles,
                                                       const int32_t *__restrict__ docno_d,
                                                       const int32_t *__restrict__ tf_d, int max_tf,
                                                       const int32_t *__restrict__ tcnt, int32_t *docno_o,
                                                       int32_t *tf_o) {
  extern __shared__ int32_t h[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, F = max_tf + 1;
  int32_t *hw = h + w * F;
  const uint64_t lt_mask = (1ull << lane) - 1;
  const int64_t nwv = (int64_t)gridDim.x * 4;
  const int64_t nl = (int64_t)*nlarge;
  for (int64_t tau = (int64_t)blockIdx.x * 4 + w; tau < ntiles; tau += nwv) {
    const int64_t q = tile_segment(toff, nl, tau), s = large[q];
    const int64_t sb = off[s];
    const int64_t b = sb + (tau - toff[q]) * kTfTile, e = min(off[s + 1], b + (int64_t)kTfTile);
    for (int j = lane; j < F; j += 64) hw[j] = tcnt[tau * F + j];
    __builtin_amdgcn_wave_barrier();
    // the next chunk's (tf, docno) are loaded before this chunk's placement
    int32_t tn = b + lane < e ? tf_d[b + lane] : -1, dnx = b + lane < e ? docno_d[b + lane] : 0;
    for (int64_t c = b; c < e; c += 64) {
      const bool v = c + lane < e;
      const int32_t t = tn, d = dnx;
      const int64_t in = c + 64 + lane;
      tn = in < e ? tf_d[in] : -1;
      dnx = in < e ? docno_d[in] : 0;
      uint64_t pend = __ballot(v);
      while (pend) {
        const int32_t tv = __shfl(t, __ffsll((unsigned long long)pend) - 1, 64);
        const uint64_t m = __ballot(t == tv);
        const int slot = max_tf - tv;
        const int cb = hw[slot];
        if (t == tv) {
          const int64_t p = sb + cb + __popcll(m & lt_mask);
          docno_o[p] = d;
          tf_o[p] = t;
        }
        if (lane == 0) hw[slot] = cb + __popcll(m);
        pend &= ~m;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ============================================================================
// host orchestration
// ============================================================================
static int grid_for(int64_t n, int nt = 256, int cap = 8192) {
  int64_t g = (n + nt - 1) / nt;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <typename T>
static T d2h(const T *d, hipStream_t st) {
  T h;
#if SME_D2H_PINNED
  // through a small pinned buffer of the calling thread (a pageable destination
  // takes the runtime's staged path: a longer stall per read-back, and the build
  // reads back ~30 sizes)
  static thread_local void *pin = nullptr;
  if (!pin) SME_HIP(hipHostMalloc(&pin, 64, hipHostMallocDefault));
  static_assert(sizeof(T) <= 64, "d2h");
  SME_HIP(hipMemcpyAsync(pin, d, sizeof(T), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  memcpy(&h, pin, sizeof(T));
#else
  SME_HIP(hipMemcpyAsync(&h, d, sizeof(T), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
#endif
  return h;
}

static int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (1ull << b) <= v) b++;
  return b < 1 ? 1 : b;
}

// workspace slots
enum {
  W_S, W_E, W_C, W_CNT, W_EOF, W_NEXTS, W_RS, W_RE, W_DOCNO, W_SLOW, W_SLOWLIST, W_SCROFF, W_U16, W_BOFF,
  W_TOK, W_NTOK, W_RKEYS, W_RREPS, W_POOL, W_CKEY, W_CSTR, W_NOUT, W_LONG, W_FKEYS, W_FREPS, W_CFINAL,
  W_VSLOT, W_KHI, W_KLO, W_VIDX, W_T0, W_T1, W_T2, W_T3, W_RAWTERM, W_MULTI, W_PERM, W_PREC, W_PTERM, W_PVAL,
  W_MAXNOUT, W_SS, W_SE, W_SC, W_RLIST, W_RFLAG, W_POFF, W_OVFKEY, W_FREC, W_LT, W_RADIX, W_NTOK2, W_BIGL2,
  W_BIGCAP, W_SEGB, W_VCS, W_DMARK, W_DSLOT, W_DLIST, W_DSRC, W_DKEY, W_WRANK, W_DSPAN, W_RLISTW,
  W_NSLOTS
};
constexpr int kBuildWs = 64;  // build slots live at ctx->ws[64..127]
static_assert(W_NSLOTS <= 64, "too many build workspace slots");

// K1 + K1b: record spans of the corpus exactly as XMLRecordReader yields them,
// plus the sorted positions of every '<' whose markup is not "simple" (C).
RecordSpans find_records(sme_ctx *cx, const uint8_t *t, uint64_t n, hipStream_t st, Prof *prof) {
  DevBuf *W = cx->ws + kBuildWs;
  auto cub_tmp = [&](size_t bytes) { return cx->cub_tmp.get(bytes); };
  unsigned long long *cnt = W[W_CNT].as<unsigned long long>(16);
  // ---------------- K1 scan ----------------
  // every '<' position, then the tag classification over that list
  uint64_t capL = std::max<uint64_t>(cx->lt_cap_hint, std::max<uint64_t>(4096, n / 256));
  uint64_t *ltpos = nullptr;
  int64_t nlt = 0;
  for (int attempt = 0;; attempt++) {
    ltpos = W[W_LT].as<uint64_t>(capL);
    SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_scan_lt, dim3(grid_for((int64_t)ceil_div(n, 64), 256, 4096)), dim3(kScanNT), 0, st, t,
                       (int64_t)n, ltpos, capL, cnt + 3);
    SME_CHECK_LAUNCH();
    nlt = (int64_t)d2h(cnt + 3, st);
    if ((uint64_t)nlt <= capL) break;
    if (attempt > 2) throw Error(SME_ELIMIT, "'<' list capacity");
    capL = (uint64_t)nlt + 1024;
  }
  cx->lt_cap_hint = std::max<uint64_t>(cx->lt_cap_hint, (uint64_t)nlt + (uint64_t)nlt / 8 + 1024);
  uint64_t capS = std::max<uint64_t>(1024, (uint64_t)nlt + 1), capE = capS, capC = capS;
  unsigned long long h_cnt[3];
  for (int attempt = 0;; attempt++) {
    ScanOut so;
    so.S = W[W_S].as<uint64_t>(capS);
    so.E = W[W_E].as<uint64_t>(capE);
    so.C = W[W_C].as<uint64_t>(capC);
    so.capS = (uint32_t)std::min<uint64_t>(capS, 0xFFFFFFFFu);
    so.capE = (uint32_t)std::min<uint64_t>(capE, 0xFFFFFFFFu);
    so.capC = (uint32_t)std::min<uint64_t>(capC, 0xFFFFFFFFu);
    so.cnt = cnt;
    SME_HIP(hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), st));
    if (nlt > 0)
      hipLaunchKernelGGL(k_tag_classify, dim3(grid_for(nlt, 256, 8192)), dim3(kScanNT), 0, st, t, (int64_t)n, ltpos,
                         nlt, so);
    SME_CHECK_LAUNCH();
    SME_HIP(hipMemcpyAsync(h_cnt, cnt, sizeof h_cnt, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    if (h_cnt[0] <= capS && h_cnt[1] <= capE && h_cnt[2] <= capC) break;
    if (attempt > 2) throw Error(SME_ELIMIT, "tag scan capacity");
    capS = std::max<uint64_t>(capS, h_cnt[0]);
    capE = std::max<uint64_t>(capE, h_cnt[1]);
    capC = std::max<uint64_t>(capC, h_cnt[2]);
  }
  const int64_t nS = (int64_t)h_cnt[0], nE = (int64_t)h_cnt[1], nC = (int64_t)h_cnt[2];
  if (prof) prof->mark("scan_tags");

  // sort S, E, C positions
  // sorted copies land in spare workspace slots (no device-to-device copy back)
  // (hand-written LSD radix, sme_sort.hip; the values ride along unused)
  auto sort_u64 = [&](uint64_t *buf, int64_t cnt_, int slot_alt) -> uint64_t * {
    if (cnt_ < 2) return buf;
    uint64_t *alt = W[slot_alt].as<uint64_t>(cnt_);
    uint32_t *va = cx->ws[26].as<uint32_t>(cnt_), *vb = cx->ws[27].as<uint32_t>(cnt_);
    uint32_t *rscr = cx->ws[24].as<uint32_t>(kv_sort_scratch(cnt_) / sizeof(uint32_t) + 1);
    return kv_sort<uint64_t>(buf, va, alt, vb, cnt_, bits_for(n), rscr, st, true) == va ? buf : alt;
  };
  uint64_t *S = sort_u64(W[W_S].as<uint64_t>(capS), nS, W_SS);
  uint64_t *E = sort_u64(W[W_E].as<uint64_t>(capE), nE, W_SE);
  uint64_t *C = sort_u64(W[W_C].as<uint64_t>(capC), nC, W_SC);

  // ---------------- K1b records ----------------
  int64_t *e_of = W[W_EOF].as<int64_t>(nS + 1), *next_s = W[W_NEXTS].as<int64_t>(nS + 1);
  SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
  int64_t nR = 0;
  uint64_t *rs = W[W_RS].as<uint64_t>(nS + 1), *re = W[W_RE].as<uint64_t>(nS + 1);
  if (nS > 0) {
    hipLaunchKernelGGL(k_chain, dim3(grid_for(nS)), dim3(256), 0, st, S, nS, E, nE, e_of, next_s, cnt);
    SME_CHECK_LAUNCH();
    unsigned long long hc[3];  // bad, (walk count), records with an end tag: one read
    SME_HIP(hipMemcpyAsync(hc, cnt, sizeof hc, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    const unsigned long long bad = hc[0];
    if (bad == 0) {
      // records are the prefix of S with an end tag (e_of is monotone)
      nR = (int64_t)hc[2];
      if (nR > 0)
        hipLaunchKernelGGL(k_records_direct, dim3(grid_for(nR)), dim3(256), 0, st, S, E, e_of, nR, rs, re);
    } else {
      hipLaunchKernelGGL(k_records_walk, dim3(1), dim3(64), 0, st, S, nS, E, e_of, next_s, rs, re, cnt + 1);
      SME_CHECK_LAUNCH();
      nR = (int64_t)d2h(cnt + 1, st);
    }
  }
  if (prof) prof->mark("records");
  return RecordSpans{rs, re, nR, C, nC};
}

__global__ void k_iota_docno(int32_t *d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = (int32_t)(i + 1);
}

void build_docid_hash(sme_ctx *cx, bool distinct, hipStream_t st) {
  cx->map_hash_ok = false;
  if (!distinct || cx->map_n < 2) return;
  const uint64_t cap = next_pow2(std::max<uint64_t>(1024, 2 * (uint64_t)cx->map_n));
  uint32_t *slots = cx->map_slots.as<uint32_t>(cap);
  unsigned int *ovf = cx->ws[63].as<unsigned int>(4);
  SME_HIP(hipMemsetAsync(slots, 0, cap * sizeof(uint32_t), st));
  SME_HIP(hipMemsetAsync(ovf, 0, sizeof(unsigned int), st));
  hipLaunchKernelGGL(k_map_hash, dim3(grid_for(cx->map_n)), dim3(256), 0, st, (const uint16_t *)cx->map_chars.p,
                     (const int64_t *)cx->map_off.p, cx->map_n, slots, cap - 1, ovf);
  SME_CHECK_LAUNCH();
  cx->map_mask = cap - 1;
  cx->map_hash_ok = d2h(ovf, st) == 0;
}

sme_index *build_index(sme_ctx *cx, const uint8_t *t, uint64_t n, hipStream_t st, int job) {
  // job 0: TermKGramDocIndexer; job 1: CharKGramTermIndexer (no docnos: its mapper
  // never calls getDocid, and records stay in file order = the map task's order)
  if (job == 0 && !cx->has_map) throw Error(SME_ENOMAP, "no docno mapping loaded (sme_load_docno_mapping)");
  DevBuf *W = cx->ws + kBuildWs;
  Prof prof(st, &cx->prof_events);
  auto cub_tmp = [&](size_t bytes) { return cx->cub_tmp.get(bytes); };
  unsigned long long *cnt = W[W_CNT].as<unsigned long long>(40);  // [20] max tf, [22..23] docno range, [32..34] K6b

  uint8_t early_code[128];  // vocabulary sort: unit -> code (host copy outlives its async upload)
  const RecordSpans rsp = find_records(cx, t, n, st, &prof);
  uint64_t *rs = rsp.rs, *re = rsp.re, *C = rsp.C;
  const int64_t nR = rsp.nR, nC = rsp.nC;

  // ---------------- K2 docno ----------------
  int32_t *docno = W[W_DOCNO].as<int32_t>(nR + 1);
  uint64_t *dspan = job == 0 ? W[W_DSPAN].as<uint64_t>(nR + 1) : nullptr;  // (text offset << 8 | length) of each docid
  SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
  if (nR > 0 && job == 0) {
    hipLaunchKernelGGL(k_docno, dim3(grid_for(nR)), dim3(256), 0, st, t, (int64_t)n, rs, re, nR,
                       (const uint16_t *)cx->map_chars.p, (const int64_t *)cx->map_off.p, cx->map_n,
                       cx->map_hash_ok ? (const uint32_t *)cx->map_slots.p : nullptr, cx->map_mask, docno, cnt,
                       dspan);
    SME_CHECK_LAUNCH();
  } else if (nR > 0) {
    hipLaunchKernelGGL(k_iota_docno, dim3(grid_for(nR)), dim3(256), 0, st, docno, nR);
  }
  uint8_t *slow = W[W_SLOW].as<uint8_t>(nR + 1);
  // fast-path records (ascending), for the stream tokenizer
  int32_t *frec = W[W_FREC].as<int32_t>(nR + 1);
  if (nR > 0) {
    hipLaunchKernelGGL(k_mark_slow, dim3(grid_for(nR)), dim3(256), 0, st, rs, re, nR, C, nC, slow, cnt + 1);
    // (queued before the one host read below: the docno order test and the
    // fast-record list need nothing from the host)
    hipLaunchKernelGGL(k_not_ascending, dim3(grid_for(nR)), dim3(256), 0, st, docno, nR, cnt + 3);
    uint8_t *fflag = W[W_RFLAG].as<uint8_t>(nR);
    hipLaunchKernelGGL(k_not_flags, dim3(grid_for(nR)), dim3(256), 0, st, slow, nR, fflag);
    select_flagged(fflag, nR, frec, reinterpret_cast<int32_t *>(cnt + 14), cx->ws[25], cx->ws[23], st);
    SME_CHECK_LAUNCH();
  }
  unsigned long long h2[16];  // [0] docid errors, [1] slow records, [3] docno descents, [14] fast records
  SME_HIP(hipMemcpyAsync(h2, cnt, sizeof h2, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h2[0]) throw Error(SME_EPARSE, "a record has <DOCNO> but no </DOCNO> (TrecDocument.getDocid throws)");
  const int64_t nslow = (int64_t)h2[1];
  const int64_t nF = nR > 0 ? (int64_t)(int32_t)(uint32_t)h2[14] : 0;
  prof.mark("docno");

  // records in docno order (stable) -> perm; duplicate docnos?
  int64_t *perm = W[W_PERM].as<int64_t>(nR + 1);
  bool dup_docno = false;
  // records already in strictly ascending docno order (a corpus in docid order,
  // as TREC collections and every synthetic corpus are): perm = identity, no
  // duplicates, no sort
  bool ascending = false;
  if (nR > 0) {
    ascending = h2[3] == 0;
    if (ascending) hipLaunchKernelGGL(k_iota_i64, dim3(grid_for(nR)), dim3(256), 0, st, perm, nR);
  }
  if (nR > 0 && !ascending) {
    uint32_t *k0 = W[W_T0].as<uint32_t>(nR), *k1 = W[W_T1].as<uint32_t>(nR);
    uint32_t *v0 = W[W_T2].as<uint32_t>(nR), *v1 = W[W_T3].as<uint32_t>(nR);
    hipLaunchKernelGGL(k_docno_keys, dim3(grid_for(nR)), dim3(256), 0, st, docno, nR, k0, v0);
    uint32_t *rscr = cx->ws[24].as<uint32_t>(kv_sort_scratch(nR) / sizeof(uint32_t) + 1);
    uint32_t *vs = kv_sort<uint32_t>(k0, v0, k1, v1, nR, 32, rscr, st, true);
    const uint32_t *ks = vs == v0 ? k0 : k1;
    hipLaunchKernelGGL(k_widen_u32, dim3(grid_for(nR)), dim3(256), 0, st, vs, nR, perm);
    SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_adjacent_equal, dim3(grid_for(nR)), dim3(256), 0, st, ks, nR, cnt);
    dup_docno = d2h(cnt, st) != 0;
  }
  prof.mark("docno_sort");

  // ---------------- K3 tokenize ----------------
  // Raw-vocabulary table: sized from the previous build's distinct-token count
  // (load <= 1/2, so the hot part stays cache resident), or from the corpus size
  // the first time; a probe run longer than kMaxProbe retries with a 4x table.
  uint64_t rcap = cx->raw_cap_hint
                      ? cx->raw_cap_hint
                      : next_pow2(std::max<uint64_t>(1ull << 20, std::min<uint64_t>(n / 256, 1ull << 30)));
  uint32_t *tok = W[W_TOK].as<uint32_t>(n / 2 + 2);
  int32_t *ntok = W[W_NTOK].as<int32_t>(nR + 1);
  RawTable tb;
  unsigned int *ovf = reinterpret_cast<unsigned int *>(cnt + 8);
  int64_t h_nsel = 0;  // distinct raw tokens (read with the overflow flags)

  for (int attempt = 0;; attempt++) {
    {
      uint8_t *rb = W[W_RKEYS].as<uint8_t>(rcap * kRawSlotBytes);
      tb.tok = reinterpret_cast<ulonglong2 *>(rb);
      tb.key = reinterpret_cast<unsigned long long *>(rb + rcap * sizeof(ulonglong2));
      tb.rep = tb.key + rcap;
    }
    tb.mask = rcap - 1;
    tb.text = t;
    tb.overflow = ovf;
    SME_HIP(hipMemsetAsync(tb.tok, 0, rcap * kRawSlotBytes, st));
    SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
    if (nR > 0) {
      if (nF > 0) {
        uint64_t *rsF = W[W_LT].as<uint64_t>(2 * (size_t)nF), *reF = rsF + nF;  // '<' list no longer needed
        hipLaunchKernelGGL(k_gather_bounds, dim3(grid_for(nF)), dim3(256), 0, st, frec, nF, rs, re, rsF, reF);
        // events bracket exactly this launch: "tok_kernel" is the dominant kernel's
        // duration that bench.py reports against the HBM roofline
        prof.mark("tok_setup");
        const int64_t tgrid = std::max<int64_t>(1, std::min<int64_t>(nF, cx->opt_tok_grid)),
                      rpb = (nF + tgrid - 1) / tgrid;
        int tokexp = 0;
#ifdef SME_EXPERIMENTS
        // SME_TOKEXP (timing experiments, experiment builds only; wrong results):
        // 1 no signatures / probes, 2 no token stores, 4 no raw_insert (a miss
        // takes its home slot), 8 home slot only (no probe walk, no insert),
        // 16 no token passes (positions, probes, stores), 32 no byte classes
        if (const char *tx = getenv("SME_TOKEXP")) tokexp = atoi(tx);
#endif
        hipLaunchKernelGGL(k_tok_fast, dim3((unsigned)((nF + rpb - 1) / rpb)), dim3(kTokNT), 0, st, t, (int64_t)n, rsF,
                           reF, frec, nF, rpb, tok, ntok, tb, tokexp);
        SME_CHECK_LAUNCH();
        prof.mark("tok_kernel");
      }
    }
    if (nslow > 0) {
      int64_t *slist = W[W_SLOWLIST].as<int64_t>(nslow);
      hipLaunchKernelGGL(k_compact_flags, dim3(grid_for(nR)), dim3(256), 0, st, slow, nR, slist, cnt + 2);
      int64_t *lens = W[W_T0].as<int64_t>(nslow + 1), *soff = W[W_SCROFF].as<int64_t>(nslow + 1);
      hipLaunchKernelGGL(k_fill_slow_lens, dim3(grid_for(nslow)), dim3(256), 0, st, slist, nslow, rs, re, lens);
      size_t tbb = 0;
      SME_HIP(hipMemsetAsync(lens + nslow, 0, sizeof(int64_t), st));
      excl_scan(lens, soff, (int64_t)(nslow + 1), cx->ws[23], st);
      int64_t tot = d2h(soff + nslow, st);
      uint16_t *u16s = W[W_U16].as<uint16_t>(tot + 1);
      uint32_t *boffs = W[W_BOFF].as<uint32_t>(tot + 1);
      hipLaunchKernelGGL(k_tok_slow, dim3(grid_for(nslow, 64)), dim3(64), 0, st, t, rs, re, slist, nslow, soff,
                         u16s, boffs, tok, ntok, tb);
      SME_CHECK_LAUNCH();
    }
    // the distinct raw tokens' list is queued before the one host read of the
    // overflow flags and its length (an overflowing attempt discards it)
    hipLaunchKernelGGL(k_raw_flags, dim3(grid_for((int64_t)rcap)), dim3(256), 0, st, tb.key, rcap,
                       W[W_RFLAG].as<uint8_t>(rcap));
    select_flagged(W[W_RFLAG].as<uint8_t>(rcap), (int64_t)rcap, W[W_RLIST].as<int32_t>(rcap),
                   reinterpret_cast<int32_t *>(cnt + 13), cx->ws[25], cx->ws[23], st);
    unsigned long long hov[6];  // cnt[8..13]: overflow flags (low word of [8]), ..., distinct count ([13])
    SME_HIP(hipMemcpyAsync(hov, cnt + 8, sizeof hov, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    const unsigned int of = (unsigned int)hov[0];
    h_nsel = (int64_t)(int32_t)(uint32_t)hov[5];
    if (of == 0) break;
    if (of & 2u) throw Error(SME_ELIMIT, "a raw token is longer than 16 MiB");
    if (attempt > 3 || rcap >= (1ull << 32)) throw Error(SME_ELIMIT, "raw vocabulary table overflow");
    rcap <<= 2;
  }
  prof.mark("tokenize");

  // ---------------- K4 vocabulary ----------------
  // distinct raw tokens -> rlist (ascending slot order)
  int32_t *const rlist_all = W[W_RLIST].as<int32_t>(rcap);
  const int64_t nraw_all = h_nsel;
  // next build's raw table: load <= 40 % (fewer probe collisions: c2 tokenizes in 9.2 ms at 8 M
  // slots vs 10.0 ms at 4 M; option raw_load_pct)
  {
    const uint64_t pct = (uint64_t)std::max<int64_t>(10, std::min<int64_t>(90, cx->opt_raw_load_pct));
    cx->raw_cap_hint = next_pow2(std::max<uint64_t>(1ull << 20, (uint64_t)nraw_all * 100 / pct + 1));
  }
  // ---------------- K4b docid terms (before the vocabulary: their raw slots skip it) ----------------
  bool dfast = cx->opt_docid_terms != 0 && nR > 0 && nraw_all > 0 && dspan != nullptr;
  int32_t *rlist_w = nullptr;  // the raw slots of the word vocabulary (no docid term's)
  int64_t nraw_w = 0;
  uint32_t *dmark = nullptr;
  int32_t *dslot = nullptr, *dl = nullptr;
  uint64_t *dsrc = nullptr;
  Key16 *dkey = nullptr;
  int64_t Vd = 0;
  if (dfast) {
    unsigned long long *dcnt = reinterpret_cast<unsigned long long *>(W[W_DSRC].as<uint64_t>(4));  // (reallocated below)
    dmark = W[W_DMARK].as<uint32_t>(rcap);
    dslot = W[W_DSLOT].as<int32_t>(nR + 1);
    SME_HIP(hipMemsetAsync(dmark, 0xFF, rcap * sizeof(uint32_t), st));
    hipLaunchKernelGGL(k_docid_slots, dim3(grid_for(nR)), dim3(256), 0, st, t, (int64_t)n, dspan, nR, tb, dslot,
                       dmark);
    uint8_t *dflag = reinterpret_cast<uint8_t *>(W[W_DKEY].as<Key16>(nR / 16 + 1));
    hipLaunchKernelGGL(k_docid_flags, dim3(grid_for(nR)), dim3(256), 0, st, dslot, nR, dflag);
    dl = W[W_DLIST].as<int32_t>(nR + 1);
    SME_HIP(hipMemsetAsync(dcnt, 0, 4 * sizeof(unsigned long long), st));
    select_flagged(dflag, nR, dl, reinterpret_cast<int32_t *>(dcnt), cx->ws[25], cx->ws[23], st);
    SME_CHECK_LAUNCH();
    Vd = (int64_t)(int32_t)(uint32_t)d2h(dcnt, st);
    if (Vd > 0) {
      dsrc = W[W_DSRC].as<uint64_t>(Vd + 4);
      dkey = W[W_DKEY].as<Key16>(Vd);
      unsigned long long *bad = reinterpret_cast<unsigned long long *>(dsrc + Vd);
      SME_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned long long), st));
      hipLaunchKernelGGL(k_docid_keys, dim3(grid_for(Vd)), dim3(256), 0, st, dl, Vd, dspan, t, (int64_t)n, dsrc, dkey);
      hipLaunchKernelGGL(k_docid_ascending, dim3(grid_for(Vd)), dim3(256), 0, st, dkey, dsrc, Vd, t, bad);
      SME_CHECK_LAUNCH();
      if (d2h(bad, st) != 0) dfast = false;  // not in ascending order in the file (or equal terms): general path
    } else {
      dfast = false;
    }
    if (dfast) {  // the word vocabulary's raw slots
      uint8_t *wflag = W[W_RFLAG].as<uint8_t>(rcap);
      rlist_w = W[W_RLISTW].as<int32_t>(rcap);
      unsigned long long *wcnt = reinterpret_cast<unsigned long long *>(dsrc + Vd + 1);
      SME_HIP(hipMemsetAsync(wcnt, 0, sizeof(unsigned long long), st));
      hipLaunchKernelGGL(k_raw_flags_words, dim3(grid_for((int64_t)rcap)), dim3(256), 0, st, tb.key, dmark, rcap,
                         wflag);
      select_flagged(wflag, (int64_t)rcap, rlist_w, reinterpret_cast<int32_t *>(wcnt), cx->ws[25], cx->ws[23], st);
      SME_CHECK_LAUNCH();
      nraw_w = (int64_t)(int32_t)(uint32_t)d2h(wcnt, st);
    }
  }
  prof.mark("docid_terms");
  const int32_t *rlist = rlist_all;
  int64_t nraw = nraw_all;
vocab_again:  // (a docid term equal to a word term: the general path, from here)
  rlist = dfast ? rlist_w : rlist_all;
  nraw = dfast ? nraw_w : nraw_all;
  int64_t *poff = W[W_POFF].as<int64_t>(nraw + 1);
  {
    int64_t *lens = W[W_T0].as<int64_t>(nraw + 1);
    hipLaunchKernelGGL(k_raw_lens, dim3(grid_for(nraw + 1)), dim3(256), 0, st, tb.rep, rlist, nraw, lens);
    size_t tbb = 0;
    excl_scan(lens, poff, (int64_t)(nraw + 1), cx->ws[23], st);
  }
  const int64_t pool_units = d2h(poff + nraw, st);
  CandOut co;
  co.pool = W[W_POOL].as<uint16_t>(pool_units + 1);
  co.poff = poff;
  co.nraw = nraw;
  co.raw_nout = W[W_NOUT].as<int32_t>(rcap);
  int32_t *max_nout = W[W_MAXNOUT].as<int32_t>(4);  // must survive the counter resets below
  co.max_nout = max_nout;
  co.err = ovf;
  co.pres = reinterpret_cast<unsigned int *>(cnt + 28);  // read by the one-word term sort below
  SME_HIP(hipMemsetAsync(co.pres, 0, 4 * sizeof(unsigned int), st));
  int64_t *long_list = nullptr;
  uint64_t long_cap = std::max<uint64_t>(cx->vocab_long_cap, 4096);
  uint64_t ovf_cap = std::max<uint64_t>(cx->vocab_ovf_cap, 4096);
  int64_t novf = 0, nlong = 0;
  for (int attempt = 0;; attempt++) {
    co.cand_str = W[W_CSTR].as<uint64_t>(nraw + ovf_cap);
    co.ovf_key = W[W_OVFKEY].as<uint64_t>(ovf_cap);
    co.ovf_cap = ovf_cap;
    co.novf = cnt + 4;
    long_list = W[W_LONG].as<int64_t>(long_cap);
    SME_HIP(hipMemsetAsync(cnt, 0, 13 * sizeof(unsigned long long), st));
    SME_HIP(hipMemsetAsync(max_nout, 0, sizeof(int32_t), st));
    if (nraw > 0)
      hipLaunchKernelGGL(k_vocab, dim3(grid_for(nraw, 256, 16384)), dim3(256), 0, st, tb, rlist, nraw, co,
                         long_list, cnt + 5, long_cap);
    SME_CHECK_LAUNCH();
    nlong = (int64_t)d2h(cnt + 5, st);
    if ((uint64_t)nlong > long_cap) {
      long_cap = nlong + 16;
      continue;
    }
    if (nlong > 0) {
      int64_t *lens = W[W_T0].as<int64_t>(nlong + 1), *soff = W[W_T1].as<int64_t>(nlong + 1);
      hipLaunchKernelGGL(k_long_lens, dim3(grid_for(nlong)), dim3(256), 0, st, long_list, nlong, rlist, tb.rep,
                         lens);
      SME_HIP(hipMemsetAsync(lens + nlong, 0, sizeof(int64_t), st));
      size_t tbb = 0;
      excl_scan(lens, soff, (int64_t)(nlong + 1), cx->ws[23], st);
      int64_t tot = d2h(soff + nlong, st);
      uint16_t *scr = W[W_U16].as<uint16_t>(tot + 1);
      hipLaunchKernelGGL(k_vocab_long, dim3(grid_for(nlong, 64)), dim3(64), 0, st, tb, rlist, co, long_list, nlong,
                         soff, scr);
      SME_CHECK_LAUNCH();
    }
    unsigned long long hc[2];
    SME_HIP(hipMemcpyAsync(hc, cnt + 4, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(hc + 1, cnt + 8, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    if ((unsigned)hc[1] & 1u) throw Error(SME_ELIMIT, "vocabulary pool region overrun");
    if (hc[0] <= ovf_cap) {
      novf = (int64_t)hc[0];
      cx->vocab_long_cap = long_cap;
      cx->vocab_ovf_cap = ovf_cap;
      break;
    }
    if (attempt > 3) throw Error(SME_ELIMIT, "vocabulary overflow list");
    ovf_cap = hc[0] + 1024;
  }
  const int64_t ncand = nraw + novf;
  // final-term dedup
  uint64_t fcap = next_pow2(std::max<int64_t>(1024, 2 * ncand));
  unsigned long long *fkeys = W[W_FKEYS].as<unsigned long long>(fcap);
  unsigned long long *freps = W[W_FREPS].as<unsigned long long>(fcap);
  uint32_t *cand_final = W[W_CFINAL].as<uint32_t>(ncand + 1);
  SME_HIP(hipMemsetAsync(fkeys, 0, fcap * 8, st));
  SME_HIP(hipMemsetAsync(freps, 0, fcap * 8, st));
  SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
  int32_t *maxlen = reinterpret_cast<int32_t *>(cnt + 12);
  if (ncand > 0)
    hipLaunchKernelGGL(k_final_insert, dim3(grid_for(ncand)), dim3(256), 0, st, co.pool, co.cand_str, ncand, fkeys,
                       freps, fcap - 1, cand_final, ovf, maxlen);
  uint32_t *vslot = W[W_VSLOT].as<uint32_t>(ncand + 1);
  uint32_t *vidx = W[W_VIDX].as<uint32_t>(ncand + 1);
  uint64_t *vcs = W[W_VCS].as<uint64_t>(ncand + 1);
  hipLaunchKernelGGL(k_final_compact, dim3(grid_for((int64_t)fcap)), dim3(256), 0, st, fkeys, freps, fcap - 1,
                     co.cand_str, co.pool, cnt + 1, vslot, vidx, vcs);
  SME_CHECK_LAUNCH();
  unsigned long long hv[13];
  SME_HIP(hipMemcpyAsync(hv, cnt, sizeof hv, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (d2h(ovf, st)) throw Error(SME_ELIMIT, "final term table overflow");
  const int64_t Vw = (int64_t)hv[1];  // word terms (docid terms of K4b: Vd more)
  const int term_maxlen = (int)(int32_t)(uint32_t)hv[12];
  const bool term_wide = (hv[12] >> 32) != 0;  // maxlen + 1: a term has a unit >= 128
  if (dfast) {  // a docid term equal to a word term (e.g. the docid also in lowercase in a text): general path
    unsigned long long *bad = reinterpret_cast<unsigned long long *>(dsrc + Vd);
    SME_HIP(hipMemsetAsync(bad, 0, sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_docid_collide, dim3(grid_for(Vd)), dim3(256), 0, st, dsrc, dkey, Vd, t, co.pool,
                       co.cand_str, fkeys, freps, fcap - 1, bad);
    SME_CHECK_LAUNCH();
    if (d2h(bad, st) != 0) {
      dfast = false;
      goto vocab_again;
    }
  }
  const int64_t V = Vw + (dfast ? Vd : 0);  // all terms

  sme_index *ix = new sme_index(cx);
  std::unique_ptr<sme_index> ix_guard(ix);  // freed (back to the pool) if a later stage throws
  ix->K = cx->cfg.k;
  ix->R = cx->cfg.num_partitions;
  ix->idf_mode = cx->cfg.idf_mode;
  ix->N = nR;
  ix->V = V;

  int32_t *rank_of_slot = W[W_T3].as<int32_t>(fcap);
  uint32_t *order = W[W_T2].as<uint32_t>(Vw + 1);
  int64_t *term_off = ix->d_term_off.as<int64_t>(V + 1);
  if (Vw > 0) {
    // LSD radix sort of the vocabulary in String.compareTo order: 4 UTF-16 units per
    // 64-bit key word, least significant word first, stable; terms are at most
    // 99 units and all words below the longest term's length are sorted.
    // (9 ASCII units of 7 bits per word when no unit is >= 128)
    const int cpw = term_wide ? 4 : 9, ub = term_wide ? 16 : 7, kbits = cpw * ub;
    const int nwords = std::min(8, (std::max(term_maxlen, 1) + cpw - 1) / cpw);
    uint64_t *kw = W[W_KHI].as<uint64_t>(Vw), *kw2 = W[W_KLO].as<uint64_t>(Vw);
    uint32_t *ord_a = vidx, *ord_b = order;
    uint32_t *rscr = W[W_RADIX].as<uint32_t>(kv_sort_scratch(Vw) / sizeof(uint32_t) + 1);
    bool done = false;
    if (!term_wide && nwords > 1) {
      // ONE key word of the first cpw2 units, in ceil(log2(alphabet + 1)) bits each,
      // then the short runs of terms sharing those units ordered by the whole
      // string (c2: 6 radix passes instead of 12); runs over 64 terms: the full
      // word-by-word sort below
      // the units in use: collected by the vocabulary kernels from every stem
      unsigned int *pres = co.pres;
      unsigned int hp[4];
      SME_HIP(hipMemcpyAsync(hp, pres, sizeof hp, hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      uint8_t *code_h = early_code;
      int nsym = 0;
      for (int u = 0; u < 128; u++) code_h[u] = (hp[u >> 5] >> (u & 31)) & 1u ? (uint8_t)++nsym : (uint8_t)0;
      const int ub2 = bits_for((uint64_t)nsym), cpw2 = 64 / ub2;
      if (cpw2 > cpw) {
        uint8_t *code = reinterpret_cast<uint8_t *>(W[W_SEGB].as<uint64_t>(16));
        SME_HIP(hipMemcpyAsync(code, code_h, 128, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_term_code, dim3(grid_for(Vw)), dim3(256), 0, st, ord_a, Vw, vcs, co.pool, code, cpw2, ub2,
                           kw);
        uint32_t *so = kv_sort<uint64_t>(kw, ord_a, kw2, ord_b, Vw, cpw2 * ub2, rscr, st, true);
        const uint64_t *sk = so == ord_a ? kw : kw2;
        unsigned int mr = 0;
        if (term_maxlen > cpw2) {
          unsigned int *d_mr = pres;
          SME_HIP(hipMemsetAsync(d_mr, 0, sizeof(unsigned int), st));
          hipLaunchKernelGGL(k_key_runs, dim3(grid_for(Vw)), dim3(256), 0, st, sk, Vw, d_mr);
          mr = d2h(d_mr, st);
        }
        if (mr <= 64) {
          if (mr > 1) hipLaunchKernelGGL(k_key_fixup, dim3(grid_for(Vw)), dim3(256), 0, st, sk, Vw, so, vcs, co.pool);
          if (so != order) SME_HIP(hipMemcpyAsync(order, so, Vw * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
          done = true;
        } else {
          hipLaunchKernelGGL(k_iota_u32, dim3(grid_for(Vw)), dim3(256), 0, st, ord_a, Vw);  // start over
        }
      }
    }
    for (int w = nwords - 1; w >= 0 && !done; w--) {
      hipLaunchKernelGGL(k_term_word, dim3(grid_for(Vw)), dim3(256), 0, st, ord_a, Vw, vcs, co.pool, w, cpw, ub, kw);
      if (kv_sort<uint64_t>(kw, ord_a, kw2, ord_b, Vw, kbits, rscr, st) != ord_a) std::swap(ord_a, ord_b);
    }
    if (!done && ord_a != order)
      SME_HIP(hipMemcpyAsync(order, ord_a, Vw * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    if (term_maxlen > 32)
      hipLaunchKernelGGL(k_final_fixup, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vslot, freps, co.cand_str,
                         co.pool);
  }
  int64_t *drank = nullptr, *wrank_all = nullptr;
  // K6b: docid pairs beside the term sort when the word ranks need fewer key bits
  // than the merged ids (c5: 24 -> 15 bits, one LSD pass less; the c4 shard: 24 ->
  // 22, which with the records' tf bound lets the single-pass aggregation run).  Not
  // below 23 merged bits (c2: 21 -> 20 bits saves no pass; the split costs 0.1 ms)
  bool dsplit = false;
  if (dfast && job == 0 && cx->cfg.k == 1 && !dup_docno && cx->opt_docid_split && Vd < (int64_t)kDocCode) {
    const int bm = bits_for((uint64_t)std::max<int64_t>(V - 1, 1));
    dsplit = (bm > 22 || cx->opt_docid_split == 2) && bits_for((uint64_t)std::max<int64_t>(Vw - 1, 1)) < bm;
  }
  if (V > 0 && !dfast) {
    int64_t *tlen = W[W_T0].as<int64_t>(Vw + 1);
    hipLaunchKernelGGL(k_final_rank, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vslot, vcs, rank_of_slot, tlen);
    SME_HIP(hipMemsetAsync(tlen + Vw, 0, sizeof(int64_t), st));
    excl_scan(tlen, term_off, (int64_t)(Vw + 1), cx->ws[23], st);
    int64_t tchars = d2h(term_off + Vw, st);
    uint16_t *term_chars = ix->d_term_chars.as<uint16_t>(tchars + 1);
    hipLaunchKernelGGL(k_final_gather, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vcs, co.pool, term_off,
                       term_chars);
    SME_CHECK_LAUNCH();
  } else if (V > 0) {
    // K4b: the sorted word terms and the (ascending) docid terms merged by rank
    int64_t *tlen = W[W_T0].as<int64_t>(V + 1);
    Key16 *wkey = W[W_KLO].as<Key16>(Vw + 1);  // (the word sort's second key array: free again)
    uint8_t *wexact = reinterpret_cast<uint8_t *>(W[W_T1].as<uint64_t>(Vw / 8 + 2));
    int64_t *wrank = W[W_WRANK].as<int64_t>(Vw + Vd + 1);
    drank = wrank + Vw;
    wrank_all = wrank;
    if (Vw > 0) {
      hipLaunchKernelGGL(k_word_keys, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vcs, co.pool, wkey, wexact);
      hipLaunchKernelGGL(k_word_rank, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vslot, vcs, co.pool, wkey,
                         wexact, dkey, dsrc, Vd, t, rank_of_slot, tlen, wrank, (int)dsplit);
    }
    hipLaunchKernelGGL(k_docid_rank, dim3(grid_for(Vd)), dim3(256), 0, st, dkey, dsrc, Vd, order, Vw, vcs, co.pool,
                       wkey, wexact, t, tlen, drank);
    SME_HIP(hipMemsetAsync(tlen + V, 0, sizeof(int64_t), st));
    excl_scan(tlen, term_off, (int64_t)(V + 1), cx->ws[23], st);
    int64_t tchars = d2h(term_off + V, st);
    uint16_t *term_chars = ix->d_term_chars.as<uint16_t>(tchars + 1);
    if (Vw > 0)
      hipLaunchKernelGGL(k_word_gather, dim3(grid_for(Vw)), dim3(256), 0, st, order, Vw, vcs, co.pool, wrank, term_off,
                         term_chars);
    hipLaunchKernelGGL(k_docid_gather, dim3(grid_for(Vd)), dim3(256), 0, st, dsrc, dkey, Vd, drank, t, term_off,
                       term_chars);
    SME_CHECK_LAUNCH();
  } else {
    SME_HIP(hipMemsetAsync(term_off, 0, sizeof(int64_t), st));
    ix->d_term_chars.get(16);
  }
  // raw slot -> term ids
  int32_t *raw_term = W[W_RAWTERM].as<int32_t>(rcap);
  int32_t *multi = W[W_MULTI].as<int32_t>(novf + 1);
  SME_HIP(hipMemsetAsync(raw_term, 0xFF, rcap * sizeof(int32_t), st));
  if (nraw > 0)
    hipLaunchKernelGGL(k_raw_term, dim3(grid_for(nraw)), dim3(256), 0, st, rlist, nraw, cand_final, rank_of_slot,
                       co.raw_nout, raw_term);
  if (dfast)
    hipLaunchKernelGGL(k_docid_raw, dim3(grid_for(Vd)), dim3(256), 0, st, dl, Vd, dslot, drank, raw_term, co.raw_nout,
                       (int)dsplit);
  if (novf > 0) {
    uint64_t *ok2 = W[W_T0].as<uint64_t>(novf);
    uint32_t *oi = W[W_T1].as<uint32_t>(novf), *oi2 = W[W_VIDX].as<uint32_t>(novf);
    hipLaunchKernelGGL(k_iota_u32, dim3(grid_for(novf)), dim3(256), 0, st, oi, novf);
    uint32_t *rscr = W[W_RADIX].as<uint32_t>(kv_sort_scratch(novf) / sizeof(uint32_t) + 1);
    if (kv_sort<uint64_t>(co.ovf_key, oi, ok2, oi2, novf, 64, rscr, st, true) == oi) {
      std::swap(oi, oi2);
      ok2 = co.ovf_key;
    }
    hipLaunchKernelGGL(k_raw_multi, dim3(grid_for(novf)), dim3(256), 0, st, ok2, oi2, novf, nraw, cand_final,
                       rank_of_slot, raw_term, multi);
  }
  SME_CHECK_LAUNCH();
  prof.mark("vocabulary");
  if (job == 1) {
    // CharKGramTermIndexer: term stream in file order, then the char k-gram stage
    AggIn ai;
    ai.rs = rs;
    ai.tokstream = tok;
    ai.ntok = ntok;
    ai.raw_term = raw_term;
    ai.raw_nout = co.raw_nout;
    ai.multi_term = multi;
    ai.perm = perm;  // identity (docno = record index + 1)
    ai.docno = docno;
    const unsigned g_grid = (unsigned)std::min<int64_t>(std::max<int64_t>((nR + 3) / 4, 1), 8192);
    int64_t *tcnt = W[W_T2].as<int64_t>(nR + 1), *toff = W[W_T3].as<int64_t>(nR + 1);
    if (nR > 0) hipLaunchKernelGGL(k_tcount, dim3(g_grid), dim3(kAggNT), 0, st, ai, nR, tcnt);
    SME_HIP(hipMemsetAsync(tcnt + nR, 0, sizeof(int64_t), st));
    size_t tbb = 0;
    excl_scan(tcnt, toff, (int64_t)(nR + 1), cx->ws[23], st);
    const int64_t M = d2h(toff + nR, st);
    int32_t *tstream = W[W_U16].as<int32_t>(M + 1);
    if (nR > 0) hipLaunchKernelGGL(k_twrite, dim3(g_grid), dim3(kAggNT), 0, st, ai, nR, toff, tstream);
    SME_CHECK_LAUNCH();
    prof.mark("term_stream");
    chargram_stage(cx, ix, tstream, M, V, term_off, (const uint16_t *)ix->d_term_chars.p, st, &prof);
    ix->N = nR;
    ix->V = V;
    ix->Vt = V;
    ix->profile = prof.finish();
    ix_guard.release();
    return ix;
  }

  // ---------------- K5 aggregation ----------------
  const int K = cx->cfg.k;
  int64_t Vi = V;  // index "terms": terms for K = 1, distinct k-grams for K >= 2
  AggIn ai;
  ai.rs = rs;
  ai.tokstream = tok;
  ai.ntok = ntok;
  ai.raw_term = raw_term;
  ai.raw_nout = co.raw_nout;
  ai.multi_term = multi;
  ai.max_nout = co.max_nout;
  ai.perm = perm;
  ai.docno = docno;
  int64_t P = 0;
  uint32_t *p_term = nullptr;
  uint64_t *p_val = nullptr;
  // K6b fallback: the raw slots' term codes back to merged ids (every path but the
  // split single-pass aggregation reads merged ids)
  auto to_merged = [&]() {
    hipLaunchKernelGGL(k_code_to_merged, dim3(grid_for((int64_t)rcap + novf)), dim3(256), 0, st, raw_term, rcap, multi,
                       novf, (const int64_t *)wrank_all, (const int64_t *)drank);
    SME_CHECK_LAUNCH();
    dsplit = false;
  };
  // K = 1 with distinct docnos: the count pass also finds the largest tf, so the
  // emit pass can write the term sort's packed u32 values ((docno - dmin) * F + tf)
  // directly (no 8-byte pair values, no separate pack / stats passes)
  const bool want_packed = K == 1 && !dup_docno && nR > 0;
  unsigned int *mtf = reinterpret_cast<unsigned int *>(cnt + 20);
  int *dmn = reinterpret_cast<int *>(cnt + 22), *dmx = dmn + 1;
  int32_t h_mtf = 0, h_drange[2] = {0, -1};
  if (want_packed) {
    const int h_init[2] = {INT_MAX, INT_MIN};
    SME_HIP(hipMemsetAsync(mtf, 0, sizeof(unsigned int), st));
    SME_HIP(hipMemcpyAsync(dmn, h_init, sizeof h_init, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_docno_range, dim3(grid_for(nR, 256, 1024)), dim3(256), 0, st, docno, nR, dmn, dmx);
    ai.max_tf = mtf;
  }
  bool fused = false;
  // single pass: the term sort's first pass reads pair x from the region of its record
  const int64_t *sort_reg = nullptr, *sort_xoff = nullptr;
  int64_t sort_nrec = 0;
  if (K == 1 && want_packed && !cx->opt_agg_two_pass) {
    // single-pass aggregation: record regions sized by ntok * max_nout
    int64_t *reg = W[W_T2].as<int64_t>(nR + 1), *reg_off = W[W_SEGB].as<int64_t>(nR + 1);
    SME_HIP(hipMemsetAsync(cnt + 24, 0, 4 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_agg_regions, dim3(grid_for(nR, 256, 1024)), dim3(256), 0, st, perm, ntok, nR, max_nout, reg,
                       cnt + 24);
    SME_HIP(hipMemsetAsync(reg + nR, 0, sizeof(int64_t), st));
    size_t tbb = 0;
    excl_scan(reg, reg_off, (int64_t)(nR + 1), cx->ws[23], st);
    int64_t Pb = 0;
    unsigned long long h_rmx = 0;
    SME_HIP(hipMemcpyAsync(&Pb, reg_off + nR, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(&h_rmx, cnt + 24, sizeof h_rmx, hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(h_drange, dmn, sizeof h_drange, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    // (K6b: the sort keys are word ranks -- on the c4 shard 22 bits, which with the
    // records' tf bound fit the 32 the single pass asks for, where 24-bit merged ids do not)
    const int32_t tbits0 = dsplit ? bits_for((uint64_t)std::max<int64_t>(Vw - 1, 1)) : bits_for((uint64_t)std::max<int64_t>(Vi, 1));
    const uint64_t Fq = h_rmx + 1, D = (uint64_t)((int64_t)h_drange[1] - h_drange[0] + 1);
    if (Pb > 0 && Pb < (1ll << 32) && D * Fq < (1ull << 32) && tbits0 + bits_for(Fq - 1) <= 32) {
      fused = true;
      p_term = W[W_PTERM].as<uint32_t>(Pb + 1);
      ai.v32 = W[W_PVAL].as<uint32_t>(Pb + 1);
      ai.dmin = h_drange[0];
      ai.F = (uint32_t)Fq;
      ai.reg_off = reg_off;
      ai.dcnt = W[W_T3].as<int64_t>(nR + 1);
      ai.nbig = cnt + 26;
      ai.big_out = W[W_SLOWLIST].as<int64_t>(nR + 1);
      if (dsplit) {  // K6b: docid pairs beside the regions
        ai.dk_rec = W[W_KHI].as<int32_t>(nR + 1);
        ai.dv_rec = W[W_VSLOT].as<uint32_t>(nR + 1);
        ai.dbad = cnt + 32;
      }
      auto run_fused = [&]() {
        SME_HIP(hipMemsetAsync(mtf, 0, sizeof(unsigned int), st));
        SME_HIP(hipMemsetAsync(cnt + 26, 0, sizeof(unsigned long long), st));
        if (ai.dk_rec) {
          SME_HIP(hipMemsetAsync(ai.dk_rec, 0xFF, (size_t)nR * sizeof(int32_t), st));
          SME_HIP(hipMemsetAsync(ai.dbad, 0, sizeof(unsigned long long), st));
        }
        const unsigned agg_grid = agg_grid_for(cx, nR);
        hipLaunchKernelGGL(k_agg_w<true>, dim3(agg_grid), dim3(kAggNT), 0, st, ai, nR, nullptr, nullptr, p_term,
                           nullptr);
        SME_CHECK_LAUNCH();
        const int64_t nbig = (int64_t)d2h(cnt + 26, st);
        if (nbig > 0) {
          int64_t *bl2 = W[W_BIGL2].as<int64_t>(nbig);
          sort_pairs_v64<uint64_t>(reinterpret_cast<uint64_t *>(ai.big_out), reinterpret_cast<uint64_t *>(bl2), nullptr,
                                   nullptr, nbig, 64, cx->ws[120], cx->ws[121], cx->ws[122], st);
          int64_t *bcap = W[W_BIGCAP].as<int64_t>(nbig + 1), *boff = W[W_RLIST].as<int64_t>(nbig + 1);
          hipLaunchKernelGGL(k_big_caps, dim3(grid_for(nbig)), dim3(256), 0, st, bl2, nbig, perm, ntok, max_nout, bcap);
          SME_HIP(hipMemsetAsync(bcap + nbig, 0, sizeof(int64_t), st));
          excl_scan(bcap, boff, (int64_t)(nbig + 1), cx->ws[23], st);
          const int64_t gtot = d2h(boff + nbig, st);
          int32_t *gkeys = W[W_U16].as<int32_t>(gtot), *gcnt = W[W_BOFF].as<int32_t>(gtot);
          hipLaunchKernelGGL(k_agg_big, dim3((unsigned)std::min<int64_t>(nbig, 4096)), dim3(kAggNT), 0, st, ai, bl2,
                             nbig, boff, bcap, gkeys, gcnt, nullptr, reg_off, p_term, nullptr, 2);
          SME_CHECK_LAUNCH();
        }
      };
      run_fused();
      if (dsplit && d2h(ai.dbad, st) != 0) {  // a record with two docid-term pairs: merged ids, one sort
        to_merged();
        ai.dk_rec = nullptr;
        ai.dv_rec = nullptr;
        ai.dbad = nullptr;
        run_fused();
      }
      // exact pair offsets of the records (docno order)
      int64_t *xoff = W[W_NTOK2].as<int64_t>(nR + 1);
      SME_HIP(hipMemsetAsync(ai.dcnt + nR, 0, sizeof(int64_t), st));
      excl_scan(ai.dcnt, xoff, (int64_t)(nR + 1), cx->ws[23], st);
      SME_HIP(hipMemcpyAsync(&P, xoff + nR, sizeof(int64_t), hipMemcpyDeviceToHost, st));
      SME_HIP(hipMemcpyAsync(&h_mtf, mtf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      ix->P = P;
      sort_reg = reg_off;
      sort_xoff = xoff;
      sort_nrec = nR;
    }
  }
  if (dsplit && !(fused && ai.dk_rec)) to_merged();
  if (K == 1 && !fused) {
  int32_t *prec = W[W_PREC].as<int32_t>(nR + 1);
  int64_t *pair_off = W[W_T3].as<int64_t>(nR + 1);  // rank_of_slot no longer needed
  unsigned agg_grid = agg_grid_for(cx, nR);
  if (nR > 0) {
    hipLaunchKernelGGL(k_agg_w<false>, dim3(agg_grid), dim3(kAggNT), 0, st, ai, nR, prec, nullptr, nullptr, nullptr);
    SME_CHECK_LAUNCH();
  }
  // big records
  SME_HIP(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
  int64_t *big_list = W[W_SLOWLIST].as<int64_t>(nR + 1);
  if (nR > 0) hipLaunchKernelGGL(k_big_list, dim3(grid_for(nR)), dim3(256), 0, st, prec, nR, big_list, cnt);
  const int64_t nbig = (int64_t)d2h(cnt, st);
  int64_t *bcap = nullptr, *boff = nullptr;
  int32_t *gkeys = nullptr, *gcnt = nullptr, *bcount = nullptr;
  if (nbig > 0) {
    // deterministic order of big records (atomic compaction above is unordered)
    size_t tbb = 0;
    int64_t *bl2 = W[W_SCROFF].as<int64_t>(nbig);
    sort_pairs_v64<uint64_t>(reinterpret_cast<uint64_t *>(big_list), reinterpret_cast<uint64_t *>(bl2), nullptr,
                             nullptr, nbig, 64, cx->ws[120], cx->ws[121], cx->ws[122], st);
    big_list = bl2;
    bcap = W[W_T0].as<int64_t>(nbig + 1);
    boff = W[W_T1].as<int64_t>(nbig + 1);
    hipLaunchKernelGGL(k_big_caps, dim3(grid_for(nbig)), dim3(256), 0, st, big_list, nbig, perm, ntok, max_nout, bcap);
    SME_HIP(hipMemsetAsync(bcap + nbig, 0, sizeof(int64_t), st));
    excl_scan(bcap, boff, (int64_t)(nbig + 1), cx->ws[23], st);
    int64_t gtot = d2h(boff + nbig, st);
    gkeys = W[W_U16].as<int32_t>(gtot);
    gcnt = W[W_BOFF].as<int32_t>(gtot);
    bcount = W[W_NEXTS].as<int32_t>(nR + 1);
    hipLaunchKernelGGL(k_agg_big, dim3((unsigned)std::min<int64_t>(nbig, 4096)), dim3(kAggNT), 0, st, ai, big_list,
                       nbig, boff, bcap, gkeys, gcnt, bcount, nullptr, nullptr, nullptr, 0);
    SME_CHECK_LAUNCH();
  } else {
    bcount = W[W_NEXTS].as<int32_t>(nR + 1);
  }
  int64_t *prec64 = W[W_T2].as<int64_t>(nR + 1);
  hipLaunchKernelGGL(k_pair_counts, dim3(grid_for(nR + 1)), dim3(256), 0, st, prec, bcount, nR, prec64);
  SME_HIP(hipMemsetAsync(prec64 + nR, 0, sizeof(int64_t), st));
  {
    size_t tbb = 0;
    excl_scan(prec64, pair_off, (int64_t)(nR + 1), cx->ws[23], st);
  }
  SME_HIP(hipMemcpyAsync(&P, pair_off + nR, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  if (want_packed) {
    SME_HIP(hipMemcpyAsync(&h_mtf, mtf, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(h_drange, dmn, sizeof h_drange, hipMemcpyDeviceToHost, st));
  }
  SME_HIP(hipStreamSynchronize(st));
  ix->P = P;
  p_term = W[W_PTERM].as<uint32_t>(P + 1);
  if (want_packed && P > 0) {
    const int32_t tbits0 = bits_for((uint64_t)std::max<int64_t>(Vi, 1));
    const uint64_t Fq = (uint64_t)std::max(h_mtf, 1) + 1, D = (uint64_t)((int64_t)h_drange[1] - h_drange[0] + 1);
    if (D * Fq < (1ull << 32) && tbits0 + bits_for(Fq - 1) <= 32) {
      ai.v32 = W[W_PVAL].as<uint32_t>(P + 1);
      ai.dmin = h_drange[0];
      ai.F = (uint32_t)Fq;
    }
  }
  if (!ai.v32) p_val = W[W_PVAL].as<uint64_t>(P + 1);
  if (nR > 0) {
    // big records are flagged in prec via a negative marker: keep a copy of flags
    hipLaunchKernelGGL(k_agg_w<true>, dim3(agg_grid), dim3(kAggNT), 0, st, ai, nR, prec, pair_off, p_term, p_val);
    SME_CHECK_LAUNCH();
  }
  if (nbig > 0) {
    hipLaunchKernelGGL(k_agg_big, dim3((unsigned)std::min<int64_t>(nbig, 4096)), dim3(kAggNT), 0, st, ai, big_list,
                       nbig, boff, bcap, gkeys, gcnt, bcount, pair_off, p_term, p_val, 1);
    SME_CHECK_LAUNCH();
  }
  } else if (K >= 2) {
    // K >= 2: term streams, k-gram pairs per record, gram ids in TermDF order
    const int tb = bits_for((uint64_t)std::max<int64_t>(V, 1));
    const bool ranked = (int64_t)K * tb > 63 || cx->opt_kgram_rank;  // keys by iterated ranking (k_gram_round_*)
    const unsigned g_grid = (unsigned)std::min<int64_t>(std::max<int64_t>((nR + 3) / 4, 1), 8192);
    int64_t *tcnt = W[W_T2].as<int64_t>(nR + 1), *toff = W[W_T3].as<int64_t>(nR + 1);
    if (nR > 0) hipLaunchKernelGGL(k_tcount, dim3(g_grid), dim3(kAggNT), 0, st, ai, nR, tcnt);
    SME_HIP(hipMemsetAsync(tcnt + nR, 0, sizeof(int64_t), st));
    size_t tbb = 0;
    excl_scan(tcnt, toff, (int64_t)(nR + 1), cx->ws[23], st);
    const int64_t M = d2h(toff + nR, st);
    int32_t *tstream = W[W_U16].as<int32_t>(M + 1);
    if (nR > 0) hipLaunchKernelGGL(k_twrite, dim3(g_grid), dim3(kAggNT), 0, st, ai, nR, toff, tstream);
    const uint32_t *pos_key = nullptr;
    const uint32_t *grep = nullptr;  // ranked: one position of every gram id
    int64_t Vr = 0;                  // ranked: distinct k-grams
    if (ranked && M > 0) {
      if (M > 0xFFFFFFFFll) throw Error(SME_ELIMIT, "k-gram ranking of more than 2^32 term positions");
      uint64_t *ka = W[W_FKEYS].as<uint64_t>(M + 1), *kb = W[W_OVFKEY].as<uint64_t>(M + 1);
      uint32_t *pa = W[W_FREPS].as<uint32_t>(M + 1), *pb = W[W_RREPS].as<uint32_t>(M + 1);
      uint32_t *ra = W[W_RKEYS].as<uint32_t>(M + 1), *rb = W[W_CSTR].as<uint32_t>(M + 1);
      uint32_t *head = W[W_RLIST].as<uint32_t>(M + 2), *excl = W[W_POFF].as<uint32_t>(M + 2);
      uint32_t *rep = W[W_SEGB].as<uint32_t>(M + 1);
      uint32_t *rscr = W[W_RADIX].as<uint32_t>(kv_sort_scratch(M) / sizeof(uint32_t) + 1);
      const uint32_t *rprev = nullptr;
      int64_t nprev = V;  // distinct (j-1)-grams: the ranks' range
      for (int j = 2; j <= K; j++) {
        hipLaunchKernelGGL(k_gram_round_keys, dim3(g_grid), dim3(kAggNT), 0, st, tstream, toff, nR, j, tb, rprev, ka,
                           pa);
        const int kbits = std::min(64, bits_for((uint64_t)std::max<int64_t>(nprev, 1)) + tb + 1);
        uint32_t *ps = kv_sort<uint64_t>(ka, pa, kb, pb, M, kbits, rscr, st, true);
        const uint64_t *ks = ps == pa ? ka : kb;
        hipLaunchKernelGGL(k_gram_round_heads, dim3(grid_for(M)), dim3(256), 0, st, ks, M, head);
        SME_HIP(hipMemsetAsync(head + M, 0, sizeof(uint32_t), st));
        excl_scan(head, excl, M + 1, cx->ws[23], st);
        uint32_t *rnew = (rprev == ra) ? rb : ra;
        hipLaunchKernelGGL(k_gram_round_scatter, dim3(grid_for(M)), dim3(256), 0, st, ks, ps, head, excl, M, rnew,
                           j == K ? rep : nullptr);
        SME_CHECK_LAUNCH();
        nprev = (int64_t)d2h(excl + M, st);
        rprev = rnew;
      }
      pos_key = rprev;
      grep = rep;
      Vr = nprev;
    }
    int64_t *pcount = W[W_T1].as<int64_t>(nR + 1), *pair_off = W[W_T0].as<int64_t>(nR + 1);
    uint8_t *bigf = W[W_SLOW].as<uint8_t>(nR + 1);
    if (nR > 0)
      hipLaunchKernelGGL(k_gram_agg<false>, dim3(g_grid), dim3(kAggNT), 0, st, tstream, toff, nR, perm, docno, K, tb,
                         pcount, bigf, nullptr, nullptr, nullptr, pos_key);
    SME_HIP(hipMemsetAsync(pcount + nR, 0, sizeof(int64_t), st));
    excl_scan(pcount, pair_off, (int64_t)(nR + 1), cx->ws[23], st);
    const int64_t Pg = d2h(pair_off + nR, st);
    uint64_t *pkey = W[W_KHI].as<uint64_t>(Pg + 1), *pval0 = W[W_KLO].as<uint64_t>(Pg + 1);
    if (nR > 0)
      hipLaunchKernelGGL(k_gram_agg<true>, dim3(g_grid), dim3(kAggNT), 0, st, tstream, toff, nR, perm, docno, K, tb,
                         pcount, bigf, pair_off, pkey, pval0, pos_key);
    SME_CHECK_LAUNCH();
    // sort pairs by gram key (stable: docno order within a gram)
    uint64_t *pkey_s = W[W_CKEY].as<uint64_t>(Pg + 1);
    p_val = W[W_PVAL].as<uint64_t>(Pg + 1);
    if (Pg > 0) {
      sort_pairs_v64<uint64_t>(pkey, pkey_s, pval0, p_val, Pg,
                               ranked ? bits_for((uint64_t)std::max<int64_t>(Vr, 1)) : K * tb, cx->ws[120],
                               cx->ws[121], cx->ws[122], st);
    }
    uint32_t *gflag = W[W_VSLOT].as<uint32_t>(Pg + 1), *gincl = W[W_VIDX].as<uint32_t>(Pg + 2);
    p_term = W[W_PTERM].as<uint32_t>(Pg + 1);
    int64_t Vg = 0;
    if (Pg > 0) {
      hipLaunchKernelGGL(k_gram_flags, dim3(grid_for(Pg)), dim3(256), 0, st, pkey_s, Pg, gflag);
      // inclusive sum = the exclusive scan of (flags, 0) shifted by one
      SME_HIP(hipMemsetAsync(gflag + Pg, 0, sizeof(uint32_t), st));
      excl_scan(gflag, gincl, Pg + 1, cx->ws[23], st);
      gincl += 1;
      Vg = (int64_t)d2h(gincl + Pg - 1, st);
      int32_t *gcomp = ix->d_gram.as<int32_t>(Vg * K + 1);
      // (ranked: the keys are the gram ids themselves, the components come from
      // one occurrence of each gram)
      hipLaunchKernelGGL(k_gram_ids, dim3(grid_for(Pg)), dim3(256), 0, st, pkey_s, gincl, Pg, ranked ? 0 : K, tb,
                         p_term, gcomp);
      if (ranked)
        hipLaunchKernelGGL(k_gram_comp_rep, dim3(grid_for(Vg)), dim3(256), 0, st, grep, Vg, K, tstream, gcomp);
      SME_CHECK_LAUNCH();
    } else {
      ix->d_gram.get(16);
    }
    P = Pg;
      Vi = Vg;
    ix->P = P;
    dup_docno = true;  // occurrences of big records and equal docnos merge in the reducer step
  }
  prof.mark("aggregate");

  // ---------------- K6 sort by term ----------------
  // K6b: the docid pairs (one per record at most, docno order) as a list sorted by
  // docid index j, and every word's (shift, merged id)
  const bool split = dsplit && ai.dk_rec != nullptr;
  int64_t Pw = P, Nd = 0;
  uint32_t *dk = nullptr, *dv = nullptr;
  uint2 *xw = nullptr;
  if (split) {
    uint8_t *dfl = W[W_RREPS].as<uint8_t>(nR + 1);
    int32_t *didx = W[W_CFINAL].as<int32_t>(nR + 1);
    hipLaunchKernelGGL(k_dsplit_flags, dim3(grid_for(nR)), dim3(256), 0, st, ai.dk_rec, nR, dfl);
    SME_HIP(hipMemsetAsync(cnt + 33, 0, 2 * sizeof(unsigned long long), st));
    select_flagged(dfl, nR, didx, reinterpret_cast<int32_t *>(cnt + 33), cx->ws[25], cx->ws[23], st);
    dk = W[W_CSTR].as<uint32_t>(nR + 1);
    dv = W[W_VIDX].as<uint32_t>(nR + 1);
    hipLaunchKernelGGL(k_dsplit_gather, dim3(grid_for(nR)), dim3(256), 0, st, didx, cnt + 33, ai.dk_rec, ai.dv_rec, dk,
                       dv, cnt + 34);
    SME_CHECK_LAUNCH();
    unsigned long long hd[2];
    SME_HIP(hipMemcpyAsync(hd, cnt + 33, sizeof hd, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    Nd = (int64_t)(uint32_t)hd[0];
    if (hd[1] != 0 && Nd > 1) {  // docno order is not docid order: a stable sort by j
      uint32_t *dk2 = W[W_LONG].as<uint32_t>(Nd + 1), *dv2 = reinterpret_cast<uint32_t *>(W[W_OVFKEY].as<uint64_t>(Nd / 2 + 1));
      uint32_t *rs2 = W[W_RADIX].as<uint32_t>(kv_sort_scratch(Nd) / sizeof(uint32_t) + 1);
      if (kv_sort<uint32_t>(dk, dv, dk2, dv2, Nd, bits_for((uint64_t)Vd), rs2, st, true) != dv) {
        dk = dk2;
        dv = dv2;
      }
    }
    xw = reinterpret_cast<uint2 *>(W[W_DKEY].as<Key16>(Vw / 2 + 1));
    if (Vw > 0)
      hipLaunchKernelGGL(k_word_shift, dim3(grid_for(Vw)), dim3(256), 0, st, (const int64_t *)wrank_all, Vw, dk, Nd,
                         xw);
    SME_CHECK_LAUNCH();
    P = Pw + Nd;
    if (P > 0xFFFFFFFFll) throw Error(SME_ELIMIT, "term sort of more than 2^32 pairs");
    ix->P = P;
    prof.mark("docid_pairs");
  }
  const int tbits = split ? bits_for((uint64_t)std::max<int64_t>(Vw - 1, 1)) : bits_for((uint64_t)std::max<int64_t>(Vi, 1));
  uint32_t *key_s = W[W_T0].as<uint32_t>(P + 1);
  int64_t Pm = P;
  int32_t max_tf = 1;
  // packed path: u32 keys and u32 values through both sorts (no duplicate docnos)
  bool packed = false;
  int64_t dmin = 0;
  uint32_t F = 0;
  if (ai.v32 != nullptr) {  // emitted packed by the aggregation (see want_packed)
    max_tf = std::max<int32_t>(1, h_mtf);
    packed = true;
    dmin = ai.dmin;
    F = ai.F;
  } else if (P > 0 && !dup_docno && K == 1) {
    SME_HIP(hipMemsetAsync(mtf, 0, sizeof(unsigned int), st));
    const int h_init[2] = {INT_MAX, INT_MIN};
    SME_HIP(hipMemcpyAsync(dmn, h_init, sizeof h_init, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_pair_stats, dim3(grid_for(P, 256, 2048)), dim3(256), 0, st, p_val, P, mtf);
    hipLaunchKernelGGL(k_docno_range, dim3(grid_for(nR, 256, 1024)), dim3(256), 0, st, docno, nR, dmn, dmx);
    unsigned int h_m = d2h(mtf, st);
    int h_r[2];
    SME_HIP(hipMemcpyAsync(h_r, dmn, sizeof h_r, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    const uint64_t Fq = (uint64_t)h_m + 1, D = (uint64_t)((int64_t)h_r[1] - (int64_t)h_r[0] + 1);
    max_tf = std::max<int32_t>(1, (int32_t)h_m);
    packed = D * Fq < (1ull << 32) && tbits + bits_for((uint64_t)max_tf) <= 32;
    dmin = h_r[0];
    F = (uint32_t)Fq;
  }
  int32_t *docno_d = nullptr, *tf_d = nullptr;
  int64_t *off = nullptr;
  std::vector<double> early_lut;  // the fused weight pass's LUT (outlives its async upload)
  bool weights_fused = false;
  if (packed) {
    uint32_t *v32 = ai.v32;
    if (v32 == nullptr) {
      v32 = reinterpret_cast<uint32_t *>(W[W_T1].as<uint64_t>(P + 1));
      hipLaunchKernelGGL(k_pack_pairs, dim3(grid_for(P)), dim3(256), 0, st, p_val, P, dmin, F, v32);
    }
    uint32_t *v32s = W[W_T2].as<uint32_t>(P + 1);
    docno_d = ix->d_docno_d.as<int32_t>(P + 1);
    tf_d = ix->d_tf_d.as<int32_t>(P + 1);
    // hand-written stable LSD radix sort by term id (sme_sort.hip); the last
    // pass unpacks (docno, tf) into the CSR arrays
    uint32_t *rscr = W[W_RADIX].as<uint32_t>(term_sort_scratch(P) / sizeof(uint32_t) + 1);
    // reference idf mode: one idf for every term (stored df 1, T1/T2), so the last
    // pass writes the TF-IDF weights too (no separate weight pass over tf)
    double *wf = nullptr;
    if (ix->idf_mode == SME_IDF_REFERENCE && P > 0) {
      early_lut.assign((size_t)max_tf + 1, 0.0);
      for (int i = 1; i <= max_tf; i++) early_lut[(size_t)i] = 1.0 + log((double)i);
      SME_HIP(hipMemcpyAsync(ix->d_lut.as<double>(max_tf + 1), early_lut.data(), early_lut.size() * sizeof(double),
                             hipMemcpyHostToDevice, st));
      wf = ix->d_w.as<double>(P + 1);
      weights_fused = true;
    }
    const double idf_r = log10((double)(std::max<int64_t>(nR, 0) / 1));
    // digit width (sort_digit_bits; 0 = auto): 11, or 8 past 2^30 pairs -- a pass's
    // per-(tile, digit) counts grow with the pairs, and 2048 digits over an 8192-pair
    // tile leave 4-pair runs to scatter (c4 shard, 22-bit keys: two 11-bit passes
    // 34.5 ms, three of <= 8 bits 30.9 ms; c2 / c5 keep 11)
    const int sort_bits = cx->opt_sort_bits > 0 ? (int)cx->opt_sort_bits : (Pw > (int64_t(1) << 30) ? 8 : 11);
    key_s = term_sort(p_term, v32, key_s, v32s, sort_nrec, sort_reg, sort_xoff, Pw, tbits, dmin, F, docno_d, tf_d, rscr,
                      st, wf ? (const double *)ix->d_lut.p : nullptr, idf_r, wf, sort_bits, xw, P);
    off = ix->d_off.as<int64_t>(Vi + 1);
    SME_HIP(hipMemsetAsync(off, 0, (Vi + 1) * sizeof(int64_t), st));
    if (!split) {
      hipLaunchKernelGGL(k_term_offsets<false>, dim3(grid_for(P)), dim3(256), 0, st, key_s, P, off, Vi);
    } else {
      // word terms' offsets over the sorted keys (the docid slots are holes), then
      // the docid terms' offsets and their pairs in the holes
      hipLaunchKernelGGL(k_term_offsets<true>, dim3(grid_for(P)), dim3(256), 0, st, key_s, P, off, Vi);
      hipLaunchKernelGGL(k_docid_off, dim3(grid_for(Vd)), dim3(256), 0, st, dk, Nd, Vd, (const int64_t *)drank,
                         (const int64_t *)wrank_all, Vw, xw, Pw, off);
      if (Nd > 0)
        hipLaunchKernelGGL(k_docid_place, dim3(grid_for(Nd)), dim3(256), 0, st, dk, dv, Nd, (const int64_t *)drank,
                           (const int64_t *)wrank_all, Vw, xw, off, Pw, dmin, F, docno_d, tf_d, key_s,
                           wf ? (const double *)ix->d_lut.p : nullptr, idf_r, wf);
    }
    SME_CHECK_LAUNCH();
  } else {
    uint64_t *val_s = W[W_T1].as<uint64_t>(P + 1);
    if (P > 0)
      sort_pairs_v64<uint32_t>(p_term, key_s, p_val, val_s, P, tbits, cx->ws[120], cx->ws[121], cx->ws[122], st);
    if (dup_docno && P > 0) {
      // MyReducer.reduce: equal docnos (duplicate docids) are merged by summing tf
      uint64_t *ck = W[W_PVAL].as<uint64_t>(P), *ck2 = W[W_T2].as<uint64_t>(P);
      int32_t *tfv = reinterpret_cast<int32_t *>(W[W_PTERM].as<uint32_t>(P)), *tf2 = W[W_T3].as<int32_t>(P);
      hipLaunchKernelGGL(k_dup_keys, dim3(grid_for(P)), dim3(256), 0, st, key_s, val_s, P, ck, tfv);
      int64_t *nout = reinterpret_cast<int64_t *>(cnt + 10);
      reduce_by_key_sum(ck, tfv, P, ck2, tf2, nout, cx->ws[120], cx->ws[121], cx->ws[23], st);
      Pm = d2h(nout, st);
      hipLaunchKernelGGL(k_dup_unpack, dim3(grid_for(Pm)), dim3(256), 0, st, ck2, tf2, Pm, key_s, val_s);
    }
    off = ix->d_off.as<int64_t>(Vi + 1);
    SME_HIP(hipMemsetAsync(off, 0, (Vi + 1) * sizeof(int64_t), st));
    if (Pm > 0) hipLaunchKernelGGL(k_term_offsets<false>, dim3(grid_for(Pm)), dim3(256), 0, st, key_s, Pm, off, Vi);
    docno_d = ix->d_docno_d.as<int32_t>(Pm + 1);
    tf_d = ix->d_tf_d.as<int32_t>(Pm + 1);
    if (Pm > 0) hipLaunchKernelGGL(k_unpack_vals, dim3(grid_for(Pm)), dim3(256), 0, st, val_s, Pm, docno_d, tf_d);
    SME_CHECK_LAUNCH();
    if (Pm > 0) {
      int32_t *mx = reinterpret_cast<int32_t *>(cnt + 11);
      reduce_max<int32_t>(tf_d, Pm, mx, st);
      max_tf = std::max(1, d2h(mx, st));
    }
  }
  ix->P = Pm;
  const int64_t PP = Pm;
  prof.mark("sort_term");

  // ---------------- K7 weights ----------------
  ix->max_tf = max_tf;
  {
    // LUT[tf] = 1 + ln(tf) and idf tables, evaluated once on the host with the
    // platform libm so the device weights equal the fp64 reference bit for bit.
    std::vector<double> lut(max_tf + 1, 0.0);
    for (int i = 1; i <= max_tf; i++) lut[i] = 1.0 + log((double)i);
    double *d_lut = ix->d_lut.as<double>(max_tf + 1);
    SME_HIP(hipMemcpyAsync(d_lut, lut.data(), lut.size() * sizeof(double), hipMemcpyHostToDevice, st));
    const int64_t Nn = std::max<int64_t>(nR, 0);
    double idf_ref = log10((double)(Nn / 1));  // stored df of every real term is 1 (T1)
    int64_t sdf = (int64_t)std::sqrt((double)std::max<int64_t>(Nn, 1)) + 1;
    std::vector<double> by_df(sdf + 1), by_q(Nn / std::max<int64_t>(sdf, 1) + 2);
    for (int64_t d = 1; d <= sdf; d++) by_df[d] = log10((double)(Nn / d));
    for (size_t q = 0; q < by_q.size(); q++) by_q[q] = log10((double)q);
    double *d_bydf = W[W_U16].as<double>(by_df.size() + by_q.size());
    double *d_byq = d_bydf + by_df.size();
    SME_HIP(hipMemcpyAsync(d_bydf, by_df.data(), by_df.size() * sizeof(double), hipMemcpyHostToDevice, st));
    SME_HIP(hipMemcpyAsync(d_byq, by_q.data(), by_q.size() * sizeof(double), hipMemcpyHostToDevice, st));
    double *idf = ix->d_idf.as<double>(Vi + 1);
    if (Vi > 0)
      hipLaunchKernelGGL(k_term_idf, dim3(grid_for(Vi)), dim3(256), 0, st, off, Vi, idf_ref, Nn, nullptr, d_bydf, sdf,
                         d_byq, ix->idf_mode, idf);
    double *w = ix->d_w.as<double>(PP + 1);
    if (PP > 0 && !weights_fused)
      hipLaunchKernelGGL(k_weights, dim3(grid_for(PP)), dim3(256), 0, st, key_s, tf_d, PP, d_lut, idf_ref, off, Nn,
                         d_bydf, sdf, d_byq, ix->idf_mode, w);
    SME_CHECK_LAUNCH();
    SME_HIP(hipStreamSynchronize(st));  // host vectors go out of scope
  }
  prof.mark("weights");

  // ---------------- K8 reduce-output order ----------------
  int32_t *docno_o = ix->d_docno_o.as<int32_t>(PP + 1), *tf_o = ix->d_tf_o.as<int32_t>(PP + 1);
  if (PP > 0 && max_tf <= kTfSortMaxTf) {
    // segmented counting sort over the term CSR (no full-width key sort)
    hipLaunchKernelGGL(k_tfsort_tiny, dim3(grid_for(Vi)), dim3(256), 0, st, off, Vi, docno_d, tf_d, docno_o, tf_o);
    // medium and large segments as lists (a grid-stride walk over all V terms costs a
    // dependent offset load per term and block)
    int64_t *ntl = W[W_FKEYS].as<int64_t>(3 * (Vi + 1)), *toff = W[W_FREPS].as<int64_t>(Vi + 1);
    int32_t *seg_med = reinterpret_cast<int32_t *>(ntl + Vi + 1), *seg_large = seg_med + Vi,
            *seg_small = seg_large + Vi, *seg_wave = seg_small + Vi;
    unsigned long long *nseg = cnt + 28;  // [0] medium, [1] large, [2] small, [3] wave-sized
    SME_HIP(hipMemsetAsync(nseg, 0, 4 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_tf_classify, dim3(grid_for(Vi)), dim3(256), 0, st, off, Vi, seg_med, seg_large, seg_small,
                       seg_wave, nseg);
    // the small / medium / wave-sized classes (disjoint terms, disjoint output
    // ranges) run on the auxiliary stream beside the large tiles' count / scan /
    // place chain, which also waits on a host read of the tile count (tf sort
    // 3.1 -> 2.8 ms; k_docno beside the tokenizer, tried the same way, slowed the
    // tokenizer by more than it saved)
    hipStream_t s2 = cx->aux_stream;
    SME_HIP(hipEventRecord(cx->ev_fork, st));
    SME_HIP(hipStreamWaitEvent(s2, cx->ev_fork, 0));
    // every exit from this block -- a throw between the fork and the join
    // included -- makes st wait for the auxiliary stream's kernels, so they never
    // write docno_o / tf_o after the build's workspace is released or reused
    struct AuxJoin {
      hipStream_t st, s2;
      hipEvent_t ev;
      ~AuxJoin() {
        (void)hipEventRecord(ev, s2);
        (void)hipStreamWaitEvent(st, ev, 0);
      }
    } aux_join{st, s2, cx->ev_join};
    hipLaunchKernelGGL(k_tfsort_small, dim3(grid_for(Vi * 64, 256, 8192)), dim3(256), 0, s2, off, seg_small, nseg + 2,
                       docno_d, tf_d, docno_o, tf_o);
    const size_t lds4 = (size_t)(max_tf + 1) * 4 * sizeof(int32_t);
    hipLaunchKernelGGL(k_tfsort_block<4>, dim3((unsigned)std::min<int64_t>(std::max<int64_t>(Vi, 1), 4096)),
                       dim3(256), lds4, s2, off, Vi, docno_d, tf_d, docno_o, tf_o, seg_med, nseg, max_tf);
    hipLaunchKernelGGL(k_tfsort_block<1>, dim3((unsigned)std::min<int64_t>(std::max<int64_t>(Vi, 1), 32768)),
                       dim3(64), lds4 / 4, s2, off, Vi, docno_d, tf_d, docno_o, tf_o, seg_wave, nseg + 3, max_tf);
    SME_CHECK_LAUNCH();
    // large segments: tiles spread over the whole chip
    hipLaunchKernelGGL(k_tf_ntiles, dim3(grid_for(Vi + 1)), dim3(256), 0, st, off, seg_large, nseg + 1, Vi, ntl);
    size_t tbb = 0;
    excl_scan(ntl, toff, (int64_t)(Vi + 1), cx->ws[23], st);
    const int64_t ntiles = d2h(toff + Vi, st);
    if (ntiles > 0) {
      const int F = max_tf + 1;
      int32_t *tcnt = reinterpret_cast<int32_t *>(W[W_CKEY].as<uint64_t>((ntiles * F + 1) / 2 + 1));
      const unsigned tg = (unsigned)std::min<int64_t>((ntiles + 3) / 4, 8192);
      hipLaunchKernelGGL(k_tf_tile_count, dim3(tg), dim3(256), (size_t)4 * F * sizeof(int32_t), st, off, seg_large,
                         nseg + 1, toff, ntiles, tf_d, max_tf, tcnt);
      hipLaunchKernelGGL(k_tf_tile_scan, dim3((unsigned)std::min<int64_t>(Vi, 8192)), dim3(256), 0, st, nseg + 1,
                         toff, max_tf, tcnt);
      hipLaunchKernelGGL(k_tf_tile_place, dim3(tg), dim3(256), (size_t)4 * F * sizeof(int32_t), st, off, seg_large,
                         nseg + 1, toff, ntiles, docno_d, tf_d, max_tf, tcnt, docno_o, tf_o);
    }
    SME_CHECK_LAUNCH();
  } else if (PP > 0) {  // (aux_join: st waits for the auxiliary stream here)
    const int tfb = bits_for((uint64_t)max_tf);
    if (tbits + tfb <= 32) {  // u32 composite (term, tf desc)
      const uint32_t tfmask = (uint32_t)((1ull << tfb) - 1);
      uint32_t *ck = reinterpret_cast<uint32_t *>(W[W_PVAL].as<uint64_t>(PP)), *ck2 = W[W_T2].as<uint32_t>(PP);
      hipLaunchKernelGGL(k_composite32, dim3(grid_for(PP)), dim3(256), 0, st, key_s, tf_d, PP, tfb, tfmask, ck);
      // (docno_d stays intact: the sort's values start from a copy)
      uint32_t *dv = W[W_T3].as<uint32_t>(PP);
      SME_HIP(hipMemcpyAsync(dv, docno_d, (size_t)PP * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
      sort_pairs<uint32_t>(ck, ck2, dv, reinterpret_cast<uint32_t *>(docno_o), PP, tbits + tfb, cx->ws[122], st);
      hipLaunchKernelGGL(k_composite32_tf, dim3(grid_for(PP)), dim3(256), 0, st, ck2, PP, tfmask, tf_o);
    } else {
      const uint64_t tfmask = (1ull << tfb) - 1;
      uint64_t *ck = W[W_PVAL].as<uint64_t>(PP), *ck2 = W[W_T2].as<uint64_t>(PP);
      hipLaunchKernelGGL(k_composite, dim3(grid_for(PP)), dim3(256), 0, st, key_s, tf_d, PP, tfb, tfmask, ck);
      uint32_t *dv = W[W_T3].as<uint32_t>(PP);
      SME_HIP(hipMemcpyAsync(dv, docno_d, (size_t)PP * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
      sort_pairs<uint64_t>(ck, ck2, dv, reinterpret_cast<uint32_t *>(docno_o), PP, tbits + tfb, cx->ws[122], st);
      hipLaunchKernelGGL(k_composite_tf, dim3(grid_for(PP)), dim3(256), 0, st, ck2, PP, tfmask, tf_o);
    }
    SME_CHECK_LAUNCH();
  }
  prof.mark("sort_tf");

  // doc-counter postings need every record's docno in input order
  int32_t *rdn = ix->d_rec_docno.as<int32_t>(nR + 1);
  if (nR > 0 && want_packed && h_drange[1] >= h_drange[0]) {  // range known from the aggregation
    SME_HIP(hipMemcpyAsync(rdn, docno, nR * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    ix->dmin = h_drange[0];
    ix->dmax = h_drange[1];
  } else if (nR > 0) {
    SME_HIP(hipMemcpyAsync(rdn, docno, nR * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    int *dmn = reinterpret_cast<int *>(cnt + 12), *dmx = dmn + 1;
    const int h_init[2] = {INT_MAX, INT_MIN};
    SME_HIP(hipMemcpyAsync(dmn, h_init, sizeof h_init, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_docno_range, dim3(grid_for(nR, 256, 1024)), dim3(256), 0, st, docno, nR, dmn, dmx);
    int h_r[2];
    SME_HIP(hipMemcpyAsync(h_r, dmn, sizeof h_r, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    ix->dmin = h_r[0];
    ix->dmax = h_r[1];
  }
  prof.mark("finalize");
  ix->V = Vi;
  ix->Vt = V;
  ix->profile = prof.finish();
  ix_guard.release();
  return ix;
}

// ---------------------------------------------------------------------------
// re-weight with global statistics (doc-sharded multi-GPU: N and df all-reduced)
// ---------------------------------------------------------------------------
__global__ void k_reweight(const int64_t *off, int64_t V, const int32_t *tf, const double *lut, double idf_ref,
                           const int64_t *gdf, int64_t N, const double *idf_by_df, int64_t sdf, const double *idf_by_q,
                           int mode, double *w) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t t = blockIdx.x * wpb + (threadIdx.x >> 6); t < V; t += (int64_t)gridDim.x * wpb) {
    double idf = idf_ref;
    if (mode != SME_IDF_REFERENCE) {
      int64_t df = gdf ? gdf[t] : off[t + 1] - off[t];
      idf = df <= sdf ? idf_by_df[df] : idf_by_q[N / df];
    }
    for (int64_t p = off[t] + lane; p < off[t + 1]; p += 64) w[p] = __dmul_rn(lut[tf[p]], idf);
  }
}

void reweight_index(sme_index *ix, int64_t N, const int64_t *d_gdf, hipStream_t st) {
  auto &W = ix->ctx->ws;
  std::vector<double> lut(ix->max_tf + 1, 0.0);
  for (int i = 1; i <= ix->max_tf; i++) lut[i] = 1.0 + log((double)i);
  const int64_t Nn = std::max<int64_t>(N, 0);
  double idf_ref = log10((double)(Nn / 1));
  int64_t sdf = (int64_t)std::sqrt((double)std::max<int64_t>(Nn, 1)) + 1;
  std::vector<double> by_df(sdf + 1), by_q(Nn / std::max<int64_t>(sdf, 1) + 2);
  for (int64_t d = 1; d <= sdf; d++) by_df[d] = log10((double)(Nn / d));
  for (size_t q = 0; q < by_q.size(); q++) by_q[q] = log10((double)q);
  double *d_lut = ix->d_lut.as<double>(lut.size());
  double *d_tab = W[57].as<double>(by_df.size() + by_q.size());
  SME_HIP(hipMemcpyAsync(d_lut, lut.data(), lut.size() * sizeof(double), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_tab, by_df.data(), by_df.size() * sizeof(double), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_tab + by_df.size(), by_q.data(), by_q.size() * sizeof(double), hipMemcpyHostToDevice, st));
  if (ix->V > 0)
    hipLaunchKernelGGL(k_term_idf, dim3((unsigned)std::min<int64_t>((ix->V + 255) / 256, 65536)), dim3(256), 0, st,
                       (const int64_t *)ix->d_off.p, ix->V, idf_ref, Nn, d_gdf, d_tab, sdf, d_tab + by_df.size(),
                       ix->idf_mode, (double *)ix->d_idf.p);
  if (ix->V > 0)
    hipLaunchKernelGGL(k_reweight, dim3((unsigned)std::min<int64_t>((ix->V + 3) / 4, 65536)),
                       dim3(256), 0, st, (const int64_t *)ix->d_off.p, ix->V, (const int32_t *)ix->d_tf_d.p, d_lut,
                       idf_ref, d_gdf, Nn, d_tab, sdf, d_tab + by_df.size(), ix->idf_mode, (double *)ix->d_w.p);
  SME_CHECK_LAUNCH();
  SME_HIP(hipStreamSynchronize(st));
  ix->q_ready = false;  // impact rows and alpha depend on idf (prepare_queries rebuilds them)
}

}  // namespace sme
