// sme_chargram.hip -- the CharKGramTermIndexer job on the device
// (C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:74-211; C/ = ABDURRAHMAN-PA2-3-code/src/).
//
// The mapper turns every token t of processContent(doc) into '$' t '$' and adds t to a
// HashSet per k-unit substring (in-mapper combining over the whole map task, :88-111);
// close() emits each gram with its set in HashSet iteration order (:114-129); with one
// map task the reducer's pairwise merge sees a single list and returns it (:136-171);
// TextOutputFormat writes "gram\t[t1, t2, ...]\n" per key (ArrayListWritable.toString,
// C/edu/umd/cloud9/io/array/ArrayListWritable.java:112-123), keys in Text byte order
// inside each of R HashPartitioner partitions.
//
// Device formulation (everything a function of the term vocabulary + first occurrences):
//   * a term's place in a gram's set depends only on its insertion index among the set's
//     members = the order of the terms' FIRST occurrence in the task's token stream;
//   * the JDK 6 HashMap iteration order of n keys inserted in that order has a closed
//     form: final capacity C (16, doubled while n > 3C/4), bucket = spread(hashCode) &
//     (C-1); key t was inserted at capacity c_t, and with d = log2(C / c_t) the chain of a
//     bucket lists d = 0, 2, 4, ... (newest first) then ..., 5, 3, 1 (oldest first) --
//     head insertion, and each resize transfer reverses a chain.  (Checked against a
//     direct simulation of the JDK 6 algorithm in oracle/oracle_chargram.c.)
// So: first occurrence per term (atomic min over the stream) -> (gram, term) pairs with
// UTF-8 gram keys packed big-endian into W = ceil((3k + 2) / 8) 64-bit words, the byte
// length in the last word's low 16 bits (Text order = numeric order of the word tuple,
// any k) -> LSD sort by (gram words, first occurrence), dedup -> per-element HashSet
// rank key -> sort -> one pass that writes every line at its scanned offset.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sme_internal.hpp"

namespace sme {

// key words of a k-unit gram: <= 3 bytes per unit (a surrogate pair: 4 bytes for 2
// units) + the 16-bit byte length
inline int cg_words(int K) { return (3 * K + 2 + 7) / 8; }
// byte j of a gram key (word-major layout kw[w * stride + i])
__device__ __forceinline__ uint8_t cg_byte(const uint64_t *kw, int64_t stride, int64_t i, int j) {
  return (uint8_t)(kw[(int64_t)(j >> 3) * stride + i] >> (56 - 8 * (j & 7)));
}
__device__ __forceinline__ int cg_nbytes(const uint64_t *kw, int64_t stride, int W, int64_t i) {
  return (int)(kw[(int64_t)(W - 1) * stride + i] & 0xFFFFu);
}
__device__ __forceinline__ bool cg_key_eq(const uint64_t *kw, int64_t stride, int W, int64_t a, int64_t b) {
  for (int w = 0; w < W; w++)
    if (kw[(int64_t)w * stride + a] != kw[(int64_t)w * stride + b]) return false;
  return true;
}

// String.getBytes("UTF-8") of units [0, n) (unpaired surrogate -> '?'); returns bytes
__device__ __forceinline__ int java_utf8_at(const uint16_t *u, int n, uint8_t *o) {
  int k = 0;
  for (int i = 0; i < n; i++) {
    const unsigned c = u[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && u[i + 1] >= 0xDC00 && u[i + 1] <= 0xDFFF) {
      const unsigned cp = 0x10000 + ((c - 0xD800) << 10) + (u[i + 1] - 0xDC00);
      o[k++] = (uint8_t)(0xF0 | (cp >> 18));
      o[k++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
      o[k++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      o[k++] = (uint8_t)(0x80 | (cp & 0x3F));
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      o[k++] = '?';
    } else if (c < 0x80) {
      o[k++] = (uint8_t)c;
    } else if (c < 0x800) {
      o[k++] = (uint8_t)(0xC0 | (c >> 6));
      o[k++] = (uint8_t)(0x80 | (c & 0x3F));
    } else {
      o[k++] = (uint8_t)(0xE0 | (c >> 12));
      o[k++] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
      o[k++] = (uint8_t)(0x80 | (c & 0x3F));
    }
  }
  return k;
}
__device__ __forceinline__ int java_utf8_len(const uint16_t *u, int64_t n) {
  int k = 0;
  for (int64_t i = 0; i < n; i++) {
    const unsigned c = u[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && u[i + 1] >= 0xDC00 && u[i + 1] <= 0xDFFF) {
      k += 4;
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      k += 1;
    } else {
      k += c < 0x80 ? 1 : (c < 0x800 ? 2 : 3);
    }
  }
  return k;
}

// first occurrence (stream position) of every term; read first, so the hot terms'
// words are only written a handful of times
__global__ void k_first_occ(const int32_t *ts, int64_t M, unsigned long long *first) {
  for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < M; x += (int64_t)gridDim.x * blockDim.x) {
    const int32_t t = ts[x];
    if (first[t] > (unsigned long long)x) atomicMin(&first[t], (unsigned long long)x);
  }
}

// per term: String.hashCode, Java UTF-8 length, gram count of '$' t '$'
__global__ void k_term_props(const int64_t *toff, const uint16_t *tch, int64_t V, int K, int32_t *jh, int32_t *u8len,
                             int64_t *ngram) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t <= V; t += (int64_t)gridDim.x * blockDim.x) {
    if (t == V) {
      ngram[V] = 0;
      continue;
    }
    const int64_t b = toff[t], L = toff[t + 1] - b;
    uint32_t h = 0;
    for (int64_t i = 0; i < L; i++) h = 31u * h + tch[b + i];
    jh[t] = (int32_t)h;
    u8len[t] = java_utf8_len(tch + b, L);
    ngram[t] = L + 2 - K + 1 > 0 ? L + 2 - K + 1 : 0;
  }
}

__global__ void k_rank_of(const uint32_t *order, int64_t V, uint32_t *rank) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < V; r += (int64_t)gridDim.x * blockDim.x)
    rank[order[r]] = (uint32_t)r;
}

// every (gram position, term): the gram's Java UTF-8 bytes (String.getBytes, an
// unpaired surrogate -> '?') packed big-endian into W words, the byte length in the
// low 16 bits of the last -> numeric order of the words = Text order
__global__ void k_gram_pairs(const int64_t *toff, const uint16_t *tch, int64_t V, int K, int W, const int64_t *goff,
                             const uint32_t *rank, uint64_t *kw, int64_t NP, uint32_t *kord, uint32_t *kterm) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = toff[t], L = toff[t + 1] - b, g0 = goff[t], ng = goff[t + 1] - g0;
    auto unit = [&](int64_t p) -> unsigned {  // position in '$' t '$'
      return (p == 0 || p == L + 1) ? (unsigned)'$' : (unsigned)tch[b + p - 1];
    };
    for (int64_t i = 0; i < ng; i++) {
      const int64_t x = g0 + i;
      uint64_t word = 0;
      int nb = 0, w = 0;
      auto put = [&](unsigned by) {
        word |= (uint64_t)(by & 0xFFu) << (56 - 8 * (nb & 7));
        nb++;
        if ((nb & 7) == 0) {
          kw[(int64_t)w * NP + x] = word;
          w++;
          word = 0;
        }
      };
      for (int j = 0; j < K; j++) {
        const unsigned c = unit(i + j);
        if (c >= 0xD800 && c <= 0xDBFF && j + 1 < K && unit(i + j + 1) >= 0xDC00 && unit(i + j + 1) <= 0xDFFF) {
          const unsigned cp = 0x10000 + ((c - 0xD800) << 10) + (unit(i + j + 1) - 0xDC00);
          put(0xF0 | (cp >> 18));
          put(0x80 | ((cp >> 12) & 0x3F));
          put(0x80 | ((cp >> 6) & 0x3F));
          put(0x80 | (cp & 0x3F));
          j++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
          put('?');
        } else if (c < 0x80) {
          put(c);
        } else if (c < 0x800) {
          put(0xC0 | (c >> 6));
          put(0x80 | (c & 0x3F));
        } else {
          put(0xE0 | (c >> 12));
          put(0x80 | ((c >> 6) & 0x3F));
          put(0x80 | (c & 0x3F));
        }
      }
      const int len = nb;
      for (; w < W; w++) {  // the partial word, zero words, the length
        kw[(int64_t)w * NP + x] = word | (w == W - 1 ? (uint64_t)len : 0ull);
        word = 0;
      }
      kord[x] = rank[t];
      kterm[x] = (uint32_t)t;
    }
  }
}

template <typename T>
__global__ void k_gather(const T *src, const uint32_t *idx, int64_t n, T *dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[idx[i]];
}
__global__ void k_cg_scatter(const uint32_t *idx, const uint32_t *incl, int64_t n, uint32_t *dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[idx[i]] = incl[i] - 1;
}
__global__ void k_iota32(uint32_t *a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}

// sorted pairs (order idx): keep the first of each equal (gram, term), flag gram starts
__global__ void k_cg_flags(const uint64_t *kw, int64_t NP, int W, const uint32_t *kterm, const uint32_t *idx,
                           int64_t n, uint8_t *keep) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t a = idx[i];
    bool k = true;
    if (i > 0) {
      const uint32_t p = idx[i - 1];
      k = !(kterm[a] == kterm[p] && cg_key_eq(kw, NP, W, a, p));
    }
    keep[i] = k ? 1 : 0;
  }
}

__global__ void k_cg_gstart(const uint64_t *kw, int64_t NP, int W, const uint32_t *u, int64_t n, uint32_t *gflag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gflag[i] = (i == 0 || !cg_key_eq(kw, NP, W, u[i], u[i - 1])) ? 1u : 0u;
}
__global__ void k_cg_segs(const uint32_t *gincl, int64_t n, int64_t *gstart) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (i == 0 || gincl[i] != gincl[i - 1]) gstart[gincl[i] - 1] = i;
}

__device__ __forceinline__ uint32_t spread6(int32_t h0) {
  uint32_t h = (uint32_t)h0;
  h ^= (h >> 20) ^ (h >> 12);
  return h ^ (h >> 7) ^ (h >> 4);
}
__device__ __forceinline__ int log2_pow2(int64_t c) { return 63 - __clzll((unsigned long long)c); }
// JDK 6 HashMap capacity after n insertions / at the insertion of element t (0-based)
__device__ __forceinline__ int64_t cap_after(int64_t n) {
  int64_t c = 16;
  while (n > c * 3 / 4) c <<= 1;
  return c;
}

// HashSet iteration rank key of every element: (bucket, chain class, insertion order)
__global__ void k_cg_setkey(const uint32_t *u, const uint32_t *kterm, const uint32_t *gincl, const int64_t *gstart,
                            int64_t ngr, int64_t n, const int32_t *jh, uint64_t *skey) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = gincl[i] - 1;
    const int64_t s0 = gstart[g], s1 = g + 1 < (uint64_t)ngr ? gstart[g + 1] : n;
    const int64_t cnt = s1 - s0, t = i - s0;
    const int64_t C = cap_after(cnt), c = cap_after(t);  // capacity when t was inserted
    const int d = log2_pow2(C) - log2_pow2(c);
    const uint64_t bucket = spread6(jh[kterm[u[i]]]) & (uint32_t)(C - 1);
    const uint64_t cls = (d & 1) ? (uint64_t)(31 - (d - 1) / 2) : (uint64_t)(d / 2);
    const uint64_t tk = (d & 1) ? (uint64_t)t : (uint64_t)((1ll << 26) - 1 - t);
    skey[i] = (bucket << 32) | (cls << 26) | tk;
  }
}

// per gram (in key order): line length, partition (HashPartitioner on Text.hashCode)
__global__ void k_cg_lines(const uint64_t *kw, int64_t NP, int W, const uint32_t *u, const int64_t *gstart,
                           int64_t ngr, int64_t n, const int64_t *elen_scan, int R, int64_t *llen, uint32_t *part) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < ngr; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s0 = gstart[g], s1 = g + 1 < ngr ? gstart[g + 1] : n;
    const uint32_t a = u[s0];
    const int nb = cg_nbytes(kw, NP, W, a);
    int32_t h = 1;
    for (int j = 0; j < nb; j++) h = 31 * h + (int32_t)(int8_t)cg_byte(kw, NP, a, j);
    part[g] = (uint32_t)((h & 0x7fffffff) % R);
    // "gram" '\t' '[' (terms joined by ", ") ']' '\n'
    llen[g] = nb + 4 + (elen_scan[s1] - elen_scan[s0]) - 2;
  }
}

// write the gram prefix of every line, and every element's term + separator
__global__ void k_cg_write_keys(const uint64_t *kw, int64_t NP, int W, const uint32_t *u, const int64_t *gstart,
                                const uint32_t *gorder, int64_t ngr, const int64_t *loff, uint8_t *out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < ngr; r += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = gorder[r];
    const uint32_t a = u[gstart[g]];
    const int nb = cg_nbytes(kw, NP, W, a);
    uint8_t *w = out + loff[r];
    for (int j = 0; j < nb; j++) w[j] = cg_byte(kw, NP, a, j);
    w[nb] = '\t';
    w[nb + 1] = '[';
  }
}
__global__ void k_cg_write_terms(const uint32_t *u, const uint32_t *kterm, const uint32_t *gincl, const int64_t *gstart,
                                 int64_t ngr, int64_t n, const uint32_t *rank_of_g, const int64_t *loff,
                                 const int64_t *elen_scan, const uint64_t *kw, int64_t NP, int W,
                                 const int64_t *toff, const uint16_t *tch, uint8_t *out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t g = gincl[i] - 1;
    const int64_t s0 = gstart[g], s1 = g + 1 < (uint64_t)ngr ? gstart[g + 1] : n;
    const uint32_t a0 = u[s0];
    const int nb = cg_nbytes(kw, NP, W, a0);
    uint8_t *w = out + loff[rank_of_g[g]] + nb + 2 + (elen_scan[i] - elen_scan[s0]);
    const uint32_t t = kterm[u[i]];
    const int64_t b = toff[t];
    const int bl = java_utf8_at(tch + b, (int)(toff[t + 1] - b), w);
    if (i + 1 < s1) {
      w[bl] = ',';
      w[bl + 1] = ' ';
    } else {
      w[bl] = ']';
      w[bl + 1] = '\n';
    }
  }
}
__global__ void k_cg_elen(const uint32_t *u, const uint32_t *kterm, const int32_t *u8len, int64_t n, int64_t *elen) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
    elen[i] = i < n ? (int64_t)u8len[kterm[u[i]]] + 2 : 0;
}
__global__ void k_cg_part_start(const uint32_t *psorted, const int64_t *loff, int64_t ngr, int R, int64_t total,
                                int64_t *pstart) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= ngr; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t cur = r < ngr ? (int64_t)psorted[r] : R;
    const int64_t prev = r > 0 ? (int64_t)psorted[r - 1] : -1;
    for (int64_t p = prev + 1; p <= cur && p <= R; p++) pstart[p] = r < ngr ? loff[r] : total;
  }
}

static int cg_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }
template <typename T>
static T cg_d2h(const T *d, hipStream_t st) {
  T h{};
  SME_HIP(hipMemcpyAsync(&h, d, sizeof(T), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  return h;
}

void chargram_stage(sme_ctx *cx, sme_index *ix, const int32_t *tstream, int64_t M, int64_t V, const int64_t *term_off,
                    const uint16_t *tch, hipStream_t st, Prof *prof) {
  const int K = cx->cfg.k, R = cx->cfg.num_partitions;
  if (K < 1) throw Error(SME_EINVAL, "CharKGramTermIndexer needs k >= 1");
  ix->job = 1;
  auto &W = cx->ws;  // slots 48..63 (query / serializer region) are free during a build
  ix->part_start.assign((size_t)R + 1, 0);
  ix->h_parts.clear();
  ix->h_parts.resize((size_t)R);
  ix->h_parts_ready.assign((size_t)R, 0);
  ix->ser_ready = true;
  if (V == 0) {
    ix->d_ser.get(16);
    ix->cg_ngrams = ix->cg_pairs = 0;
    return;
  }
  // first occurrences -> insertion rank of every term
  unsigned long long *first = W[48].as<unsigned long long>(V);
  SME_HIP(hipMemsetAsync(first, 0xFF, V * sizeof(unsigned long long), st));
  if (M > 0) hipLaunchKernelGGL(k_first_occ, dim3(cg_grid(M)), dim3(256), 0, st, tstream, M, first);
  uint32_t *ti = W[49].as<uint32_t>(V), *order = W[50].as<uint32_t>(V), *rank = W[51].as<uint32_t>(V);
  unsigned long long *first_s = W[52].as<unsigned long long>(V);
  hipLaunchKernelGGL(k_iota32, dim3(cg_grid(V)), dim3(256), 0, st, ti, V);
  // (the hand-written LSD sorts clobber their inputs; none is read afterwards unless copied)
  DevBuf &rs = cx->ws[122];
  sort_pairs<uint64_t>(reinterpret_cast<uint64_t *>(first), reinterpret_cast<uint64_t *>(first_s), ti, order, V, 64,
                       rs, st);
  hipLaunchKernelGGL(k_rank_of, dim3(cg_grid(V)), dim3(256), 0, st, order, V, rank);
  int32_t *jh = W[53].as<int32_t>(V), *u8len = W[54].as<int32_t>(V);
  int64_t *ng = W[55].as<int64_t>(V + 1), *goff = W[56].as<int64_t>(V + 1);
  hipLaunchKernelGGL(k_term_props, dim3(cg_grid(V + 1)), dim3(256), 0, st, term_off, tch, V, K, jh, u8len, ng);
  excl_scan(ng, goff, (int64_t)(V + 1), cx->ws[23], st);
  const int64_t NP = cg_d2h(goff + V, st);
  SME_CHECK_LAUNCH();
  if (prof) prof->mark("cg_terms");
  if (NP == 0) {
    ix->d_ser.get(16);
    ix->cg_ngrams = ix->cg_pairs = 0;
    return;
  }
  if (NP >= (1ll << 31)) throw Error(SME_ELIMIT, "more than 2^31 (gram, term) pairs");
  // (gram, term) pairs sorted by (gram bytes, first occurrence): stable LSD passes,
  // the insertion rank first, then the key words from the last to the first
  const int KW = cg_words(K);
  uint64_t *kw = W[57].as<uint64_t>((size_t)KW * NP);
  uint32_t *kord = W[59].as<uint32_t>(NP), *kterm = W[60].as<uint32_t>(NP);
  hipLaunchKernelGGL(k_gram_pairs, dim3(cg_grid(V)), dim3(256), 0, st, term_off, tch, V, K, KW, goff, rank, kw, NP,
                     kord, kterm);
  // (either buffer ends up holding the permutation, then the gram-start flags: NP + 1)
  uint32_t *ia = W[61].as<uint32_t>(NP + 1), *ib = W[62].as<uint32_t>(NP + 1);
  uint64_t *k64 = W[52].as<uint64_t>(NP), *k64s = W[48].as<uint64_t>(NP);
  uint32_t *k32s = W[49].as<uint32_t>(NP);
  hipLaunchKernelGGL(k_iota32, dim3(cg_grid(NP)), dim3(256), 0, st, ia, NP);
  sort_pairs<uint32_t>(kord, k32s, ia, ib, NP, 32, rs, st);
  for (int w = KW - 1; w >= 0; w--) {  // permutation in ib; each pass: gather the word, sort, back into ib
    hipLaunchKernelGGL(k_gather<uint64_t>, dim3(cg_grid(NP)), dim3(256), 0, st, kw + (int64_t)w * NP, ib, NP, k64);
    sort_pairs<uint64_t>(k64, k64s, ib, ia, NP, 64, rs, st);
    std::swap(ia, ib);
  }
  // dedup equal (gram, term) -> u: pair indices in (gram, insertion) order
  uint8_t *keep = W[63].as<uint8_t>(NP);
  hipLaunchKernelGGL(k_cg_flags, dim3(cg_grid(NP)), dim3(256), 0, st, kw, NP, KW, kterm, ib, NP, keep);
  uint32_t *u = ia;
  int32_t *d_nu = reinterpret_cast<int32_t *>(W[55].as<int64_t>(V + 1));
  int32_t *sel = cx->ws[120].as<int32_t>(NP + 1);
  select_flagged(keep, NP, sel, d_nu, cx->ws[25], cx->ws[23], st);
  const int64_t n = cg_d2h(d_nu, st);
  hipLaunchKernelGGL(k_gather<uint32_t>, dim3(cg_grid(n)), dim3(256), 0, st, ib, reinterpret_cast<const uint32_t *>(sel),
                     n, u);
  // gram segments
  uint32_t *gflag = ib, *gincl = W[50].as<uint32_t>(std::max<int64_t>(NP, V) + 1);
  hipLaunchKernelGGL(k_cg_gstart, dim3(cg_grid(n)), dim3(256), 0, st, kw, NP, KW, u, n, gflag);
  // inclusive sum = the exclusive scan of (flags, 0) shifted by one
  SME_HIP(hipMemsetAsync(gflag + n, 0, sizeof(uint32_t), st));
  excl_scan(gflag, gincl, n + 1, cx->ws[23], st);
  gincl += 1;
  const int64_t ngr = cg_d2h(gincl + n - 1, st);
  int64_t *gstart = W[56].as<int64_t>(std::max<int64_t>(ngr + 1, V + 1));
  hipLaunchKernelGGL(k_cg_segs, dim3(cg_grid(n)), dim3(256), 0, st, gincl, n, gstart);
  if (prof) prof->mark("cg_pairs");
  // HashSet iteration order inside every gram: sort by set key, then stably by gram
  uint64_t *skey = W[52].as<uint64_t>(n), *skey_s = W[48].as<uint64_t>(n);
  hipLaunchKernelGGL(k_cg_setkey, dim3(cg_grid(n)), dim3(256), 0, st, u, kterm, gincl, gstart, ngr, n, jh, skey);
  uint32_t *u2 = ib;
  {  // u is read again below: sort a copy of it
    uint32_t *uc = cx->ws[121].as<uint32_t>(n + 1);
    SME_HIP(hipMemcpyAsync(uc, u, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    sort_pairs<uint64_t>(skey, skey_s, uc, u2, n, 64, rs, st);
  }
  uint32_t *g_of = W[59].as<uint32_t>(n), *g_of_s = W[49].as<uint32_t>(n);
  // gram of each element of u2: gincl is by position in u -> scatter by pair index, gather by u2
  {
    uint32_t *gid_by_pair = W[51].as<uint32_t>(NP);
    hipLaunchKernelGGL(k_cg_scatter, dim3(cg_grid(n)), dim3(256), 0, st, u, gincl, n, gid_by_pair);
    hipLaunchKernelGGL(k_gather<uint32_t>, dim3(cg_grid(n)), dim3(256), 0, st, gid_by_pair, u2, n, g_of);
  }
  uint32_t *u3 = W[61].as<uint32_t>(n);
  sort_pairs<uint32_t>(g_of, g_of_s, u2, u3, n, 32, rs, st);
  // u3: elements in (gram key, HashSet order); gincl / gstart still describe the segments
  if (prof) prof->mark("cg_sets");
  // line lengths, partitions, offsets
  int64_t *elen = W[53].as<int64_t>(n + 1), *escan = W[54].as<int64_t>(n + 1);
  hipLaunchKernelGGL(k_cg_elen, dim3(cg_grid(n + 1)), dim3(256), 0, st, u3, kterm, u8len, n, elen);
  excl_scan(elen, escan, (int64_t)(n + 1), cx->ws[23], st);
  // kw/kterm (slots 57, 60) stay live until the lines are written
  DevBuf b_llen, b_loff, b_part;
  int64_t *llen = b_llen.as<int64_t>(ngr + 1), *loff = b_loff.as<int64_t>(ngr + 1);
  uint32_t *part = b_part.as<uint32_t>(ngr + 1), *part_s = W[62].as<uint32_t>(ngr + 1);
  hipLaunchKernelGGL(k_cg_lines, dim3(cg_grid(ngr)), dim3(256), 0, st, kw, NP, KW, u3, gstart, ngr, n, escan, R, llen,
                     part);
  uint32_t *gseq = W[51].as<uint32_t>(ngr + 1), *gorder = W[63].as<uint32_t>(ngr + 1);
  hipLaunchKernelGGL(k_iota32, dim3(cg_grid(ngr)), dim3(256), 0, st, gseq, ngr);
  sort_pairs<uint32_t>(part, part_s, gseq, gorder, ngr, 32, rs, st);
  int64_t *llen_s = W[52].as<int64_t>(ngr + 1);
  hipLaunchKernelGGL(k_gather<int64_t>, dim3(cg_grid(ngr)), dim3(256), 0, st, llen, gorder, ngr, llen_s);
  SME_HIP(hipMemsetAsync(llen_s + ngr, 0, sizeof(int64_t), st));
  excl_scan(llen_s, loff, (int64_t)(ngr + 1), cx->ws[23], st);
  const int64_t total = cg_d2h(loff + ngr, st);
  uint32_t *rank_of_g = W[51].as<uint32_t>(ngr + 1);  // gseq no longer needed
  hipLaunchKernelGGL(k_rank_of, dim3(cg_grid(ngr)), dim3(256), 0, st, gorder, ngr, rank_of_g);
  uint8_t *out = ix->d_ser.as<uint8_t>(total + 16);
  hipLaunchKernelGGL(k_cg_write_keys, dim3(cg_grid(ngr)), dim3(256), 0, st, kw, NP, KW, u3, gstart, gorder, ngr, loff,
                     out);
  hipLaunchKernelGGL(k_cg_write_terms, dim3(cg_grid(n)), dim3(256), 0, st, u3, kterm, gincl, gstart, ngr, n, rank_of_g,
                     loff, escan, kw, NP, KW, term_off, tch, out);
  int64_t *pstart = W[53].as<int64_t>((size_t)R + 1);
  hipLaunchKernelGGL(k_cg_part_start, dim3(cg_grid(ngr + 1)), dim3(256), 0, st, part_s, loff, ngr, R, total, pstart);
  SME_CHECK_LAUNCH();
  SME_HIP(hipMemcpyAsync(ix->part_start.data(), pstart, ((size_t)R + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  ix->cg_ngrams = ngr;
  ix->cg_pairs = n;
  if (prof) prof->mark("cg_output");
}

}  // namespace sme
