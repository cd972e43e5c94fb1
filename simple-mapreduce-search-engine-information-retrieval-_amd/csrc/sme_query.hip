// sme_query.hip -- batched rank() (IntDocVectorsForwardIndex.rank, C/sa/edu/kaust/fwindex/
// IntDocVectorsForwardIndex.java:192-223), query-string tokenization
// (GalagoTokenizer.processContent on the REPL line, :292-295) and term lookup
// (getValue's forward-index lookup, :148-184).
//
// Scoring semantics: for each query token in order (unknown ones skipped,
// duplicates twice), for each posting of that term, score[d] += w where
// w = (1 + ln tf) * idf was precomputed in fp64 by the build's weight pass.
// A document's score is therefore the left-to-right fp64 sum of its weights in
// query-token order, exactly as the JVM accumulates `score.score += ...`.
// Output order: score desc, docno asc (north-star tie-break; equals the
// reference's stable Collections.sort for single-term queries).
//
// Kernel shape: one 256-lane workgroup per query, sweeping the docno axis in
// tiles of kTile documents whose fp64 accumulators live in LDS (32 KiB, so four
// workgroups share a CU).  Postings are docno-sorted per term; for each tile the
// workgroup streams every query term's postings that fall in it, 1024 per step
// (4 per lane, coalesced), in query-token order -- one barrier per step, and
// postings of one term have distinct docnos, so a document's adds happen in
// token order and the fp64 sum is the reference's.  The weight of a posting is
// lut[tf] * idf[term] (fp64, no contraction: bit-identical to the build's
// TF-IDF pass), so a posting costs 8 bytes of HBM (docno, tf), not 12.  Each
// lane keeps its best KMAX (score, docno) in registers; the lists are merged by
// k rounds of block arg-max at the end.
#include <hip/hip_runtime.h>
#include <math.h>

#include "sme_internal.hpp"
#include "sme_text.hpp"

namespace sme {

constexpr int kQNT = 256;
constexpr int kTile = 4096;
constexpr int kQPer = 4;  // postings per lane per step
constexpr int kMaxQTerms = 128;
constexpr int kLutLds = 256;  // 1 + ln(tf) for tf < 256 from LDS, the rare rest from HBM

__device__ __forceinline__ bool better(double as, int32_t ad, double bs, int32_t bd) {
  return as > bs || (as == bs && ad < bd);
}

// insert (s, d) into the descending register list ts/td (fully unrolled: no
// dynamic register indexing)
template <int K>
__device__ __forceinline__ void topk_insert(double (&ts)[K], int32_t (&td)[K], double s, int32_t d) {
  if (!better(s, d, ts[K - 1], td[K - 1])) return;
  bool done = false;
#pragma unroll
  for (int i = K - 1; i >= 1; i--) {
    if (!done) {
      if (better(s, d, ts[i - 1], td[i - 1])) {
        ts[i] = ts[i - 1];
        td[i] = td[i - 1];
      } else {
        ts[i] = s;
        td[i] = d;
        done = true;
      }
    }
  }
  if (!done) {
    ts[0] = s;
    td[0] = d;
  }
}

template <int KMAX>
__global__ __launch_bounds__(kQNT) void k_query(const int64_t *__restrict__ off, const int32_t *__restrict__ docno,
                                                const int32_t *__restrict__ tf, const double *__restrict__ lut,
                                                int max_tf, const double *__restrict__ idf,
                                                const int32_t *__restrict__ terms, const int64_t *__restrict__ qoff,
                                                int nq, int k, int32_t *out_d, double *out_s, int *err) {
  __shared__ double acc[kTile];
  __shared__ double s_lut[kLutLds];
  __shared__ int64_t cur[kMaxQTerms], endp[kMaxQTerms];
  __shared__ double tidf[kMaxQTerms];
  __shared__ int32_t s_next;
  __shared__ unsigned long long s_stop;
  __shared__ double red_s[kQNT / 64];
  __shared__ int32_t red_d[kQNT / 64], red_t[kQNT / 64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int j = tid; j < kTile; j += kQNT) acc[j] = -1.0;  // untouched (weights are >= 0)
  for (int j = tid; j < kLutLds; j += kQNT) s_lut[j] = j <= max_tf ? lut[j] : 0.0;
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int64_t q0 = qoff[q];
    int nt = (int)(qoff[q + 1] - q0);
    if (nt > kMaxQTerms) {
      if (tid == 0) atomicOr(err, 1);
      nt = kMaxQTerms;
    }
    if (tid == 0) s_next = 0x7FFFFFFF;
    __syncthreads();
    for (int i = tid; i < nt; i += kQNT) {
      const int32_t t = terms[q0 + i];
      const int64_t b = t >= 0 ? off[t] : 0, e = t >= 0 ? off[t + 1] : 0;
      cur[i] = b;
      endp[i] = e;
      tidf[i] = t >= 0 ? idf[t] : 0.0;
      if (b < e) atomicMin(&s_next, docno[b]);
    }
    double ts[KMAX];
    int32_t td[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; j++) {
      ts[j] = -INFINITY;
      td[j] = 0x7FFFFFFF;
    }
    __syncthreads();
    while (s_next != 0x7FFFFFFF) {  // uniform: read after a barrier
      const int32_t lo = s_next;
      const int64_t hi = (int64_t)lo + kTile;
      __syncthreads();
      if (tid == 0) s_next = 0x7FFFFFFF;
      for (int i = 0; i < nt; i++) {
        const int64_t c = cur[i], e = endp[i];
        if (c >= e) continue;  // uniform
        const double w_idf = tidf[i];
        if (tid == 0) s_stop = (unsigned long long)e;
        __syncthreads();
        // Each lane walks its stride of the term's postings until the first docno
        // >= hi; the smallest stop over lanes is the term's first posting beyond
        // the tile, and the docno there is that term's next docno.
        int64_t p = c + tid;
        int32_t dstop = 0x7FFFFFFF;
        for (;;) {
          int32_t dv[kQPer], fv[kQPer];
#pragma unroll
          for (int u = 0; u < kQPer; u++) {
            const int64_t pu = p + (int64_t)u * kQNT;
            dv[u] = pu < e ? docno[pu] : 0x7FFFFFFF;
            fv[u] = pu < e ? tf[pu] : 0;
          }
          bool stop = false;
#pragma unroll
          for (int u = 0; u < kQPer; u++) {
            if (stop) continue;
            if ((int64_t)dv[u] >= hi || p + (int64_t)u * kQNT >= e) {
              stop = true;
              p += (int64_t)u * kQNT;
              dstop = p < e ? dv[u] : 0x7FFFFFFF;
              continue;
            }
            const int d = dv[u] - lo;
            const double l = fv[u] < kLutLds ? s_lut[fv[u]] : lut[fv[u]];
            const double w = __dmul_rn(l, w_idf);
            const double v = acc[d];
            acc[d] = v < 0.0 ? w : __dadd_rn(v, w);
          }
          if (stop) break;
          p += (int64_t)kQPer * kQNT;
        }
        // wave minima first: one LDS atomic per wave, not per lane
        unsigned long long pm = (unsigned long long)p;
        int32_t dm = dstop;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long po = __shfl_xor(pm, o, 64);
          const int32_t dd = __shfl_xor(dm, o, 64);
          pm = po < pm ? po : pm;
          dm = dd < dm ? dd : dm;
        }
        if (lane == 0) {
          atomicMin(&s_stop, pm);
          if (dm != 0x7FFFFFFF) atomicMin(&s_next, dm);
        }
        __syncthreads();  // also orders this term's adds before the next term's
        if (tid == 0) cur[i] = (int64_t)s_stop;
      }
      __syncthreads();
      for (int j = tid; j < kTile; j += kQNT) {
        const double sc = acc[j];
        if (sc < 0.0) continue;
        acc[j] = -1.0;
        topk_insert<KMAX>(ts, td, sc, lo + j);
      }
      __syncthreads();
    }
    // merge the per-lane lists: k rounds of block arg-max over list heads
    for (int r = 0; r < k; r++) {
      double bs = ts[0];
      int32_t bd = td[0];
      int32_t bt = tid;
      for (int o = 32; o > 0; o >>= 1) {
        double os = __shfl_xor(bs, o, 64);
        int32_t od = __shfl_xor(bd, o, 64), ot = __shfl_xor(bt, o, 64);
        if (better(os, od, bs, bd)) {
          bs = os;
          bd = od;
          bt = ot;
        }
      }
      if (lane == 0) {
        red_s[wave] = bs;
        red_d[wave] = bd;
        red_t[wave] = bt;
      }
      __syncthreads();
      bs = red_s[0];
      bd = red_d[0];
      bt = red_t[0];
      for (int x = 1; x < kQNT / 64; x++)
        if (better(red_s[x], red_d[x], bs, bd)) {
          bs = red_s[x];
          bd = red_d[x];
          bt = red_t[x];
        }
      if (tid == bt) {  // pop the head: shift the winner's list left
#pragma unroll
        for (int j = 0; j < KMAX - 1; j++) {
          ts[j] = ts[j + 1];
          td[j] = td[j + 1];
        }
        ts[KMAX - 1] = -INFINITY;
        td[KMAX - 1] = 0x7FFFFFFF;
      }
      if (tid == 0) {
        const bool valid = bs != -INFINITY;
        out_d[(int64_t)q * k + r] = valid ? bd : -1;
        out_s[(int64_t)q * k + r] = valid ? bs : 0.0;
      }
      __syncthreads();
    }
  }
}

void query_topk(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k, int32_t *d_out_docno,
                double *d_out_score, hipStream_t st) {
  if (k < 1) throw Error(SME_EINVAL, "k must be >= 1");
  if (nq <= 0) return;
  int *err = ix->ctx->ws[63].as<int>(4);
  SME_HIP(hipMemsetAsync(err, 0, sizeof(int), st));
  const int64_t *off = (const int64_t *)ix->d_off.p;
  const int32_t *dn = (const int32_t *)ix->d_docno_d.p;
  const int32_t *tf = (const int32_t *)ix->d_tf_d.p;
  const double *lut = (const double *)ix->d_lut.p;
  const double *idf = (const double *)ix->d_idf.p;
  unsigned grid = (unsigned)std::min(nq, 1 << 20);
  // events on the launch stream bracket the scoring kernel (bench.py roofline)
  hipEvent_t e0, e1;
  SME_HIP(hipEventCreate(&e0));
  SME_HIP(hipEventCreate(&e1));
  SME_HIP(hipEventRecord(e0, st));
  if (k <= 16) {
    hipLaunchKernelGGL(k_query<16>, dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, d_terms, d_qoff, nq, k,
                       d_out_docno, d_out_score, err);
  } else if (k <= 32) {
    hipLaunchKernelGGL(k_query<32>, dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, d_terms, d_qoff, nq, k,
                       d_out_docno, d_out_score, err);
  } else {
    throw Error(SME_ENOTIMPL, "top-k with k > 32 is not built yet");
  }
  SME_CHECK_LAUNCH();
  SME_HIP(hipEventRecord(e1, st));
  int h_err = 0;
  SME_HIP(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  float ms = 0;
  SME_HIP(hipEventElapsedTime(&ms, e0, e1));
  ix->ctx->last_query_ms = ms;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (h_err) throw Error(SME_ELIMIT, "a query has more than 128 terms");
}

// ---------------------------------------------------------------------------
// processContent on one string (query parsing), single lane
// ---------------------------------------------------------------------------
__global__ void k_tokenize_one(const uint8_t *b, int64_t n, uint16_t *units, uint16_t *work, int64_t work_cap,
                               uint16_t *out, int64_t out_cap, int64_t *offs, int cap_tok, int *ntok, int *err) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t nu = 0;
  for (int64_t p = 0; p < n;) {
    uint16_t tmp[2];
    int k;
    int used = utf8_step(b, p, n, tmp, &k);
    for (int x = 0; x < k; x++) units[nu++] = tmp[x];
    p += used;
  }
  int cnt = 0;
  int64_t o = 0;
  offs[0] = 0;
  TagScan sc;
  sc.t = units;
  sc.n = (int)nu;
  Stemmer stm;
  sc.run([&](int u0, int u1) {
    normalize_raw(units + u0, u1 - u0, work, (int)work_cap, [&](const uint16_t *p, int l) {
      if (is_stopword(p, l)) return;
      for (int i = 0; i < l; i++) stm.b[i] = p[i];
      stm.len = l;
      stm.run();
      if (cnt >= cap_tok || o + stm.len > out_cap) {
        *err = 1;
        return;
      }
      for (int i = 0; i < stm.len; i++) out[o + i] = stm.b[i];
      o += stm.len;
      offs[++cnt] = o;
    });
  });
  *ntok = cnt;
}

void tokenize_string(sme_ctx *cx, const uint8_t *h_utf8, size_t n, std::vector<std::vector<uint16_t>> &out,
                     hipStream_t st) {
  auto &W = cx->ws;
  const int64_t cap_tok = (int64_t)n + 4;
  uint8_t *d_b = W[48].as<uint8_t>(n + 1);
  uint16_t *units = W[49].as<uint16_t>(n + 4);
  uint16_t *work = W[50].as<uint16_t>(4 * n + 64);
  uint16_t *tokbuf = W[51].as<uint16_t>(2 * n + 16);
  int64_t *offs = W[52].as<int64_t>(cap_tok + 1);
  int *cnt = W[53].as<int>(4);
  if (n) SME_HIP(hipMemcpyAsync(d_b, h_utf8, n, hipMemcpyHostToDevice, st));
  SME_HIP(hipMemsetAsync(cnt, 0, 4 * sizeof(int), st));
  hipLaunchKernelGGL(k_tokenize_one, dim3(1), dim3(64), 0, st, d_b, (int64_t)n, units, work, (int64_t)(4 * n + 64),
                     tokbuf, (int64_t)(2 * n + 16), offs, (int)cap_tok, cnt, cnt + 1);
  SME_CHECK_LAUNCH();
  int h[2];
  SME_HIP(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h[1]) throw Error(SME_ELIMIT, "tokenize output capacity");
  std::vector<int64_t> ho(h[0] + 1);
  SME_HIP(hipMemcpy(ho.data(), offs, ho.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<uint16_t> hb(ho.back());
  if (!hb.empty()) SME_HIP(hipMemcpy(hb.data(), tokbuf, hb.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
  out.clear();
  for (int i = 0; i < h[0]; i++) out.emplace_back(hb.begin() + ho[i], hb.begin() + ho[i + 1]);
}

// ---------------------------------------------------------------------------
// term lookup: binary search over the rank-ordered vocabulary
// ---------------------------------------------------------------------------
__global__ void k_lookup(const int64_t *toff, const uint16_t *tchars, int64_t V, const int64_t *qo,
                         const uint16_t *qc, int n, int32_t *ids) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint16_t *a = qc + qo[i];
    const int64_t al = qo[i + 1] - qo[i];
    int64_t lo = 0, hi = V - 1, res = -1;
    while (lo <= hi) {
      int64_t mid = (lo + hi) >> 1;
      const uint16_t *b = tchars + toff[mid];
      int64_t bl = toff[mid + 1] - toff[mid], m = al < bl ? al : bl;
      int c = 0;
      for (int64_t x = 0; x < m && c == 0; x++) c = (int)b[x] - (int)a[x];
      if (c == 0) c = (int)(bl - al);
      if (c == 0) {
        res = mid;
        break;
      }
      if (c < 0)
        lo = mid + 1;
      else
        hi = mid - 1;
    }
    ids[i] = (int32_t)res;
  }
}

// K > 1: the forward index is keyed by k_gram[0] and its Hashtable keeps the
// LAST k-gram (TermDF order) with that first element (IntDocVectorsForwardIndex
// .java:107-120, T11): the last gram whose first component is the term id.
__global__ void k_gram_last(const int32_t *gram, int64_t V, int K, int n, int32_t *ids) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int32_t t = ids[i];
    if (t < 0) continue;
    int64_t lo = 0, hi = V;  // first gram with first component > t
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (gram[m * K] <= t)
        lo = m + 1;
      else
        hi = m;
    }
    ids[i] = (lo > 0 && gram[(lo - 1) * K] == t) ? (int32_t)(lo - 1) : -1;
  }
}

void lookup_terms(sme_index *ix, const std::vector<std::vector<uint16_t>> &terms, int32_t *ids, hipStream_t st) {
  const int n = (int)terms.size();
  if (n == 0) return;
  std::vector<int64_t> qo(n + 1, 0);
  for (int i = 0; i < n; i++) qo[i + 1] = qo[i] + (int64_t)terms[i].size();
  std::vector<uint16_t> qc(qo[n] + 1);
  for (int i = 0; i < n; i++) std::copy(terms[i].begin(), terms[i].end(), qc.begin() + qo[i]);
  auto &W = ix->ctx->ws;
  int64_t *d_qo = W[54].as<int64_t>(n + 1);
  uint16_t *d_qc = W[48].as<uint16_t>(qc.size());
  int32_t *d_ids = W[49].as<int32_t>(n);
  SME_HIP(hipMemcpyAsync(d_qo, qo.data(), qo.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_qc, qc.data(), qc.size() * sizeof(uint16_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_lookup, dim3((n + 255) / 256), dim3(256), 0, st, (const int64_t *)ix->d_term_off.p,
                     (const uint16_t *)ix->d_term_chars.p, ix->Vt, d_qo, d_qc, n, d_ids);
  if (ix->K > 1)
    hipLaunchKernelGGL(k_gram_last, dim3((n + 255) / 256), dim3(256), 0, st, (const int32_t *)ix->d_gram.p, ix->V,
                       ix->K, n, d_ids);
  SME_CHECK_LAUNCH();
  SME_HIP(hipMemcpyAsync(ids, d_ids, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
}

}  // namespace sme
