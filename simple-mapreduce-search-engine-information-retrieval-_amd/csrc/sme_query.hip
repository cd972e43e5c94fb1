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
// Kernel shape: one 256-lane workgroup per query.  Postings are docno-sorted
// per term, so the workgroup sweeps the docno axis in tiles of kTile docs held
// as an fp64 accumulator in LDS; for each tile it streams every query term's
// postings that fall in the tile (coalesced, 256 at a time, the block barrier
// of __syncthreads_count separates terms so the add order per doc is the
// query-token order).  Touched accumulator entries feed a per-lane top-k list
// in LDS; the lists are merged by k rounds of block arg-max.
#include <hip/hip_runtime.h>
#include <math.h>

#include "sme_internal.hpp"
#include "sme_text.hpp"

namespace sme {

constexpr int kQNT = 256;
constexpr int kTile = 4096;
constexpr int kMaxQTerms = 128;

__device__ __forceinline__ bool better(double as, int32_t ad, double bs, int32_t bd) {
  return as > bs || (as == bs && ad < bd);
}

template <int KMAX>
__global__ __launch_bounds__(kQNT) void k_query(const int64_t *__restrict__ off, const int32_t *__restrict__ docno,
                                                const double *__restrict__ w, const int32_t *__restrict__ terms,
                                                const int64_t *__restrict__ qoff, int nq, int k, int32_t *out_d,
                                                double *out_s, int *err) {
  __shared__ double acc[kTile];
  __shared__ double topS[KMAX * kQNT];
  __shared__ int32_t topD[KMAX * kQNT];
  __shared__ int64_t cur[kMaxQTerms], endp[kMaxQTerms];
  __shared__ int32_t s_lo;
  __shared__ double red_s[kQNT / 64];
  __shared__ int32_t red_d[kQNT / 64], red_t[kQNT / 64];
  const int tid = threadIdx.x;
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int64_t q0 = qoff[q];
    int nt = (int)(qoff[q + 1] - q0);
    if (nt > kMaxQTerms) {
      if (tid == 0) atomicOr(err, 1);
      nt = kMaxQTerms;
    }
    for (int i = tid; i < nt; i += kQNT) {
      int32_t t = terms[q0 + i];
      cur[i] = t >= 0 ? off[t] : 0;
      endp[i] = t >= 0 ? off[t + 1] : 0;
    }
    for (int j = 0; j < KMAX; j++) {
      topS[j * kQNT + tid] = -INFINITY;
      topD[j * kQNT + tid] = 0x7FFFFFFF;
    }
    __syncthreads();
    for (;;) {
      // next tile starts at the smallest unprocessed docno of any term
      if (tid == 0) s_lo = 0x7FFFFFFF;
      __syncthreads();
      bool any = false;
      for (int i = tid; i < nt; i += kQNT)
        if (cur[i] < endp[i]) {
          atomicMin(&s_lo, docno[cur[i]]);
          any = true;
        }
      if (__syncthreads_count(any) == 0) break;
      const int32_t lo = s_lo;
      const int64_t hi = (int64_t)lo + kTile;
      for (int j = tid; j < kTile; j += kQNT) acc[j] = -1.0;  // untouched (weights are >= 0)
      __syncthreads();
      for (int i = 0; i < nt; i++) {
        int64_t c = cur[i];
        const int64_t e = endp[i];
        for (;;) {
          const int64_t p = c + tid;
          bool in = p < e && (int64_t)docno[p] < hi;
          int n_in = __syncthreads_count(in);
          if (in) {
            const int d = docno[p] - lo;
            const double v = acc[d];
            acc[d] = v < 0.0 ? w[p] : v + w[p];
          }
          c += n_in;
          if (n_in < kQNT) break;
        }
        if (tid == 0) cur[i] = c;
      }
      __syncthreads();
      for (int j = tid; j < kTile; j += kQNT) {
        const double sc = acc[j];
        if (sc < 0.0) continue;
        const int32_t dn = lo + j;
        const int last = (k - 1) * kQNT + tid;
        if (!better(sc, dn, topS[last], topD[last])) continue;
        int pos = k - 1;
        while (pos > 0 && better(sc, dn, topS[(pos - 1) * kQNT + tid], topD[(pos - 1) * kQNT + tid])) {
          topS[pos * kQNT + tid] = topS[(pos - 1) * kQNT + tid];
          topD[pos * kQNT + tid] = topD[(pos - 1) * kQNT + tid];
          pos--;
        }
        topS[pos * kQNT + tid] = sc;
        topD[pos * kQNT + tid] = dn;
      }
      __syncthreads();
    }
    // merge the per-lane lists: k rounds of block arg-max over list heads
    int head = 0;
    for (int r = 0; r < k; r++) {
      double bs = head < k ? topS[head * kQNT + tid] : -INFINITY;
      int32_t bd = head < k ? topD[head * kQNT + tid] : 0x7FFFFFFF;
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
      if ((tid & 63) == 0) {
        red_s[tid >> 6] = bs;
        red_d[tid >> 6] = bd;
        red_t[tid >> 6] = bt;
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
      if (tid == bt) head++;
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
  const double *w = (const double *)ix->d_w.p;
  unsigned grid = (unsigned)std::min(nq, 65536);
  if (k <= 16) {
    hipLaunchKernelGGL(k_query<16>, dim3(grid), dim3(kQNT), 0, st, off, dn, w, d_terms, d_qoff, nq, k, d_out_docno,
                       d_out_score, err);
  } else if (k <= 32) {
    hipLaunchKernelGGL(k_query<32>, dim3(grid), dim3(kQNT), 0, st, off, dn, w, d_terms, d_qoff, nq, k, d_out_docno,
                       d_out_score, err);
  } else {
    throw Error(SME_ENOTIMPL, "top-k with k > 32 is not built yet");
  }
  SME_CHECK_LAUNCH();
  int h_err = 0;
  SME_HIP(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
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
                     (const uint16_t *)ix->d_term_chars.p, ix->V, d_qo, d_qc, n, d_ids);
  SME_CHECK_LAUNCH();
  SME_HIP(hipMemcpyAsync(ids, d_ids, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
}

}  // namespace sme
