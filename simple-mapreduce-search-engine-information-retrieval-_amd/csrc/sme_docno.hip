// sme_docno.hip -- docno assignment (NumberTrecDocuments):
//
//   map      docid of every record (TrecDocument.getDocid), as Text (UTF-8)
//            C/edu/umd/cloud9/collection/trec/NumberTrecDocuments.java:82-95
//   shuffle  [Hadoop] Text keys sorted by their UTF-8 bytes (unsigned, shorter
//            prefix first), one reducer
//   reduce   distinct docids numbered 1.. in that order            :97-107
//   write    TrecDocnoMapping.writeDocnoData: int32 N, N x writeUTF(docid)
//            C/edu/umd/cloud9/collection/trec/TrecDocnoMapping.java:92-125
//
// Device: record split (shared with the index build), docid spans, re-encoding
// of each docid as Text.set(String) would (UTF-8 with U+FFFD for malformed
// input), an LSD radix sort over 8-byte big-endian words (length first, so a
// proper prefix sorts first), adjacent-distinct compaction.  Host: the
// writeUTF (modified UTF-8) framing of the distinct docids.
//
// Parity note: a docid containing '\t', '\r' or '\n' is split by the
// reference's text round trip (split("\\t")[0] per line); this path keeps the
// docid whole.  Such docids are "parity unpinned".
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sme_internal.hpp"
#include "sme_text.hpp"
#include "sme_trec.hpp"

namespace sme {

__device__ __forceinline__ int utf8_put(uint32_t cp, uint8_t *o) {
  if (cp < 0x80) {
    if (o) o[0] = (uint8_t)cp;
    return 1;
  }
  if (cp < 0x800) {
    if (o) {
      o[0] = (uint8_t)(0xC0 | (cp >> 6));
      o[1] = (uint8_t)(0x80 | (cp & 0x3F));
    }
    return 2;
  }
  if (cp < 0x10000) {
    if (o) {
      o[0] = (uint8_t)(0xE0 | (cp >> 12));
      o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      o[2] = (uint8_t)(0x80 | (cp & 0x3F));
    }
    return 3;
  }
  if (o) {
    o[0] = (uint8_t)(0xF0 | (cp >> 18));
    o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
    o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
    o[3] = (uint8_t)(0x80 | (cp & 0x3F));
  }
  return 4;
}

// decode [b, e) as Text.toString (replacement per maximal ill-formed subpart),
// re-encode as UTF-8; returns the length, writes when o != nullptr
__device__ int64_t docid_text(const uint8_t *t, int64_t b, int64_t e, uint8_t *o) {
  int64_t len = 0;
  for (int64_t p = b; p < e;) {
    uint16_t u[2];
    int k;
    const int used = utf8_step(t, p, e, u, &k);
    uint32_t cp = u[0];
    if (k == 2) cp = 0x10000 + (((uint32_t)u[0] - 0xD800) << 10) + ((uint32_t)u[1] - 0xDC00);
    len += utf8_put(cp, o ? o + len : nullptr);
    p += used;
  }
  return len;
}

__global__ void k_docid_len(const uint8_t *t, const uint64_t *rs, const uint64_t *re, int64_t nR, int64_t *ib_,
                            int64_t *ie_, int64_t *len, unsigned long long *err) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t ib, ie;
    if (!docid_span(t, (int64_t)rs[r], (int64_t)re[r], &ib, &ie)) {
      atomicAdd(err, 1ull);
      ib = ie = 0;
    }
    ib_[r] = ib;
    ie_[r] = ie;
    len[r] = docid_text(t, ib, ie, nullptr);
  }
}

__global__ void k_docid_write(const uint8_t *t, const int64_t *ib, const int64_t *ie, const int64_t *off, int64_t nR,
                              uint8_t *out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nR; r += (int64_t)gridDim.x * blockDim.x)
    docid_text(t, ib[r], ie[r], out + off[r]);
}

// sort key of record order[i]: length (pass 0) or big-endian bytes [8w, 8w + 8)
__global__ void k_docid_word(const uint32_t *order, int64_t nR, const uint8_t *ids, const int64_t *off, int w,
                             uint64_t *key) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = order[i];
    const int64_t b = off[r], l = off[r + 1] - off[r];
    if (w < 0) {
      key[i] = (uint64_t)l;
      continue;
    }
    uint64_t k = 0;
    for (int j = 0; j < 8; j++) {
      const int64_t x = 8 * (int64_t)w + j;
      k = (k << 8) | (x < l ? ids[b + x] : 0u);
    }
    key[i] = k;
  }
}

__global__ void k_docid_distinct(const uint32_t *order, int64_t nR, const uint8_t *ids, const int64_t *off,
                                 uint32_t *flag) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nR; i += (int64_t)gridDim.x * blockDim.x) {
    if (i == 0) {
      flag[i] = 1;
      continue;
    }
    const uint32_t a = order[i - 1], b = order[i];
    const int64_t la = off[a + 1] - off[a], lb = off[b + 1] - off[b];
    bool same = la == lb;
    for (int64_t x = 0; same && x < la; x++) same = ids[off[a] + x] == ids[off[b] + x];
    flag[i] = same ? 0u : 1u;
  }
}

static int bits_of(uint64_t v) {
  int b = 1;
  while (b < 64 && (1ull << b) <= v) b++;
  return b;
}

void number_documents(sme_ctx *cx, const uint8_t *t, uint64_t n, hipStream_t st, std::vector<uint8_t> &out) {
  const RecordSpans rsp = find_records(cx, t, n, st, nullptr);
  const int64_t nR = rsp.nR;
  auto &W = cx->ws;  // 48..63: transient per call
  auto cub_tmp = [&](size_t bytes) { return cx->cub_tmp.get(bytes); };
  unsigned long long *err = W[48].as<unsigned long long>(2);
  SME_HIP(hipMemsetAsync(err, 0, sizeof(unsigned long long), st));
  int64_t *ib = W[49].as<int64_t>(nR + 1), *ie = W[50].as<int64_t>(nR + 1);
  int64_t *len = W[51].as<int64_t>(nR + 1), *off = W[52].as<int64_t>(nR + 1);
  auto grid = [](int64_t m) { return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 8192))); };
  if (nR > 0) hipLaunchKernelGGL(k_docid_len, grid(nR), dim3(256), 0, st, t, rsp.rs, rsp.re, nR, ib, ie, len, err);
  SME_HIP(hipMemsetAsync(len + nR, 0, sizeof(int64_t), st));
  size_t tb = 0;
  excl_scan(len, off, (int64_t)(nR + 1), cx->ws[23], st);
  int64_t h2[1];
  unsigned long long h_err = 0;
  SME_HIP(hipMemcpyAsync(h2, off + nR, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipMemcpyAsync(&h_err, err, sizeof h_err, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h_err) throw Error(SME_EPARSE, "a record has <DOCNO> but no </DOCNO> (TrecDocument.getDocid throws)");
  const int64_t tot = h2[0];
  uint8_t *ids = W[53].as<uint8_t>(tot + 8);
  if (nR > 0) hipLaunchKernelGGL(k_docid_write, grid(nR), dim3(256), 0, st, t, ib, ie, off, nR, ids);
  // longest docid -> number of 8-byte words
  int64_t maxlen = 0;
  if (nR > 0) {
    int64_t *mx = W[54].as<int64_t>(1);
    reduce_max<int64_t>(len, nR, mx, st);
    SME_HIP(hipMemcpyAsync(&maxlen, mx, sizeof maxlen, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
  }
  // LSD: length, then words from the last to the first (stable)
  uint32_t *oa = W[55].as<uint32_t>(nR + 1), *ob = W[56].as<uint32_t>(nR + 1);
  uint64_t *ka = W[57].as<uint64_t>(nR + 1), *kb = W[58].as<uint64_t>(nR + 1);
  std::vector<uint32_t> iota(nR);
  for (int64_t i = 0; i < nR; i++) iota[i] = (uint32_t)i;
  if (nR > 0) SME_HIP(hipMemcpyAsync(oa, iota.data(), nR * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  const int nwords = (int)((maxlen + 7) / 8);
  uint32_t *rscr = W[60].as<uint32_t>(kv_sort_scratch(nR) / sizeof(uint32_t) + 1);
  for (int w = -1; w < nwords && nR > 1; w++) {
    const int pw = w < 0 ? -1 : nwords - 1 - w;  // after the length pass: last word first
    hipLaunchKernelGGL(k_docid_word, grid(nR), dim3(256), 0, st, oa, nR, ids, off, pw, ka);
    const int bits = pw < 0 ? bits_of((uint64_t)maxlen) : 64;
    if (kv_sort<uint64_t>(ka, oa, kb, ob, nR, bits, rscr, st) != oa) std::swap(oa, ob);
  }
  uint32_t *flag = W[59].as<uint32_t>(nR + 1);
  if (nR > 0) hipLaunchKernelGGL(k_docid_distinct, grid(nR), dim3(256), 0, st, oa, nR, ids, off, flag);
  SME_CHECK_LAUNCH();
  // host: the distinct docids in order, framed as writeDocnoData writes them
  std::vector<uint32_t> h_order(nR), h_flag(nR);
  std::vector<int64_t> h_off(nR + 1);
  std::vector<uint8_t> h_ids(tot + 1);
  if (nR > 0) {
    SME_HIP(hipMemcpyAsync(h_order.data(), oa, nR * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(h_flag.data(), flag, nR * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  }
  SME_HIP(hipMemcpyAsync(h_off.data(), off, (nR + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  if (tot > 0) SME_HIP(hipMemcpyAsync(h_ids.data(), ids, tot, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  out.clear();
  out.resize(4);
  int32_t cntd = 0;
  for (int64_t i = 0; i < nR; i++) {
    if (!h_flag[i]) continue;
    const uint32_t r = h_order[i];
    const uint8_t *p = h_ids.data() + h_off[r];
    const int64_t l = h_off[r + 1] - h_off[r];
    // writeUTF: the String's UTF-16 units as modified UTF-8 (U+0000 -> C0 80,
    // supplementary code points -> two 3-byte surrogates)
    std::vector<uint8_t> m;
    for (int64_t x = 0; x < l;) {
      uint32_t c = p[x];
      int k = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
      uint32_t cp = k == 1 ? c : k == 2 ? (c & 0x1F) : k == 3 ? (c & 0x0F) : (c & 0x07);
      for (int y = 1; y < k; y++) cp = (cp << 6) | (p[x + y] & 0x3F);
      x += k;
      auto unit = [&](uint32_t u) {
        if (u >= 1 && u <= 0x7F) {
          m.push_back((uint8_t)u);
        } else if (u > 0x7FF) {
          m.push_back((uint8_t)(0xE0 | ((u >> 12) & 0x0F)));
          m.push_back((uint8_t)(0x80 | ((u >> 6) & 0x3F)));
          m.push_back((uint8_t)(0x80 | (u & 0x3F)));
        } else {
          m.push_back((uint8_t)(0xC0 | ((u >> 6) & 0x1F)));
          m.push_back((uint8_t)(0x80 | (u & 0x3F)));
        }
      };
      if (cp >= 0x10000) {
        unit(0xD800 + ((cp - 0x10000) >> 10));
        unit(0xDC00 + ((cp - 0x10000) & 0x3FF));
      } else {
        unit(cp);
      }
    }
    if (m.size() > 65535) throw Error(SME_ELIMIT, "a docid exceeds writeUTF's 65535 bytes");
    out.push_back((uint8_t)(m.size() >> 8));
    out.push_back((uint8_t)m.size());
    out.insert(out.end(), m.begin(), m.end());
    cntd++;
  }
  out[0] = (uint8_t)(cntd >> 24);
  out[1] = (uint8_t)(cntd >> 16);
  out[2] = (uint8_t)(cntd >> 8);
  out[3] = (uint8_t)cntd;
}

}  // namespace sme

namespace sme {
// cuts[g] = the first record start (XMLRecordReader match position of "<DOC>")
// at or after n * g / world, n if none: the records a Hadoop split
// [n g / W, n (g+1) / W) owns (XMLInputFormat.java:173-198, a record belongs to
// the split its start tag's match begins in), taken from ONE reader pass over
// the whole input so that a shard reader started at a cut sees exactly the
// records the single reader does (no "<<DOC>" or nested "<DOC>" cut).
__global__ void k_split_cuts(const uint64_t *rs, int64_t nR, uint64_t n, int world, uint64_t *cuts) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g > world) return;
  if (g == 0 || g == world) {
    cuts[g] = g == 0 ? 0 : n;
    return;
  }
  const uint64_t target = n / (uint64_t)world * (uint64_t)g + n % (uint64_t)world * (uint64_t)g / (uint64_t)world;
  int64_t lo = 0, hi = nR;  // first rs >= target
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (rs[m] < target) lo = m + 1;
    else hi = m;
  }
  cuts[g] = lo < nR ? rs[lo] : n;
}

void split_points(sme_ctx *cx, const uint8_t *d_text, uint64_t n, int world, uint64_t *h_cuts, hipStream_t st) {
  const RecordSpans rsp = find_records(cx, d_text, n, st, nullptr);
  DevBuf out;
  uint64_t *d = out.as<uint64_t>((size_t)world + 1);
  hipLaunchKernelGGL(k_split_cuts, dim3((world + 64) / 64), dim3(64), 0, st, rsp.rs, rsp.nR, n, world, d);
  SME_CHECK_LAUNCH();
  SME_HIP(hipMemcpyAsync(h_cuts, d, ((size_t)world + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
}
}  // namespace sme
