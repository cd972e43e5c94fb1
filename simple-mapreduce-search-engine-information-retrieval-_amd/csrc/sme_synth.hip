// sme_synth.hip -- on-device generator of the synthetic Zipfian TREC corpora
// (same bytes as synth.py's host generator).  Used by bench.py
// to put the c2 corpus (~3.3 GB) straight into HBM.
#include <hip/hip_runtime.h>

#include "sme_internal.hpp"

namespace sme {

constexpr int kHeadLen = 39;  // "<DOC>\n<DOCNO>D%09d</DOCNO>\n<TEXT>\n"
constexpr int kTailLen = 15;  // "</TEXT>\n</DOC>\n"

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Syn {
  const uint8_t *vocab;
  const int64_t *voff;
  int64_t V;
  const double *cdf;
  int64_t d0;
  uint64_t seed;
  int lo, hi;
};

__device__ __forceinline__ int doc_len(const Syn &s, int64_t d) {
  uint64_t key = (s.seed << 40) + ((uint64_t)d << 12) + 4095ull;
  return s.lo + (int)(splitmix64(key) % (uint64_t)(s.hi - s.lo + 1));
}
__device__ __forceinline__ int64_t tok_rank(const Syn &s, int64_t d, int j) {
  uint64_t key = (s.seed << 40) + ((uint64_t)d << 12) + (uint64_t)j;
  double x = (double)(splitmix64(key) >> 11) * (1.0 / 9007199254740992.0);
  int64_t a = 0, b = s.V;
  while (a < b) {
    int64_t m = (a + b) >> 1;
    if (s.cdf[m] <= x)
      a = m + 1;
    else
      b = m;
  }
  return a;
}

__global__ void k_syn_sizes(Syn s, int64_t ndocs, int64_t *size) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t i = blockIdx.x * wpb + (threadIdx.x >> 6); i < ndocs; i += (int64_t)gridDim.x * wpb) {
    const int64_t d = s.d0 + i;
    const int L = doc_len(s, d);
    int64_t body = 0;
    for (int j = lane; j < L; j += 64) {
      int64_t r = tok_rank(s, d, j);
      body += s.voff[r + 1] - s.voff[r] + 1;
    }
    for (int o = 32; o > 0; o >>= 1) body += __shfl_xor(body, o, 64);
    if (lane == 0) size[i] = kHeadLen + body + kTailLen;
  }
}

__global__ void k_syn_write(Syn s, int64_t ndocs, const int64_t *off, uint8_t *out) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t i = blockIdx.x * wpb + (threadIdx.x >> 6); i < ndocs; i += (int64_t)gridDim.x * wpb) {
    const int64_t d = s.d0 + i;
    uint8_t *o = out + off[i];
    const int64_t end = off[i + 1];
    if (lane == 0) {
      const char *h1 = "<DOC>\n<DOCNO>D";
      for (int k = 0; k < 14; k++) o[k] = (uint8_t)h1[k];
      int64_t v = d;
      for (int k = 8; k >= 0; k--) {
        o[14 + k] = (uint8_t)('0' + v % 10);
        v /= 10;
      }
      const char *h2 = "</DOCNO>\n<TEXT>\n";
      for (int k = 0; k < 16; k++) o[23 + k] = (uint8_t)h2[k];
      const char *t = "</TEXT>\n</DOC>\n";
      uint8_t *q = out + end - kTailLen;
      for (int k = 0; k < kTailLen; k++) q[k] = (uint8_t)t[k];
    }
    const int L = doc_len(s, d);
    int64_t carry = kHeadLen;
    for (int j0 = 0; j0 < L; j0 += 64) {
      const int j = j0 + lane;
      int64_t r = 0, wl = 0;
      if (j < L) {
        r = tok_rank(s, d, j);
        wl = s.voff[r + 1] - s.voff[r];
      }
      int64_t inc = j < L ? wl + 1 : 0;
      int64_t x = inc;
      for (int dlt = 1; dlt < 64; dlt <<= 1) {
        int64_t y = __shfl_up(x, dlt, 64);
        if (lane >= dlt) x += y;
      }
      const int64_t pos = carry + x - inc;
      if (j < L) {
        const uint8_t *w = s.vocab + s.voff[r];
        for (int64_t k = 0; k < wl; k++) o[pos + k] = w[k];
        o[pos + wl] = (j == L - 1 || (j + 1) % 12 == 0) ? '\n' : ' ';
      }
      carry += __shfl(x, 63, 64);
    }
  }
}

}  // namespace sme

extern "C" int sme_synth_corpus(int device, const uint8_t *vocab, const int64_t *vocab_off, int64_t V,
                                const double *cdf, int64_t n_docs, int64_t d0, uint64_t seed, int len_lo,
                                int len_hi, void **d_corpus, size_t *nbytes) {
  try {
    SME_HIP(hipSetDevice(device));
    hipStream_t st;
    SME_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t *dv;
    int64_t *dvo, *size, *off;
    double *dc;
    SME_HIP(hipMalloc(&dv, vocab_off[V] + 1));
    SME_HIP(hipMalloc(&dvo, (V + 1) * sizeof(int64_t)));
    SME_HIP(hipMalloc(&dc, V * sizeof(double)));
    SME_HIP(hipMalloc(&size, (n_docs + 1) * sizeof(int64_t)));
    SME_HIP(hipMalloc(&off, (n_docs + 1) * sizeof(int64_t)));
    SME_HIP(hipMemcpyAsync(dv, vocab, vocab_off[V], hipMemcpyHostToDevice, st));
    SME_HIP(hipMemcpyAsync(dvo, vocab_off, (V + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
    SME_HIP(hipMemcpyAsync(dc, cdf, V * sizeof(double), hipMemcpyHostToDevice, st));
    sme::Syn s{dv, dvo, V, dc, d0, seed, len_lo, len_hi};
    const unsigned g = (unsigned)std::min<int64_t>((n_docs + 3) / 4, 65536);
    hipLaunchKernelGGL(sme::k_syn_sizes, dim3(g), dim3(256), 0, st, s, n_docs, size);
    SME_HIP(hipMemsetAsync(size + n_docs, 0, sizeof(int64_t), st));
    sme::DevBuf scan_tmp;
    sme::excl_scan(size, off, n_docs + 1, scan_tmp, st);
    int64_t total = 0;
    SME_HIP(hipMemcpyAsync(&total, off + n_docs, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    uint8_t *out;
    SME_HIP(hipMalloc(&out, total + 64));
    hipLaunchKernelGGL(sme::k_syn_write, dim3(g), dim3(256), 0, st, s, n_docs, off, out);
    SME_HIP(hipGetLastError());
    SME_HIP(hipStreamSynchronize(st));
    (void)hipFree(dv);
    (void)hipFree(dvo);
    (void)hipFree(dc);
    (void)hipFree(size);
    (void)hipFree(off);
    (void)hipStreamDestroy(st);
    *d_corpus = out;
    *nbytes = (size_t)total;
    return SME_OK;
  } catch (const sme::Error &e) {
    return e.code;
  }
}

extern "C" void sme_synth_free(void *d) {
  if (d) (void)hipFree(d);
}

// ---- calibration: achievable HBM bandwidth on this device -------------------
// A streaming copy (16-byte nontemporal loads and stores, grid-stride, 8 x 256
// workgroups per CU), the measured ceiling beside the 8 TB/s spec that bench.py
// reports its roofline fractions against.
namespace sme {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_hbm_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < 4; u++) __builtin_nontemporal_store(v[u], dst + i + u * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}
}  // namespace sme

/* HBM copy calibration (bench.py): copies `bytes` (rounded down to 16) between
 * two device buffers `reps` times after one warm-up; *gbps = 2 x bytes / mean
 * kernel time (read + write). */
extern "C" int sme_hbm_copy_bench(int device, size_t bytes, int reps, double *gbps) {
  try {
    if (!gbps || reps < 1 || bytes < 16) return SME_EINVAL;
    SME_HIP(hipSetDevice(device));
    const int64_t n16 = (int64_t)(bytes / 16);
    void *a = nullptr, *b = nullptr;
    SME_HIP(hipMalloc(&a, n16 * 16));
    SME_HIP(hipMalloc(&b, n16 * 16));
    hipStream_t st;
    SME_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    SME_HIP(hipMemsetAsync(a, 1, n16 * 16, st));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const dim3 grid((unsigned)(8 * cus));
    hipEvent_t e0, e1;
    SME_HIP(hipEventCreate(&e0));
    SME_HIP(hipEventCreate(&e1));
    hipLaunchKernelGGL(sme::k_hbm_copy, grid, dim3(256), 0, st, (const sme::u32x4 *)a, (sme::u32x4 *)b, n16);
    SME_HIP(hipEventRecord(e0, st));
    for (int r = 0; r < reps; r++)
      hipLaunchKernelGGL(sme::k_hbm_copy, grid, dim3(256), 0, st, (const sme::u32x4 *)(r & 1 ? b : a),
                         (sme::u32x4 *)(r & 1 ? a : b), n16);
    SME_HIP(hipGetLastError());
    SME_HIP(hipEventRecord(e1, st));
    SME_HIP(hipEventSynchronize(e1));
    float ms = 0;
    SME_HIP(hipEventElapsedTime(&ms, e0, e1));
    *gbps = 2.0 * (double)(n16 * 16) * reps / (ms * 1e-3) / 1e9;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    (void)hipFree(a);
    (void)hipFree(b);
    return SME_OK;
  } catch (const sme::Error &e) {
    return e.code;
  }
}
