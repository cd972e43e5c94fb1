// sme_dfx.hip -- the multi-GPU df exchange's device steps (dist.df_exchange).
//
// The reducer's df of a term is its postings length summed over every map
// output (TermKGramDocIndexer.java:175-183, 189-211).  Doc shards agree on terms
// through 128-bit fingerprints (sme_index_term_fingerprints); each fingerprint
// has ONE owner rank, fp.w0 mod world.  Per rank:
//
//   pack    local rows (fp, df) grouped by owner for one all_to_all: a counting
//           scatter (per-block owner histograms in LDS, one device-wide scan of
//           the owner-major (owner, block) counts, the scatter), plus pos[i] =
//           the send slot of local row i
//   sum     on the owner, every received row's df summed over the rows of its
//           fingerprint (all shards'), in an open-addressing table keyed by w0
//           (64-bit CAS) with w1 verified after the inserts; a w0 shared by two
//           different w1 (probability 2^-64 per pair) is answered exactly by a
//           host regrouping instead
//   unpack  the summed df returned in send order -> local row order (gather by pos)
//
// No torch sort / unique on this path: dist.df_exchange only moves the buffers.
#include "sme_common.hpp"
#include "sme_internal.hpp"

#include <algorithm>
#include <map>
#include <utility>

namespace sme {
namespace {

constexpr int kDfxNT = 256;
constexpr int kDfxItems = 8;                       // rows per thread per block
constexpr int kDfxRows = kDfxNT * kDfxItems;       // rows per block
constexpr int kDfxMaxWorld = 1024;
constexpr uint64_t kDfxEmpty = ~0ull;

__device__ __forceinline__ uint64_t dfx_mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// cnt[w * nb + b] = rows of block b owned by rank w
__global__ __launch_bounds__(kDfxNT) void k_dfx_hist(const uint64_t *fp, int64_t n, int world, int64_t nb,
                                                     int64_t *cnt) {
  __shared__ int32_t h[kDfxMaxWorld];
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    for (int w = threadIdx.x; w < world; w += kDfxNT) h[w] = 0;
    __syncthreads();
    const int64_t r0 = b * kDfxRows;
    for (int u = 0; u < kDfxItems; u++) {
      const int64_t i = r0 + u * kDfxNT + threadIdx.x;
      if (i < n) atomicAdd(&h[(int)(fp[2 * i] % (uint64_t)world)], 1);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < world; w += kDfxNT) cnt[(int64_t)w * nb + b] = h[w];
    __syncthreads();
  }
}

// scatter: row i -> base[owner][block] + its rank among the block's rows of that
// owner (rank order inside a block is the LDS atomic order: any order is valid,
// pos[] records it)
__global__ __launch_bounds__(kDfxNT) void k_dfx_scatter(const uint64_t *fp, const int64_t *df, int64_t n, int world,
                                                        int64_t nb, const int64_t *base, uint64_t *sfp, int64_t *sdf,
                                                        int64_t *pos) {
  __shared__ int32_t h[kDfxMaxWorld];
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    for (int w = threadIdx.x; w < world; w += kDfxNT) h[w] = 0;
    __syncthreads();
    const int64_t r0 = b * kDfxRows;
    for (int u = 0; u < kDfxItems; u++) {
      const int64_t i = r0 + u * kDfxNT + threadIdx.x;
      if (i < n) {
        const uint64_t w0 = fp[2 * i];
        const int w = (int)(w0 % (uint64_t)world);
        const int64_t p = base[(int64_t)w * nb + b] + atomicAdd(&h[w], 1);
        sfp[2 * p] = w0;
        sfp[2 * p + 1] = fp[2 * i + 1];
        sdf[p] = df[i];
        pos[i] = p;
      }
    }
    __syncthreads();
  }
}

__global__ void k_dfx_insert(const uint64_t *fp, const int64_t *df, int64_t n, uint64_t *k0, uint64_t *k1,
                             unsigned long long *sum, uint64_t mask, int64_t *slot, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t w0 = fp[2 * i];
    if (w0 == kDfxEmpty) {  // the table's empty marker: exact host regrouping
      atomicAdd(cnt + 1, 1ull);
      slot[i] = -1;
      continue;
    }
    uint64_t h = dfx_mix(w0) & mask;
    for (;;) {
      const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(k0 + h),
                                               (unsigned long long)kDfxEmpty, (unsigned long long)w0);
      if (old == kDfxEmpty) {  // claimed: this row's w1 is the slot's
        k1[h] = fp[2 * i + 1];
        atomicAdd(cnt, 1ull);
        break;
      }
      if (old == w0) break;
      h = (h + 1) & mask;
    }
    atomicAdd(sum + h, (unsigned long long)df[i]);
    slot[i] = (int64_t)h;
  }
}

// per row: the slot's sum, and a flag if the slot's w1 differs (a w0 collision)
__global__ void k_dfx_read(const uint64_t *fp, int64_t n, const uint64_t *k1, const unsigned long long *sum,
                           const int64_t *slot, int64_t *out, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = slot[i];
    if (h < 0) continue;
    if (k1[h] != fp[2 * i + 1]) atomicAdd(cnt + 1, 1ull);
    out[i] = (int64_t)sum[h];
  }
}

__global__ void k_dfx_gather(const int64_t *src, const int64_t *pos, int64_t n, int64_t *out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = src[pos[i]];
}

unsigned grid_of(int64_t n, int64_t per, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, cap));
}

}  // namespace

void dfx_pack(sme_ctx *cx, const uint64_t *fp, const int64_t *df, int64_t n, int world, uint64_t *sfp, int64_t *sdf,
              int64_t *pos, int64_t *h_counts, hipStream_t st) {
  if (world < 1 || world > kDfxMaxWorld) throw Error(SME_EINVAL, "world out of range (1..1024)");
  const int64_t nb = std::max<int64_t>(1, (n + kDfxRows - 1) / kDfxRows);
  int64_t *cnt = cx->ws[123].as<int64_t>((size_t)world * nb + 1);
  int64_t *base = cx->ws[124].as<int64_t>((size_t)world * nb + 1);
  SME_HIP(hipMemsetAsync(cnt, 0, ((size_t)world * nb + 1) * sizeof(int64_t), st));
  if (n > 0) hipLaunchKernelGGL(k_dfx_hist, dim3(grid_of(nb, 1, 65536)), dim3(kDfxNT), 0, st, fp, n, world, nb, cnt);
  SME_CHECK_LAUNCH();
  excl_scan(cnt, base, (int64_t)world * nb + 1, cx->ws[23], st);
  if (n > 0)
    hipLaunchKernelGGL(k_dfx_scatter, dim3(grid_of(nb, 1, 65536)), dim3(kDfxNT), 0, st, fp, df, n, world, nb, base,
                       sfp, sdf, pos);
  SME_CHECK_LAUNCH();
  // per-owner totals: base[(w + 1) * nb] - base[w * nb]
  std::vector<int64_t> starts((size_t)world + 1);
  for (int w = 0; w <= world; w++)
    SME_HIP(hipMemcpyAsync(&starts[(size_t)w], base + (int64_t)w * nb, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  for (int w = 0; w < world; w++) h_counts[w] = starts[(size_t)w + 1] - starts[(size_t)w];
}

void dfx_sum(sme_ctx *cx, const uint64_t *fp, const int64_t *df, int64_t n, int64_t *out, int64_t *h_distinct,
             hipStream_t st) {
  *h_distinct = 0;
  if (n <= 0) return;
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  uint64_t *k0 = cx->ws[125].as<uint64_t>(cap);
  uint64_t *k1 = cx->ws[126].as<uint64_t>(cap);
  unsigned long long *sum = reinterpret_cast<unsigned long long *>(cx->ws[127].as<uint64_t>(cap + 2));
  unsigned long long *cnt = sum + cap;
  int64_t *slot = cx->ws[124].as<int64_t>((size_t)n);
  SME_HIP(hipMemsetAsync(k0, 0xFF, cap * sizeof(uint64_t), st));
  SME_HIP(hipMemsetAsync(sum, 0, (cap + 2) * sizeof(uint64_t), st));
  hipLaunchKernelGGL(k_dfx_insert, dim3(grid_of(n, 256, 16384)), dim3(256), 0, st, fp, df, n, k0, k1, sum, cap - 1,
                     slot, cnt);
  hipLaunchKernelGGL(k_dfx_read, dim3(grid_of(n, 256, 16384)), dim3(256), 0, st, fp, n, k1, sum, slot, out, cnt);
  SME_CHECK_LAUNCH();
  unsigned long long h[2] = {0, 0};
  SME_HIP(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h[1] == 0) {
    *h_distinct = (int64_t)h[0];
    return;
  }
  // a w0 shared by different w1 (or a w0 equal to the empty marker): regroup
  // every row exactly on the host by the full 128-bit fingerprint
  std::vector<uint64_t> hf(2 * (size_t)n);
  std::vector<int64_t> hd((size_t)n), ho((size_t)n);
  SME_HIP(hipMemcpy(hf.data(), fp, 2 * n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  SME_HIP(hipMemcpy(hd.data(), df, n * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::map<std::pair<uint64_t, uint64_t>, int64_t> g;
  for (int64_t i = 0; i < n; i++) g[{hf[2 * i], hf[2 * i + 1]}] += hd[(size_t)i];
  for (int64_t i = 0; i < n; i++) ho[(size_t)i] = g[{hf[2 * i], hf[2 * i + 1]}];
  SME_HIP(hipMemcpy(out, ho.data(), n * sizeof(int64_t), hipMemcpyHostToDevice));
  *h_distinct = (int64_t)g.size();
}

void dfx_unpack(const int64_t *ret, const int64_t *pos, int64_t n, int64_t *out, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(k_dfx_gather, dim3(grid_of(n, 256, 16384)), dim3(256), 0, st, ret, pos, n, out);
  SME_CHECK_LAUNCH();
}

}  // namespace sme
