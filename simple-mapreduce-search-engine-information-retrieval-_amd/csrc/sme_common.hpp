// sme_common.hpp -- host/device plumbing shared by the sme kernels:
// error propagation, a reusable device workspace, and wave64 / block scans.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sme.h"

namespace sme {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define SME_HIP(x)                                                                      \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess)                                                               \
      throw ::sme::Error(e_ == hipErrorOutOfMemory ? SME_ENOMEM : SME_EHIP,             \
                         std::string(#x) + ": " + hipGetErrorString(e_) + " @" __FILE__ \
                         ":" + std::to_string(__LINE__));                               \
  } while (0)

#define SME_CHECK_LAUNCH() SME_HIP(hipGetLastError())

// Freed device blocks kept for reuse (index arrays are rebuilt every step:
// hipMalloc/hipFree of gigabytes per build stalls for hundreds of ms).
struct BufPool {
  std::vector<std::pair<void *, size_t>> blocks;
  void *take(size_t bytes, size_t *cap) {
    size_t best = blocks.size();
    for (size_t i = 0; i < blocks.size(); i++)
      if (blocks[i].second >= bytes && blocks[i].second <= 2 * bytes + (64u << 20) &&
          (best == blocks.size() || blocks[i].second < blocks[best].second))
        best = i;
    if (best == blocks.size()) return nullptr;
    void *p = blocks[best].first;
    *cap = blocks[best].second;
    blocks.erase(blocks.begin() + (ptrdiff_t)best);
    return p;
  }
  void put(void *p, size_t cap) { blocks.emplace_back(p, cap); }
  size_t idle() const {  // bytes held for reuse (free to this context, not in hipMemGetInfo's free)
    size_t s = 0;
    for (const auto &b : blocks) s += b.second;
    return s;
  }
  ~BufPool() {
    for (auto &b : blocks) (void)hipFree(b.first);
  }
};

// A device buffer that grows on demand and is kept across builds, so the
// timed path does no hipMalloc once warmed up.  With a pool, blocks come from
// and go back to it instead of hipMalloc/hipFree.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  BufPool *pool = nullptr;
  void *get(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes > cap) {
      if (p) {
        SME_HIP(hipDeviceSynchronize());  // in-flight kernels may still use the old block
        if (pool)
          pool->put(p, cap);
        else
          SME_HIP(hipFree(p));
      }
      p = nullptr;
      size_t nc = 0;
      if (pool) p = pool->take(bytes, &nc);
      if (!p) {
        nc = bytes + bytes / 8;
        SME_HIP(hipMalloc(&p, nc));
      }
      cap = nc;
    }
    return p;
  }
  template <typename T>
  T *as(size_t n) {
    return reinterpret_cast<T *>(get(n * sizeof(T)));
  }
  void release() {
    if (p) {
      if (pool)
        pool->put(p, cap);
      else
        (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
  ~DevBuf() { release(); }
};

__host__ __device__ inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
inline uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// ---- device scans ---------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Inclusive wave sum (every lane of the wave active).  32-bit values scan with
// DPP moves and no LDS: shifts 1, 2, 4, 8 inside each 16-lane row, then the
// row_bcast:15 / row_bcast:31 carries into rows 1, 3 and 2, 3 (6 adds, where
// the ds_bpermute ladder took 6 LDS round trips and ~24 VALU).
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  if constexpr (sizeof(T) == 4) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return (T)x;
  } else {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      T u = __shfl_up(v, o, 64);
      if (l >= o) v += u;
    }
    return v;
  }
}
// Inclusive wave max (every lane active); signed 32-bit values by the DPP ladder
// of wave_incl_sum with INT32_MIN for the lanes a move does not reach.
template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  if constexpr (sizeof(T) == 4 && T(-1) < T(0)) {
    int x = (int)v;
    constexpr int kLo = (int)0x80000000;
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x111, 0xF, 0xF, false));  // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x112, 0xF, 0xF, false));  // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x114, 0xF, 0xF, false));  // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x118, 0xF, 0xF, false));  // row_shr:8
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    x = max(x, __builtin_amdgcn_update_dpp(kLo, x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return (T)x;
  } else {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      T u = __shfl_up(v, o, 64);
      if (l >= o) v = v > u ? v : u;
    }
    return v;
  }
}

// Block-wide exclusive sum for blockDim.x == NT (multiple of 64); scratch >= NT/64+1.
template <int NT, typename T>
__device__ __forceinline__ T block_excl_sum(T v, T *scratch, T *total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  T inc = wave_incl_sum(v);
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int i = 0; i < NT / 64; i++) {
      T t = scratch[i];
      scratch[i] = run;
      run += t;
    }
    scratch[NT / 64] = run;
  }
  __syncthreads();
  T r = scratch[w] + inc - v;
  *total = scratch[NT / 64];
  __syncthreads();
  return r;
}
// Block-wide exclusive max (identity `lo`).
template <int NT, typename T>
__device__ __forceinline__ T block_excl_max(T v, T lo, T *scratch, T *total) {
  const int w = threadIdx.x >> 6, l = lane_id();
  T inc = wave_incl_max(v);
  T exc;
  if constexpr (sizeof(T) == 4) {
    exc = (T)__builtin_amdgcn_update_dpp((int)lo, (int)inc, 0x138, 0xF, 0xF, false);  // wave_shr:1 (lane 0: lo)
  } else {
    exc = __shfl_up(inc, 1, 64);
    if (l == 0) exc = lo;
  }
  if (l == 63) scratch[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = lo;
    for (int i = 0; i < NT / 64; i++) {
      T t = scratch[i];
      scratch[i] = run;
      run = run > t ? run : t;
    }
    scratch[NT / 64] = run;
  }
  __syncthreads();
  T pre = scratch[w];
  T r = pre > exc ? pre : exc;
  *total = scratch[NT / 64];
  __syncthreads();
  return r;
}

// 64-bit token hash (FNV-1a + murmur3 fmix); 0 is reserved for "empty".
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

}  // namespace sme
