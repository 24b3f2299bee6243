// vqa_common.h — shared device helpers for libvqa (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "vqa.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace vqa {

// thread-local error text behind vqa_get_last_error()
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// one-output-channel conv (vqa_conv_ends.hip): forward and fused data + weight gradient
bool co1_supported(int C, int O, int K, int S, int D, int dtype, int flags);
size_t co1_bwd_workspace(int C, int K);
int co1_fwd(const void* x, const float* w, const float* bias, const void* resid, void* y, int B, int T, int C, int K,
            int D, int P, int flags, int dtype, hipStream_t s);
int co1_bwd(const void* dy, const float* w, const void* x, const void* resid, void* dx, int B, int T, int C, int K,
            int D, int P, int flags, int dtype, void* ws, int* nparts, hipStream_t s);

template <class T> __device__ __forceinline__ float ld(const T* p);
template <> __device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld<bf16>(const bf16* p) { return (float)(*p); }
template <class T> __device__ __forceinline__ void st(T* p, float v);
template <> __device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<bf16>(bf16* p, float v) { *p = (bf16)v; }

// 4 consecutive elements <-> f32x4 (8 B for bf16, 16 B for f32; caller guarantees alignment)
template <class T> __device__ __forceinline__ f32x4 ld4(const T* p);
template <> __device__ __forceinline__ f32x4 ld4<float>(const float* p) { return *(const f32x4*)p; }
template <> __device__ __forceinline__ f32x4 ld4<bf16>(const bf16* p) {
  bf16x4 v = *(const bf16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <class T> __device__ __forceinline__ void st4(T* p, f32x4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, f32x4 v) { *(f32x4*)p = v; }
template <> __device__ __forceinline__ void st4<bf16>(bf16* p, f32x4 v) {
  bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *(bf16x4*)p = o;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block (256 threads) sum; result valid in all threads. red must hold >= 4 floats.
__device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = red[0] + red[1] + red[2] + red[3];
  return s;
}

// ---- reset permutation (shared host/device) ------------------------------------------------------
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__host__ __device__ inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint64_t perm_key(uint64_t seed, int64_t counter, int level) {
  return splitmix64(splitmix64(seed + (uint64_t)level) + (uint64_t)counter);
}
// keyed 4-round balanced Feistel on 2^(2h) >= M, cycle-walked into [0, M). Bijective on [0, M).
__host__ __device__ inline int64_t perm_index(uint64_t key, int64_t M, int64_t i) {
  int h = 1;
  while ((1ll << (2 * h)) < M) ++h;
  const uint32_t mask = (h >= 32) ? 0xFFFFFFFFu : ((1u << h) - 1u);
  const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
  const uint32_t rk[4] = {k0, k1, k0 ^ 0x9E3779B9u, k1 ^ 0x85EBCA6Bu};
  uint64_t x = (uint64_t)i;
  do {
    uint32_t L = (uint32_t)(x >> h) & mask, R = (uint32_t)x & mask;
    for (int r = 0; r < 4; ++r) {
      uint32_t F = mix32((R ^ rk[r]) + (uint32_t)r) & mask;
      uint32_t nL = R;
      R = L ^ F;
      L = nL;
    }
    x = ((uint64_t)L << h) | (uint64_t)R;
  } while ((int64_t)x >= M);
  return (int64_t)x;
}

}  // namespace vqa

#define VQA_REQUIRE(cond, code, ...)          \
  do {                                        \
    if (!(cond)) {                            \
      vqa::set_error(__VA_ARGS__);            \
      return code;                            \
    }                                         \
  } while (0)

#define VQA_ARG(cond, ...) VQA_REQUIRE(cond, VQA_E_INVALID_ARG, __VA_ARGS__)

#define VQA_LAUNCHED(name)                                                              \
  do {                                                                                  \
    hipError_t e_ = hipGetLastError();                                                  \
    if (e_ != hipSuccess) {                                                             \
      vqa::set_error("%s: launch failed: %s", name, hipGetErrorString(e_));             \
      return VQA_E_HIP;                                                                 \
    }                                                                                   \
  } while (0)
