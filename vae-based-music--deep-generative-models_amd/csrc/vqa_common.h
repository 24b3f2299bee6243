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

// ---- cross-lane moves on the VALU (DPP, v_permlane*_swap, v_readlane) ------------------------------------
// The library's reductions and lane exchanges use these instead of __shfl* (ds_bpermute_b32 through the LDS
// crossbar): no LDS instruction, no LDS allocation needed, and — where the values are summed — a fixed pairing
// whose result is bitwise the same in every lane. Every caller below has all 64 lanes active.
// Partner helpers return the value of one partner lane; each step of a reduction pairs the two halves of the group
// the previous steps reduced, so a reduction over a 16-lane row is xor1 -> xor2 -> hmirror -> mirror, and the
// same fp32 sums are formed in both lanes of every pair (a + b = b + a: every lane ends with identical bits).
namespace xl {
template <int CTRL> __device__ __forceinline__ int dpp(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }
template <int CTRL> __device__ __forceinline__ float dpp(float v) { return __int_as_float(dpp<CTRL>(__float_as_int(v))); }
template <class T> __device__ __forceinline__ T xor1(T v) { return dpp<0xB1>(v); }      // quad_perm [1,0,3,2]
template <class T> __device__ __forceinline__ T xor2(T v) { return dpp<0x4E>(v); }      // quad_perm [2,3,0,1]
template <class T> __device__ __forceinline__ T hmirror(T v) { return dpp<0x141>(v); }  // row_half_mirror: 7 - i
template <class T> __device__ __forceinline__ T mirror(T v) { return dpp<0x140>(v); }   // row_mirror: 15 - i
template <class T> __device__ __forceinline__ T ror4(T v) { return dpp<0x124>(v); }     // row_ror:4
template <class T> __device__ __forceinline__ T ror8(T v) { return dpp<0x128>(v); }     // row_ror:8
// the values of lanes l and l ^ 16 (resp. l ^ 32), in an order the caller must not rely on (symmetric use only)
__device__ __forceinline__ void pair16(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair32(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void pair16(int v, int& a, int& b) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  a = (int)r[0];
  b = (int)r[1];
}
__device__ __forceinline__ void pair32(int v, int& a, int& b) {
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  a = (int)r[0];
  b = (int)r[1];
}
__device__ __forceinline__ float sum16(float v) { float a, b; pair16(v, a, b); return a + b; }  // v[l] + v[l ^ 16]
__device__ __forceinline__ float sum32(float v) { float a, b; pair32(v, a, b); return a + b; }  // v[l] + v[l ^ 32]
__device__ __forceinline__ float max16(float v) { float a, b; pair16(v, a, b); return fmaxf(a, b); }
__device__ __forceinline__ float max32(float v) { float a, b; pair32(v, a, b); return fmaxf(a, b); }
// sum over the lane's 16-lane row, in every lane of the row
__device__ __forceinline__ float row_sum(float v) {
  v += xor1(v);
  v += xor2(v);
  v += hmirror(v);
  return v + mirror(v);
}
__device__ __forceinline__ float row_max(float v) {
  v = fmaxf(v, xor1(v));
  v = fmaxf(v, xor2(v));
  v = fmaxf(v, hmirror(v));
  return fmaxf(v, mirror(v));
}
// sum over the aligned group of R consecutive lanes (R a power of two <= 64), in every lane of the group
template <int R> __device__ __forceinline__ float grp_sum(float v) {
  if constexpr (R >= 2) v += xor1(v);
  if constexpr (R >= 4) v += xor2(v);
  if constexpr (R >= 8) v += hmirror(v);
  if constexpr (R >= 16) v += mirror(v);
  if constexpr (R >= 32) v = sum16(v);
  if constexpr (R >= 64) v = sum32(v);
  return v;
}
// sum over the lanes with equal (lane mod R), R a power of two <= 64 (in lane q the rotations pair q with q + 4,
// q + 8 inside its row: every lane of a residue class ends with the class sum, the lanes < R with the same
// association)
template <int R> __device__ __forceinline__ float grp_combine(float v) {
  if constexpr (R <= 1) v += xor1(v);
  if constexpr (R <= 2) v += xor2(v);
  if constexpr (R <= 4) v += ror4(v);
  if constexpr (R <= 8) v += ror8(v);
  if constexpr (R <= 16) v = sum16(v);
  if constexpr (R <= 32) v = sum32(v);
  return v;
}
// inclusive scan over the wave: Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8; lanes shifted in from
// outside the row add 0), then the totals of the rows below (lanes 15, 31, 47 by v_readlane)
template <int CTRL> __device__ __forceinline__ int dpp0(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ int incl_scan(int x) {
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);
  const int t0 = __builtin_amdgcn_readlane(x, 15), t1 = __builtin_amdgcn_readlane(x, 31),
            t2 = __builtin_amdgcn_readlane(x, 47), row = (threadIdx.x & 63) >> 4;
  return x + (row > 0 ? t0 : 0) + (row > 1 ? t1 : 0) + (row > 2 ? t2 : 0);
}
// value of lane `src` (wave-uniform) in every lane
__device__ __forceinline__ float bcast(float v, int src) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src)); }
}  // namespace xl

// sum over the 64 lanes, in every lane
__device__ __forceinline__ float warp_sum(float v) { return xl::sum32(xl::sum16(xl::row_sum(v))); }
__device__ __forceinline__ float warp_max(float v) { return xl::max32(xl::max16(xl::row_max(v))); }

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
