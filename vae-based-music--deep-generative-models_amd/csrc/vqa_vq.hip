// vqa_vq.hip — EMA vector quantizer kernels (gfx950).
//
// Replaces the TF op sequence of VectorQuantizer.call (VectorQuantizer.py:75-165):
//   get_code_indices :170-186  -> vq_argmin_mfma_kernel (fp32 MFMA distance tiles + wave argmin);
//                                 no N x K distance matrix is materialised.
//   one_hot @ E^T    :86-90    -> a row gather from ET = E^T (K, D) kept by the EMA kernel.
//   commit loss      :97-99, straight-through :114 -> vq_quantize_kernel; EMA sums :123-124 -> a counting
//                                 sort by code + fixed-order segment sums (deterministic, no float atomics).
//   EMA + dead-code reset :126-145, metrics :149-159 -> vq_ema_apply_kernel / vq_metrics_kernel.
// The reset candidates (tf.random.shuffle, :137) use an injected, seeded Feistel permutation.
#include "vqa_common.h"
#include <algorithm>

namespace vqa {

// out[r] = v of lane 4 (lane >> 4) + r, for v equal in the wave's 4 rows (row 0's lanes 0-15 serve every group)
__device__ __forceinline__ void gather_row4(float v, float (&out)[4]) {
  const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float a = xl::bcast(v, r), b = xl::bcast(v, 4 + r), c = xl::bcast(v, 8 + r), d = xl::bcast(v, 12 + r);
    out[r] = g == 0 ? a : g == 1 ? b : g == 2 ? c : d;
  }
}

// ---- argmin -------------------------------------------------------------------------------------
// One workgroup = 4 waves x 32 rows. Distances d = (|z|^2 + |e|^2) - 2 z.e exactly as the reference
// orders them (VectorQuantizer.py:175-182), in fp32; z.e on v_mfma_f32_16x16x4_f32 (an exact fp32
// FMA chain over d). Codebook chunks of 128 codes are staged through LDS and shared by the waves.
template <class T, int D>
__global__ __launch_bounds__(256) void vq_argmin_mfma_kernel(const T* z, const float* E, const float* esq,
                                                            int64_t* idx, float* mind, long long N, int K) {
  constexpr int KC = 128, DS = D / 4, RT = 2;
  __shared__ float El[D * KC];
  __shared__ float el2[KC];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long long n0 = (long long)blockIdx.x * 128 + wave * 32;

  // A fragments: z[n0 + rt*16 + (lane&15)][4*ds + (lane>>4)]
  float af[RT][DS];
  float zsq[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const long long row = n0 + rt * 16 + (lane & 15);
    float s = 0.f;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      const float v = row < N ? ld(z + row * D + 4 * ds + (lane >> 4)) : 0.f;
      af[rt][ds] = v;
      s += v * v;
    }
    // full row |z|^2: the sum over the 4 lanes {l, l^16, l^32, l^48}
    zsq[rt] = xl::sum32(xl::sum16(s));
  }
  // accumulator lane holds rows 4*(lane>>4)+r: their |z|^2 from lane (4*(lane>>4)+r)
  float zq[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) gather_row4(zsq[rt], zq[rt]);

  float best[RT][4];
  int bidx[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      best[rt][r] = __builtin_inff();
      bidx[rt][r] = 0;  // a row with no finite distance (NaN / inf in z) resolves to code 0, as tf.argmin
    }

  for (int k0 = 0; k0 < K; k0 += KC) {
    __syncthreads();
    for (int e = threadIdx.x; e < D * KC; e += 256) {
      const int d = e / KC, kk = e - d * KC;
      El[e] = (k0 + kk < K) ? E[(long long)d * K + k0 + kk] : 0.f;
    }
    for (int e = threadIdx.x; e < KC; e += 256) el2[e] = (k0 + e < K) ? esq[k0 + e] : 0.f;
    __syncthreads();
#pragma unroll 1
    for (int ct = 0; ct < KC / 16; ++ct) {
      const int kl = ct * 16 + (lane & 15);
      float bf[DS];
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) bf[ds] = El[(4 * ds + (lane >> 4)) * KC + kl];
      const int kg = k0 + kl;
      const float e2 = el2[kl];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ds = 0; ds < DS; ++ds) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(af[rt][ds], bf[ds], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = zq[rt][r] + e2;
          const float dist = t - 2.0f * acc[r];
          if (kg < K && dist < best[rt][r]) {
            best[rt][r] = dist;
            bidx[rt][r] = kg;
          }
        }
      }
    }
  }
  // reduce over the 16 lanes holding the same rows (lane bits 0..3), ties -> lowest index
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float b = best[rt][r];
      int bi = bidx[rt][r];
      auto take = [&](float ob, int oi) {
        if (ob < b || (ob == b && oi < bi)) {
          b = ob;
          bi = oi;
        }
      };
      take(xl::xor1(b), xl::xor1(bi));
      take(xl::xor2(b), xl::xor2(bi));
      take(xl::hmirror(b), xl::hmirror(bi));
      take(xl::mirror(b), xl::mirror(bi));
      const long long row = n0 + rt * 16 + 4 * (lane >> 4) + r;
      if ((lane & 15) == 0 && row < N) {
        idx[row] = bi;
        if (mind) mind[row] = b;
      }
    }
}

// ---- argmin for bf16 z on bf16 MFMA, exact to fp32 products ----------------------------------------
// E is split once per codebook update into three bf16 planes hi + mid + lo (= E exactly: 3 x 8 mantissa
// bits) and z (bf16) is exact in bf16, so z.e = z.lo + z.mid + z.hi sums exact products with fp32
// accumulation — the same quality as the fp32 FMA chain at 3/16 of the MFMA time (16x16x32 bf16 vs
// 16x16x4 f32). The distance and the tie rule are those of vq_argmin_mfma_kernel.
// WG = 4 waves x 64 rows; code chunks of KC codes (3 planes, padded rows) staged in LDS.
constexpr int kSplitKC = 64;

// (distance, index) -> one uint64 whose unsigned order is (distance, then index): the K-split partial results
// combine with atomicMin in any order to the same winner (ties -> lowest index, as tf.argmin)
__device__ __forceinline__ unsigned long long vq_pack(float d, int k) {
  unsigned u = __float_as_uint(d);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)k;
}
__device__ __forceinline__ float vq_unpack_dist(unsigned long long p) {
  unsigned u = (unsigned)(p >> 32);
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __uint_as_float(u);
}

// blockIdx.y = code split: codes [y*kspan, (y+1)*kspan); with more than one split the row results go to
// idx as packed keys through atomicMin (vq_argmin_unpack_kernel turns them into indices / distances).
// Code chunks are double-buffered in LDS: the next chunk's global loads are in flight (registers) while the
// current chunk runs its MFMAs, and land in the other buffer behind ONE barrier per chunk. Codes past the span
// carry |e|^2 = +inf (their key is -inf and never wins), so the epilogue is one compare and two selects.
template <int D>
__global__ __launch_bounds__(256) void vq_argmin_split_kernel(const bf16* z, const bf16* E3, const float* esq,
                                                             int64_t* idx, float* mind, long long N, int K,
                                                             int kspan) {
  const int kbeg = blockIdx.y * kspan, kend = min(K, kbeg + kspan);
  const bool packed = gridDim.y > 1;
  constexpr int KC = kSplitKC, KS = D / 32, RT = 4;
  constexpr int CS = 3 * D + 8;          // LDS code stride (bf16): +16 B so 16 codes hit distinct banks
  constexpr int PPC = 3 * D * 2 / 16;    // 16-byte pieces per code
  constexpr int NPT = KC * PPC / 256;    // pieces per thread per chunk
  static_assert(KC * PPC % 256 == 0 && KC <= 256, "chunk staging");
  __shared__ __attribute__((aligned(16))) bf16 El[2][KC * CS];
  __shared__ float el2[2][KC];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long long n0 = (long long)blockIdx.x * 256 + wave * 64;

  bf16x8 af[RT][KS];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const long long row = n0 + rt * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 v;
      if (row < N) {
        v = *(const bf16x8*)(z + row * D + ks * 32 + 8 * (lane >> 4));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)0.f;
      }
      af[rt][ks] = v;
    }
  }
  // |z|^2 of the rows this lane reports (row 4 (lane >> 4) + r of tile rt), from the A fragments: needed only by
  // the epilogue, so it is evaluated there (16 fewer live registers in the code loop: 3 waves per SIMD)
  auto row_sqnorms = [&](float (&zq)[RT][4]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float s = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)af[rt][ks][j];
          s += f * f;
        }
      gather_row4(xl::sum32(xl::sum16(s)), zq[rt]);
    }
  };
#ifdef VQA_ARGMIN_DIST_FORM
  float zq[RT][4];
  row_sqnorms(zq);
#endif

  // the kernel maximises key = z.e - |e|^2 / 2 (distance = |z|^2 - 2 key): the MFMA accumulator starts at
  // -|e|^2 / 2, so a code costs one compare and two selects per row (the distance form took an add and an fma
  // more); the argmin is the distance's on every row whose top-2 margin exceeds the last-bit roundings
  float best[RT][4];
  int bidx[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      best[rt][r] = -__builtin_inff();
      bidx[rt][r] = kbeg;  // no finite key in this span: (inf distance, first code); the merge keeps code 0
    }

  // chunk staging: piece e = threadIdx.x + 256 p of code e / PPC
  uint4 st[NPT];
  float se2 = 0.f;
  auto load_chunk = [&](int k0) {
#pragma unroll
    for (int p = 0; p < NPT; ++p) {
      const int e = threadIdx.x + 256 * p, c = e / PPC, pc = e - c * PPC;
      st[p] = k0 + c < kend ? *(const uint4*)(E3 + (size_t)(k0 + c) * 3 * D + pc * 8) : uint4{0u, 0u, 0u, 0u};
    }
    if (threadIdx.x < KC) se2 = k0 + (int)threadIdx.x < kend ? esq[k0 + threadIdx.x] : __builtin_inff();
  };
  auto store_chunk = [&](int b) {
#pragma unroll
    for (int p = 0; p < NPT; ++p) {
      const int e = threadIdx.x + 256 * p, c = e / PPC, pc = e - c * PPC;
      *(uint4*)(&El[b][c * CS + pc * 8]) = st[p];
    }
    if (threadIdx.x < KC) el2[b][threadIdx.x] = se2;
  };
  load_chunk(kbeg);
  store_chunk(0);
  __syncthreads();
  int b = 0;
  for (int k0 = kbeg; k0 < kend; k0 += KC, b ^= 1) {
    const bool more = k0 + KC < kend;
    if (more) load_chunk(k0 + KC);  // lands while this chunk is compared
#pragma unroll 1
    for (int ct = 0; ct < KC / 16; ++ct) {
      const int kl = ct * 16 + (lane & 15);
      const bf16* eb = &El[b][kl * CS + 8 * (lane >> 4)];
      bf16x8 bfr[3][KS];
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) bfr[s][ks] = *(const bf16x8*)(eb + s * D + ks * 32);
      const int kg = k0 + kl;
#ifdef VQA_ARGMIN_DIST_FORM  // A/B only: the round-3 distance-form epilogue (add, fma, compare, two selects)
      const float e2 = el2[b][kl];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 2; s >= 0; --s)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][ks], bfr[s][ks], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // timing only (best holds -distance; the reported min distance is not meaningful in this build)
          const float dist = __builtin_fmaf(-2.0f, acc[r], zq[rt][r] + e2);
          if (-dist > best[rt][r]) {
            best[rt][r] = -dist;
            bidx[rt][r] = kg;
          }
        }
      }
#else
      const float c = -0.5f * el2[b][kl];  // exact; codes past the span: -inf, never chosen
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        f32x4 acc = {c, c, c, c};
#pragma unroll
        for (int s = 2; s >= 0; --s)  // smallest plane first
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt][ks], bfr[s][ks], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (acc[r] > best[rt][r]) {  // strict: the lowest code wins a tie (codes visited in increasing order)
            best[rt][r] = acc[r];
            bidx[rt][r] = kg;
          }
        }
      }
#endif
    }
    if (more) store_chunk(b ^ 1);  // buffer b ^ 1 was last read before the previous barrier
    __syncthreads();
  }
#ifndef VQA_ARGMIN_DIST_FORM
  float zq[RT][4];
  row_sqnorms(zq);
#endif
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float b = best[rt][r];
      int bi = bidx[rt][r];
      auto take = [&](float ob, int oi) {
        if (ob > b || (ob == b && oi < bi)) {
          b = ob;
          bi = oi;
        }
      };
      take(xl::xor1(b), xl::xor1(bi));
      take(xl::xor2(b), xl::xor2(bi));
      take(xl::hmirror(b), xl::hmirror(bi));
      take(xl::mirror(b), xl::mirror(bi));
      const long long row = n0 + rt * 16 + 4 * (lane >> 4) + r;
      if ((lane & 15) == 0 && row < N) {
        // |z|^2 - 2 key (+inf for a row with no finite key). A row with a non-finite |z|^2 has no finite distance
        // to any code (inf - inf or NaN): code 0 of the span, as the distance form resolves it, and min distance
        // +inf, as the distance form reports it (a NaN would also break the packed keys' order in the merge)
        const float zr = zq[rt][r];
        const bool finite = zr < __builtin_inff();
        const float dist = finite ? __builtin_fmaf(-2.0f, b, zr) : __builtin_inff();
        if (!finite) bi = kbeg;
        if (packed) {
          atomicMin((unsigned long long*)idx + row, vq_pack(dist, bi));
        } else {
          idx[row] = bi;
          if (mind) mind[row] = dist;
        }
      }
    }
}

__global__ __launch_bounds__(256) void vq_argmin_init_kernel(int64_t* idx, long long N) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < N) idx[i] = (int64_t)~0ull;
}
__global__ __launch_bounds__(256) void vq_argmin_unpack_kernel(int64_t* idx, float* mind, long long N) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const unsigned long long p = (unsigned long long)idx[i];
  idx[i] = (int64_t)(unsigned)(p & 0xffffffffu);
  if (mind) mind[i] = vq_unpack_dist(p);
}

// E (D, K) fp32 -> E3 (K, 3, D) bf16 planes with hi + mid + lo = E
__global__ __launch_bounds__(256) void vq_split3_kernel(const float* E, bf16* E3, int D, int K) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)D * K) return;
  const int d = (int)(e / K), k = (int)(e - (long long)d * K);
  const float v = E[e];
  const bf16 hi = (bf16)v;
  const float r1 = v - (float)hi;
  const bf16 mid = (bf16)r1;
  const bf16 lo = (bf16)(r1 - (float)mid);
  bf16* o = E3 + (size_t)k * 3 * D + d;
  o[0] = hi;
  o[D] = mid;
  o[2 * D] = lo;
}

// generic argmin (any D): one thread per row
template <class T>
__global__ __launch_bounds__(256) void vq_argmin_direct_kernel(const T* z, const float* E, const float* esq,
                                                              int64_t* idx, float* mind, long long N, int D, int K) {
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float zsq = 0.f;
  for (int d = 0; d < D; ++d) {
    const float v = ld(z + n * D + d);
    zsq += v * v;
  }
  float best = __builtin_inff();
  int bi = 0;
  for (int k = 0; k < K; ++k) {
    float dot = 0.f;
    for (int d = 0; d < D; ++d) dot += ld(z + n * D + d) * E[(long long)d * K + k];
    const float t = zsq + esq[k];
    const float dist = t - 2.0f * dot;
    if (dist < best) {
      best = dist;
      bi = k;
    }
  }
  idx[n] = bi;
  if (mind) mind[n] = best;
}

// |e_k|^2, one wave per code: lane d squares e[d][k] (d, d + 64, ... for D > 64), then a butterfly sum over the
// wave — the summation order of vq_ema_apply_kernel's fused |e|^2, so both give the same bits for the same E
__global__ __launch_bounds__(256) void vq_sqnorm_kernel(const float* E, float* esq, int D, int K) {
  const int k = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= K) return;  // wave-uniform
  float s = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float v = E[(long long)d * K + k];
    s += v * v;
  }
  s = warp_sum(s);
  if (lane == 0) esq[k] = s;
}

// ---- quantize / straight-through / commitment ----------------------------------------------------
// thread per (row, d); partial sums of (q - z)^2 per workgroup -> ws (reduced in a fixed order)
template <class T>
__global__ __launch_bounds__(256) void vq_quantize_kernel(const T* z, const float* ET, const int64_t* idx, T* qst,
                                                         long long N, int D, float* ws) {
  __shared__ float red[4];
  const long long total = N * D;
  float part = 0.f;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long n = e / D;
    const int d = (int)(e - n * D);
    const long long k = idx[n];
    const float zf = ld(z + e);
    const float q = ET[k * D + d];
    const float diff = q - zf;
    part += diff * diff;
    st(qst + e, zf + diff);
  }
  const float s = block_sum_256(part, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// out[0] = scale * sum(ws[0..n))  (single workgroup, fixed order)
__global__ __launch_bounds__(256) void reduce_scalar_kernel(const float* ws, int n, float scale, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += ws[i];
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

template <class T>
__global__ __launch_bounds__(256) void vq_backward_kernel(const T* dq, const T* z, const float* ET,
                                                         const int64_t* idx, T* dz, float scale, long long N, int D) {
  const long long total = N * D;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long n = e / D;
    const int d = (int)(e - n * D);
    const float zf = ld(z + e);
    const float q = ET[idx[n] * D + d];
    st(dz + e, ld(dq + e) + scale * (zf - q));
  }
}

// Vectorised forms for D = 32 / 64 (the model's latent widths): a thread owns 8 consecutive channels of one row,
// so z / dq / q_st / dz move in 16-byte (bf16) pieces, the row's code is one load per 8 channels, and the
// element -> (row, channel) map is a shift of a 32-bit index instead of a 64-bit division per element. The
// per-element arithmetic is the scalar kernels' (fp32, no contraction), so q_st and dz are bitwise the same;
// the commitment partials are summed in another order (a float sum: within the tests' tolerance).
template <class T, int D>
__global__ __launch_bounds__(256) void vq_quantize8_kernel(const T* z, const float* ET, const int64_t* idx, T* qst,
                                                          int N, float* ws) {
  __shared__ float red[4];
  constexpr int OPR = D / 8;  // 8-channel pieces per row
  const int total = N * OPR;
  float part = 0.f;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < total; o += gridDim.x * 256) {
    const int n = o / OPR, c = (o - n * OPR) * 8;
    const size_t e = (size_t)n * D + c;
    const float* q = ET + idx[n] * D + c;
    const f32x4 z0 = ld4(z + e), z1 = ld4(z + e + 4);
    const f32x4 d0 = *(const f32x4*)q - z0, d1 = *(const f32x4*)(q + 4) - z1;
#pragma unroll
    for (int i = 0; i < 4; ++i) part += d0[i] * d0[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) part += d1[i] * d1[i];
    st4(qst + e, z0 + d0);
    st4(qst + e + 4, z1 + d1);
  }
  const float s = block_sum_256(part, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

template <class T, int D>
__global__ __launch_bounds__(256) void vq_backward8_kernel(const T* dq, const T* z, const float* ET,
                                                          const int64_t* idx, T* dz, float scale, int N) {
  constexpr int OPR = D / 8;
  const int total = N * OPR;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < total; o += gridDim.x * 256) {
    const int n = o / OPR, c = (o - n * OPR) * 8;
    const size_t e = (size_t)n * D + c;
    const float* q = ET + idx[n] * D + c;
    const f32x4 z0 = ld4(z + e), z1 = ld4(z + e + 4);
    const f32x4 g0 = ld4(dq + e), g1 = ld4(dq + e + 4);
    const f32x4 t0 = z0 - *(const f32x4*)q, t1 = z1 - *(const f32x4*)(q + 4);
    st4(dz + e, g0 + scale * t0);
    st4(dz + e + 4, g1 + scale * t1);
  }
}

template <class T>
__global__ __launch_bounds__(256) void vq_reset_rows_kernel(const T* z, float* RT, long long N_local,
                                                           long long row_offset, long long N_global, int D, int K,
                                                           uint64_t seed, const int64_t* counter, int level) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)K * D) return;
  const int k = (int)(e / D), d = (int)(e - (long long)k * D);
  const long long M = N_global >= K ? N_global : N_global * ((K + N_global - 1) / N_global);
  const uint64_t key = perm_key(seed, counter[0], level);
  const long long g = perm_index(key, M, k) % N_global;
  const long long loc = g - row_offset;
  RT[e] = (loc >= 0 && loc < N_local) ? ld(z + loc * D + d) : 0.f;
}

// one wave per code, lane = d (D <= 64)
// One wave per code k, lane d = embedding dimension. With esq / E3 (nullable) the codebook's derived state is
// written in the same pass: |e_k|^2 (the butterfly order of vq_sqnorm_kernel) and the bf16 hi/mid/lo planes
// (vq_split3_kernel's arithmetic) — the two launches the next step's argmin needs, off the step's serial tail.
__global__ __launch_bounds__(256) void vq_ema_apply_kernel(float* E, float* ET, float* m_t, float* N_t,
                                                          const float* m_sumT, const float* n_sum, const float* RT,
                                                          float g, float omg, float thresh, int64_t* counter,
                                                          float* esq, bf16* E3, int D, int K) {
  const int k = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int d = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) counter[0] += 1;
  if (k >= K) return;  // wave-uniform
  float e = 0.f;
  if (d < D) {
    // TF: gamma * N_t + (1 - gamma) * N_t_  — two products then a sum (no contraction: -ffp-contract=off)
    const float Nn = g * N_t[k] + omg * n_sum[k];
    const float mn = g * m_t[(long long)d * K + k] + omg * m_sumT[(long long)k * D + d];
    const bool use = Nn >= thresh;
    const float Nc = fminf(fmaxf(Nn, 1e-8f), 1e8f);
    e = use ? mn / Nc : RT[(long long)k * D + d];
    m_t[(long long)d * K + k] = mn;
    E[(long long)d * K + k] = e;
    ET[(long long)k * D + d] = e;
    if (d == 0) N_t[k] = Nn;
    if (E3) {
      const bf16 hi = (bf16)e;
      const float r1 = e - (float)hi;
      const bf16 mid = (bf16)r1;
      const bf16 lo = (bf16)(r1 - (float)mid);
      bf16* o = E3 + (size_t)k * 3 * D + d;
      o[0] = hi;
      o[D] = mid;
      o[2 * D] = lo;
    }
  }
  if (esq) {
    const float s = warp_sum(e * e);
    if (d == 0) esq[k] = s;
  }
}

// metrics: [0] #(n_sum >= thr), [1] #(N_t >= thr), [2] -sum p log(p + 1e-8), p = n_sum / sum(n_sum)
__global__ __launch_bounds__(256) void vq_metrics_kernel(const float* n_sum, const float* N_t, float thresh, int K,
                                                        float* metrics) {
  __shared__ float red[4];
  float tot = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) tot += n_sum[k];
  tot = block_sum_256(tot, red);
  float bu = 0.f, ru = 0.f, ent = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float c = n_sum[k];
    bu += c >= thresh ? 1.f : 0.f;
    ru += N_t[k] >= thresh ? 1.f : 0.f;
    const float p = c / tot;
    ent += p * logf(p + 1e-8f);
  }
  __syncthreads();
  bu = block_sum_256(bu, red);
  __syncthreads();
  ru = block_sum_256(ru, red);
  __syncthreads();
  ent = block_sum_256(ent, red);
  if (threadIdx.x == 0) {
    metrics[0] = bu;
    metrics[1] = ru;
    metrics[2] = -ent;
  }
}

static int quantize_blocks(long long total) {
  long long b = (total + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

// the vectorised forms apply: D = 32 / 64, 16-byte aligned rows, 32-bit piece indices — including the grid-stride
// loop's last increment (a piece index plus the largest stride, 4096 blocks x 256, stays below 2^31)
static bool vq_vec8_ok(long long N, int D, std::initializer_list<const void*> ptrs) {
  if ((D != 32 && D != 64) || N * (D / 8) + 4096ll * 256 >= (1ll << 31)) return false;
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16) return false;
  return true;
}
static int vec8_blocks(long long N, int D) { return quantize_blocks(N * D / 8); }

// ---- EMA sums by code (VectorQuantizer.py:123-124: m_sum = z^T onehot, n_sum = column sums of onehot) ----
// Deterministic: the rows are counting-sorted by code (stable: by code, then row), and every code's sum is
// taken over its rows in that order — sequential runs within 64-position tiles, tile partials added in tile
// order. No floating-point atomics anywhere, so the sums (and the codebook they drive) are bitwise
// reproducible run to run and independent of scheduling. Counts are exact integers.
//   1 vq_sort_count_kernel   per 1024-row chunk: per-code counts, each row's rank among its chunk's equal codes
//   2 vq_sort_scan_kernel    per code: exclusive prefix of the chunk counts; totals (n_sum += total)
//   3 vq_sort_scatter_kernel segment starts (exclusive scan of the totals), perm[pos] = row, scode[pos] = code
//   4 vq_seg_sum_kernel      one wave per 64 sorted positions, lanes = channels: run sums in row order; a run
//                            that is its code's whole segment is added to m_sumT, others go to tile partials
//   5 vq_seg_combine_kernel  codes spanning tiles: tile partials summed in tile order -> m_sumT
constexpr int kSortChunk = 1024;  // rows per chunk (= threads of kernels 1 and 3)
constexpr int kSegTile = 64;      // sorted positions per wave in kernel 4
constexpr int kMaxSortK = 16384;  // LDS histogram bound (64 KB)

struct SortWs {
  int* cnt;    // [nch][K] chunk counts -> exclusive offsets within the code
  int* tot;    // [K] rows per code
  int* seg;    // [K + 1] segment starts in sorted order
  int* lrank;  // [N] rank of the row among the equal codes of its chunk
  int* perm;   // [N] sorted position -> row
  int* scode;  // [N] sorted position -> code
  float* tfirst;  // [ntile][D] sum of the tile's first run (when that run is not a whole segment)
  float* tlast;   // [ntile][D] sum of the tile's last run (idem, when it is not also the first)
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }
static size_t sort_ws_bytes(long long N, int D, int K) {
  const long long nch = (N + kSortChunk - 1) / kSortChunk, ntile = (N + kSegTile - 1) / kSegTile;
  return align256((size_t)nch * K * 4) + align256((size_t)K * 4) + align256((size_t)(K + 1) * 4) +
         3 * align256((size_t)N * 4) + 2 * align256((size_t)ntile * D * 4);
}
static SortWs sort_ws(void* base, long long N, int D, int K) {
  const long long nch = (N + kSortChunk - 1) / kSortChunk, ntile = (N + kSegTile - 1) / kSegTile;
  char* p = (char*)base;
  SortWs w;
  w.cnt = (int*)p;   p += align256((size_t)nch * K * 4);
  w.tot = (int*)p;   p += align256((size_t)K * 4);
  w.seg = (int*)p;   p += align256((size_t)(K + 1) * 4);
  w.lrank = (int*)p; p += align256((size_t)N * 4);
  w.perm = (int*)p;  p += align256((size_t)N * 4);
  w.scode = (int*)p; p += align256((size_t)N * 4);
  w.tfirst = (float*)p; p += align256((size_t)ntile * D * 4);
  w.tlast = (float*)p;
  return w;
}

__global__ __launch_bounds__(kSortChunk) void vq_sort_count_kernel(const int64_t* idx, SortWs w, int N, int K) {
  extern __shared__ int hist[];  // [K]
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, row = c * kSortChunk + tid;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t v = row < N ? idx[row] : -1;
  const int k = (v >= 0 && v < K) ? (int)v : -1;  // an index outside [0, K) contributes to no code
  for (int i = tid; i < K; i += kSortChunk) hist[i] = 0;
  // stable rank = equal codes at lower lanes of the row's wave + equal codes in the chunk's earlier waves
  int r = 0;
#pragma unroll
  for (int j = 0; j < 63; ++j) r += (__builtin_amdgcn_readlane(k, j) == k) & (j < lane);
  // the waves take turns in row order: read the running histogram (the earlier waves' counts), then add
  // their own rows (integer LDS atomics; a wave's read completes before its adds are issued)
  for (int t = 0; t < kSortChunk / 64; ++t) {
    __syncthreads();
    if (wv == t && k >= 0) {
      r += hist[k];
      w.lrank[row] = r;
      atomicAdd(hist + k, 1);
    }
  }
  __syncthreads();
  for (int i = tid; i < K; i += kSortChunk) w.cnt[(size_t)c * K + i] = hist[i];
}

// block = 16 waves x 64 codes: wave v scans its contiguous range of chunks, the 16 range totals are
// prefixed in LDS, then each wave writes its range's exclusive offsets
__global__ __launch_bounds__(1024) void vq_sort_scan_kernel(SortWs w, float* n_sum, int nch, int K) {
  __shared__ int part[16][64];
  const int lane = threadIdx.x & 63, v = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), k = blockIdx.x * 64 + lane;
  const int per = (nch + 15) / 16, c0 = min(nch, v * per), c1 = min(nch, c0 + per);
  int s = 0;
  if (k < K)
    for (int c = c0; c < c1; ++c) s += w.cnt[(size_t)c * K + k];
  part[v][lane] = s;
  __syncthreads();
  if (v == 0) {
    int run = 0;
    for (int i = 0; i < 16; ++i) {
      const int t = part[i][lane];
      part[i][lane] = run;
      run += t;
    }
    if (k < K) {
      w.tot[k] = run;
      if (n_sum) n_sum[k] += (float)run;
    }
  }
  __syncthreads();
  if (k < K) {
    int run = part[v][lane];
    for (int c = c0; c < c1; ++c) {
      const int t = w.cnt[(size_t)c * K + k];
      w.cnt[(size_t)c * K + k] = run;
      run += t;
    }
  }
}

// exclusive scan of tot[0..K) into seg (LDS, K + 1 ints) by the block's 1024 threads
__device__ void seg_scan(const int* tot, int* seg, int K) {
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, v = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int per = (K + kSortChunk - 1) / kSortChunk, i0 = min(K, tid * per), i1 = min(K, i0 + per);
  int s = 0;
  for (int i = i0; i < i1; ++i) s += tot[i];
  const int incl = xl::incl_scan(s);  // inclusive wave scan
  if (lane == 63) wsum[v] = incl;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < v; ++i) base += wsum[i];
  int run = base + incl - s;
  for (int i = i0; i < i1; ++i) {
    seg[i] = run;
    run += tot[i];
  }
  if (tid == kSortChunk - 1) seg[K] = run;
  __syncthreads();
}

__global__ __launch_bounds__(kSortChunk) void vq_sort_scatter_kernel(const int64_t* idx, SortWs w, int N, int K) {
  extern __shared__ int seg[];  // [K + 1]
  seg_scan(w.tot, seg, K);
  const int c = blockIdx.x, row = c * kSortChunk + threadIdx.x;
  if (c == 0)
    for (int i = threadIdx.x; i <= K; i += kSortChunk) w.seg[i] = seg[i];
  if (row >= N) return;
  const int64_t v = idx[row];
  if (v < 0 || v >= K) return;
  const int k = (int)v;
  const int pos = seg[k] + w.cnt[(size_t)c * K + k] + w.lrank[row];
  w.perm[pos] = row;
  w.scode[pos] = k;
}

template <class T>
__global__ __launch_bounds__(256) void vq_seg_sum_kernel(const T* z, SortWs w, float* m_sumT, int K, int D) {
  const int lane = threadIdx.x & 63;
  // wave-uniform tile (readfirstlane): np and the run bookkeeping stay scalar, and the 64 row loads below are
  // unconditional, so they are all in flight at once (a per-lane `i < np` guard made the compiler wrap each
  // load in its own branch and wait on it: 64 serialised HBM round trips per wave)
  const int tile = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p0 = tile * kSegTile;
  const int N = w.seg[K];  // sorted positions = rows with a valid code
  if (p0 >= N) return;
  const int np = min(kSegTile, N - p0);
  const int myrow = w.perm[p0 + min(lane, np - 1)];  // positions past np repeat a valid row (never summed)
  const int mycode = lane < np ? w.scode[p0 + lane] : -1;
  for (int d0 = 0; d0 < D; d0 += 64) {
    const int d = d0 + lane;
    const bool on = d < D;
    const int dl = min(d, D - 1);
    float v[kSegTile];
#pragma unroll
    for (int i = 0; i < kSegTile; ++i) {
      const int row = __builtin_amdgcn_readlane(myrow, i);
      v[i] = ld(z + (size_t)row * D + dl);
    }
    float s = 0.f;
    int a = 0;
#pragma unroll
    for (int i = 0; i < kSegTile; ++i) {
      if (i >= np) continue;  // uniform (partial last tile); keeps the loop unrolled (v[] in registers)
      s += v[i];
      const int k = __builtin_amdgcn_readlane(mycode, i);
      const int kn = i + 1 < np ? __builtin_amdgcn_readlane(mycode, i + 1) : -1;
      if (kn != k) {  // run [a, i] of code k ends
        const int S = w.seg[k], E = w.seg[k + 1];
        if (on) {
          if (S >= p0 && E <= p0 + np) m_sumT[(size_t)k * D + d] += s;       // whole segment in this tile
          else if (a == 0) w.tfirst[(size_t)tile * D + d] = s;                // segment continues across a tile edge
          else w.tlast[(size_t)tile * D + d] = s;
        }
        s = 0.f;
        a = i + 1;
      }
    }
  }
}

// one workgroup (4 waves) per code whose segment spans several tiles: the waves sum contiguous quarters of
// the tile range in order, then the quarters are added in order (a fixed tree for a given segment)
__global__ __launch_bounds__(256) void vq_seg_combine_kernel(SortWs w, float* m_sumT, int D) {
  __shared__ float q[4][64];
  const int k = blockIdx.x, lane = threadIdx.x & 63, v = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int S = w.seg[k], E = w.seg[k + 1];
  if (E <= S) return;
  const int ta = S / kSegTile, tb = (E - 1) / kSegTile;
  if (ta == tb) return;  // whole segment inside one tile: added by vq_seg_sum_kernel
  const int n = tb - ta;  // tiles ta+1 .. tb read tfirst
  const int per = (n + 3) / 4, i0 = ta + 1 + min(n, v * per), i1 = ta + 1 + min(n, (v + 1) * per);
  for (int d0 = 0; d0 < D; d0 += 64) {
    const int d = d0 + lane, dl = min(d, D - 1);
    float s = 0.f;
    if (v == 0) s = (S == ta * kSegTile ? w.tfirst : w.tlast)[(size_t)ta * D + dl];
    // 8 tile partials in flight per wave (clamped indices, unconditional loads), added in tile order: the
    // same sum as one load-add at a time, without a full HBM round trip per tile of a long segment
    for (int t = i0; t < i1; t += 8) {
      float u[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = w.tfirst[(size_t)min(t + j, i1 - 1) * D + dl];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t + j < i1) s += u[j];
    }
    q[v][lane] = s;
    __syncthreads();
    if (v == 0 && d < D) m_sumT[(size_t)k * D + d] += ((q[0][lane] + q[1][lane]) + q[2][lane]) + q[3][lane];
    __syncthreads();
  }
}

template <class T>
static int launch_ema_sums(const T* z, const int64_t* idx, float* m_sumT, float* n_sum, long long N, int D, int K,
                           void* ws, hipStream_t s) {
  const int nch = (int)((N + kSortChunk - 1) / kSortChunk), ntile = (int)((N + kSegTile - 1) / kSegTile);
  const SortWs w = sort_ws(ws, N, D, K);
  hipLaunchKernelGGL(vq_sort_count_kernel, dim3(nch), dim3(kSortChunk), (size_t)K * 4, s, idx, w, (int)N, K);
  VQA_LAUNCHED("vq_sort_count_kernel");
  hipLaunchKernelGGL(vq_sort_scan_kernel, dim3((K + 63) / 64), dim3(1024), 0, s, w, n_sum, nch, K);
  VQA_LAUNCHED("vq_sort_scan_kernel");
  hipLaunchKernelGGL(vq_sort_scatter_kernel, dim3(nch), dim3(kSortChunk), (size_t)(K + 1) * 4, s, idx, w, (int)N, K);
  VQA_LAUNCHED("vq_sort_scatter_kernel");
  hipLaunchKernelGGL(vq_seg_sum_kernel<T>, dim3((ntile + 3) / 4), dim3(256), 0, s, z, w, m_sumT, K, D);
  VQA_LAUNCHED("vq_seg_sum_kernel");
  hipLaunchKernelGGL(vq_seg_combine_kernel, dim3(K), dim3(256), 0, s, w, m_sumT, D);
  VQA_LAUNCHED("vq_seg_combine_kernel");
  return VQA_OK;
}

}  // namespace vqa

using namespace vqa;

extern "C" int vqa_vq_sqnorm(const float* E, float* e_sqnorm, int D, int K, vqa_stream_t stream) {
  VQA_ARG(E && e_sqnorm && D > 0 && K > 0, "vq_sqnorm: bad arguments");
  hipLaunchKernelGGL(vq_sqnorm_kernel, dim3((K + 3) / 4), dim3(256), 0, (hipStream_t)stream, E, e_sqnorm, D, K);
  VQA_LAUNCHED("vq_sqnorm_kernel");
  return VQA_OK;
}

template <class T>
static int launch_argmin(const void* z, const float* E, const float* esq, int64_t* idx, float* mind, long long N,
                         int D, int K, hipStream_t s) {
  const dim3 g((unsigned)((N + 127) / 128));
  switch (D) {
    case 4: hipLaunchKernelGGL((vq_argmin_mfma_kernel<T, 4>), g, dim3(256), 0, s, (const T*)z, E, esq, idx, mind, N, K); break;
    case 8: hipLaunchKernelGGL((vq_argmin_mfma_kernel<T, 8>), g, dim3(256), 0, s, (const T*)z, E, esq, idx, mind, N, K); break;
    case 16: hipLaunchKernelGGL((vq_argmin_mfma_kernel<T, 16>), g, dim3(256), 0, s, (const T*)z, E, esq, idx, mind, N, K); break;
    case 32: hipLaunchKernelGGL((vq_argmin_mfma_kernel<T, 32>), g, dim3(256), 0, s, (const T*)z, E, esq, idx, mind, N, K); break;
    case 64: hipLaunchKernelGGL((vq_argmin_mfma_kernel<T, 64>), g, dim3(256), 0, s, (const T*)z, E, esq, idx, mind, N, K); break;
    default:
      hipLaunchKernelGGL(vq_argmin_direct_kernel<T>, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, (const T*)z, E,
                         esq, idx, mind, N, D, K);
  }
  VQA_LAUNCHED("vq_argmin");
  return VQA_OK;
}

extern "C" int vqa_vq_argmin(const void* z, const float* E, const float* e_sqnorm, int64_t* idx, float* min_dist,
                             int64_t N, int D, int K, int dtype, vqa_stream_t stream) {
  VQA_ARG(z && E && e_sqnorm && idx, "vq_argmin: null pointer");
  VQA_ARG(N > 0 && D > 0 && K > 0, "vq_argmin: bad shape N=%lld D=%d K=%d", (long long)N, D, K);
  VQA_ARG(dtype == VQA_F32 || dtype == VQA_BF16, "vq_argmin: unknown dtype %d", dtype);
  if (dtype == VQA_BF16) return launch_argmin<bf16>(z, E, e_sqnorm, idx, min_dist, N, D, K, (hipStream_t)stream);
  return launch_argmin<float>(z, E, e_sqnorm, idx, min_dist, N, D, K, (hipStream_t)stream);
}

extern "C" int vqa_vq_split_bf16x3(const float* E, void* E3, int D, int K, vqa_stream_t stream) {
  VQA_ARG(E && E3 && D > 0 && K > 0, "vq_split_bf16x3: bad arguments");
  const long long n = (long long)D * K;
  hipLaunchKernelGGL(vq_split3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, E,
                     (bf16*)E3, D, K);
  VQA_LAUNCHED("vq_split3_kernel");
  return VQA_OK;
}

extern "C" int vqa_vq_argmin_split(const void* z, const void* E3, const float* e_sqnorm, int64_t* idx, float* min_dist,
                                   int64_t N, int D, int K, vqa_stream_t stream) {
  VQA_ARG(z && E3 && e_sqnorm && idx, "vq_argmin_split: null pointer");
  VQA_ARG(N > 0 && K > 0 && (D == 32 || D == 64), "vq_argmin_split: bad shape N=%lld D=%d K=%d (D in {32, 64})",
          (long long)N, D, K);
  // rows blocks of 256; small batches also split the codebook so that >= ~512 workgroups run
  const long long rb = (N + 255) / 256;
  int nsplit = (int)std::min<long long>(std::max<long long>(1, 512 / rb), (K + kSplitKC - 1) / kSplitKC);
  const int kspan = ((K + nsplit - 1) / nsplit + kSplitKC - 1) / kSplitKC * kSplitKC;
  nsplit = (K + kspan - 1) / kspan;
  const dim3 g((unsigned)rb, (unsigned)nsplit);
  hipStream_t s = (hipStream_t)stream;
  const unsigned nb = (unsigned)((N + 255) / 256);
  if (nsplit > 1) {
    hipLaunchKernelGGL(vq_argmin_init_kernel, dim3(nb), dim3(256), 0, s, idx, (long long)N);
    VQA_LAUNCHED("vq_argmin_init_kernel");
  }
  if (D == 64)
    hipLaunchKernelGGL(vq_argmin_split_kernel<64>, g, dim3(256), 0, s, (const bf16*)z, (const bf16*)E3, e_sqnorm, idx,
                       min_dist, (long long)N, K, kspan);
  else
    hipLaunchKernelGGL(vq_argmin_split_kernel<32>, g, dim3(256), 0, s, (const bf16*)z, (const bf16*)E3, e_sqnorm, idx,
                       min_dist, (long long)N, K, kspan);
  VQA_LAUNCHED("vq_argmin_split_kernel");
  if (nsplit > 1) {
    hipLaunchKernelGGL(vq_argmin_unpack_kernel, dim3(nb), dim3(256), 0, s, idx, min_dist, (long long)N);
    VQA_LAUNCHED("vq_argmin_unpack_kernel");
  }
  return VQA_OK;
}

extern "C" size_t vqa_vq_quantize_workspace(int64_t N, int D, int K, int dtype) {
  if (N < 1 || D < 1 || K < 1) return 0;
  (void)dtype;
  return align256((size_t)quantize_blocks((long long)N * D) * sizeof(float)) + sort_ws_bytes(N, D, K);
}

extern "C" int vqa_vq_quantize(const void* z, const float* ET, const int64_t* idx, void* q_st, float* commit_out,
                               float* m_sumT, float* n_sum, int64_t N, int D, int K, float beta, int dtype,
                               void* workspace, size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(z && ET && idx && q_st && commit_out, "vq_quantize: null pointer");
  VQA_ARG(!m_sumT == !n_sum, "vq_quantize: m_sumT and n_sum must both be set or both NULL");
  VQA_ARG(N > 0 && D > 0 && K > 0, "vq_quantize: bad shape");
  const int nb = quantize_blocks((long long)N * D);
  VQA_ARG(dtype == VQA_BF16 || dtype == VQA_F32, "vq_quantize: unknown dtype %d", dtype);
  VQA_ARG(N < (1ll << 31) - kSortChunk && D <= 1024 && K <= kMaxSortK, "vq_quantize: N=%lld D=%d K=%d out of range",
          (long long)N, D, K);
  VQA_ARG(workspace && ws_bytes >= vqa_vq_quantize_workspace(N, D, K, dtype), "vq_quantize: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  // q, straight-through output and the commitment partials (nparts <= nb: the workspace's partial rows)
  int nparts = nb;
  if (vq_vec8_ok(N, D, {z, ET, q_st})) {
    nparts = vec8_blocks(N, D);
    float* ws = (float*)workspace;
    const int n = (int)N;
    if (dtype == VQA_BF16 && D == 64)
      hipLaunchKernelGGL((vq_quantize8_kernel<bf16, 64>), dim3(nparts), dim3(256), 0, s, (const bf16*)z, ET, idx,
                         (bf16*)q_st, n, ws);
    else if (dtype == VQA_BF16)
      hipLaunchKernelGGL((vq_quantize8_kernel<bf16, 32>), dim3(nparts), dim3(256), 0, s, (const bf16*)z, ET, idx,
                         (bf16*)q_st, n, ws);
    else if (D == 64)
      hipLaunchKernelGGL((vq_quantize8_kernel<float, 64>), dim3(nparts), dim3(256), 0, s, (const float*)z, ET, idx,
                         (float*)q_st, n, ws);
    else
      hipLaunchKernelGGL((vq_quantize8_kernel<float, 32>), dim3(nparts), dim3(256), 0, s, (const float*)z, ET, idx,
                         (float*)q_st, n, ws);
    VQA_LAUNCHED("vq_quantize8_kernel");
  } else {
    if (dtype == VQA_BF16)
      hipLaunchKernelGGL(vq_quantize_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)z, ET, idx, (bf16*)q_st,
                         (long long)N, D, (float*)workspace);
    else
      hipLaunchKernelGGL(vq_quantize_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)z, ET, idx, (float*)q_st,
                         (long long)N, D, (float*)workspace);
    VQA_LAUNCHED("vq_quantize_kernel");
  }
  if (m_sumT) {
    void* sws = (char*)workspace + align256((size_t)nb * sizeof(float));
    const int rc = dtype == VQA_BF16
                       ? launch_ema_sums<bf16>((const bf16*)z, idx, m_sumT, n_sum, N, D, K, sws, s)
                       : launch_ema_sums<float>((const float*)z, idx, m_sumT, n_sum, N, D, K, sws, s);
    if (rc) return rc;
  }
  // beta * mean((q - z)^2) over N*D elements (VectorQuantizer.py:97-99)
  const float scale = (float)((double)beta / ((double)N * (double)D));
  hipLaunchKernelGGL(reduce_scalar_kernel, dim3(1), dim3(256), 0, s, (const float*)workspace, nparts, scale, commit_out);
  VQA_LAUNCHED("reduce_scalar_kernel");
  return VQA_OK;
}

extern "C" int vqa_vq_backward(const void* dq, const void* z, const float* ET, const int64_t* idx, void* dz,
                               float scale, int64_t N, int D, int dtype, vqa_stream_t stream) {
  VQA_ARG(dq && z && ET && idx && dz && N > 0 && D > 0, "vq_backward: bad arguments");
  const int nb = quantize_blocks((long long)N * D);
  hipStream_t s = (hipStream_t)stream;
  if ((dtype == VQA_BF16 || dtype == VQA_F32) && vq_vec8_ok(N, D, {dq, z, ET, dz})) {
    const int g = vec8_blocks(N, D), n = (int)N;
    if (dtype == VQA_BF16 && D == 64)
      hipLaunchKernelGGL((vq_backward8_kernel<bf16, 64>), dim3(g), dim3(256), 0, s, (const bf16*)dq, (const bf16*)z,
                         ET, idx, (bf16*)dz, scale, n);
    else if (dtype == VQA_BF16)
      hipLaunchKernelGGL((vq_backward8_kernel<bf16, 32>), dim3(g), dim3(256), 0, s, (const bf16*)dq, (const bf16*)z,
                         ET, idx, (bf16*)dz, scale, n);
    else if (D == 64)
      hipLaunchKernelGGL((vq_backward8_kernel<float, 64>), dim3(g), dim3(256), 0, s, (const float*)dq,
                         (const float*)z, ET, idx, (float*)dz, scale, n);
    else
      hipLaunchKernelGGL((vq_backward8_kernel<float, 32>), dim3(g), dim3(256), 0, s, (const float*)dq,
                         (const float*)z, ET, idx, (float*)dz, scale, n);
    VQA_LAUNCHED("vq_backward8_kernel");
    return VQA_OK;
  }
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(vq_backward_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)dq, (const bf16*)z, ET, idx,
                       (bf16*)dz, scale, (long long)N, D);
  else if (dtype == VQA_F32)
    hipLaunchKernelGGL(vq_backward_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dq, (const float*)z, ET,
                       idx, (float*)dz, scale, (long long)N, D);
  else
    VQA_ARG(false, "vq_backward: unknown dtype %d", dtype);
  VQA_LAUNCHED("vq_backward_kernel");
  return VQA_OK;
}

extern "C" int vqa_vq_reset_rows(const void* z, float* RT, int64_t N_local, int64_t row_offset, int64_t N_global,
                                 int D, int K, uint64_t seed, const int64_t* counter, int level, int dtype,
                                 vqa_stream_t stream) {
  VQA_ARG(z && RT && counter && N_local > 0 && N_global >= N_local && D > 0 && K > 0, "vq_reset_rows: bad arguments");
  VQA_ARG(row_offset >= 0 && row_offset + N_local <= N_global, "vq_reset_rows: bad row range");
  const long long total = (long long)K * D;
  const dim3 g((unsigned)((total + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(vq_reset_rows_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)z, RT, (long long)N_local,
                       (long long)row_offset, (long long)N_global, D, K, seed, counter, level);
  else if (dtype == VQA_F32)
    hipLaunchKernelGGL(vq_reset_rows_kernel<float>, g, dim3(256), 0, s, (const float*)z, RT, (long long)N_local,
                       (long long)row_offset, (long long)N_global, D, K, seed, counter, level);
  else
    VQA_ARG(false, "vq_reset_rows: unknown dtype %d", dtype);
  VQA_LAUNCHED("vq_reset_rows_kernel");
  return VQA_OK;
}

extern "C" int vqa_vq_ema_apply(float* E, float* ET, float* m_t, float* N_t, const float* m_sumT, const float* n_sum,
                                const float* RT, float gamma, float one_minus_gamma, float thresh, float* metrics,
                                int64_t* counter, int D, int K, vqa_stream_t stream) {
  return vqa_vq_ema_apply_derived(E, ET, m_t, N_t, m_sumT, n_sum, RT, gamma, one_minus_gamma, thresh, metrics, counter,
                                  nullptr, nullptr, D, K, stream);
}

extern "C" int vqa_vq_ema_apply_derived(float* E, float* ET, float* m_t, float* N_t, const float* m_sumT,
                                        const float* n_sum, const float* RT, float gamma, float one_minus_gamma,
                                        float thresh, float* metrics, int64_t* counter, float* e_sqnorm, void* E3,
                                        int D, int K, vqa_stream_t stream) {
  VQA_ARG(E && ET && m_t && N_t && m_sumT && n_sum && RT && counter, "vq_ema_apply: null pointer");
  VQA_ARG(D > 0 && D <= 64 && K > 0, "vq_ema_apply: supports D <= 64 (got D=%d)", D);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(vq_ema_apply_kernel, dim3((K + 3) / 4), dim3(256), 0, s, E, ET, m_t, N_t, m_sumT, n_sum, RT, gamma,
                     one_minus_gamma, thresh, counter, e_sqnorm, (bf16*)E3, D, K);
  VQA_LAUNCHED("vq_ema_apply_kernel");
  if (metrics) {
    hipLaunchKernelGGL(vq_metrics_kernel, dim3(1), dim3(256), 0, s, n_sum, (const float*)N_t, thresh, K, metrics);
    VQA_LAUNCHED("vq_metrics_kernel");
  }
  return VQA_OK;
}

extern "C" int64_t vqa_reset_perm_index(uint64_t seed, int64_t counter, int level, int64_t M, int64_t k) {
  if (M <= 0 || k < 0 || k >= M) return -1;
  return perm_index(perm_key(seed, counter, level), M, k);
}

extern "C" size_t vqa_embedding_bwd_workspace(int64_t N, int D, int K) {
  return N < 1 || D < 1 || K < 1 ? 0 : sort_ws_bytes(N, D, K);
}

extern "C" int vqa_embedding_bwd(const void* dy, const int64_t* idx, float* dtable, int64_t N, int D, int K, int dtype,
                                 void* workspace, size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(dy && idx && dtable && N > 0 && D > 0 && K > 0, "embedding_bwd: bad arguments");
  VQA_ARG(N < (1ll << 31) - kSortChunk && D <= 1024 && K <= kMaxSortK, "embedding_bwd: N=%lld D=%d K=%d out of range",
          (long long)N, D, K);
  VQA_ARG(dtype == VQA_BF16 || dtype == VQA_F32, "embedding_bwd: unknown dtype %d", dtype);
  VQA_ARG(workspace && ws_bytes >= sort_ws_bytes(N, D, K), "embedding_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  return dtype == VQA_BF16 ? launch_ema_sums<bf16>((const bf16*)dy, idx, dtable, nullptr, N, D, K, workspace, s)
                           : launch_ema_sums<float>((const float*)dy, idx, dtable, nullptr, N, D, K, workspace, s);
}
