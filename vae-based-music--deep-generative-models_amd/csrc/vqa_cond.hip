// vqa_cond.hip — the non-conv layers of the upper-level conditioner (gfx950).
//
// Replaces the Keras layers of src/conditioner/conditioners.py:42-72 (ConditionerNet.model):
//   layers.Embedding(bins, width)                 -> embed_fwd_kernel (row gather; the backward is the
//                                                    deterministic segment sum of vqa_embedding_bwd, vqa_vq.hip)
//   layers.LayerNormalization(axis=-1, eps=1e-6)  -> layernorm_fwd_kernel / layernorm_bwd_kernel
// The DecoderConvBlock between them runs on the conv / residual-block kernels.
#include "vqa_common.h"
#include <algorithm>

namespace vqa {

// out[n][:] = table[idx[n]][:] (fp32 table -> activation dtype); an index outside [0, K) gives a zero row (TF's
// GPU embedding_lookup semantics). One thread per (row, 4 channels).
template <class T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const float* table, const int64_t* idx, T* out, long long N,
                                                       int D, int K) {
  const long long total = N * (D / 4);
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long n = e / (D / 4);
    const int d = (int)(e - n * (D / 4)) * 4;
    const int64_t k = idx[n];
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (k >= 0 && k < K) v = *(const f32x4*)(table + k * D + d);
    st4(out + n * D + d, v);
  }
}

// ---- LayerNormalization over the last axis (keras, TF 2.7: tf.nn.moments + tf.nn.batch_normalization) ----
// y = (x - mean) * rsqrt(var + eps) * gamma + beta, biased variance, fp32 statistics. One wave per row, lane
// owns channels lane, lane + 64, ... (C <= 64 * LC); wave reductions in a fixed butterfly order.
constexpr int kLnMaxLC = 16;  // C <= 1024

__device__ __forceinline__ float wave_sum(float v) { return warp_sum(v); }

template <class T, int LC>
__device__ __forceinline__ void ln_row_stats(const T* xr, int C, float (&xv)[LC], float& mean, float& inv, float eps) {
  const int lane = threadIdx.x & 63;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LC; ++i) {
    const int c = lane + 64 * i;
    xv[i] = c < C ? ld(xr + c) : 0.f;
    s += xv[i];
  }
  mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LC; ++i) {
    const int c = lane + 64 * i;
    const float dlt = c < C ? xv[i] - mean : 0.f;
    q += dlt * dlt;
  }
  inv = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
}

template <class T, int LC>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const T* x, const float* gamma, const float* beta, T* y,
                                                           long long rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  for (long long r = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); r < rows; r += (long long)gridDim.x * 4) {
    float xv[LC], mean, inv;
    ln_row_stats<T, LC>(x + r * C, C, xv, mean, inv, eps);
#pragma unroll
    for (int i = 0; i < LC; ++i) {
      const int c = lane + 64 * i;
      if (c < C) st(y + r * C + c, (xv[i] - mean) * inv * gamma[c] + beta[c]);
    }
  }
}

// dx = inv * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; dgamma += dy * xhat, dbeta += dy per channel,
// accumulated over the workgroup's contiguous row range, combined over its 4 waves in LDS in wave order ->
// one partial row [dgamma (C) | dbeta (C)] per workgroup (reduced in a fixed order by vqa_reduce_partials).
template <class T, int LC>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* x, const T* dy, const float* gamma, T* dx,
                                                           float* part, long long rows, int C, float eps,
                                                           long long rows_per_wg) {
  extern __shared__ float red[];  // [4][2C]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float gg[LC], gb[LC];
#pragma unroll
  for (int i = 0; i < LC; ++i) gg[i] = gb[i] = 0.f;
  const long long r0 = (long long)blockIdx.x * rows_per_wg, r1 = std::min(rows, r0 + rows_per_wg);
  for (long long r = r0 + wave; r < r1; r += 4) {
    float xv[LC], mean, inv;
    ln_row_stats<T, LC>(x + r * C, C, xv, mean, inv, eps);
    float g[LC], sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < LC; ++i) {
      const int c = lane + 64 * i;
      const float d = c < C ? ld(dy + r * C + c) : 0.f;
      xv[i] = (xv[i] - mean) * inv;  // xhat
      g[i] = c < C ? d * gamma[c] : 0.f;
      sg += g[i];
      sgx += g[i] * xv[i];
      gg[i] += d * xv[i];
      gb[i] += d;
    }
    const float mg = wave_sum(sg) / (float)C, mgx = wave_sum(sgx) / (float)C;
#pragma unroll
    for (int i = 0; i < LC; ++i) {
      const int c = lane + 64 * i;
      if (c < C) st(dx + r * C + c, inv * ((g[i] - mg) - xv[i] * mgx));
    }
  }
#pragma unroll
  for (int i = 0; i < LC; ++i) {
    const int c = lane + 64 * i;
    if (c < C) {
      red[wave * 2 * C + c] = gg[i];
      red[wave * 2 * C + C + c] = gb[i];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C; e += 256)
    part[(size_t)blockIdx.x * 2 * C + e] = ((red[e] + red[2 * C + e]) + red[4 * C + e]) + red[6 * C + e];
}

// Vectorised forms for C = 8R (R = lanes per row, a power of two <= 64): each lane owns 8 consecutive channels
// (one 16-byte bf16 access), a wave holds 64/R rows at once, row statistics by R-lane butterflies (fixed order).
template <int R>
__device__ __forceinline__ float grp_sum_r(float v) { return xl::grp_sum<R>(v); }

template <class T> __device__ __forceinline__ void ld8v(const T* p, float (&v)[8]);
template <> __device__ __forceinline__ void ld8v<bf16>(const bf16* p, float (&v)[8]) {
  const bf16x8 b = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)b[i];
}
template <> __device__ __forceinline__ void ld8v<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
template <class T> __device__ __forceinline__ void st8v(T* p, const float (&v)[8]);
template <> __device__ __forceinline__ void st8v<bf16>(bf16* p, const float (&v)[8]) {
  bf16x8 b;
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (bf16)v[i];
  *(bf16x8*)p = b;
}
template <> __device__ __forceinline__ void st8v<float>(float* p, const float (&v)[8]) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

template <class T, int R>
__global__ __launch_bounds__(256) void layernorm8_fwd_kernel(const T* x, const float* gamma, const float* beta, T* y,
                                                            long long rows, float eps) {
  constexpr int C = 8 * R, RPW = 64 / R;
  const int lane = threadIdx.x & 63, sub = lane / R, c0 = 8 * (lane % R);
  float gm[8], bt[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { gm[i] = gamma[c0 + i]; bt[i] = beta[c0 + i]; }
  const long long rstep = (long long)gridDim.x * 4 * RPW;
  for (long long r = ((long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * RPW + sub; r < rows; r += rstep) {
    float v[8];
    ld8v(x + r * C + c0, v);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    const float mean = grp_sum_r<R>(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) q += (v[i] - mean) * (v[i] - mean);
    const float inv = 1.0f / sqrtf(grp_sum_r<R>(q) / (float)C + eps);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (v[i] - mean) * inv * gm[i] + bt[i];
    st8v(y + r * C + c0, v);
  }
}

template <class T, int R>
__global__ __launch_bounds__(256) void layernorm8_bwd_kernel(const T* x, const T* dy, const float* gamma, T* dx,
                                                            float* part, long long rows, float eps,
                                                            long long rows_per_wg) {
  constexpr int C = 8 * R, RPW = 64 / R;
  extern __shared__ float red[];  // [4][2C]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), sub = lane / R, c0 = 8 * (lane % R);
  float gm[8], gg[8], gb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { gm[i] = gamma[c0 + i]; gg[i] = gb[i] = 0.f; }
  const long long r0 = (long long)blockIdx.x * rows_per_wg, r1 = std::min(rows, r0 + rows_per_wg);
  for (long long r = r0 + wave * RPW + sub; r < r1; r += 4 * RPW) {
    float v[8], d[8];
    ld8v(x + r * C + c0, v);
    ld8v(dy + r * C + c0, d);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
    const float mean = grp_sum_r<R>(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) q += (v[i] - mean) * (v[i] - mean);
    const float inv = 1.0f / sqrtf(grp_sum_r<R>(q) / (float)C + eps);
    float g[8], sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] = (v[i] - mean) * inv;  // xhat
      g[i] = d[i] * gm[i];
      sg += g[i];
      sgx += g[i] * v[i];
      gg[i] += d[i] * v[i];
      gb[i] += d[i];
    }
    const float mg = grp_sum_r<R>(sg) / (float)C, mgx = grp_sum_r<R>(sgx) / (float)C;
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = inv * ((g[i] - mg) - v[i] * mgx);
    st8v(dx + r * C + c0, g);
  }
  // combine the wave's row groups (lanes with the same channels: xor R, 2R, ...), then the 4 waves in order
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    gg[i] = xl::grp_combine<R>(gg[i]);
    gb[i] = xl::grp_combine<R>(gb[i]);
  }
  if (sub == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[wave * 2 * C + c0 + i] = gg[i];
      red[wave * 2 * C + C + c0 + i] = gb[i];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * C; e += 256)
    part[(size_t)blockIdx.x * 2 * C + e] = ((red[e] + red[2 * C + e]) + red[4 * C + e]) + red[6 * C + e];
}

template <class T, int R>
static int launch_ln8(bool fwd, const void* x, const void* dy, const float* gamma, const float* beta, void* out,
                      float* part, long long rows, float eps, int nwg, hipStream_t s) {
  constexpr int C = 8 * R, RPW = 64 / R;
  if (fwd) {
    const unsigned g = (unsigned)std::min<long long>((rows + 4 * RPW - 1) / (4 * RPW), 2048);
    hipLaunchKernelGGL((layernorm8_fwd_kernel<T, R>), dim3(g), dim3(256), 0, s, (const T*)x, gamma, beta, (T*)out,
                       rows, eps);
    VQA_LAUNCHED("layernorm8_fwd_kernel");
  } else {
    const long long rpw = (rows + nwg - 1) / nwg;
    hipLaunchKernelGGL((layernorm8_bwd_kernel<T, R>), dim3(nwg), dim3(256), (size_t)8 * C * sizeof(float), s,
                       (const T*)x, (const T*)dy, gamma, (T*)out, part, rows, eps, rpw);
    VQA_LAUNCHED("layernorm8_bwd_kernel");
  }
  return VQA_OK;
}

static int ln_wgs(long long rows) {
  long long w = (rows + 63) / 64;  // >= 16 rows per wave
  return (int)std::max<long long>(1, std::min<long long>(w, 512));
}

template <class T, int LC>
static int launch_ln(bool fwd, const void* x, const void* dy, const float* gamma, const float* beta, void* out,
                     float* part, long long rows, int C, float eps, int nwg, hipStream_t s) {
  if (fwd) {
    const unsigned g = (unsigned)std::min<long long>((rows + 3) / 4, 4096);
    hipLaunchKernelGGL((layernorm_fwd_kernel<T, LC>), dim3(g), dim3(256), 0, s, (const T*)x, gamma, beta, (T*)out,
                       rows, C, eps);
    VQA_LAUNCHED("layernorm_fwd_kernel");
  } else {
    const long long rpw = (rows + nwg - 1) / nwg;
    hipLaunchKernelGGL((layernorm_bwd_kernel<T, LC>), dim3(nwg), dim3(256), (size_t)8 * C * sizeof(float), s,
                       (const T*)x, (const T*)dy, gamma, (T*)out, part, rows, C, eps, rpw);
    VQA_LAUNCHED("layernorm_bwd_kernel");
  }
  return VQA_OK;
}

template <class T>
static int dispatch_ln(bool fwd, const void* x, const void* dy, const float* gamma, const float* beta, void* out,
                       float* part, long long rows, int C, float eps, int nwg, hipStream_t s) {
  if (C == 128) return launch_ln8<T, 16>(fwd, x, dy, gamma, beta, out, part, rows, eps, nwg, s);
  if (C == 256) return launch_ln8<T, 32>(fwd, x, dy, gamma, beta, out, part, rows, eps, nwg, s);
  if (C == 64) return launch_ln8<T, 8>(fwd, x, dy, gamma, beta, out, part, rows, eps, nwg, s);
  const int lc = (C + 63) / 64;
  if (lc <= 1) return launch_ln<T, 1>(fwd, x, dy, gamma, beta, out, part, rows, C, eps, nwg, s);
  if (lc <= 2) return launch_ln<T, 2>(fwd, x, dy, gamma, beta, out, part, rows, C, eps, nwg, s);
  if (lc <= 4) return launch_ln<T, 4>(fwd, x, dy, gamma, beta, out, part, rows, C, eps, nwg, s);
  if (lc <= 8) return launch_ln<T, 8>(fwd, x, dy, gamma, beta, out, part, rows, C, eps, nwg, s);
  return launch_ln<T, kLnMaxLC>(fwd, x, dy, gamma, beta, out, part, rows, C, eps, nwg, s);
}

}  // namespace vqa

using namespace vqa;

extern "C" int vqa_embedding_fwd(const float* table, const int64_t* idx, void* out, int64_t N, int D, int K, int dtype,
                                 vqa_stream_t stream) {
  VQA_ARG(table && idx && out && N > 0 && D > 0 && K > 0, "embedding_fwd: bad arguments");
  VQA_ARG(D % 4 == 0, "embedding_fwd: width %d not a multiple of 4", D);
  const long long total = (long long)N * (D / 4);
  const unsigned g = (unsigned)std::min<long long>((total + 255) / 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(embed_fwd_kernel<bf16>, dim3(g), dim3(256), 0, s, table, idx, (bf16*)out, (long long)N, D, K);
  else if (dtype == VQA_F32)
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3(g), dim3(256), 0, s, table, idx, (float*)out, (long long)N, D, K);
  else
    VQA_ARG(false, "embedding_fwd: unknown dtype %d", dtype);
  VQA_LAUNCHED("embed_fwd_kernel");
  return VQA_OK;
}

extern "C" int vqa_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, int64_t rows, int C,
                                 float eps, int dtype, vqa_stream_t stream) {
  VQA_ARG(x && gamma && beta && y && rows > 0 && C > 0 && C <= 64 * kLnMaxLC, "layernorm_fwd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == VQA_BF16) return dispatch_ln<bf16>(true, x, nullptr, gamma, beta, y, nullptr, rows, C, eps, 0, s);
  VQA_ARG(dtype == VQA_F32, "layernorm_fwd: unknown dtype %d", dtype);
  return dispatch_ln<float>(true, x, nullptr, gamma, beta, y, nullptr, rows, C, eps, 0, s);
}

extern "C" size_t vqa_layernorm_bwd_workspace(int64_t rows, int C) {
  if (rows < 1 || C < 1) return 0;
  return (size_t)ln_wgs(rows) * 2 * (size_t)C * sizeof(float);
}

extern "C" int vqa_layernorm_bwd(const void* x, const void* dy, const float* gamma, void* dx, float* dgamma,
                                 float* dbeta, int64_t rows, int C, float eps, int dtype, void* workspace,
                                 size_t ws_bytes, vqa_partials_desc* desc, vqa_stream_t stream) {
  VQA_ARG(x && dy && gamma && dx && dgamma && dbeta && rows > 0 && C > 0 && C <= 64 * kLnMaxLC,
          "layernorm_bwd: bad arguments");
  VQA_ARG(workspace && ws_bytes >= vqa_layernorm_bwd_workspace(rows, C), "layernorm_bwd: workspace too small");
  const int nwg = ln_wgs(rows);
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if (dtype == VQA_BF16)
    rc = dispatch_ln<bf16>(false, x, dy, gamma, nullptr, dx, (float*)workspace, rows, C, eps, nwg, s);
  else if (dtype == VQA_F32)
    rc = dispatch_ln<float>(false, x, dy, gamma, nullptr, dx, (float*)workspace, rows, C, eps, nwg, s);
  else
    VQA_ARG(false, "layernorm_bwd: unknown dtype %d", dtype);
  if (rc) return rc;
  const vqa_partials_desc d{(const float*)workspace, dgamma, dbeta, nwg, 2 * C, C, 0};
  if (desc) {
    *desc = d;
    return VQA_OK;
  }
  return vqa_reduce_partials(&d, 1, stream);
}
