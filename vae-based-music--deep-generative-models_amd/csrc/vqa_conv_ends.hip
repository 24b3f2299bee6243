// vqa_conv_ends.hip — the waveform-end convolution with ONE output channel (gfx950):
//   encdec.py:148  Decoder output Conv1D(output_dim=1, 3, padding="same") over the 64-channel decoder
//                  output — forward and its GradientTape backward (vqvae.py:143).
//
// With O = 1 the conv is a row-dot: p_k[r] = sum_c act(x[r][c]) w[k][c] per input row r and tap k, and
// y[t] = b + sum_k p_k[t + k*D - P]. Each input row is read once as C/VEC lanes x 16 bytes (fully coalesced
// HBM streaming); the per-row dot products are reduced across those lanes with shuffles and combined
// through LDS. The backward reads x once and writes dx once, computing the weight gradient from the same
// registers: dx[r][c] = sum_k dy[r - k*D + P] w[k][c], dW[k][c] += act(x[r][c]) dy[r - k*D + P]
// (per-workgroup fp32 partials, reduced in a fixed order by vqa_reduce_partials: deterministic).
#include "vqa_common.h"

namespace vqa {

template <class T> struct Vec16;
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void unpack(uint4 u, float* v) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    bf16x8 x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
    return __builtin_bit_cast(uint4, x);
  }
};
template <> struct Vec16<float> {
  static constexpr int N = 4;
  static __device__ __forceinline__ void unpack(uint4 u, float* v) {
    v[0] = __uint_as_float(u.x);
    v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z);
    v[3] = __uint_as_float(u.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    return uint4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  }
};

struct Co1Args {
  const void* x;      // (B, T, C) conv input
  const float* w;     // (K, C, 1)
  const float* bias;  // (1) or null
  const void* resid;  // fwd: y-side residual (B, T); bwd: x-side residual (B, T, C)
  void* y;            // fwd output (B, T)
  const void* dy;     // bwd: (B, T)
  void* dx;           // bwd: (B, T, C)
  float* wpart;       // bwd: [nwg][K*C + 1]
  int B, T, K, D, P, flags;
  int ntb, ntiles, tpw;
};

constexpr int kCo1TB = 256;  // rows per tile

template <class TX, int C> constexpr int co1_rpp() { return 256 / (C / Vec16<TX>::N); }

// ---- forward: one 256-row output tile per workgroup ----
template <class TX, class TY, int C>
__global__ __launch_bounds__(256) void co1_fwd_kernel(Co1Args a) {
  constexpr int VEC = Vec16<TX>::N, G = C / VEC, RPP = co1_rpp<TX, C>(), TB = kCo1TB;
  constexpr int NP = TB / RPP + 1;  // input passes incl. the (K-1)*D <= RPP halo rows
  __shared__ float ps[4 * (TB + RPP)];
  const int n = blockIdx.x / a.ntb, t0 = (blockIdx.x - n * a.ntb) * TB;
  const int rows_in = TB + (a.K - 1) * a.D, r0 = t0 - a.P;
  const int g = threadIdx.x % G, rr = threadIdx.x / G;
  const TX* X = (const TX*)a.x + (size_t)n * a.T * C + g * VEC;
  uint4 xv[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int lr = p * RPP + rr, r = r0 + lr;
    xv[p] = (lr < rows_in && r >= 0 && r < a.T) ? *(const uint4*)(X + (size_t)r * C) : uint4{0u, 0u, 0u, 0u};
  }
  float wr[4][VEC];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) wr[k][j] = k < a.K ? a.w[k * C + g * VEC + j] : 0.f;
  const bool relu = a.flags & VQA_PRE_RELU;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    float v[VEC];
    Vec16<TX>::unpack(xv[p], v);
    float pk[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float xj = relu ? fmaxf(v[j], 0.f) : v[j];
#pragma unroll
      for (int k = 0; k < 4; ++k) pk[k] += xj * wr[k][j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) pk[k] = xl::grp_sum<G>(pk[k]);
    const int lr = p * RPP + rr;
    if (g == 0 && lr < rows_in)
#pragma unroll
      for (int k = 0; k < 4; ++k) ps[k * (TB + RPP) + lr] = pk[k];
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= a.T) return;
  float acc = 0.f;
  for (int k = 0; k < a.K; ++k) acc += ps[k * (TB + RPP) + threadIdx.x + k * a.D];
  float v = acc;
  if (a.bias) v = v + a.bias[0];
  const size_t oi = (size_t)n * a.T + t;
  if (a.flags & VQA_ADD_RESIDUAL) v = ld((const TY*)a.resid + oi) + v;
  st((TY*)a.y + oi, v);
}

// ---- fused backward: persistent over 256-row tiles; dx and (WGRAD) the weight-gradient partials ----
// x is the conv input (WGRAD) or the ReLU' mask tensor (data gradient only; null without a mask); with
// VQA_PRE_RELU, dx = (x > 0) ? dx : 0 and dW uses relu(x). dx is the same arithmetic in both modes.
template <class TX, class TG, int C, bool WGRAD>
__global__ __launch_bounds__(256) void co1_bwd_kernel(Co1Args a) {
  constexpr int VEC = Vec16<TX>::N, G = C / VEC, RPP = co1_rpp<TX, C>(), TB = kCo1TB, NP = TB / RPP;
  __shared__ float dys[TB + 3 * 64];
  __shared__ float red[4];
  extern __shared__ float wsum[];  // [256][4 * VEC] thread partials for the final reduction
  const int g = threadIdx.x % G, rr = threadIdx.x / G;
  const bool relu = a.flags & VQA_PRE_RELU, do_res = a.flags & VQA_ADD_RESIDUAL;
  const bool need_x = WGRAD || relu;
  const int halo = (a.K - 1) * a.D;
  float wr[4][VEC], wacc[4][VEC];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      wr[k][j] = k < a.K ? a.w[k * C + g * VEC + j] : 0.f;
      wacc[k][j] = 0.f;
    }
  float dbacc = 0.f;
  const int tbeg = blockIdx.x * a.tpw, tend = min(a.ntiles, tbeg + a.tpw);
  for (int tile = tbeg; tile < tend; ++tile) {
    const int n = tile / a.ntb, r0 = (tile - n * a.ntb) * TB;
    const TX* X = (const TX*)a.x + (size_t)n * a.T * C + g * VEC;
    uint4 xv[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int r = r0 + p * RPP + rr;
      xv[p] = (need_x && r < a.T) ? *(const uint4*)(X + (size_t)r * C) : uint4{0u, 0u, 0u, 0u};
    }
    // dy window: local i <-> t = r0 - halo + P + i, i in [0, TB + halo)
    const TG* DY = (const TG*)a.dy + (size_t)n * a.T;
    for (int i = threadIdx.x; i < TB + halo; i += 256) {
      const int t = r0 - halo + a.P + i;
      dys[i] = (t >= 0 && t < a.T) ? ld(DY + t) : 0.f;
    }
    {
      const int t = r0 + threadIdx.x;
      if (t < a.T) dbacc += ld(DY + t);
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int lr = p * RPP + rr, r = r0 + lr;
      float v[VEC], dv[VEC], dk[4];
      Vec16<TX>::unpack(xv[p], v);
#pragma unroll
      for (int k = 0; k < 4; ++k) dk[k] = k < a.K ? dys[lr + halo - k * a.D] : 0.f;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += dk[k] * wr[k][j];
        const float xa = relu ? fmaxf(v[j], 0.f) : v[j];
        dv[j] = (relu && !(v[j] > 0.f)) ? 0.f : s;
        if constexpr (WGRAD) {
#pragma unroll
          for (int k = 0; k < 4; ++k) wacc[k][j] += xa * dk[k];
        }
      }
      if (r < a.T) {
        const size_t off = ((size_t)n * a.T + r) * C + g * VEC;
        if (do_res) {
          float rv[VEC];
          Vec16<TX>::unpack(*(const uint4*)((const TX*)a.resid + off), rv);
#pragma unroll
          for (int j = 0; j < VEC; ++j) dv[j] = rv[j] + dv[j];
        }
        *(uint4*)((TX*)a.dx + off) = Vec16<TX>::pack(dv);
      }
    }
    __syncthreads();
  }
  if constexpr (!WGRAD) return;
  // workgroup partial: dW[k][c] (c = g*VEC + j) summed over rr in a fixed order, then db
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) wsum[threadIdx.x * 4 * VEC + k * VEC + j] = wacc[k][j];
  __syncthreads();
  float* out = a.wpart + (size_t)blockIdx.x * (a.K * C + 1);
  for (int e = threadIdx.x; e < a.K * C; e += 256) {
    const int k = e / C, c = e - k * C, gg = c / VEC, j = c - gg * VEC;
    float s = 0.f;
    for (int q = 0; q < RPP; ++q) s += wsum[(q * G + gg) * 4 * VEC + k * VEC + j];
    out[e] = s;
  }
  const float db = block_sum_256(dbacc, red);
  if (threadIdx.x == 0) out[a.K * C] = db;
}

static int co1_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}
constexpr int kCo1PerCU = 4;

bool co1_supported(int C, int O, int K, int S, int D, int dtype, int flags) {
  if (O != 1 || S != 1 || K < 1 || K > 4 || !(C == 32 || C == 64)) return false;
  const bool xf = dtype == VQA_F32 || (flags & VQA_X_F32);
  const int rpp = 256 / (C / (xf ? 4 : 8));
  return (K - 1) * D <= rpp && (K - 1) * D <= 3 * 64;
}

size_t co1_bwd_workspace(int C, int K) { return (size_t)co1_cus() * kCo1PerCU * (K * C + 1) * sizeof(float); }

template <class TX, class TY, int C>
static int co1_fwd_launch(const Co1Args& a, hipStream_t s) {
  hipLaunchKernelGGL((co1_fwd_kernel<TX, TY, C>), dim3(a.B * a.ntb), dim3(256), 0, s, a);
  VQA_LAUNCHED("co1_fwd_kernel");
  return VQA_OK;
}

template <class TX, class TG, int C>
static int co1_bwd_launch(const Co1Args& a, hipStream_t s) {
  const dim3 grid((a.ntiles + a.tpw - 1) / a.tpw);
  if (!a.wpart) {
    hipLaunchKernelGGL((co1_bwd_kernel<TX, TG, C, false>), grid, dim3(256), 0, s, a);
    VQA_LAUNCHED("co1_bwd_kernel");
    return VQA_OK;
  }
  const size_t lds = (size_t)256 * 4 * Vec16<TX>::N * sizeof(float);
  hipLaunchKernelGGL((co1_bwd_kernel<TX, TG, C, true>), grid, dim3(256), lds, s, a);
  VQA_LAUNCHED("co1_bwd_kernel");
  return VQA_OK;
}

int co1_fwd(const void* x, const float* w, const float* bias, const void* resid, void* y, int B, int T, int C, int K,
            int D, int P, int flags, int dtype, hipStream_t s) {
  Co1Args a{x, w, bias, resid, y, nullptr, nullptr, nullptr, B, T, K, D, P, flags, 0, 0, 0};
  a.ntb = (T + kCo1TB - 1) / kCo1TB;
  const bool xf = dtype == VQA_F32 || (flags & VQA_X_F32);
  const bool yf = dtype == VQA_F32 || (flags & VQA_Y_F32);
  if (C == 64) {
    if (xf) return yf ? co1_fwd_launch<float, float, 64>(a, s) : co1_fwd_launch<float, bf16, 64>(a, s);
    return yf ? co1_fwd_launch<bf16, float, 64>(a, s) : co1_fwd_launch<bf16, bf16, 64>(a, s);
  }
  if (xf) return yf ? co1_fwd_launch<float, float, 32>(a, s) : co1_fwd_launch<float, bf16, 32>(a, s);
  return yf ? co1_fwd_launch<bf16, float, 32>(a, s) : co1_fwd_launch<bf16, bf16, 32>(a, s);
}

// ws == NULL: data gradient only (x = the ReLU' mask or NULL). Else also the weight-gradient partials;
// *nparts receives their row count.
int co1_bwd(const void* dy, const float* w, const void* x, const void* resid, void* dx, int B, int T, int C, int K,
            int D, int P, int flags, int dtype, void* ws, int* nparts, hipStream_t s) {
  Co1Args a{x, w, nullptr, resid, nullptr, dy, dx, (float*)ws, B, T, K, D, P, flags, 0, 0, 0};
  a.ntb = (T + kCo1TB - 1) / kCo1TB;
  a.ntiles = a.ntb * B;
  int nwg = co1_cus() * kCo1PerCU;
  if (nwg > a.ntiles) nwg = a.ntiles;
  a.tpw = (a.ntiles + nwg - 1) / nwg;
  if (nparts) *nparts = (a.ntiles + a.tpw - 1) / a.tpw;
  const bool xf = dtype == VQA_F32 || (flags & VQA_X_F32);
  const bool gf = dtype == VQA_F32 || (flags & VQA_Y_F32);
  if (C == 64) {
    if (xf) return gf ? co1_bwd_launch<float, float, 64>(a, s) : co1_bwd_launch<float, bf16, 64>(a, s);
    return gf ? co1_bwd_launch<bf16, float, 64>(a, s) : co1_bwd_launch<bf16, bf16, 64>(a, s);
  }
  if (xf) return gf ? co1_bwd_launch<float, float, 32>(a, s) : co1_bwd_launch<float, bf16, 32>(a, s);
  return gf ? co1_bwd_launch<bf16, float, 32>(a, s) : co1_bwd_launch<bf16, bf16, 32>(a, s);
}

}  // namespace vqa
