// vqa_resblock.hip — the fused residual block of the dilated ResNet stacks (gfx950).
//
// Replaces resnet.py:7-29 ResnetConv1DBlock for C = 32 channels:
//     h = conv_a(relu(x)) + b_a       (k3, dilation d, SAME)
//     y = x + conv_b(relu(h)) + b_b   (k3, dilation 1, SAME)
// and its GradientTape backward (vqvae.py:143).
//
// Forward: one workgroup tile = 128 output rows; x (with a d+1 row halo) is staged once in LDS, h is
// computed for the 144 rows conv_b needs and kept in LDS (relu'd, in the activation dtype — the same
// rounding as the unfused path's h tensor), then y = x + conv_b(relu h) is written. HBM traffic: x read,
// y written — h never leaves the chip.
// Backward (recompute): h is recomputed from x instead of being saved, so the block's backward reads dy
// and x and writes dx only:
//     dh = conv_b^T(dy) * (h > 0)            over rows [t0-d, t0+128+d) (conv_a^T's halo)
//     dx = dy + conv_a^T(dh) * (x > 0)       over the tile's 128 rows
//     dW_b += relu(h)^T dy,  dW_a += relu(x)^T dh (shifted per tap), db_b += sum dy, db_a += sum dh
// the weight gradients accumulate in registers across the persistent workgroup's tiles and leave as one
// fp32 partial row per workgroup (reduced in a fixed order by vqa_reduce_partials: deterministic).
// All products are MFMA (bf16 16x16x32 or the exact fp32 16x16x4 in parity mode), fp32 accumulation.
#include "vqa_common.h"
#include "vqa_mfma.h"
#include <stdlib.h>

namespace vqa {

constexpr int RC = 32;    // block width (residual_width of the SMALL_VQ_VAE configs)
constexpr int RTM = 128;  // output rows per tile
constexpr int RMAXD = 32; // largest dilation the LDS plan covers (the model uses 1, 3, 9, 27)

struct ResArgs {
  const void* x;   // block input (B, T, C)
  const void* dy;  // backward: d loss / d y
  void* y;         // forward: y; backward: dx
  void* h;         // forward, optional: relu(h) of the tile's own rows (B, T, C)
  const float* wa;
  const float* ba;
  const float* wb;
  const float* bb;
  float* part_a;  // backward: [nwg][3*C*C + C] (dW_a | db_a)
  float* part_b;  // backward: [nwg][3*C*C + C] (dW_b | db_b)
  int B, T, d;
  int ntm, ntiles, tpw;
  int skip;  // development ablation only (VQA_RESBLOCK_SKIP): bit p skips backward phase p (outputs wrong)
};

template <class T> constexpr int rs_stride() { return RC + lds_pad<T>(); }
constexpr int round16(int v) { return (v + 15) & ~15; }

// weights -> LDS image [3][32][WS]: TRANSPOSE=true gives [k][o][c] (A operand of a forward conv),
// false the Keras layout [k][c][o] (A operand of the transposed conv)
template <class T, bool TRANSPOSE>
__device__ __forceinline__ void stage_wimg(T* img, const float* w) {
  constexpr int WS = rs_stride<T>();
  for (int e = threadIdx.x; e < 3 * RC * RC; e += 256) {
    const int k = e / (RC * RC), rem = e - k * RC * RC, r = rem / RC, c = rem - r * RC;
    // e enumerates the Keras layout: w[k][r][c] with r = input channel, c = output channel
    if (TRANSPOSE) img[(k * RC + c) * WS + r] = (T)w[e];
    else img[(k * RC + r) * WS + c] = (T)w[e];
  }
}

// The same through a per-item buffer descriptor: the hardware range check returns zeros for rows outside
// [0, T) (SAME padding; negative offsets wrap past num_records), so a chunk costs one add and one
// buffer_load, and the per-thread chunk offsets are fixed for the launch.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs_rsrc(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kRsOOB = -0x40000000;  // chunk offset that stays out of range for any row base

template <class T, int PV>
struct Rows32Buf {
  static constexpr int VEC = 16 / (int)sizeof(T), CPR = RC / VEC, ROWB = RC * (int)sizeof(T);
  uint4 v[PV];
  int goff[PV], loff[PV];  // byte offset from the tile's first row; LDS element offset (-1: none)
  __device__ __forceinline__ void init(int nrows) {
    constexpr int XS = RC + 16 / (int)sizeof(T);
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = threadIdx.x + i * 256;
      const int rr = e / CPR, q = e - rr * CPR;
      const bool in = e < nrows * CPR;
      goff[i] = in ? rr * ROWB + q * 16 : kRsOOB;
      loff[i] = in ? rr * XS + q * VEC : -1;
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int row0) {
    const int base = row0 * ROWB;
#pragma unroll
    for (int i = 0; i < PV; ++i)
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, goff[i] + base, 0, 0));
  }
  __device__ __forceinline__ void store(T* dst) const {
#pragma unroll
    for (int i = 0; i < PV; ++i)
      if (loff[i] >= 0) *(uint4*)(dst + loff[i]) = v[i];
  }
};

// chunks per thread for the largest tile of a launch (rows <= 256 at RMAXD)
template <class T> constexpr int rs_pv() { return sizeof(T) == 2 ? 4 : 8; }

// acc[mt] (16 output channels each) for 16 output rows: out[row][o] = sum_k sum_c img[k][o][c] *
// act(in[row_base + k*tap_step + row][c]); lane: row = lane & 15, channels mt*16 + 4*(lane>>4) + 0..3.
// Tap order k = 0, 1, 2 then channel blocks — the accumulation order of the unfused gather kernels.
template <class T, bool RELU_IN>
__device__ __forceinline__ void conv_rows16(f32x4 (&acc)[2], const T* img, const T* in, int row_base, int tap_step) {
  typedef Mfma<T> M;
  constexpr int WS = rs_stride<T>(), XS = rs_stride<T>();
  const int lane = threadIdx.x & 63, ko = M::koff(lane);
  acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T* wk = img + (k * RC + (lane & 15)) * WS + ko;
    const T* xr = in + (row_base + k * tap_step + (lane & 15)) * XS + ko;
#pragma unroll
    for (int cc = 0; cc < RC; cc += M::KS) {
      const typename M::frag a0 = M::load(wk + cc), a1 = M::load(wk + 16 * WS + cc);
      typename M::frag b = M::load(xr + cc);
      if (RELU_IN) b = relu_frag(b);
      acc[0] = M::mma(a0, b, acc[0]);
      acc[1] = M::mma(a1, b, acc[1]);
    }
  }
}

// The same with the weights held in registers: wf[k][mt][cc-step] = A fragments of a forward conv
// (A[m = o][K = c] = W[k][c][o], Keras layout), loaded once per workgroup by load_wfrags.
template <class T> constexpr int rs_ncc() { return RC / Mfma<T>::KS; }

template <class T>
__device__ __forceinline__ void load_wfrags(typename Mfma<T>::frag (&wf)[3][2][rs_ncc<T>()], const float* w) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < rs_ncc<T>(); ++s) {
        const int o = mt * 16 + (lane & 15);
        if constexpr (sizeof(T) == 2) {
          const int c0 = s * 32 + 8 * (lane >> 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) wf[k][mt][s][j] = (bf16)w[(k * RC + c0 + j) * RC + o];
        } else {
          wf[k][mt][s] = w[(k * RC + s * 4 + (lane >> 4)) * RC + o];
        }
      }
}

template <class T, bool RELU_IN>
__device__ __forceinline__ void conv_rows16r(f32x4 (&acc)[2], const typename Mfma<T>::frag (&wf)[3][2][rs_ncc<T>()],
                                             const T* in, int row_base, int tap_step) {
  typedef Mfma<T> M;
  constexpr int XS = rs_stride<T>();
  const int lane = threadIdx.x & 63, ko = M::koff(lane);
  acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T* xr = in + (row_base + k * tap_step + (lane & 15)) * XS + ko;
#pragma unroll
    for (int s = 0; s < rs_ncc<T>(); ++s) {
      typename M::frag b = M::load(xr + s * M::KS);
      if (RELU_IN) b = relu_frag(b);
      acc[0] = M::mma(wf[k][0][s], b, acc[0]);
      acc[1] = M::mma(wf[k][1][s], b, acc[1]);
    }
  }
}

// NJ 16-row n-tiles at once: every B fragment is loaded before the first MFMA, then the MFMAs run tap-major
// over the n-tiles (2*NJ independent accumulator chains), so the LDS latency and the MFMA dependency chain
// are hidden inside the wave. afrag(k, mt, s) supplies the A fragment (registers or an LDS image). Same
// accumulation order per output as conv_rows16.
template <class T, bool RELU_IN, int NJ, class AFrag>
__device__ __forceinline__ void conv_multi(f32x4 (&acc)[NJ][2], AFrag afrag, const T* in, const int (&rb)[NJ],
                                           int tap_step) {
  typedef Mfma<T> M;
  constexpr int XS = rs_stride<T>(), NCC = rs_ncc<T>();
  const int lane = threadIdx.x & 63, ko = M::koff(lane);
  typename M::frag b[NJ][3][NCC];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int s = 0; s < NCC; ++s) {
        b[j][k][s] = M::load(in + (rb[j] + k * tap_step + (lane & 15)) * XS + ko + s * M::KS);
        if (RELU_IN) b[j][k][s] = relu_frag(b[j][k][s]);
      }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    acc[j][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int s = 0; s < NCC; ++s) {
      const typename M::frag a0 = afrag(k, 0, s), a1 = afrag(k, 1, s);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[j][0] = M::mma(a0, b[j][k][s], acc[j][0]);
        acc[j][1] = M::mma(a1, b[j][k][s], acc[j][1]);
      }
    }
}

__device__ __forceinline__ f32x4 bias4(const float* b, int o) { return f32x4{b[o], b[o + 1], b[o + 2], b[o + 3]}; }

// ---------------------------------------------------------------------------------------------------
// 3 waves/SIMD for bf16 (<= 168 VGPRs without spilling); the fp32 parity build needs more registers
template <class T> constexpr int rs_fwd_waves() { return sizeof(T) == 2 ? 3 : 2; }

template <class T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(rs_fwd_waves<T>(), 8)))
void resblock_fwd_kernel(ResArgs a) {
  typedef Mfma<T> M;
  constexpr int XS = rs_stride<T>(), HR = RTM + 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* X = (T*)smem;  // local j <-> row t0 - 1 - d + j, XR = HR + 2d rows (raw x)
  const int d = a.d, XR = HR + 2 * d;
  T* H = X + XR * XS;  // local i <-> row t0 - 1 + i, relu(h)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tbeg = blockIdx.x * a.tpw, tend = min(a.ntiles, tbeg + a.tpw);
  if (tbeg >= tend) return;
  typename M::frag wfa[3][2][rs_ncc<T>()], wfb[3][2][rs_ncc<T>()];
  load_wfrags<T>(wfa, a.wa);
  load_wfrags<T>(wfb, a.wb);
  f32x4 bav[2], bbv[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int o = mt * 16 + 4 * (lane >> 4);
    bav[mt] = a.ba ? bias4(a.ba, o) : f32x4{0.f, 0.f, 0.f, 0.f};
    bbv[mt] = a.bb ? bias4(a.bb, o) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const unsigned ibytes = (unsigned)a.T * RC * (unsigned)sizeof(T);
  auto item_x = [&](int tile) { return rs_rsrc((const T*)a.x + (size_t)(tile / a.ntm) * a.T * RC, ibytes); };
  auto row0 = [&](int tile) { return (tile - (tile / a.ntm) * a.ntm) * RTM - 1 - d; };
  Rows32Buf<T, rs_pv<T>()> nx;
  nx.init(XR);
  nx.load(item_x(tbeg), row0(tbeg));
  nx.store(X);
  if (tbeg + 1 < tend) nx.load(item_x(tbeg + 1), row0(tbeg + 1));
  __syncthreads();
  for (int tile = tbeg; tile < tend; ++tile) {
    const int n = tile / a.ntm, t0 = (tile - n * a.ntm) * RTM;
    // h rows t0-1 .. t0+142 (conv_b reads t0-1 .. t0+128); rows outside the item are conv_b's SAME zeros
    const bool interior = t0 - 1 >= 0 && t0 - 1 + HR <= a.T;  // uniform: no SAME-padding rows in h
    auto wa_frag = [&](int k, int mt, int sc) { return wfa[k][mt][sc]; };
    auto wb_frag = [&](int k, int mt, int sc) { return wfb[k][mt][sc]; };
    {
      // h n-tiles wave, wave+4, wave+8 of HR/16 = 9 (an out-of-range slot computes a valid tile, unstored)
      int rb[3];
      f32x4 acc[3][2];
#pragma unroll
      for (int j = 0; j < 3; ++j) rb[j] = min(wave + 4 * j, HR / 16 - 1) * 16;
      conv_multi<T, true, 3>(acc, wa_frag, X, rb, d);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (wave + 4 * j >= HR / 16) continue;
        const int i = rb[j] + (lane & 15), r = t0 - 1 + i;
        const bool live = interior || (r >= 0 && r < a.T);
        const bool own = a.h && live && i >= 1 && i <= RTM;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          f32x4 v = acc[j][mt] + bav[mt];
          if (interior) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = live ? fmaxf(v[q], 0.f) : 0.f;
          }
          st4(H + i * XS + mt * 16 + 4 * (lane >> 4), v);
          if (own) st4((T*)a.h + ((size_t)n * a.T + r) * RC + mt * 16 + 4 * (lane >> 4), v);
        }
      }
    }
    __syncthreads();
    T* yi = (T*)a.y + (size_t)n * a.T * RC;
    {
      int rb[2];
      f32x4 acc[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[j] = (wave + 4 * j) * 16;
      conv_multi<T, false, 2>(acc, wb_frag, H, rb, 1);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int tl = rb[j] + (lane & 15), t = t0 + tl;
        if (t < a.T) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int o = mt * 16 + 4 * (lane >> 4);
            f32x4 v = acc[j][mt] + bbv[mt];
            v = ld4(X + (tl + 1 + d) * XS + o) + v;
            st4(yi + (size_t)t * RC + o, v);
          }
        }
      }
    }
    if (tile + 1 < tend) {
      __syncthreads();  // every read of X and H for this tile is done
      nx.store(X);
      if (tile + 2 < tend) nx.load(item_x(tile + 2), row0(tile + 2));
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------------
template <class T>
__global__ __launch_bounds__(256) void resblock_bwd_kernel(ResArgs a) {
  typedef Mfma<T> M;
  constexpr int WS = rs_stride<T>(), XS = WS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = a.d, HR = round16(RTM + 2 * d), XR = HR + 2 * d, YR = HR + 2;
  T* waF = (T*)smem;            // conv_a forward (recompute h): [k][o][c]
  T* waT = waF + 3 * RC * WS;   // conv_a^T: Keras [k][c][o]
  T* wbT = waT + 3 * RC * WS;   // conv_b^T: Keras [k][c][o]
  T* X = wbT + 3 * RC * WS;     // local j <-> row t0 - 2d + j (raw x)
  T* Y = X + XR * XS;           // local m <-> row t0 - d - 1 + m (dy)
  T* H = Y + YR * XS;           // local i <-> row t0 - d + i: relu(h), then dh
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tbeg = blockIdx.x * a.tpw, tend = min(a.ntiles, tbeg + a.tpw);
  if (tbeg >= tend) return;
  stage_wimg<T, true>(waF, a.wa);
  stage_wimg<T, false>(waT, a.wa);
  stage_wimg<T, false>(wbT, a.wb);
  f32x4 bav[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) bav[mt] = a.ba ? bias4(a.ba, mt * 16 + 4 * (lane >> 4)) : f32x4{0.f, 0.f, 0.f, 0.f};

  // weight-gradient accumulators: wave w owns input-channel tile ct = w >> 1, output-channel tile ot = w & 1
  const int ct = wave >> 1, ot = wave & 1;
  f32x4 gwa[3], gwb[3], gba = {0.f, 0.f, 0.f, 0.f}, gbb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    gwa[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    gwb[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nht = HR / 16;  // <= 12

  const unsigned ibytes = (unsigned)a.T * RC * (unsigned)sizeof(T);
  auto item_off = [&](int tile) { return (size_t)(tile / a.ntm) * a.T * RC; };
  auto tstart = [&](int tile) { return (tile - (tile / a.ntm) * a.ntm) * RTM; };
  auto load_tile = [&](Rows32Buf<T, rs_pv<T>()>& bx, Rows32Buf<T, rs_pv<T>()>& by, int tile) {
    const size_t o = item_off(tile);
    bx.load(rs_rsrc((const T*)a.x + o, ibytes), tstart(tile) - 2 * d);
    by.load(rs_rsrc((const T*)a.dy + o, ibytes), tstart(tile) - d - 1);
  };
  Rows32Buf<T, rs_pv<T>()> nx, ny;
  nx.init(XR);
  ny.init(YR);
  load_tile(nx, ny, tbeg);
  nx.store(X);
  ny.store(Y);
  if (tbeg + 1 < tend) load_tile(nx, ny, tbeg + 1);
  __syncthreads();
  for (int tile = tbeg; tile < tend; ++tile) {
    const int n = tile / a.ntm, t0 = (tile - n * a.ntm) * RTM;
    // 1. recompute relu(h) over the dh rows (zero outside the item)
    const bool interior = t0 - d >= 0 && t0 - d + HR <= a.T;  // uniform: no SAME-padding rows
    const int ko = M::koff(lane);
    auto img_frag = [&](const T* img) {
      return [=](int k, int mt, int sc) { return M::load(img + (k * RC + mt * 16 + (lane & 15)) * WS + ko + sc * M::KS); };
    };
    int rh[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) rh[j] = min(wave + 4 * j, nht - 1) * 16;
    if (!(a.skip & 1)) {
      f32x4 acc[3][2];
      conv_multi<T, true, 3>(acc, img_frag(waF), X, rh, d);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (wave + 4 * j >= nht) continue;
        const int i = rh[j] + (lane & 15), r = t0 - d + i;
        const bool live = r >= 0 && r < a.T;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          f32x4 v = acc[j][mt] + bav[mt];
          if (interior) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = live ? fmaxf(v[q], 0.f) : 0.f;
          }
          st4(H + i * XS + mt * 16 + 4 * (lane >> 4), v);
        }
      }
    }
    __syncthreads();
    // 2a. dW_b[k][c][o] += sum_t relu(h)[t+k-1][c] dy[t][o], db_b += sum_t dy[t] (the tile's own rows)
#pragma unroll 4
    for (int kk = 0; kk < (a.skip & 2 ? 0 : RTM); kk += M::KS) {
      const typename M::frag bf = M::rows(Y + (d + 1 + kk) * XS + ot * 16, XS);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const typename M::frag af = M::rows(H + (d + k - 1 + kk) * XS + ct * 16, XS);
        gwb[k] = M::mma(af, bf, gwb[k]);
      }
      if (ct == 0) gbb = M::mma(M::ones(), bf, gbb);
    }
    // 2b. dh = conv_b^T(dy) * (h > 0), held in registers until every read of relu(h) is done
    f32x4 dh[3][2];
    if (!(a.skip & 4)) {
      int rb[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) rb[j] = rh[j] + 2;
      conv_multi<T, false, 3>(dh, img_frag(wbT), Y, rb, -1);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int i = rh[j] + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const f32x4 hm = ld4(H + i * XS + mt * 16 + 4 * (lane >> 4));
#pragma unroll
          for (int q = 0; q < 4; ++q) dh[j][mt][q] = hm[q] > 0.f ? dh[j][mt][q] : 0.f;
        }
      }
    }
    __syncthreads();
    if (!(a.skip & 4)) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (wave + 4 * j >= nht) continue;
        const int i = rh[j] + (lane & 15);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) st4(H + i * XS + mt * 16 + 4 * (lane >> 4), dh[j][mt]);
      }
    }
    __syncthreads();
    // 3. dx = dy + conv_a^T(dh) * (x > 0) on the tile's rows
    T* dxi = (T*)a.y + (size_t)n * a.T * RC;
    if (!(a.skip & 8)) {
      int rb[2];
      f32x4 acc[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) rb[j] = (wave + 4 * j) * 16 + 2 * d;
      conv_multi<T, false, 2>(acc, img_frag(waT), H, rb, -d);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int tl = (wave + 4 * j) * 16 + (lane & 15), t = t0 + tl;
        if (t < a.T) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int o = mt * 16 + 4 * (lane >> 4);
            const f32x4 xm = ld4(X + (tl + 2 * d) * XS + o);
            f32x4 v = acc[j][mt];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = xm[q] > 0.f ? v[q] : 0.f;
            v = ld4(Y + (tl + d + 1) * XS + o) + v;
            st4(dxi + (size_t)t * RC + o, v);
          }
        }
      }
    }
    // 4. dW_a[k][c][o] += sum_t relu(x)[t+(k-1)d][c] dh[t][o], db_a += sum_t dh[t]
#pragma unroll 4
    for (int kk = 0; kk < (a.skip & 16 ? 0 : RTM); kk += M::KS) {
      const typename M::frag bf = M::rows(H + (d + kk) * XS + ot * 16, XS);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const typename M::frag af = relu_frag(M::rows(X + ((k + 1) * d + kk) * XS + ct * 16, XS));
        gwa[k] = M::mma(af, bf, gwa[k]);
      }
      if (ct == 0) gba = M::mma(M::ones(), bf, gba);
    }
    if (tile + 1 < tend) {
      __syncthreads();  // every read of X, Y and H for this tile is done
      nx.store(X);
      ny.store(Y);
      if (tile + 2 < tend) load_tile(nx, ny, tile + 2);
      __syncthreads();
    }
  }
  // partial rows: Keras dW[k][c][o] (c = ct*16 + 4*(lane>>4) + r, o = ot*16 + (lane&15)), then the bias
  float* pa = a.part_a + (size_t)blockIdx.x * (3 * RC * RC + RC);
  float* pb = a.part_b + (size_t)blockIdx.x * (3 * RC * RC + RC);
  const int o = ot * 16 + (lane & 15);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = ct * 16 + 4 * (lane >> 4) + r;
      pa[(k * RC + c) * RC + o] = gwa[k][r];
      pb[(k * RC + c) * RC + o] = gwb[k][r];
    }
  if (ct == 0 && lane < 16) {
    pa[3 * RC * RC + o] = gba[0];
    pb[3 * RC * RC + o] = gbb[0];
  }
}

// ---------------------------------------------------------------------------------------------------
static int rs_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}
constexpr int kResPerCU = 2;  // persistent workgroups per CU (also bounds the partial rows)

static size_t fwd_lds(int d, int esz) {
  const int s = RC + 16 / esz, HR = RTM + 16;
  return ((size_t)(HR + 2 * d) * s + (size_t)HR * s) * esz;
}
static size_t bwd_lds(int d, int esz) {
  const int s = RC + 16 / esz, HR = round16(RTM + 2 * d);
  return ((size_t)9 * RC * s + (size_t)(HR + 2 * d) * s + (size_t)(HR + 2) * s + (size_t)HR * s) * esz;
}

static int set_lds(const void* fn, size_t bytes) {
  static size_t done[4] = {0, 0, 0, 0};
  static const void* fns[4] = {nullptr, nullptr, nullptr, nullptr};
  if (bytes <= 65536) return VQA_OK;
  int slot = 0;
  while (slot < 3 && fns[slot] && fns[slot] != fn) ++slot;
  if (fns[slot] == fn && done[slot] >= bytes) return VQA_OK;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    (void)hipGetLastError();
    set_error("resblock: cannot reserve %zu B of LDS", bytes);
    return VQA_E_UNSUPPORTED;
  }
  fns[slot] = fn;
  done[slot] = bytes;
  return VQA_OK;
}

static void plan(ResArgs& a, int per_cu) {
  a.ntm = (a.T + RTM - 1) / RTM;
  a.ntiles = a.ntm * a.B;
  int nwg = rs_cus() * per_cu;
  if (nwg > a.ntiles) nwg = a.ntiles;
  a.tpw = (a.ntiles + nwg - 1) / nwg;
}

}  // namespace vqa

using namespace vqa;

extern "C" int vqa_resblock_supported(int C, int dilation, int dtype) {
  if (C != RC || dilation < 1 || dilation > RMAXD || !(dtype == VQA_F32 || dtype == VQA_BF16)) return 0;
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  return bwd_lds(dilation, esz) <= 160 * 1024 && fwd_lds(dilation, esz) <= 160 * 1024;
}

extern "C" int vqa_resblock_fwd(const void* x, const float* wa, const float* ba, const float* wb, const float* bb,
                                void* y, void* h_out, int B, int T, int C, int dilation, int dtype,
                                vqa_stream_t stream) {
  VQA_ARG(x && wa && wb && y && B > 0 && T > 0, "resblock_fwd: bad arguments");
  VQA_REQUIRE(vqa_resblock_supported(C, dilation, dtype), VQA_E_UNSUPPORTED,
              "resblock_fwd: unsupported C=%d dilation=%d dtype=%d", C, dilation, dtype);
  VQA_ARG((long long)T * C * 4 < (1ll << 30), "resblock_fwd: item too long for 32-bit buffer offsets (T=%d)", T);
  ResArgs a{x, nullptr, y, h_out, wa, ba, wb, bb, nullptr, nullptr, B, T, dilation, 0, 0, 0, 0};
  plan(a, 3);
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  const size_t lds = fwd_lds(RMAXD, esz);  // one LDS reservation for every dilation
  const hipStream_t s = (hipStream_t)stream;
  const dim3 grid((a.ntiles + a.tpw - 1) / a.tpw);
  if (dtype == VQA_BF16) {
    if (int rc = set_lds((const void*)resblock_fwd_kernel<bf16>, lds)) return rc;
    hipLaunchKernelGGL(resblock_fwd_kernel<bf16>, grid, dim3(256), lds, s, a);
  } else {
    if (int rc = set_lds((const void*)resblock_fwd_kernel<float>, lds)) return rc;
    hipLaunchKernelGGL(resblock_fwd_kernel<float>, grid, dim3(256), lds, s, a);
  }
  VQA_LAUNCHED("resblock_fwd_kernel");
  return VQA_OK;
}

extern "C" size_t vqa_resblock_bwd_workspace(int B, int T, int C, int dilation, int dtype) {
  (void)B;
  (void)T;
  (void)dilation;
  (void)dtype;
  return (size_t)2 * rs_cus() * kResPerCU * (3 * C * C + C) * sizeof(float);
}

extern "C" int vqa_resblock_bwd(const void* dy, const void* x, const float* wa, const float* ba, const float* wb,
                                const float* bb, void* dx, float* dwa, float* dba, float* dwb, float* dbb, int B,
                                int T, int C, int dilation, int dtype, void* workspace, size_t ws_bytes,
                                vqa_partials_desc* desc, vqa_stream_t stream) {
  (void)bb;
  VQA_ARG(dy && x && wa && wb && dx && dwa && dwb && B > 0 && T > 0, "resblock_bwd: bad arguments");
  VQA_ARG((long long)T * C * 4 < (1ll << 30), "resblock_bwd: item too long for 32-bit buffer offsets (T=%d)", T);
  VQA_REQUIRE(vqa_resblock_supported(C, dilation, dtype), VQA_E_UNSUPPORTED,
              "resblock_bwd: unsupported C=%d dilation=%d dtype=%d", C, dilation, dtype);
  const size_t need = vqa_resblock_bwd_workspace(B, T, C, dilation, dtype);
  VQA_ARG(workspace && ws_bytes >= need, "resblock_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  const int E = 3 * RC * RC + RC;
  ResArgs a{x, dy, dx, nullptr, wa, ba, wb, nullptr, (float*)workspace, nullptr, B, T, dilation, 0, 0, 0, 0};
  static const int dbg_skip = [] {
    const char* e = getenv("VQA_RESBLOCK_SKIP");
    return e ? atoi(e) : 0;
  }();
  a.skip = dbg_skip;
  plan(a, kResPerCU);
  const int nwg = (a.ntiles + a.tpw - 1) / a.tpw;
  a.part_b = a.part_a + (size_t)nwg * E;
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  const size_t lds = bwd_lds(dilation, esz);
  const size_t lds_max = bwd_lds(RMAXD, esz);
  const hipStream_t s = (hipStream_t)stream;
  if (dtype == VQA_BF16) {
    if (int rc = set_lds((const void*)resblock_bwd_kernel<bf16>, lds_max)) return rc;
    hipLaunchKernelGGL(resblock_bwd_kernel<bf16>, dim3(nwg), dim3(256), lds, s, a);
  } else {
    if (int rc = set_lds((const void*)resblock_bwd_kernel<float>, lds_max)) return rc;
    hipLaunchKernelGGL(resblock_bwd_kernel<float>, dim3(nwg), dim3(256), lds, s, a);
  }
  VQA_LAUNCHED("resblock_bwd_kernel");
  const vqa_partials_desc da{a.part_a, dwa, dba, nwg, E, 3 * RC * RC, 0};
  const vqa_partials_desc dbd{a.part_b, dwb, dbb, nwg, E, 3 * RC * RC, 0};
  if (desc) {
    desc[0] = da;
    desc[1] = dbd;
    return VQA_OK;
  }
  const vqa_partials_desc both[2] = {da, dbd};
  return vqa_reduce_partials(both, 2, stream);
}
