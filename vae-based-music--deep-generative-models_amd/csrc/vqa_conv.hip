// vqa_conv.hip — 1-D convolution kernels for the dilated-conv encoder/decoder (gfx950).
//
// Replaces the TF ops behind keras Conv1D / Conv1DTranspose on the reference's hot path:
//   resnet.py:13,17 (dilated residual convs), encdec.py:33 (strided down conv), :38 (projection),
//   :60 (decoder pre-conv), :67-68 (Conv1DTranspose up conv), :148 (decoder output conv).
//
// Every forward and data-gradient is ONE "gather" convolution
//     y[n, t, o] = sum_{k, c} act(x[n, t*S + k*D - P, c]) * Weff[k][c][o]      (+bias, mask, residual)
// with three ways of reading the fp32 Keras weight ("wmode"):
//   DIRECT : Weff = W[k][c][o]                       conv fwd; conv-transpose data-grad (stride 2)
//   FLIP_T : Weff = W[Kb-1-k][o][c]                  stride-1 conv data-grad
//   PAIR   : out pair j holds full rows 2j, 2j+1:    conv-transpose fwd; stride-2 conv data-grad
//            Weff[a+1][c][p*Ob+ob] = W[p + Pb - 2a][ob][c]  (a in {-1,0,1}, zero when out of range)
// so the MFMA kernel below covers all of them; the PAIR layout (n, j, p, ob) is exactly the NTC
// layout of the full-resolution tensor. Weight gradients are split-row MFMA reductions with
// per-workgroup fp32 partials and a deterministic second pass.
#include "vqa_common.h"
#include "vqa_mfma.h"
#include <algorithm>

namespace vqa {

enum { W_DIRECT = 0, W_FLIP_T = 1, W_PAIR = 2 };

struct GatherArgs {
  const void* x;
  const float* w;
  const float* bias;
  const void* resid;
  const void* mask;
  void* y;
  int B, T_in, T_out;  // x rows per item, gather-output rows per item
  int C, O;            // gather input / output channels
  int K, S, D, P;      // gather taps, stride, dilation, left pad
  int wmode, Kb, Pb;   // weight mapping; base taps; base pad (PAIR)
  int T_full;          // PAIR: full-resolution rows per item (store guard)
  int flags;
  // fused weight gradient (stride-1 data-gradient only): `mask` is the conv input u (always staged),
  // wpart receives one fp32 partial [K*O*C dW | C db] per workgroup, wrelu: dW uses relu(u)
  float* wpart = nullptr;
  int wrelu = 0;
};

__device__ __forceinline__ float weff(const GatherArgs& a, int k, int c, int o) {
  if (a.wmode == W_DIRECT) return a.w[((size_t)k * a.C + c) * a.O + o];
  if (a.wmode == W_FLIP_T) return a.w[((size_t)(a.Kb - 1 - k) * a.O + o) * a.C + c];
  const int Ob = a.O >> 1;
  const int p = o >= Ob ? 1 : 0;
  const int ob = o - p * Ob;
  const int kb = p + a.Pb - 2 * (k - 1);
  return (kb >= 0 && kb < a.Kb) ? a.w[((size_t)kb * Ob + ob) * a.C + c] : 0.f;
}

// output element index (n, t, o) -> linear offset in y / resid / mask, or -1 if outside (PAIR tail)
__device__ __forceinline__ long long out_index(const GatherArgs& a, int n, int t, int o) {
  if (a.wmode == W_PAIR) {
    const int Ob = a.O >> 1;
    const int p = o >= Ob ? 1 : 0;
    const int u = 2 * t + p;
    if (u >= a.T_full) return -1;
    return ((long long)n * a.T_full + u) * Ob + (o - p * Ob);
  }
  return ((long long)n * a.T_out + t) * a.O + o;
}

__device__ __forceinline__ int bias_index(const GatherArgs& a, int o) {
  return a.wmode == W_PAIR ? (o >= (a.O >> 1) ? o - (a.O >> 1) : o) : o;
}

// ------------------------------------------------------------------------------------------------
// Generic VALU gather conv: any C/O/K/S/D, mixed fp32/bf16 ends. Used for the 1-channel layers at
// the waveform ends (first encoder conv C=1, decoder output conv O=1 and its data-gradient).
template <class TX, class TY>
__global__ __launch_bounds__(256) void gather_direct_kernel(GatherArgs a) {
  const TX* X = (const TX*)a.x;
  const long long total = (long long)a.B * a.T_out * a.O;
  const bool relu = a.flags & VQA_PRE_RELU;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(e % a.O);
    const long long r = e / a.O;
    const int t = (int)(r % a.T_out);
    const int n = (int)(r / a.T_out);
    float acc = 0.f;
    for (int k = 0; k < a.K; ++k) {
      const int ti = t * a.S + k * a.D - a.P;
      if (ti < 0 || ti >= a.T_in) continue;
      const TX* xr = X + ((long long)n * a.T_in + ti) * a.C;
      for (int c = 0; c < a.C; ++c) {
        float xv = ld(xr + c);
        if (relu) xv = fmaxf(xv, 0.f);
        acc += xv * weff(a, k, c, o);
      }
    }
    const long long oi = out_index(a, n, t, o);
    if (oi < 0) continue;
    float v = acc;
    if (a.bias) v = v + a.bias[bias_index(a, o)];
    if (a.flags & VQA_POST_MASK) v = ld((const TY*)a.mask + oi) > 0.f ? v : 0.f;
    if (a.flags & VQA_ADD_RESIDUAL) v = ld((const TY*)a.resid + oi) + v;
    st((TY*)a.y + oi, v);
  }
}

// ------------------------------------------------------------------------------------------------
// Thin gather conv for the 1-channel waveform layers (C <= 8 or O <= 8): weights in LDS (fp32), each
// thread owns OV consecutive output channels of one row; 16-byte loads along C when C % 8 == 0.
template <class T> __device__ __forceinline__ void ld8_(const T* p, float* v);
template <> __device__ __forceinline__ void ld8_<bf16>(const bf16* p, float* v) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> __device__ __forceinline__ void ld8_<float>(const float* p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = a[j];
    v[j + 4] = b[j];
  }
}

template <class T> __device__ __forceinline__ void st8_(T* p, const float* v);
template <> __device__ __forceinline__ void st8_<bf16>(bf16* p, const float* v) {
  *(bf16x8*)p = bf16x8{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3], (bf16)v[4], (bf16)v[5], (bf16)v[6], (bf16)v[7]};
}
template <> __device__ __forceinline__ void st8_<float>(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

template <class TX, class TY, int OV>
__global__ __launch_bounds__(256) void gather_thin_kernel(GatherArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* wl = (float*)smem;  // [K][C][O]
  const int KCO = a.K * a.C * a.O;
  for (int e = threadIdx.x; e < KCO; e += blockDim.x) {
    const int o = e % a.O, c = (e / a.O) % a.C, k = e / (a.O * a.C);
    wl[e] = weff(a, k, c, o);
  }
  __syncthreads();
  const TX* X = (const TX*)a.x;
  const int OG = a.O / OV;
  const int total = a.B * a.T_out * OG;  // < 2^31 (host-checked)
  const bool relu = a.flags & VQA_PRE_RELU;
  const bool vec = (a.C % 8) == 0;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int og = e % OG;
    const int r = e / OG;
    const int t = r % a.T_out;
    const int n = r / a.T_out;
    float acc[OV];
#pragma unroll
    for (int q = 0; q < OV; ++q) acc[q] = 0.f;
    for (int k = 0; k < a.K; ++k) {
      const int ti = t * a.S + k * a.D - a.P;
      if (ti < 0 || ti >= a.T_in) continue;
      const TX* xr = X + ((long long)n * a.T_in + ti) * a.C;
      const float* wk = wl + (size_t)k * a.C * a.O + og * OV;
      if (vec) {
        for (int c0 = 0; c0 < a.C; c0 += 8) {
          float xv[8];
          ld8_(xr + c0, xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xj = relu ? fmaxf(xv[j], 0.f) : xv[j];
#pragma unroll
            for (int q = 0; q < OV; ++q) acc[q] += xj * wk[(c0 + j) * a.O + q];
          }
        }
      } else {
        for (int c = 0; c < a.C; ++c) {
          float xs = ld(xr + c);
          if (relu) xs = fmaxf(xs, 0.f);
#pragma unroll
          for (int q = 0; q < OV; ++q) acc[q] += xs * wk[c * a.O + q];
        }
      }
    }
    const int o0 = og * OV;
    const long long oi = out_index(a, n, t, o0);
    if (oi < 0) continue;
    const int bo = bias_index(a, o0);
    if constexpr (OV == 8) {
      if (a.O % 16 == 0) {  // the 8 channels are contiguous and 16-byte aligned in every mode: one vector access
        float v[8], m[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = a.bias ? acc[q] + a.bias[bo + q] : acc[q];
        if (a.flags & VQA_POST_MASK) {
          ld8_((const TY*)a.mask + oi, m);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = m[q] > 0.f ? v[q] : 0.f;
        }
        if (a.flags & VQA_ADD_RESIDUAL) {
          ld8_((const TY*)a.resid + oi, m);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = m[q] + v[q];
        }
        st8_((TY*)a.y + oi, v);
        continue;
      }
    }
#pragma unroll
    for (int q = 0; q < OV; ++q) {
      float v = acc[q];
      if (a.bias) v = v + a.bias[bo + q];
      if (a.flags & VQA_POST_MASK) v = ld((const TY*)a.mask + oi + q) > 0.f ? v : 0.f;
      if (a.flags & VQA_ADD_RESIDUAL) v = ld((const TY*)a.resid + oi + q) + v;
      st((TY*)a.y + oi + q, v);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Stage rows [r0, r0+rows) of one item (Xi = that item's row 0, channels C) into LDS with padded row
// stride XS, zero-filling rows outside [lo, hi), optional ReLU. 16-byte vector loads.
template <class T, int C>
__device__ __forceinline__ void stage_rows(T* xl, int XS, const T* Xi, int lo, int hi, int r0, int rows,
                                           bool relu) {
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int CPR = C / VEC;
  for (int e = threadIdx.x; e < rows * CPR; e += blockDim.x) {
    const int rr = e / CPR, q = e - rr * CPR;
    const int ti = r0 + rr;
    uint4 v = {0u, 0u, 0u, 0u};
    if (ti >= lo && ti < hi) v = *((const uint4*)(Xi + (long long)ti * C) + q);
    if (relu) relu_bits<T>(v);
    *(uint4*)(xl + rr * XS + q * VEC) = v;
  }
}

// Narrow-output gather conv (O <= 8, C in {32, 64}; the decoder output conv C=64 -> O=1): one block =
// TB output rows of one item; the input rows are staged through LDS with coalesced 16-byte loads and
// every thread reduces one output row from LDS.
template <class TX, class TY, int C>
__global__ __launch_bounds__(256) void gather_thinO_kernel(GatherArgs a, int ntb) {
  constexpr int TB = 256;
  constexpr int XS = C + 16 / (int)sizeof(TX);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* wl = (float*)smem;  // [K][C][O]
  const int KCO = a.K * C * a.O;
  TX* xl = (TX*)(smem + ((KCO * 4 + 15) / 16) * 16);
  const int n = blockIdx.x / ntb, t0 = (blockIdx.x - n * ntb) * TB;
  for (int e = threadIdx.x; e < KCO; e += 256) {
    const int o = e % a.O, c = (e / a.O) % C, k = e / (a.O * C);
    wl[e] = weff(a, k, c, o);
  }
  const int rows_in = (TB - 1) * a.S + (a.K - 1) * a.D + 1;
  stage_rows<TX, C>(xl, XS, (const TX*)a.x + (long long)n * a.T_in * C, 0, a.T_in, t0 * a.S - a.P, rows_in,
                    a.flags & VQA_PRE_RELU);
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= a.T_out) return;
  float acc[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) acc[o] = 0.f;
  for (int k = 0; k < a.K; ++k) {
    const TX* xr = xl + (threadIdx.x * a.S + k * a.D) * XS;
    const float* wk = wl + k * C * a.O;
#pragma unroll
    for (int c0 = 0; c0 < C; c0 += 8) {
      float xv[8];
      ld8_(xr + c0, xv);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int o = 0; o < 8; ++o)
          if (o < a.O) acc[o] += xv[j] * wk[(c0 + j) * a.O + o];
    }
  }
  const long long oi = out_index(a, n, t, 0);
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    if (o < a.O) {
      float v = acc[o];
      if (a.bias) v = v + a.bias[o];
      if (a.flags & VQA_POST_MASK) v = ld((const TY*)a.mask + oi + o) > 0.f ? v : 0.f;
      if (a.flags & VQA_ADD_RESIDUAL) v = ld((const TY*)a.resid + oi + o) + v;
      st((TY*)a.y + oi + o, v);
    }
  }
}

template <class T> struct Raw4;
template <> struct Raw4<bf16> { typedef bf16x4 type; };
template <> struct Raw4<float> { typedef f32x4 type; };

// Register-staged row loader (issue early, write late — cdna_hip_programming.md T14): chunk
// e = threadIdx.x + i*256 of a rows x C tile, 16 B each, PV chunks per thread held in VGPRs; chunks
// beyond 256*PV are staged synchronously by tail().
template <class T, int C, int PV>
struct RowStager {
  static constexpr int VEC = 16 / (int)sizeof(T), CPR = C / VEC;
  uint4 v[PV];
  unsigned ok;
  // branch-free issue (see TileRegs::load); requires lo < hi (a non-empty row range)
  __device__ __forceinline__ void load(const T* Xi, int lo, int hi, int r0, int rows) {
    ok = 0u;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = threadIdx.x + i * 256;
      const int rr = e / CPR, q = e - rr * CPR, ti = r0 + rr;
      const bool val = e < rows * CPR && ti >= lo && ti < hi;
      const int tc = val ? ti : lo;
      v[i] = *((const uint4*)(Xi + (long long)tc * C) + (val ? q : 0));
      ok |= val ? (1u << i) : 0u;
    }
  }
  __device__ __forceinline__ void store(T* xl, int XS, int rows, bool relu) {
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e < rows * CPR) {
        const int rr = e / CPR, q = e - rr * CPR;
        uint4 t = v[i];
        if (!(ok & (1u << i))) t = uint4{0u, 0u, 0u, 0u};
        if (relu) relu_bits<T>(t);
        *(uint4*)(xl + rr * XS + q * VEC) = t;
      }
    }
  }
  __device__ __forceinline__ void tail(T* xl, int XS, const T* Xi, int lo, int hi, int r0, int rows, bool relu) {
    for (int e = threadIdx.x + PV * 256; e < rows * CPR; e += 256) {
      const int rr = e / CPR, q = e - rr * CPR, ti = r0 + rr;
      uint4 t = {0u, 0u, 0u, 0u};
      if (ti >= lo && ti < hi) t = *((const uint4*)(Xi + (long long)ti * C) + q);
      if (relu) relu_bits<T>(t);
      *(uint4*)(xl + rr * XS + q * VEC) = t;
    }
  }
};

// Weights -> LDS image [K][O][C + pad] in T: 16-byte loads along the Keras kernel's contiguous axis, every
// load of a batch issued before any store. DIRECT (w[k][c][o]: o contiguous) moves (tap, input-channel pair,
// output quad) items — two float4 loads, four packed-pair stores; FLIP_T / PAIR (c contiguous) move (tap,
// output channel, input quad) items — one float4 load, one 4-element store. (The per-element form — a scalar
// load and a 2-byte store per weight — took ~5 us at the start of every workgroup: 0.41 ms of the step's
// 1.98 ms of conv time, tools/conv_sweep.py.)
template <class T> __device__ __forceinline__ void st2w(T* p, float a, float b);
template <> __device__ __forceinline__ void st2w<float>(float* p, float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  *(f2*)p = f2{a, b};
}
template <> __device__ __forceinline__ void st2w<bf16>(bf16* p, float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  *(b2*)p = __builtin_convertvector((f2){a, b}, b2);
}

template <class T, int C, int O>
__device__ __forceinline__ void stage_weights(const GatherArgs& a, T* wl, int WS) {
  static_assert(C % 4 == 0 && O % 4 == 0, "vector weight staging");
  constexpr int NB = 4;  // items in flight per thread
  if (a.wmode == W_DIRECT) {
    constexpr int OQ = O / 4, CP = C / 2;
    const int items = a.K * CP * OQ;
    for (int e0 = 0; e0 < items; e0 += 256 * NB) {
      f32x4 lo[NB], hi[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int e = e0 + threadIdx.x + j * 256;
        lo[j] = hi[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (e < items) {
          const int oq = e % OQ, cp = (e / OQ) % CP, k = e / (OQ * CP);
          const float* src = a.w + ((size_t)k * C + 2 * cp) * O + 4 * oq;
          lo[j] = *(const f32x4*)src;
          hi[j] = *(const f32x4*)(src + O);
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int e = e0 + threadIdx.x + j * 256;
        if (e < items) {
          const int oq = e % OQ, cp = (e / OQ) % CP, k = e / (OQ * CP);
          T* dst = wl + ((size_t)k * O + 4 * oq) * WS + 2 * cp;
#pragma unroll
          for (int i = 0; i < 4; ++i) st2w<T>(dst + i * WS, lo[j][i], hi[j][i]);
        }
      }
    }
  } else {
    constexpr int CQ = C / 4;
    const int items = a.K * O * CQ;
    for (int e0 = 0; e0 < items; e0 += 256 * NB) {
      f32x4 v[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int e = e0 + threadIdx.x + j * 256;
        v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (e < items) {
          const int cq = e % CQ, o = (e / CQ) % O, k = e / (CQ * O);
          const float* src = nullptr;
          if (a.wmode == W_FLIP_T) {
            src = a.w + ((size_t)(a.Kb - 1 - k) * O + o) * C + 4 * cq;
          } else {  // PAIR: out pair column o = (p, ob) takes base tap kb = p + Pb - 2 (k - 1), zero outside
            const int Ob = O >> 1, p = o >= Ob ? 1 : 0, ob = o - p * Ob, kb = p + a.Pb - 2 * (k - 1);
            if (kb >= 0 && kb < a.Kb) src = a.w + ((size_t)kb * Ob + ob) * C + 4 * cq;
          }
          if (src) v[j] = *(const f32x4*)src;
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int e = e0 + threadIdx.x + j * 256;
        if (e < items) {
          const int cq = e % CQ, o = (e / CQ) % O, k = e / (CQ * O);
          st4<T>(wl + ((size_t)k * O + o) * WS + 4 * cq, v[j]);
        }
      }
    }
  }
}

// One tile's global -> LDS copy in 16-byte chunks, held in registers between load() and store():
// chunks [0, nx) are the input rows (with halo; padded LDS rows, compile-time chunks per row), then ne
// chunks of the ReLU' mask and ne of the residual — the output rows of the tile, contiguous in global
// memory, copied chunk-linearly (unpadded) into their LDS tiles. Chunk e = threadIdx.x + i*256.
struct TileSrc {
  const char* x;      // this item's input row 0
  int r0, nx;         // first input row of the tile, input chunks
  const char* m;      // mask bytes of the tile's first output row (nullptr: unused)
  const char* r;      // residual bytes of the tile's first output row (nullptr: unused)
  int ne, elim;       // chunks per epilogue tensor; bytes valid from m / r (rows past the item read 0)
};

template <class T, int C, int PV>
struct TileRegs {
  static constexpr int VEC = 16 / (int)sizeof(T), CPR = C / VEC;
  uint4 v[PV];
  unsigned ok;  // bit i: chunk i is real data (else it is stored as zeros)
  // Branch-free: every chunk issues its load (an out-of-range chunk reads a valid dummy address and is
  // zeroed at store time) so the PV loads go out back to back. A per-chunk `if (valid) load` makes hipcc
  // branch around each load and wait vmcnt(0) per chunk (cdna_hip_programming.md, trap (c)).
  __device__ __forceinline__ void load(const TileSrc& s, int T_in) {
    ok = 0u;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = threadIdx.x + i * 256;
      const int row = e / CPR, q = e % CPR, gr = s.r0 + row;
      const bool in_x = e < s.nx;
      const bool vx = in_x && gr >= 0 && gr < T_in;
      const int e2 = e - s.nx;
      const bool in_m = s.m != nullptr && e2 < s.ne;
      const int e3 = s.m != nullptr ? e2 - s.ne : e2;
      const int ei = in_m ? e2 : e3;
      const char* eb = in_m ? s.m : s.r;
      const bool ve = !in_x && eb != nullptr && ei < s.ne && ei * 16 < s.elim;
      const char* px = s.x + (long long)gr * C * (int)sizeof(T) + q * 16;
      const char* pe = eb + (long long)ei * 16;
      const char* p = vx ? px : (ve ? pe : s.x);
      v[i] = *(const uint4*)p;
      ok |= (vx || ve) ? (1u << i) : 0u;
    }
  }
  __device__ __forceinline__ void store(const TileSrc& s, T* xl, int XS, char* ml, char* rl, bool relu) {
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = threadIdx.x + i * 256;
      uint4 t = v[i];
      if (!(ok & (1u << i))) t = uint4{0u, 0u, 0u, 0u};
      if (e < s.nx) {
        const int row = e / CPR, q = e % CPR;
        if (relu) relu_bits<T>(t);
        *(uint4*)(xl + row * XS + q * VEC) = t;
      } else {
        int e2 = e - s.nx;
        char* b = s.m ? ml : nullptr;
        if (!b || e2 >= s.ne) {
          if (s.m) e2 -= s.ne;
          b = s.r ? rl : nullptr;
        }
        if (b && e2 < s.ne) *((uint4*)b + e2) = t;
      }
    }
  }
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t item_rsrc(const void* base, long long off, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base + (unsigned long long)off;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  void* q = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}


// MFMA gather conv, persistent and software-pipelined. Each workgroup (4 waves) owns a contiguous range
// of TM-row tiles of one or more items (a tile's halo rows were just read by its predecessor on the
// same CU), stages the weights once, and keeps TWO tiles in flight in registers (tiles i+1, i+2) while
// tile i runs its MFMAs and epilogue out of LDS — so neither the input rows nor the epilogue operands
// (residual, ReLU' mask) are ever waited for inside a tile (cdna_hip_programming.md T14, two deep).
// D[o][t] = sum_{k,c} Weff^T[o][(k,c)] * X[(k,c)][t]: A = weights (rows = output channels), B = a 16-byte
// channel run of one input row; each accumulator lane holds 4 consecutive output channels of one row.
// occupancy target: 4 waves/SIMD (<= 128 VGPRs) for the 4-chunk stager, 3 (<= 168) for 8, 2 for 12;
// O = 128 tiles (and fp32 O = 64 with 8 chunks) need more registers than that without spilling
template <class T, int O, int PV> constexpr int gather_waves() {
  if (O >= 128 || (sizeof(T) == 4 && O >= 64 && PV > 4)) return 2;
  return PV <= 4 ? 4 : (PV <= 5 ? (O <= 32 ? 4 : 3) : (PV <= 8 ? 3 : 2));
}

template <class T, int C, int O, int TM, int PV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gather_waves<T, O, PV>(), 8)))
void gather_mfma_kernel(GatherArgs a, int ntm, int ntiles, int tpw) {
  typedef Mfma<T> M;
  constexpr int NW = 4, RW = TM / NW, NT = RW / 16, MT = O / 16;
  constexpr int XS = C + lds_pad<T>();
  constexpr int WS = C + lds_pad<T>();
  static_assert(RW % 16 == 0 && O % 16 == 0 && C % M::KS == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* wl = (T*)smem;
  T* xl = wl + (size_t)a.K * O * WS;
  const int rows_in = (TM - 1) * a.S + (a.K - 1) * a.D + 1;
  // epilogue tiles, unpadded and chunk-linear: [TM][O], or in PAIR mode [2TM][O/2] (full-resolution rows)
  T* ml = xl + (size_t)rows_in * XS;
  T* rl = ml + (size_t)TM * O;

  const int tbeg = blockIdx.x * tpw, tend = min(ntiles, tbeg + tpw);
  if (tbeg >= tend) return;
  const bool pair = a.wmode == W_PAIR;
  const bool do_mask = a.flags & VQA_POST_MASK, do_res = a.flags & VQA_ADD_RESIDUAL;
  const bool relu = a.flags & VQA_PRE_RELU;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ko = M::koff(lane);
  constexpr int ESZ = (int)sizeof(T);
  const int erow = pair ? O / 2 : O;  // elements per output row (full resolution)

  auto source = [&](int tile) {
    const int n = tile / ntm, t0 = (tile - n * ntm) * TM;
    TileSrc src;
    src.x = (const char*)a.x + (long long)n * a.T_in * C * ESZ;
    src.r0 = t0 * a.S - a.P;
    src.nx = rows_in * (C * ESZ / 16);
    const int r0e = pair ? 2 * t0 : t0;                 // first output row of the tile
    const int rvalid = pair ? a.T_full : a.T_out;        // output rows of this item
    const long long eoff = ((long long)n * rvalid + r0e) * erow * ESZ;
    src.m = do_mask ? (const char*)a.mask + eoff : nullptr;
    src.r = do_res ? (const char*)a.resid + eoff : nullptr;
    src.ne = TM * O * ESZ / 16;
    src.elim = (rvalid - r0e) * erow * ESZ;
    return src;
  };

  // the bias per output channel (PAIR: both halves), staged once: the epilogue reads it from LDS (a global load
  // per output block in the epilogue was waited for in turn: 8 serial round trips per tile at O = 128)
  __shared__ __attribute__((aligned(16))) float bias_l[O];
  for (int i = threadIdx.x; i < O; i += 256) bias_l[i] = a.bias ? a.bias[bias_index(a, i)] : 0.f;
  stage_weights<T, C, O>(a, wl, WS);
  TileSrc S0, S1;
  TileRegs<T, C, PV> A, B;
  S0 = source(tbeg);
  A.load(S0, a.T_in);
  if (tbeg + 1 < tend) {
    S1 = source(tbeg + 1);
    B.load(S1, a.T_in);
  }
  A.store(S0, xl, XS, (char*)ml, (char*)rl, relu);
  __syncthreads();

  // bf16 tiles without epilogue operands: the output rows staged in the (then unused) epilogue-operand region and
  // stored as contiguous 16-byte chunks (the 8-byte per-lane stores wrote a quarter of a cache line each)
  constexpr int OP = O + 8;
  const int rvalid_ = pair ? a.T_full : a.T_out;
  const bool se = sizeof(T) == 2 && !do_mask && !do_res && (long long)rvalid_ * erow * ESZ < (1ll << 31);
  T* stg = ml + (size_t)wave * RW * OP;
  static_assert(TM * (O + 8) <= 2 * TM * O, "staged tile fits the two epilogue-operand tiles");

  // one tile: MFMAs out of LDS, epilogue operands out of LDS, stores to global
  auto run_tile = [&](int tile) {
    const int n = tile / ntm, t0 = (tile - n * ntm) * TM;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // K <= 4 (host-checked): unrolled, uniform exit
      if (k >= a.K) break;
      const T* wk = wl + (size_t)k * O * WS + (lane & 15) * WS + ko;
      const T* xk = xl + (size_t)(k * a.D) * XS + ko;
#pragma unroll
      for (int cc = 0; cc < C; cc += M::KS) {
        typename M::frag af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = M::load(wk + mt * 16 * WS + cc);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int tl = wave * RW + nt * 16 + (lane & 15);
          const typename M::frag bf = M::load(xk + (size_t)(tl * a.S) * XS + cc);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = M::mma(af[mt], bf, acc[mt][nt]);
        }
      }
    }
    if (se) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int o = mt * 16 + 4 * (lane >> 4);
          f32x4 v = acc[mt][nt];
          if (a.bias) {
            const f32x4 bp = *(const f32x4*)(bias_l + o);
            v = f32x4{v[0] + bp[0], v[1] + bp[1], v[2] + bp[2], v[3] + bp[3]};
          }
          const bf16x4 ob = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *(bf16x4*)(stg + (nt * 16 + (lane & 15)) * OP + o) = ob;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // the wave's RW output rows are contiguous (PAIR: row t holds full-resolution rows 2t, 2t+1); rows past the
      // item are dropped by the range check (a 16-byte chunk never straddles a PAIR half)
      const unsigned ib = (unsigned)((long long)rvalid_ * erow * ESZ);
      const __amdgpu_buffer_rsrc_t ry = item_rsrc(a.y, (long long)n * ib, ib);
      constexpr int CPRO = O * 2 / 16, NCH = RW * CPRO / 64;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int e = lane + 64 * i, r = e / CPRO, q = e - r * CPRO;
        const u32x4 c = *(const u32x4*)(stg + r * OP + q * 8);
        __builtin_amdgcn_raw_buffer_store_b128(c, ry, ((t0 + wave * RW + r) * O + q * 8) * 2, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tl = wave * RW + nt * 16 + (lane & 15);
      const int t = t0 + tl;
      if (t >= a.T_out) continue;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int o = mt * 16 + 4 * (lane >> 4);
        const long long oi = out_index(a, n, t, o);
        if (oi < 0) continue;
        // this element inside the staged (unpadded) epilogue tile
        int eidx;
        if (pair) {
          const int Ob = O / 2, p = o >= Ob ? 1 : 0;
          eidx = (2 * tl + p) * Ob + (o - p * Ob);
        } else {
          eidx = tl * O + o;
        }
        f32x4 v = acc[mt][nt];
        if (a.bias) {
          const f32x4 bp = *(const f32x4*)(bias_l + o);
          v = f32x4{v[0] + bp[0], v[1] + bp[1], v[2] + bp[2], v[3] + bp[3]};
        }
        if (do_mask) {
          const f32x4 m = ld4(ml + eidx);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] : 0.f;
        }
        if (do_res) {
          const f32x4 r = ld4(rl + eidx);
          v = f32x4{r[0] + v[0], r[1] + v[1], r[2] + v[2], r[3] + v[3]};
        }
        st4((T*)a.y + oi, v);
      }
    }
  };

  // steady state, unrolled by two so each register set has a static name (rule 20)
  for (int tile = tbeg; tile < tend; tile += 2) {
    // LDS: tile; B: tile+1 (in flight); A: free
    if (tile + 2 < tend) {
      S0 = source(tile + 2);
      A.load(S0, a.T_in);
    }
    run_tile(tile);
    __syncthreads();
    if (tile + 1 >= tend) break;
    B.store(S1, xl, XS, (char*)ml, (char*)rl, relu);
    __syncthreads();
    // LDS: tile+1; A: tile+2 (in flight); B: free
    if (tile + 3 < tend) {
      S1 = source(tile + 3);
      B.load(S1, a.T_in);
    }
    run_tile(tile + 1);
    __syncthreads();
    if (tile + 2 >= tend) break;
    A.store(S0, xl, XS, (char*)ml, (char*)rl, relu);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// The 32-channel residual convs (C = O = 32, direct or stride-1 data-gradient weights, any K <= 4,
// stride 1 or 2) — 80 % of the model's conv traffic — get a leaner kernel than gather_mfma_kernel:
//  * every global access is a raw buffer access through a per-item descriptor, so the hardware range
//    check supplies the SAME zero padding and drops stores past the item end (no per-element guards);
//  * all per-thread chunk offsets are computed once per launch: staging costs one add per 16-byte chunk
//    and the epilogue tensors (ReLU' mask / conv input, residual) are plain contiguous spans;
//  * the ReLU is one packed integer max per dword (a bf16 / fp32 is negative iff its int16 / int32 is);
//  * the tile is held in registers two tiles ahead (T14) exactly as in gather_mfma_kernel.
// FW additionally accumulates the weight gradient of a stride-1 data-gradient from the staged tiles
// (vqa_conv1d_bwd_data_weight): epilogue tensor 0 is then the conv input u.
template <class T> __device__ __forceinline__ u32x4 relu_chunk(u32x4 v);
__device__ __forceinline__ unsigned relu_pk_bf16(unsigned w) {
  const s16x2 z = {0, 0};
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(s16x2, w), z));
}
template <> __device__ __forceinline__ u32x4 relu_chunk<bf16>(u32x4 v) {
  return u32x4{relu_pk_bf16(v.x), relu_pk_bf16(v.y), relu_pk_bf16(v.z), relu_pk_bf16(v.w)};
}
__device__ __forceinline__ unsigned relu_f32_bits(unsigned w) { return (unsigned)max((int)w, 0); }
template <> __device__ __forceinline__ u32x4 relu_chunk<float>(u32x4 v) {
  return u32x4{relu_f32_bits(v.x), relu_f32_bits(v.y), relu_f32_bits(v.z), relu_f32_bits(v.w)};
}

template <class T> __device__ __forceinline__ void store_out4(__amdgpu_buffer_rsrc_t r, int voff, f32x4 v);
template <> __device__ __forceinline__ void store_out4<bf16>(__amdgpu_buffer_rsrc_t r, int voff, f32x4 v) {
  bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), r, voff, 0, 0);
}
template <> __device__ __forceinline__ void store_out4<float>(__amdgpu_buffer_rsrc_t r, int voff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, voff, 0, 0);
}

template <class T, int O, int PVX, int NEP, bool FW> constexpr int conv32_waves() {
  if (FW) return sizeof(T) == 2 ? 3 : 2;
  const int regs = PVX + NEP * (int)sizeof(T) * (O / 32) + (O / 32 - 1) * 4;
  return regs <= 7 ? 4 : (regs <= 11 ? 3 : 2);
}

// x-row byte offset that stays out of range after adding any tile base (|base| < 2^30)
constexpr int kOOB = -0x40000000;

// bf16 output tiles (no fused weight gradient) are staged through LDS over the x rows before they are stored: each
// lane then writes whole 16-byte chunks of contiguous output rows (1 KB per wave store) instead of 8-byte pieces of
// 16 rows (a quarter of a cache line each); the x region is sized for the staged tile (row pitch O + 8)
template <class T, bool FW> constexpr bool conv32_staged() { return !FW && sizeof(T) == 2; }
template <class T, int O, int PVX, bool FW> constexpr int conv32_xelems() {
  constexpr int XS = 32 + 16 / (int)sizeof(T), XROWS = 256 / (32 / (16 / (int)sizeof(T))) * PVX;
  return conv32_staged<T, FW>() && 128 * (O + 8) > XROWS * XS ? 128 * (O + 8) : XROWS * XS;
}

// O = 64: a 32 -> 64 conv, or the PAIR layout (conv-transpose forward, stride-2 data-gradient) whose
// output row j holds the two full-resolution rows 2j, 2j+1 (32 channels each) — the bytes of (B, 2T, 32).
template <class T, int O, int PVX, int NEP, bool FW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(conv32_waves<T, O, PVX, NEP, FW>(), 8)))
void conv32_kernel(GatherArgs a, int ntm, int ntiles, int tpw) {
  typedef Mfma<T> M;
  static_assert(O == 32 || (O == 64 && !FW), "conv32: O = 32 or 64 (64 without FW)");
  constexpr int C = 32, TM = 128, NW = 4, RW = TM / NW, NT = RW / 16, MT = O / 16;
  constexpr int ESZ = (int)sizeof(T), VEC = 16 / ESZ, CPR = C / VEC, ROWB = C * ESZ;
  constexpr int XS = C + lds_pad<T>(), WS = XS;
  constexpr int RSTEP = 256 / CPR;  // x rows between a thread's consecutive chunks
  constexpr int XROWS = RSTEP * PVX;
  constexpr int ECH = TM * O * ESZ / 16 / 256;  // chunks per thread per epilogue tensor
  constexpr int EBYTES = TM * O * ESZ;
  static_assert(NEP >= (FW ? 1 : 0) && NEP <= 2, "epilogue tensors");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* wl = (T*)smem;
  T* xl = wl + (size_t)a.K * O * WS;
  char* el = (char*)(xl + (size_t)conv32_xelems<T, O, PVX, FW>());
  constexpr bool SE = conv32_staged<T, FW>();
  constexpr int OP = O + 8;  // staged row pitch (elements)

  const int tbeg = blockIdx.x * tpw, tend = min(ntiles, tbeg + tpw);
  if (tbeg >= tend) return;
  const bool do_mask = a.flags & VQA_POST_MASK, do_res = a.flags & VQA_ADD_RESIDUAL;
  const bool relu = a.flags & VQA_PRE_RELU;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int ko = M::koff(lane);
  const int rows_in = (TM - 1) * a.S + (a.K - 1) * a.D + 1;
  // epilogue tensor slots: [mask or conv input (FW)] then [residual]
  const bool has_m = do_mask || FW;
  const void* ep0 = has_m ? a.mask : a.resid;
  const void* ep1 = a.resid;
  const T* ml = (const T*)el;                                   // valid when has_m
  const T* rl = (const T*)(el + (has_m ? EBYTES : 0));          // valid when do_res
  const unsigned xbytes = (unsigned)a.T_in * ROWB;
  // PAIR: the item's valid bytes end at full-resolution row T_full (the range check drops the rest)
  const bool pair = a.wmode == W_PAIR;
  const unsigned obytes = pair ? (unsigned)a.T_full * (O / 2) * ESZ : (unsigned)a.T_out * O * ESZ;

  // per-thread chunk geometry, fixed for the launch
  const int q = threadIdx.x % CPR, row0 = threadIdx.x / CPR;
  int gx[PVX];
#pragma unroll
  for (int i = 0; i < PVX; ++i) gx[i] = (row0 + i * RSTEP < rows_in) ? (row0 + i * RSTEP) * ROWB + q * 16 : kOOB;
  const int lx = (row0 * XS) * ESZ + q * 16;  // + i * RSTEP * XS * ESZ
  const int ge = threadIdx.x * 16;            // + j * 4096 (epilogue chunks)

  u32x4 ra[PVX + NEP * ECH], rb[PVX + NEP * ECH];
  auto load = [&](u32x4* r, int tile) {
    const int n = tile / ntm, t0 = (tile - n * ntm) * TM;
    const __amdgpu_buffer_rsrc_t rx = item_rsrc(a.x, (long long)n * xbytes, xbytes);
    const int xb = (t0 * a.S - a.P) * ROWB;
#pragma unroll
    for (int i = 0; i < PVX; ++i) r[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, gx[i] + xb, 0, 0);
    if constexpr (NEP > 0) {
      const int eb = t0 * O * ESZ;
      const __amdgpu_buffer_rsrc_t r0 = item_rsrc(ep0, (long long)n * obytes, obytes);
#pragma unroll
      for (int j = 0; j < ECH; ++j) r[PVX + j] = __builtin_amdgcn_raw_buffer_load_b128(r0, ge + j * 4096 + eb, 0, 0);
      if constexpr (NEP > 1) {
        const __amdgpu_buffer_rsrc_t r1 = item_rsrc(ep1, (long long)n * obytes, obytes);
#pragma unroll
        for (int j = 0; j < ECH; ++j)
          r[PVX + ECH + j] = __builtin_amdgcn_raw_buffer_load_b128(r1, ge + j * 4096 + eb, 0, 0);
      }
    }
  };
  auto store = [&](const u32x4* r) {
#pragma unroll
    for (int i = 0; i < PVX; ++i)
      *(u32x4*)((char*)xl + lx + i * RSTEP * XS * ESZ) = relu ? relu_chunk<T>(r[i]) : r[i];
#pragma unroll
    for (int j = 0; j < NEP * ECH; ++j) *(u32x4*)(el + ge + j * 4096) = r[PVX + j];
  };

  // fused weight gradient accumulators (C = O = 32: wave w owns ci-tile w>>1, co-tile w&1 of every tap)
  f32x4 wacc[4], wdb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) wacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias of this lane's 4 output channels per 16-channel block
  f32x4 bias[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int o = mt * 16 + 4 * (lane >> 4), bo = pair ? (o & (O / 2 - 1)) : o;  // PAIR: halves share the bias
    bias[mt] = a.bias ? f32x4{a.bias[bo], a.bias[bo + 1], a.bias[bo + 2], a.bias[bo + 3]} : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  stage_weights<T, C, O>(a, wl, WS);
  load(ra, tbeg);
  if (tbeg + 1 < tend) load(rb, tbeg + 1);
  store(ra);
  __syncthreads();

  auto run_tile = [&](int tile) {
    const int n = tile / ntm, t0 = (tile - n * ntm) * TM;
    // the accumulators start at the bias (the fused residual block's convs do the same: bit-identical outputs)
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = bias[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // K <= 4 (host-checked): unrolled, uniform exit
      if (k >= a.K) break;
      const T* wk = wl + (size_t)k * O * WS + (lane & 15) * WS + ko;
      const T* xk = xl + (size_t)(k * a.D) * XS + ko;
#pragma unroll
      for (int cc = 0; cc < C; cc += M::KS) {
        typename M::frag af[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) af[mt] = M::load(wk + mt * 16 * WS + cc);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int tl = wave * RW + nt * 16 + (lane & 15);
          const typename M::frag bf = M::load(xk + (size_t)(tl * a.S) * XS + cc);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = M::mma(af[mt], bf, acc[mt][nt]);
        }
      }
    }
    const __amdgpu_buffer_rsrc_t ry = item_rsrc(a.y, (long long)n * obytes, obytes);
    const int yb = t0 * O * ESZ;
    T* stg = xl + (size_t)wave * RW * OP;  // SE: this wave's staged rows
    if constexpr (SE) __syncthreads();     // every wave's MFMA reads of the x rows are done
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tl = wave * RW + nt * 16 + (lane & 15);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int o = mt * 16 + 4 * (lane >> 4);
        const int eidx = tl * O + o;
        f32x4 v = acc[mt][nt];
        if (do_mask) {
          const f32x4 m = ld4(ml + eidx);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = m[i] > 0.f ? v[i] : 0.f;
        }
        if (do_res) v = ld4(rl + eidx) + v;
        if constexpr (SE) {
          const bf16x4 ob = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *(bf16x4*)(stg + (nt * 16 + (lane & 15)) * OP + o) = ob;
        } else {
          store_out4<T>(ry, eidx * ESZ + yb, v);
        }
      }
    }
    if constexpr (SE) {
      // the wave's RW rows are contiguous in the output: 16-byte chunks, rows past the item dropped by the range
      // check (a chunk never straddles a PAIR half: 32 channels = 4 chunks)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      constexpr int CPRO = O * 2 / 16, NCH = RW * CPRO / 64;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int e = lane + 64 * i, r = e / CPRO, q = e - r * CPRO;
        const u32x4 c = *(const u32x4*)(stg + r * OP + q * 8);
        __builtin_amdgcn_raw_buffer_store_b128(c, ry, ((wave * RW + r) * O + q * 8) * 2 + yb, 0, 0);
      }
    }
    if constexpr (FW) {
      const int it = wave >> 1, jt = wave & 1;
      const T* up = ml + it * 16;
      const T* gp = xl + jt * 16;
#pragma unroll 1
      for (int kk = 0; kk < TM; kk += M::KS) {
        typename M::frag af = M::rows(up + (size_t)kk * O, O);
        if (a.wrelu) af = relu_frag(af);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < a.K) {
            const typename M::frag bf = M::rows(gp + (size_t)(kk + (a.K - 1 - k) * a.D) * XS, XS);
            wacc[k] = M::mma(af, bf, wacc[k]);
          }
        }
        if (it == 0) {
          const typename M::frag bo = M::rows(gp + (size_t)(kk + a.P) * XS, XS);
          wdb = M::mma(M::ones(), bo, wdb);
        }
      }
    }
  };

  for (int tile = tbeg; tile < tend; tile += 2) {
    // LDS: tile; rb: tile+1 (in flight); ra: free
    if (tile + 2 < tend) load(ra, tile + 2);
    run_tile(tile);
    __syncthreads();
    if (tile + 1 >= tend) break;
    store(rb);
    __syncthreads();
    if (tile + 3 < tend) load(rb, tile + 3);
    run_tile(tile + 1);
    __syncthreads();
    if (tile + 2 >= tend) break;
    store(ra);
    __syncthreads();
  }
  if constexpr (FW) {
    float* out = a.wpart + (size_t)blockIdx.x * (size_t)(a.K * O * C + C);
    const int it = wave >> 1, jt = wave & 1;
    const int co = jt * 16 + (lane & 15);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < a.K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) out[((size_t)k * O + it * 16 + 4 * (lane >> 4) + r) * C + co] = wacc[k][r];
      }
    }
    if (it == 0 && lane < 16) out[a.K * O * C + co] = wdb[0];
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient: dW[k][c][o] = sum_{n,t} act(x[n, t*S + k*D - P, c]) * g[n, t, o],
// db[o] = sum_{n,t} g[n, t, o]. Grid = (chunks per item, items); each workgroup reduces CH output
// rows in TT-row sub-tiles staged in LDS and writes fp32 partials [wg][K*C*O + O]; a second
// kernel sums the partials in a fixed order (deterministic).
struct WgradArgs {
  const void* x;
  const void* g;
  float* ws;
  int B, T_in, T_out, C, O, K, S, D, P;
  int CH, nchunk;
  int flags;  // VQA_PRE_RELU, VQA_X_F32, VQA_Y_F32, WG_DB_FROM_X
  int nb;     // bias entries per partial: O (bias = column sums of g) or C (WG_DB_FROM_X)
};

// bias gradient = column sums of the INPUT x over the rows this workgroup owns (conv-transpose bias:
// its output-gradient is the gather input of the weight gradient)
constexpr int WG_DB_FROM_X = 1 << 8;

template <class T, int C, int O, int TT>
__global__ __launch_bounds__(256) void wgrad_mfma_kernel(WgradArgs a) {
  typedef Mfma<T> M;
  constexpr int XS = C + lds_pad<T>();
  constexpr int GS = O + lds_pad<T>();
  constexpr int CT = C / 16, OT = O / 16;
  constexpr int MAXTW = CT * OT;  // max tiles per wave (K <= 4 taps over 4 waves)
  constexpr int KT = (int)sizeof(T) == 2 ? 32 : 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* gl = (T*)smem;
  T* xl = gl + TT * GS;
  __shared__ float red[256];

  const int n = blockIdx.y, ch = blockIdx.x;
  const int tbeg = ch * a.CH, tend = min(a.T_out, tbeg + a.CH);
  const int rows_in = (TT - 1) * a.S + (a.K - 1) * a.D + 1;
  const int ntile = a.K * CT * OT;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;

  f32x4 acc[MAXTW];
#pragma unroll
  for (int i = 0; i < MAXTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  const bool db_x = a.flags & WG_DB_FROM_X;
  const int NB = db_x ? C : O;
  const int dbo = threadIdx.x % NB, dbr = threadIdx.x / NB, dbstep = 256 / NB;

  const bool relu = a.flags & VQA_PRE_RELU;
  const T* Gi = (const T*)a.g + (long long)n * a.T_out * O;
  const T* Xi = (const T*)a.x + (long long)n * a.T_in * C;
  RowStager<T, O, 4> sg;
  // input chunks per thread: the model's input spans without the tail loop (whose loads were waited for one by one
  // before every sub-tile's store): bf16 C = 32 stride 2 K = 4 (258 rows x 4 chunks) -> 5; C = 64 stride 1 K = 3
  // (130 x 8) and stride 2 K = 4 (258 x 8) -> 9
  RowStager<T, C, sizeof(T) == 2 ? (C == 32 ? 5 : (C == 64 ? 9 : 4)) : 4> sx;
  if (tbeg < tend) {
    const int nrows = min(TT, tend - tbeg);
    sg.load(Gi, tbeg, tbeg + nrows, tbeg, TT);
    sx.load(Xi, 0, a.T_in, tbeg * a.S - a.P, rows_in);
    sg.store(gl, GS, TT, false);
    sg.tail(gl, GS, Gi, tbeg, tbeg + nrows, tbeg, TT, false);
    sx.store(xl, XS, rows_in, relu);
    sx.tail(xl, XS, Xi, 0, a.T_in, tbeg * a.S - a.P, rows_in, relu);
  }
  __syncthreads();
  for (int t0 = tbeg; t0 < tend; t0 += TT) {
    const int nrows = min(TT, tend - t0);
    const int t1 = t0 + TT;
    const bool has_next = t1 < tend;
    const int nrows1 = has_next ? min(TT, tend - t1) : 0;
    if (has_next) {  // prefetch the next sub-tile while this one is reduced
      sg.load(Gi, t1, t1 + nrows1, t1, TT);
      sx.load(Xi, 0, a.T_in, t1 * a.S - a.P, rows_in);
    }
    if (db_x) {
      for (int r = a.P + dbr; r < a.P + nrows * a.S; r += dbstep) dbacc += (float)xl[r * XS + dbo];
    } else {
      for (int r = dbr; r < nrows; r += dbstep) dbacc += (float)gl[r * GS + dbo];
    }
#pragma unroll
    for (int ti = 0; ti < MAXTW; ++ti) {
      const int tile = wave + 4 * ti;
      if (tile < ntile) {
        const int ot = tile % OT, rest = tile / OT, ct = rest % CT, k = rest / CT;
        // K = output rows: transposed LDS reads of both operands (same even/odd K order)
        const T* xp = xl + (size_t)(k * a.D) * XS + ct * 16;
        const T* gp = gl + ot * 16;
        f32x4 c = acc[ti];
#pragma unroll
        for (int kk = 0; kk < TT; kk += KT) {
          const typename M::frag af = M::rows_eo(xp + (size_t)(kk * a.S) * XS, a.S * XS);
          const typename M::frag bf = M::rows_eo(gp + (size_t)kk * GS, GS);
          c = M::mma(af, bf, c);
        }
        acc[ti] = c;
      }
    }
    __syncthreads();
    if (has_next) {
      sg.store(gl, GS, TT, false);
      sg.tail(gl, GS, Gi, t1, t1 + nrows1, t1, TT, false);
      sx.store(xl, XS, rows_in, relu);
      sx.tail(xl, XS, Xi, 0, a.T_in, t1 * a.S - a.P, rows_in, relu);
    }
    __syncthreads();
  }

  float* out = a.ws + (size_t)(n * a.nchunk + ch) * (size_t)(a.K * C * O + NB);
#pragma unroll
  for (int ti = 0; ti < MAXTW; ++ti) {
    const int tile = wave + 4 * ti;
    if (tile < ntile) {
      const int ot = tile % OT, rest = tile / OT, ct = rest % CT, k = rest / CT;
      const int o = ot * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = ct * 16 + 4 * (lane >> 4) + r;
        out[((size_t)k * C + c) * O + o] = acc[ti][r];
      }
    }
  }
  red[threadIdx.x] = dbacc;
  __syncthreads();
  if (threadIdx.x < NB) {
    float s = 0.f;
    for (int r = 0; r < dbstep; ++r) s += red[r * NB + threadIdx.x];
    out[a.K * C * O + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// Thin weight gradients for the 1-channel waveform layers. Threads = RL row lanes x VL lanes of 8
// consecutive channels along the WIDE side; 16-byte loads along it; LDS reduction over row lanes.
//   WIDE_X: C % 8 == 0, O <= 2 (decoder output conv, C=64 -> O=1)
//   WIDE_G: O % 8 == 0, C <= 2 (first encoder conv, C=1 -> O=32)
template <class T> __device__ __forceinline__ void ld8(const T* p, float* v);
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, float* v) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> __device__ __forceinline__ void ld8<float>(const float* p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = a[j];
    v[j + 4] = b[j];
  }
}
template <class T> __device__ __forceinline__ void st8(T* p, const float* v);
template <> __device__ __forceinline__ void st8<bf16>(bf16* p, const float* v) {
  bf16x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
  *(bf16x8*)p = x;
}
template <> __device__ __forceinline__ void st8<float>(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

// buffer loads converting to fp32 (an out-of-range offset reads zeros)
template <class T> __device__ __forceinline__ float ld1_buf(__amdgpu_buffer_rsrc_t r, int off);
template <> __device__ __forceinline__ float ld1_buf<float>(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <> __device__ __forceinline__ float ld1_buf<bf16>(__amdgpu_buffer_rsrc_t r, int off) {
  return __uint_as_float((unsigned)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0) << 16);
}
template <class T> __device__ __forceinline__ void ld8_buf(__amdgpu_buffer_rsrc_t r, int off, float* v);
template <> __device__ __forceinline__ void ld8_buf<bf16>(__amdgpu_buffer_rsrc_t r, int off, float* v) {
  const u32x4 w = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
template <> __device__ __forceinline__ void ld8_buf<float>(__amdgpu_buffer_rsrc_t r, int off, float* v) {
  const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __uint_as_float(a[i]);
    v[i + 4] = __uint_as_float(b[i]);
  }
}

// NM: the narrow side's width bound (1 for the model's 1-channel ends: half the accumulators and tap registers of
// NM = 2, 29.4 vs 33.6 us for the first encoder conv at cfg2, the same sums in the same order)
template <class TX, class TG, bool WIDE_X, int NM>
__global__ __launch_bounds__(256) void wgrad_thin_kernel(WgradArgs a) {
  constexpr int KM = 4, U = 8;  // max taps, rows in flight per thread
  const int W = WIDE_X ? a.C : a.O;
  const int NN = WIDE_X ? a.O : a.C;
  const int VL = W / 8, RL = 256 / VL;
  const int v = threadIdx.x % VL, rl = threadIdx.x / VL;
  const int n = blockIdx.y, ch = blockIdx.x;
  const int tbeg = ch * a.CH, tend = min(a.T_out, tbeg + a.CH);
  const bool relu = a.flags & VQA_PRE_RELU;
  // the item's rows as buffer resources (host-checked: an item is < 2^30 bytes)
  const unsigned xbytes = (unsigned)a.T_in * a.C * (unsigned)sizeof(TX), gbytes = (unsigned)a.T_out * a.O * (unsigned)sizeof(TG);
  const __amdgpu_buffer_rsrc_t rx = item_rsrc(a.x, (long long)n * xbytes, xbytes);
  const __amdgpu_buffer_rsrc_t rg = item_rsrc(a.g, (long long)n * gbytes, gbytes);
  float acc[KM][NM][8];
  float bacc[8];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int i = 0; i < NM; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][i][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) bacc[j] = 0.f;
  if (rl < RL) {
    // U rows per iteration, all loads issued before the FMAs (memory-level parallelism)
    for (int t = tbeg + rl; t < tend; t += U * RL) {
      float gv[U][WIDE_X ? NM : 8];
      float xv[U][KM][WIDE_X ? 8 : NM];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // every load issued unconditionally: rows past the chunk and taps outside the item get an out-of-range
        // buffer offset (kOOB), which reads zeros (a load in a branch was waited for right there: 8 serial round
        // trips per iteration, 33 us at the first conv)
        const int tt = t + u * RL;
        const bool okr = tt < tend;
        const int goff = okr ? (tt * a.O + (WIDE_X ? 0 : v * 8)) * (int)sizeof(TG) : kOOB;
        if (WIDE_X) {
#pragma unroll
          for (int i = 0; i < NM; ++i) gv[u][i] = ld1_buf<TG>(rg, i < NN ? goff + i * (int)sizeof(TG) : kOOB);
        } else {
          ld8_buf<TG>(rg, goff, gv[u]);
        }
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          const int ti = tt * a.S + k * a.D - a.P;
          const bool ok = okr && k < a.K && ti >= 0 && ti < a.T_in;
          const int xoff = ok ? (ti * a.C + (WIDE_X ? v * 8 : 0)) * (int)sizeof(TX) : kOOB;
          if (WIDE_X) {
            ld8_buf<TX>(rx, xoff, xv[u][k]);
          } else {
#pragma unroll
            for (int i = 0; i < NM; ++i) xv[u][k][i] = ld1_buf<TX>(rx, i < NN ? xoff + i * (int)sizeof(TX) : kOOB);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (WIDE_X) {
          if (v == 0)
#pragma unroll
            for (int i = 0; i < NM; ++i) bacc[i] += gv[u][i];
#pragma unroll
          for (int k = 0; k < KM; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float x = relu ? fmaxf(xv[u][k][j], 0.f) : xv[u][k][j];
#pragma unroll
              for (int i = 0; i < NM; ++i) acc[k][i][j] += x * gv[u][i];
            }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) bacc[j] += gv[u][j];
#pragma unroll
          for (int k = 0; k < KM; ++k)
#pragma unroll
            for (int i = 0; i < NM; ++i) {
              const float x = relu ? fmaxf(xv[u][k][i], 0.f) : xv[u][k][i];
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[k][i][j] += x * gv[u][j];
            }
        }
      }
    }
  }
  // reduce over row lanes: per thread KM*NM*8 + 8 values
  constexpr int PER = KM * NM * 8 + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = (float*)smem;  // [256][PER]
  {
    float* r = red + threadIdx.x * PER;
    int q = 0;
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int i = 0; i < NM; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[q++] = acc[k][i][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[q++] = bacc[j];
  }
  __syncthreads();
  const int KCO = a.K * a.C * a.O;
  float* out = a.ws + (size_t)(n * a.nchunk + ch) * (size_t)(KCO + a.nb);
  for (int e = threadIdx.x; e < KCO + a.nb; e += 256) {
    int vv, q;
    if (e < KCO) {
      const int o = e % a.O, c = (e / a.O) % a.C, k = e / (a.O * a.C);
      const int wide = WIDE_X ? c : o, narrow = WIDE_X ? o : c;
      vv = wide / 8;
      q = (k * NM + narrow) * 8 + (wide % 8);
    } else {
      const int o = e - KCO;
      vv = WIDE_X ? 0 : o / 8;
      q = KM * NM * 8 + (WIDE_X ? o : o % 8);
    }
    float sum = 0.f;
    for (int r = 0; r < RL; ++r) sum += red[(r * VL + vv) * PER + q];
    out[e] = sum;
  }
}

// Generic VALU weight gradient (small K*C*O: the 1-channel layers). Same partial layout.
template <class TX, class TG, int TT>
__global__ __launch_bounds__(256) void wgrad_direct_kernel(WgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* gl = (float*)smem;           // [TT][O]
  float* xl = gl + TT * a.O;          // [rows_in][C]
  constexpr int EPT = 16;
  const int n = blockIdx.y, ch = blockIdx.x;
  const int tbeg = ch * a.CH, tend = min(a.T_out, tbeg + a.CH);
  const int rows_in = (TT - 1) * a.S + (a.K - 1) * a.D + 1;
  const int E = a.K * a.C * a.O;
  const int e0 = blockIdx.z * EPT * 256;  // this slice's weight elements [e0, e0 + 4096) (gridDim.z slices)
  const bool relu = a.flags & VQA_PRE_RELU;
  float acc[EPT];
#pragma unroll
  for (int i = 0; i < EPT; ++i) acc[i] = 0.f;
  float dbacc = 0.f;
  for (int t0 = tbeg; t0 < tend; t0 += TT) {
    const int nrows = min(TT, tend - t0);
    for (int e = threadIdx.x; e < TT * a.O; e += blockDim.x) {
      const int r = e / a.O, o = e - r * a.O;
      gl[e] = r < nrows ? ld((const TG*)a.g + ((long long)n * a.T_out + t0 + r) * a.O + o) : 0.f;
    }
    for (int e = threadIdx.x; e < rows_in * a.C; e += blockDim.x) {
      const int r = e / a.C, c = e - r * a.C;
      const int ti = t0 * a.S - a.P + r;
      float v = (ti >= 0 && ti < a.T_in) ? ld((const TX*)a.x + ((long long)n * a.T_in + ti) * a.C + c) : 0.f;
      xl[e] = relu ? fmaxf(v, 0.f) : v;
    }
    __syncthreads();
    if (blockIdx.z == 0) {
      if (a.flags & WG_DB_FROM_X) {
        if (threadIdx.x < a.C)
          for (int r = a.P; r < a.P + nrows * a.S; ++r) dbacc += xl[r * a.C + threadIdx.x];
      } else if (threadIdx.x < a.O) {
        for (int r = 0; r < nrows; ++r) dbacc += gl[r * a.O + threadIdx.x];
      }
    }
#pragma unroll
    for (int i = 0; i < EPT; ++i) {
      const int e = e0 + threadIdx.x + i * 256;
      if (e < E) {
        const int o = e % a.O, c = (e / a.O) % a.C, k = e / (a.O * a.C);
        float s = acc[i];
        for (int r = 0; r < nrows; ++r) s += xl[(r * a.S + k * a.D) * a.C + c] * gl[r * a.O + o];
        acc[i] = s;
      }
    }
    __syncthreads();
  }
  float* out = a.ws + (size_t)(n * a.nchunk + ch) * (size_t)(E + a.nb);
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int e = e0 + threadIdx.x + i * 256;
    if (e < E) out[e] = acc[i];
  }
  if (blockIdx.z == 0 && threadIdx.x < a.nb) out[E + threadIdx.x] = dbacc;
}

// out1[e] = sum_p ws[p*E + e] for e < E1, out2[e - E1] likewise for e >= E1. Block = 16 elements x 16 part
// groups (64-byte row segments); each thread keeps 8 independent partial sums (memory-level parallelism);
// the sums and then the groups are combined in a fixed order, so the result is deterministic.
constexpr int kRedCols = 16;
__device__ __forceinline__ float reduce_col16(const float* ws, int nparts, int E, int e, float (*red)[kRedCols]) {
  const int el = threadIdx.x & (kRedCols - 1), grp = threadIdx.x / kRedCols;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (e < E) {
    int p = grp;
    for (; p + 7 * 16 < nparts; p += 8 * 16)
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += ws[(size_t)(p + 16 * u) * E + e];
    for (; p < nparts; p += 16) s[0] += ws[(size_t)p * E + e];
  }
  red[grp][el] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  float t = 0.f;
  if (grp == 0)
    for (int g = 0; g < 16; ++g) t += red[g][el];
  return t;
}

// Wide form (rows whose length and base keep float4 alignment): block = 256 elements (64 lanes x 4) of every
// partial row, each wave reading 1 KB of one row per load (4 rows at a time over the 4 waves, 8 rows in flight
// per wave); the 8 per-thread sums, then the 4 waves, are combined in a fixed order: deterministic.
constexpr int kRedCols256 = 256;
__device__ __forceinline__ f32x4 reduce_col256(const float* ws, int nparts, int E, int e, f32x4 (*red)[64]) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  f32x4 s[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (e < E) {
    int p = wave;
    for (; p + 4 * 7 < nparts; p += 4 * 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += *(const f32x4*)(ws + (size_t)(p + 4 * u) * E + e);
    for (; p < nparts; p += 4) s[0] += *(const f32x4*)(ws + (size_t)p * E + e);
  }
  red[wave][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  f32x4 t = {0.f, 0.f, 0.f, 0.f};
  if (wave == 0) t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
  return t;
}

static bool desc_vec4(const vqa_partials_desc& d) {
  return d.n % 4 == 0 && ((uintptr_t)d.partials & 15) == 0;
}

__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* ws, int nparts, int E, int E1,
                                                             float* out1, float* out2) {
  __shared__ float red[16][kRedCols];
  const int e = blockIdx.x * kRedCols + (threadIdx.x & (kRedCols - 1));
  const float s = reduce_col16(ws, nparts, E, e, red);
  if (threadIdx.x < kRedCols && e < E) {
    if (e < E1) {
      if (out1) out1[e] = s;
    } else if (out2) {
      out2[e - E1] = s;
    }
  }
}

// Batched form: one launch reduces up to kMaxDescs layers; block b belongs to the descriptor whose
// [start, start + ceil(n/16)) range contains it. Same fixed summation order as reduce_partials_kernel.
constexpr int kMaxDescs = 48;
struct ReduceBatch {
  vqa_partials_desc d[kMaxDescs];
  int start[kMaxDescs + 1];
  int vec4[kMaxDescs];
  int count;
};

__global__ __launch_bounds__(256) void reduce_partials_batched_kernel(ReduceBatch rb) {
  __shared__ f32x4 red4[16][16];
  int i = 0;
  while (i + 1 < rb.count && (int)blockIdx.x >= rb.start[i + 1]) ++i;
  const vqa_partials_desc& d = rb.d[i];
  if (rb.vec4[i]) {
#ifdef VQA_REDUCE_COL64  // A/B only: the round-3 layout (64 columns x 16 row groups per block)
    const int e = ((int)blockIdx.x - rb.start[i]) * 64 + 4 * (threadIdx.x & 15);
    f32x4 s;
    {
      const int el = threadIdx.x & 15, grp = threadIdx.x >> 4;
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e < d.n) {
        int p = grp;
        for (; p + 7 * 16 < d.nparts; p += 8 * 16)
#pragma unroll
          for (int u = 0; u < 8; ++u) t[u] += *(const f32x4*)(d.partials + (size_t)(p + 16 * u) * d.n + e);
        for (; p < d.nparts; p += 16) t[0] += *(const f32x4*)(d.partials + (size_t)p * d.n + e);
      }
      red4[grp][el] = ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
      __syncthreads();
      s = f32x4{0.f, 0.f, 0.f, 0.f};
      if (grp == 0)
        for (int g = 0; g < 16; ++g) s += red4[g][el];
    }
    if (threadIdx.x < 16 && e < d.n) {
#else
    const int e = ((int)blockIdx.x - rb.start[i]) * kRedCols256 + 4 * (threadIdx.x & 63);
    const f32x4 s = reduce_col256(d.partials, d.nparts, d.n, e, (f32x4(*)[64])red4);
    if (threadIdx.x < 64 && e < d.n) {
#endif
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int eq = e + q;
        if (eq < d.n_w) {
          if (d.dw) d.dw[eq] = s[q];
        } else if (d.db) {
          d.db[eq - d.n_w] = s[q];
        }
      }
    }
    return;
  }
  float(*red)[kRedCols] = (float(*)[kRedCols])red4;
  const int e = ((int)blockIdx.x - rb.start[i]) * kRedCols + (threadIdx.x & (kRedCols - 1));
  const float s = reduce_col16(d.partials, d.nparts, d.n, e, red);
  if (threadIdx.x < kRedCols && e < d.n) {
    if (e < d.n_w) {
      if (d.dw) d.dw[e] = s;
    } else if (d.db) {
      d.db[e - d.n_w] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// Raise a kernel's dynamic-LDS limit only when a launch needs more than the 64 KiB default; the value is
// the exact need (static LDS counts against the 160 KiB too). Cached per kernel, so it runs during the
// eager warm-up, never inside a hipGraph capture.
static int ensure_dyn_lds(const void* fn, size_t bytes, size_t* cached, const char* name) {
  if (bytes <= 65536 || bytes <= *cached) return VQA_OK;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    vqa::set_error("%s: cannot reserve %zu B of LDS: %s", name, bytes, hipGetErrorString(e));
    return VQA_E_UNSUPPORTED;
  }
  *cached = bytes;
  return VQA_OK;
}
static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

// resident workgroups per CU the persistent grid assumes at most (also bounds the fused-wgrad partials)
constexpr int kMaxGatherPerCU = 4;

// rows per workgroup tile: all O channels x TM rows; TM keeps VGPRs <= ~128 (3 waves/SIMD)
static int gather_tm(int O, int S) {
  (void)S;
  return O == 32 ? 128 : 64;
}

// persistent grid = the resident workgroups (VGPR- and LDS-limited), so no workgroup waits for a second
// round; tiles are split into contiguous ranges (a tile's halo rows were just read by its predecessor)
static int persistent_grid(const void* fn, size_t lds, int* per_cu, size_t* per_cu_lds, int ntiles, int* tpw) {
  if (*per_cu == 0 || *per_cu_lds != lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, 256, lds) != hipSuccess || nb < 1) {
      (void)hipGetLastError();
      nb = 1;
    }
    *per_cu = nb > kMaxGatherPerCU ? kMaxGatherPerCU : nb;
    *per_cu_lds = lds;
  }
  int nwg = num_cus() * *per_cu;
  if (nwg > ntiles) nwg = ntiles;
  *tpw = (ntiles + nwg - 1) / nwg;
  return (ntiles + *tpw - 1) / *tpw;
}

template <class T, int C, int O, int TM, int PV>
static int launch_gather_mfma_pv(const GatherArgs& a, size_t lds, hipStream_t s) {
  const void* fn = (const void*)gather_mfma_kernel<T, C, O, TM, PV>;
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds(fn, lds, &lds_set, "gather_mfma_kernel");
  if (rc != VQA_OK) return rc;
  const int ntm = (a.T_out + TM - 1) / TM;
  const int ntiles = ntm * a.B;
  static int per_cu = 0;
  static size_t per_cu_lds = 0;
  int tpw = 0;
  const int nwg = persistent_grid(fn, lds, &per_cu, &per_cu_lds, ntiles, &tpw);
  hipLaunchKernelGGL((gather_mfma_kernel<T, C, O, TM, PV>), dim3(nwg), dim3(256), lds, s, a, ntm, ntiles, tpw);
  VQA_LAUNCHED("gather_mfma_kernel");
  return VQA_OK;
}

// epilogue tiles staged per tile: ReLU' mask / conv input (fused wgrad), residual
static int gather_nep(const GatherArgs& a, bool fw) {
  return (((a.flags & VQA_POST_MASK) || fw) ? 1 : 0) + ((a.flags & VQA_ADD_RESIDUAL) ? 1 : 0);
}

template <class T, int C, int O, int TM>
static int launch_gather_mfma_t(const GatherArgs& a, hipStream_t s) {
  constexpr int XS = C + lds_pad<T>(), WS = C + lds_pad<T>();
  const int rows_in = (TM - 1) * a.S + (a.K - 1) * a.D + 1;
  const int nep = gather_nep(a, false);
  const size_t ebytes = (size_t)TM * O * sizeof(T);
  const size_t lds = ((size_t)a.K * O * WS + (size_t)rows_in * XS) * sizeof(T) + 2 * ebytes;
  VQA_REQUIRE(lds <= 160 * 1024, VQA_E_UNSUPPORTED, "gather conv: LDS tile too large (%zu B)", lds);
  // 16-byte chunks per tile held in registers per thread; a tile only a few chunks over a multiple of
  // 256 must not pay for the next size up
  const long long chunks = (long long)rows_in * C * sizeof(T) / 16 + (long long)nep * TM * O * sizeof(T) / 16;
  const int pv = (int)((chunks + 255) / 256);
  if (pv <= 3) return launch_gather_mfma_pv<T, C, O, TM, 3>(a, lds, s);
  if (pv <= 4) return launch_gather_mfma_pv<T, C, O, TM, 4>(a, lds, s);
  if (pv <= 5) return launch_gather_mfma_pv<T, C, O, TM, 5>(a, lds, s);
  if (pv <= 8) return launch_gather_mfma_pv<T, C, O, TM, 8>(a, lds, s);
  if (pv <= 12) return launch_gather_mfma_pv<T, C, O, TM, 12>(a, lds, s);
  vqa::set_error("gather conv: tile of %lld chunks exceeds the register stager", chunks);
  return VQA_E_UNSUPPORTED;
}

template <class T, int C, int O>
static int launch_gather_mfma_o(const GatherArgs& a, hipStream_t s) {
  if constexpr (O == 32) return launch_gather_mfma_t<T, C, O, 128>(a, s);
  else return launch_gather_mfma_t<T, C, O, 64>(a, s);
}

template <class T>
static int launch_gather_mfma(const GatherArgs& a, hipStream_t s) {
  if (a.C == 32) {
    if (a.O == 32) return launch_gather_mfma_o<T, 32, 32>(a, s);
    if (a.O == 64) return launch_gather_mfma_o<T, 32, 64>(a, s);
    if (a.O == 128) return launch_gather_mfma_o<T, 32, 128>(a, s);
  } else if (a.C == 64) {
    if (a.O == 32) return launch_gather_mfma_o<T, 64, 32>(a, s);
    if (a.O == 64) return launch_gather_mfma_o<T, 64, 64>(a, s);
    if (a.O == 128) return launch_gather_mfma_o<T, 64, 128>(a, s);
  }
  vqa::set_error("gather conv: no MFMA tile for C=%d O=%d", a.C, a.O);
  return VQA_E_UNSUPPORTED;
}

// ---- the 32-channel kernel
template <class T, int O, int PVX, int NEP, bool FW>
static int launch_conv32_k(const GatherArgs& a, hipStream_t s, int* nwg_out) {
  constexpr int ESZ = (int)sizeof(T), XS = 32 + lds_pad<T>();
  const size_t lds = ((size_t)a.K * O * XS + (size_t)conv32_xelems<T, O, PVX, FW>()) * ESZ + (size_t)NEP * 128 * O * ESZ;
  const void* fn = (const void*)conv32_kernel<T, O, PVX, NEP, FW>;
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds(fn, lds, &lds_set, "conv32_kernel");
  if (rc != VQA_OK) return rc;
  const int ntm = (a.T_out + 127) / 128;
  const int ntiles = ntm * a.B;
  static int per_cu = 0;
  static size_t per_cu_lds = 0;
  int tpw = 0;
  const int nwg = persistent_grid(fn, lds, &per_cu, &per_cu_lds, ntiles, &tpw);
  if (nwg_out) *nwg_out = nwg;
  hipLaunchKernelGGL((conv32_kernel<T, O, PVX, NEP, FW>), dim3(nwg), dim3(256), lds, s, a, ntm, ntiles, tpw);
  VQA_LAUNCHED("conv32_kernel");
  return VQA_OK;
}

template <class T, int PVX, bool FW>
static int launch_conv32_n(const GatherArgs& a, int nep, hipStream_t s, int* nwg_out) {
  if constexpr (!FW) {
    if (a.O == 64) {
      if (nep == 0) return launch_conv32_k<T, 64, PVX, 0, false>(a, s, nwg_out);
      if (nep == 1) return launch_conv32_k<T, 64, PVX, 1, false>(a, s, nwg_out);
      return launch_conv32_k<T, 64, PVX, 2, false>(a, s, nwg_out);
    }
    if (nep == 0) return launch_conv32_k<T, 32, PVX, 0, FW>(a, s, nwg_out);
  }
  if (nep == 1) return launch_conv32_k<T, 32, PVX, 1, FW>(a, s, nwg_out);
  return launch_conv32_k<T, 32, PVX, 2, FW>(a, s, nwg_out);
}

// x chunks per thread the 32-channel kernel stages for this launch (0: not applicable)
static int conv32_pvx(const GatherArgs& a, int dtype, bool fw) {
  if ((uintptr_t)a.w & 15) return 0;  // stage_weights reads the kernel in 16-byte vectors
  const bool o64 = a.O == 64 && !fw && (a.wmode != W_PAIR || a.T_full <= 2 * a.T_out);
  if (a.C != 32 || !((a.O == 32 && a.wmode != W_PAIR) || o64) || a.K > 4 || a.S > 2) return 0;
  if (a.flags & (VQA_X_F32 | VQA_Y_F32)) return 0;
  if (fw && (a.S != 1 || a.K > 3 || a.wmode != W_FLIP_T)) return 0;
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  if ((long long)a.T_in * 32 * esz >= (1ll << 29) || (long long)a.T_out * a.O * esz >= (1ll << 29)) return 0;
  const int rows_in = 127 * a.S + (a.K - 1) * a.D + 1;
  const int chunks = rows_in * 32 * esz / 16;
  const int pv = (chunks + 255) / 256;
  const int opts_bf16[] = {3, 5}, opts_f32[] = {5, 6, 9};
  const int* opts = esz == 2 ? opts_bf16 : opts_f32;
  const int nopt = esz == 2 ? 2 : 3;
  for (int i = 0; i < nopt; ++i) {
    if (pv <= opts[i]) {
      const int xs = 32 + 16 / esz, xrows = 256 / (32 * esz / 16) * opts[i];
      const size_t lds = ((size_t)a.K * a.O * xs + (size_t)xrows * xs) * esz + 2 * 128 * (size_t)a.O * esz;
      return lds <= 150 * 1024 ? opts[i] : 0;
    }
  }
  return 0;
}

template <class T, bool FW>
static int launch_conv32(const GatherArgs& a, int pvx, hipStream_t s, int* nwg_out) {
  const int nep = gather_nep(a, FW);
  if constexpr (sizeof(T) == 2) {
    if (pvx == 3) return launch_conv32_n<T, 3, FW>(a, nep, s, nwg_out);
    return launch_conv32_n<T, 5, FW>(a, nep, s, nwg_out);
  } else {
    if (pvx == 5) return launch_conv32_n<T, 5, FW>(a, nep, s, nwg_out);
    if (pvx == 6) return launch_conv32_n<T, 6, FW>(a, nep, s, nwg_out);
    return launch_conv32_n<T, 9, FW>(a, nep, s, nwg_out);
  }
}

static bool mfma_ok(const GatherArgs& a, int dtype) {
  if ((uintptr_t)a.w & 15) return false;  // stage_weights reads the kernel in 16-byte vectors
  if (a.flags & (VQA_X_F32 | VQA_Y_F32)) return false;
  if (a.K > 4) return false;  // the kernel's tap loop is unrolled for K <= 4
  if (!((a.C == 32 || a.C == 64) && (a.O == 32 || a.O == 64 || a.O == 128))) return false;
  const int tm = gather_tm(a.O, a.S);
  const int rows_in = (tm - 1) * a.S + (a.K - 1) * a.D + 1;
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  const long long chunks = (long long)rows_in * a.C * esz / 16 + (long long)gather_nep(a, false) * tm * a.O * esz / 16;
  if (chunks > 12 * 256) return false;
  return (size_t)rows_in * (a.C + 8) * 4 + (size_t)a.K * a.O * (a.C + 8) * 4 <= 150 * 1024;
}

template <class TX, class TY>
static int launch_gather_direct(const GatherArgs& a, hipStream_t s) {
  const long long total = (long long)a.B * a.T_out * a.O;
  long long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((gather_direct_kernel<TX, TY>), dim3((unsigned)blocks), dim3(256), 0, s, a);
  VQA_LAUNCHED("gather_direct_kernel");
  return VQA_OK;
}

template <class TX, class TY, int C>
static int launch_gather_thinO_c(const GatherArgs& a, hipStream_t s) {
  const int ntb = (a.T_out + 255) / 256;
  const int rows_in = 255 * a.S + (a.K - 1) * a.D + 1;
  const size_t lds = ((size_t)a.K * C * a.O * 4 + 15) / 16 * 16 + (size_t)rows_in * (C + 16 / sizeof(TX)) * sizeof(TX);
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds((const void*)gather_thinO_kernel<TX, TY, C>, lds, &lds_set, "gather_thinO_kernel");
  if (rc != VQA_OK) return rc;
  hipLaunchKernelGGL((gather_thinO_kernel<TX, TY, C>), dim3(ntb * a.B), dim3(256), lds, s, a, ntb);
  VQA_LAUNCHED("gather_thinO_kernel");
  return VQA_OK;
}

template <class TX, class TY>
static int launch_gather_thinO(const GatherArgs& a, hipStream_t s) {
  return a.C == 32 ? launch_gather_thinO_c<TX, TY, 32>(a, s) : launch_gather_thinO_c<TX, TY, 64>(a, s);
}

template <class TX, class TY>
static int launch_gather_thin(const GatherArgs& a, hipStream_t s) {
  VQA_REQUIRE((long long)a.B * a.T_out * a.O < (1ll << 31), VQA_E_UNSUPPORTED, "thin conv: tensor too large");
  const int OV = (a.O % 8 == 0) ? 8 : 1;
  const long long total = (long long)a.B * a.T_out * (a.O / OV);
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const size_t lds = (size_t)a.K * a.C * a.O * sizeof(float);
  if (OV == 8)
    hipLaunchKernelGGL((gather_thin_kernel<TX, TY, 8>), dim3((unsigned)blocks), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((gather_thin_kernel<TX, TY, 1>), dim3((unsigned)blocks), dim3(256), lds, s, a);
  VQA_LAUNCHED("gather_thin_kernel");
  return VQA_OK;
}

// ------------------------------------------------------------------------------------------------
// One-input-channel conv (the encoder's first conv on the waveform, encdec.py:33 with C = 1): a workgroup
// owns CI1_RB output rows of one item; their input span is staged once in LDS (fp32), each lane holds the
// K x 8 weights of its 8 output channels in registers and writes its rows' 8 channels as one 16-byte
// (bf16) store — consecutive lanes write consecutive bytes. Per-row tap order k = 0..K-1 (as the gather
// kernels).
constexpr int CI1_RB = 512, CI1_KMAX = 8;
// input values staged per thread by the unrolled path (span <= 256 CI1_SPT: stride 2, K <= 4 at CI1_RB = 512); the
// loads are issued together from clamped addresses, zeros selected (the loop form waited on every load in turn)
constexpr int CI1_SPT = 5;

// KT: the tap count as a compile-time constant (4: the model's first conv; fewer registers, all tap reads issued
// together) or 0 (any K <= CI1_KMAX from the arguments). Same sums in the same order either way.
template <class TX, class TY, int O, int KT>
__global__ __launch_bounds__(256) void gather_ci1_kernel(GatherArgs a) {
  constexpr int L = O / 8, RPP = 256 / L;  // lanes per row, rows per pass
  constexpr int KK = KT > 0 ? KT : CI1_KMAX;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* xl = (float*)smem;
  const int n = blockIdx.y, t0 = blockIdx.x * CI1_RB;
  const int span = (CI1_RB - 1) * a.S + (a.K - 1) * a.D + 1, i0 = t0 * a.S - a.P;
  const TX* X = (const TX*)a.x + (size_t)n * a.T_in;
  const bool relu = a.flags & VQA_PRE_RELU;
  if (span <= 256 * CI1_SPT) {
    float v[CI1_SPT];
#pragma unroll
    for (int i = 0; i < CI1_SPT; ++i) {
      const int e = threadIdx.x + 256 * i, ti = i0 + e;
      const bool ok = e < span && ti >= 0 && ti < a.T_in;
      const float x = ld(X + min(max(ti, 0), a.T_in - 1));
      v[i] = ok ? x : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CI1_SPT; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < span) xl[e] = relu ? fmaxf(v[i], 0.f) : v[i];
    }
  } else {
    for (int e = threadIdx.x; e < span; e += 256) {
      const int ti = i0 + e;
      float v = (ti >= 0 && ti < a.T_in) ? ld(X + ti) : 0.f;
      xl[e] = relu ? fmaxf(v, 0.f) : v;
    }
  }
  const int o8 = (threadIdx.x % L) * 8, rl = threadIdx.x / L;
  float w[KK][8], b[8];
#pragma unroll
  for (int k = 0; k < KK; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) w[k][j] = (KT > 0 || k < a.K) ? a.w[k * O + o8 + j] : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) b[j] = a.bias ? a.bias[o8 + j] : 0.f;
  __syncthreads();
  TY* Y = (TY*)a.y + (size_t)n * a.T_out * O;
  for (int r = rl; r < CI1_RB && t0 + r < a.T_out; r += RPP) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) {
      if (KT == 0 && k >= a.K) break;
      const float xv = xl[r * a.S + k * a.D];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += xv * w[k][j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = acc[j] + b[j];
    st8_(Y + (size_t)(t0 + r) * O + o8, acc);
  }
}

template <class TX, class TY, int KT>
static void launch_gather_ci1_k(const GatherArgs& a, const dim3& grid, size_t lds, hipStream_t s) {
  if (a.O == 32) hipLaunchKernelGGL((gather_ci1_kernel<TX, TY, 32, KT>), grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL((gather_ci1_kernel<TX, TY, 64, KT>), grid, dim3(256), lds, s, a);
}

template <class TX, class TY>
static int launch_gather_ci1(const GatherArgs& a, hipStream_t s) {
  const size_t lds = (size_t)((CI1_RB - 1) * a.S + (a.K - 1) * a.D + 1) * sizeof(float);
  const dim3 grid((a.T_out + CI1_RB - 1) / CI1_RB, a.B);
  if (a.K == 4) launch_gather_ci1_k<TX, TY, 4>(a, grid, lds, s);
  else launch_gather_ci1_k<TX, TY, 0>(a, grid, lds, s);
  VQA_LAUNCHED("gather_ci1_kernel");
  return VQA_OK;
}

static bool ci1_ok(const GatherArgs& a) {
  return a.C == 1 && a.wmode == W_DIRECT && (a.O == 32 || a.O == 64) && a.K <= CI1_KMAX &&
         !(a.flags & (VQA_POST_MASK | VQA_ADD_RESIDUAL)) &&
         (size_t)((CI1_RB - 1) * a.S + (a.K - 1) * a.D + 1) * sizeof(float) <= 64 * 1024;
}

int run_gather(const GatherArgs& a, int dtype, hipStream_t s) {
  VQA_ARG(dtype == VQA_F32 || dtype == VQA_BF16, "unknown dtype %d", dtype);
  VQA_ARG(a.x && a.w && a.y, "null tensor pointer");
  VQA_ARG(a.B > 0 && a.T_in > 0 && a.T_out > 0 && a.C > 0 && a.O > 0 && a.K > 0 && a.S > 0 && a.D > 0,
          "non-positive shape");
  VQA_ARG(!(a.flags & VQA_POST_MASK) || a.mask, "VQA_POST_MASK without mask");
  VQA_ARG(!(a.flags & VQA_ADD_RESIDUAL) || a.resid, "VQA_ADD_RESIDUAL without residual");
  if (const int pvx = conv32_pvx(a, dtype, false)) {
    return dtype == VQA_BF16 ? launch_conv32<bf16, false>(a, pvx, s, nullptr)
                             : launch_conv32<float, false>(a, pvx, s, nullptr);
  }
  if (mfma_ok(a, dtype)) return dtype == VQA_BF16 ? launch_gather_mfma<bf16>(a, s) : launch_gather_mfma<float>(a, s);
  const bool xf = dtype == VQA_F32 || (a.flags & VQA_X_F32);
  const bool yf = dtype == VQA_F32 || (a.flags & VQA_Y_F32);
  if (ci1_ok(a)) {
    if (xf && yf) return launch_gather_ci1<float, float>(a, s);
    if (xf) return launch_gather_ci1<float, bf16>(a, s);
    if (yf) return launch_gather_ci1<bf16, float>(a, s);
    return launch_gather_ci1<bf16, bf16>(a, s);
  }
  if (a.O <= 8 && (a.C == 32 || a.C == 64) && a.wmode != W_PAIR && a.K <= 4 && a.S <= 2 && a.D <= 64) {
    if (xf && yf) return launch_gather_thinO<float, float>(a, s);
    if (xf) return launch_gather_thinO<float, bf16>(a, s);
    if (yf) return launch_gather_thinO<bf16, float>(a, s);
    return launch_gather_thinO<bf16, bf16>(a, s);
  }
  if ((a.C <= 8 || a.O <= 8) && (size_t)a.K * a.C * a.O * 4 <= 64 * 1024 &&
      (a.wmode != W_PAIR || (a.O / 2) % 8 == 0 || a.O % 8 != 0)) {
    if (xf && yf) return launch_gather_thin<float, float>(a, s);
    if (xf) return launch_gather_thin<float, bf16>(a, s);
    if (yf) return launch_gather_thin<bf16, float>(a, s);
    return launch_gather_thin<bf16, bf16>(a, s);
  }
  if (xf && yf) return launch_gather_direct<float, float>(a, s);
  if (xf) return launch_gather_direct<float, bf16>(a, s);
  if (yf) return launch_gather_direct<bf16, float>(a, s);
  return launch_gather_direct<bf16, bf16>(a, s);
}

// ---- weight gradient planning ----
enum { WG_MFMA = 0, WG_THIN_X = 1, WG_THIN_G = 2, WG_DIRECT = 3 };
struct WgradPlan {
  int kind;
  int TT, CH, nchunk, nwg, E, nb;
  size_t lds, ws_bytes;
};

static WgradPlan plan_wgrad(int dtype, int B, int T_in, int T_out, int C, int O, int K, int S, int D, int flags) {
  WgradPlan p{};
  const bool anyf32 = (flags & (VQA_X_F32 | VQA_Y_F32)) != 0;
  const size_t esz = dtype == VQA_BF16 ? 2 : 4;
  p.nb = (flags & WG_DB_FROM_X) ? C : O;
  // the thin kernels address an item's rows through 32-bit buffer offsets
  const bool thin_fits = (long long)T_in * C * 4 < (1ll << 30) && (long long)T_out * O * 4 < (1ll << 30);
  if (!anyf32 && (C == 32 || C == 64) && (O == 32 || O == 64) && K <= 4) {
    p.kind = WG_MFMA;
    p.TT = dtype == VQA_BF16 ? 128 : 64;
    const int rows_in = (p.TT - 1) * S + (K - 1) * D + 1;
    p.lds = ((size_t)p.TT * (O + 16 / esz) + (size_t)rows_in * (C + 16 / esz)) * esz;
    if (p.lds > 150 * 1024) {
      p.TT = 64;
      const int r2 = (p.TT - 1) * S + (K - 1) * D + 1;
      p.lds = ((size_t)p.TT * (O + 16 / esz) + (size_t)r2 * (C + 16 / esz)) * esz;
    }
  } else if (K <= 4 && C % 8 == 0 && C <= 256 && O <= 2 && !(flags & WG_DB_FROM_X) && thin_fits) {
    p.kind = WG_THIN_X;
    p.TT = 64;
    p.lds = (size_t)256 * (4 * 2 * 8 + 8) * sizeof(float);
  } else if (K <= 4 && O % 8 == 0 && O <= 256 && C <= 2 && !(flags & WG_DB_FROM_X) && thin_fits) {
    p.kind = WG_THIN_G;
    p.TT = 64;
    p.lds = (size_t)256 * (4 * 2 * 8 + 8) * sizeof(float);
  } else {
    p.kind = WG_DIRECT;
    p.TT = 64;
    const int rows_in = (p.TT - 1) * S + (K - 1) * D + 1;
    p.lds = ((size_t)p.TT * O + (size_t)rows_in * C) * 4;
  }
  // ~512 workgroups (two per CU): each streams its rows once (4 rows in flight per thread in the thin
  // kinds) and the partials stay small
  const long long target = 512;
  const long long per_item = (target + B - 1) / B;
  int ch = (int)((T_out + per_item - 1) / per_item);
  ch = ((ch + p.TT - 1) / p.TT) * p.TT;
  if (ch < p.TT) ch = p.TT;
  p.CH = ch;
  p.nchunk = (T_out + ch - 1) / ch;
  p.nwg = p.nchunk * B;
  p.E = K * C * O + p.nb;
  p.ws_bytes = (size_t)p.nwg * p.E * sizeof(float);
  return p;
}

template <class T, int C, int O, int TT>
static int launch_wgrad_mfma_t(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds((const void*)wgrad_mfma_kernel<T, C, O, TT>, p.lds, &lds_set, "wgrad_mfma_kernel");
  if (rc != VQA_OK) return rc;
  hipLaunchKernelGGL((wgrad_mfma_kernel<T, C, O, TT>), dim3(p.nchunk, a.B), dim3(256), p.lds, s, a);
  VQA_LAUNCHED("wgrad_mfma_kernel");
  return VQA_OK;
}

template <class T, int C, int O>
static int launch_wgrad_mfma_co(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  if (p.TT == 128) return launch_wgrad_mfma_t<T, C, O, 128>(a, p, s);
  return launch_wgrad_mfma_t<T, C, O, 64>(a, p, s);
}

template <class T>
static int launch_wgrad_mfma(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  if (a.C == 32 && a.O == 32) return launch_wgrad_mfma_co<T, 32, 32>(a, p, s);
  if (a.C == 32 && a.O == 64) return launch_wgrad_mfma_co<T, 32, 64>(a, p, s);
  if (a.C == 64 && a.O == 32) return launch_wgrad_mfma_co<T, 64, 32>(a, p, s);
  if (a.C == 64 && a.O == 64) return launch_wgrad_mfma_co<T, 64, 64>(a, p, s);
  vqa::set_error("wgrad: no MFMA tile for C=%d O=%d", a.C, a.O);
  return VQA_E_UNSUPPORTED;
}

template <class TX, class TG>
static int launch_wgrad_direct(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds((const void*)wgrad_direct_kernel<TX, TG, 64>, p.lds, &lds_set, "wgrad_direct_kernel");
  if (rc != VQA_OK) return rc;
  const unsigned slices = (unsigned)((a.K * a.C * a.O + 4095) / 4096);  // 16 weight elements per thread per slice
  hipLaunchKernelGGL((wgrad_direct_kernel<TX, TG, 64>), dim3(p.nchunk, a.B, slices), dim3(256), p.lds, s, a);
  VQA_LAUNCHED("wgrad_direct_kernel");
  return VQA_OK;
}

template <class TX, class TG, bool WX, int NM>
static int launch_wgrad_thin_nm(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  static size_t lds_set = 0;
  const int rc = ensure_dyn_lds((const void*)wgrad_thin_kernel<TX, TG, WX, NM>, p.lds, &lds_set, "wgrad_thin_kernel");
  if (rc != VQA_OK) return rc;
  hipLaunchKernelGGL((wgrad_thin_kernel<TX, TG, WX, NM>), dim3(p.nchunk, a.B), dim3(256), p.lds, s, a);
  VQA_LAUNCHED("wgrad_thin_kernel");
  return VQA_OK;
}

template <class TX, class TG, bool WX>
static int launch_wgrad_thin(const WgradArgs& a, const WgradPlan& p, hipStream_t s) {
  return (WX ? a.O : a.C) == 1 ? launch_wgrad_thin_nm<TX, TG, WX, 1>(a, p, s) : launch_wgrad_thin_nm<TX, TG, WX, 2>(a, p, s);
}

template <bool WX>
static int launch_wgrad_thin_t(const WgradArgs& a, const WgradPlan& p, bool xf, bool gf, hipStream_t s) {
  if (xf && gf) return launch_wgrad_thin<float, float, WX>(a, p, s);
  if (xf) return launch_wgrad_thin<float, bf16, WX>(a, p, s);
  if (gf) return launch_wgrad_thin<bf16, float, WX>(a, p, s);
  return launch_wgrad_thin<bf16, bf16, WX>(a, p, s);
}

int run_wgrad(const void* x, const void* g, float* dw, float* db, int B, int T_in, int T_out, int C, int O, int K,
              int S, int D, int P, int flags, int dtype, void* ws, size_t ws_bytes, hipStream_t s,
              vqa_partials_desc* defer) {
  VQA_ARG(dtype == VQA_F32 || dtype == VQA_BF16, "unknown dtype %d", dtype);
  VQA_ARG(x && g && dw, "null tensor pointer");
  VQA_ARG(B > 0 && T_in > 0 && T_out > 0 && C > 0 && O > 0 && K > 0 && S > 0 && D > 0, "non-positive shape");
  WgradPlan p = plan_wgrad(dtype, B, T_in, T_out, C, O, K, S, D, flags);
  VQA_ARG(ws && ws_bytes >= p.ws_bytes, "workspace too small: need %zu bytes, got %zu", p.ws_bytes, ws_bytes);
  VQA_REQUIRE(p.lds <= 150 * 1024, VQA_E_UNSUPPORTED, "wgrad: LDS tile too large (%zu B)", p.lds);
  VQA_REQUIRE(p.kind != WG_DIRECT || K * C * O <= 16 * 256 * 64, VQA_E_UNSUPPORTED,
              "wgrad: generic path limited to K*C*O<=262144");
  VQA_REQUIRE(p.nb <= 256 && 256 % p.nb == 0, VQA_E_UNSUPPORTED, "wgrad: bias width must divide 256");
  WgradArgs a{x, g, (float*)ws, B, T_in, T_out, C, O, K, S, D, P, p.CH, p.nchunk, flags, p.nb};
  const bool xf = dtype == VQA_F32 || (flags & VQA_X_F32);
  const bool gf = dtype == VQA_F32 || (flags & VQA_Y_F32);
  int rc;
  switch (p.kind) {
    case WG_MFMA:
      rc = dtype == VQA_BF16 ? launch_wgrad_mfma<bf16>(a, p, s) : launch_wgrad_mfma<float>(a, p, s);
      break;
    case WG_THIN_X: rc = launch_wgrad_thin_t<true>(a, p, xf, gf, s); break;
    case WG_THIN_G: rc = launch_wgrad_thin_t<false>(a, p, xf, gf, s); break;
    default:
      if (xf && gf) rc = launch_wgrad_direct<float, float>(a, p, s);
      else if (xf) rc = launch_wgrad_direct<float, bf16>(a, p, s);
      else if (gf) rc = launch_wgrad_direct<bf16, float>(a, p, s);
      else rc = launch_wgrad_direct<bf16, bf16>(a, p, s);
  }
  if (rc != VQA_OK) return rc;
  const int KCO = K * C * O;
  if (defer) {
    *defer = vqa_partials_desc{(const float*)ws, dw, db, p.nwg, p.E, KCO, 0};
    return VQA_OK;
  }
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((p.E + kRedCols - 1) / kRedCols), dim3(256), 0, s, (const float*)ws, p.nwg, p.E,
                     KCO, dw, db);
  VQA_LAUNCHED("reduce_partials_kernel");
  return VQA_OK;
}

size_t wgrad_ws(int dtype, int B, int T_in, int T_out, int C, int O, int K, int S, int D, int flags) {
  if (B < 1 || T_in < 1 || T_out < 1 || C < 1 || O < 1 || K < 1 || S < 1 || D < 1) return 0;  // no such conv
  return plan_wgrad(dtype, B, T_in, T_out, C, O, K, S, D, flags).ws_bytes;
}

}  // namespace vqa

// ================================================================================================
// C ABI
using namespace vqa;

// -1 for a shape TF's "same" padding does not define (stride or dilation < 1, K < 1, T_in < 0)
extern "C" int vqa_same_out_len(int T_in, int stride) {
  if (stride < 1 || T_in < 0) return -1;
  return (T_in + stride - 1) / stride;
}
extern "C" int vqa_same_pad_left(int T_in, int K, int stride, int dilation) {
  if (stride < 1 || dilation < 1 || K < 1 || T_in < 0) return -1;
  const int out = (T_in + stride - 1) / stride;
  const int pad = std::max((out - 1) * stride + (K - 1) * dilation + 1 - T_in, 0);
  return pad / 2;
}

extern "C" int vqa_conv1d_fwd(const void* x, const float* w, const float* bias, const void* residual, void* y, int B,
                              int T_in, int T_out, int C_in, int C_out, int K, int stride, int dilation, int pad_left,
                              int flags, int dtype, vqa_stream_t stream) {
  VQA_ARG(stride >= 1 && dilation >= 1 && K >= 1, "conv1d_fwd: stride %d, dilation %d, K %d must be >= 1", stride,
          dilation, K);
  VQA_ARG(T_out == (T_in + stride - 1) / stride, "conv1d_fwd: T_out %d != ceil(T_in/stride)", T_out);
  if (co1_supported(C_in, C_out, K, stride, dilation, dtype, flags) && (dtype == VQA_F32 || dtype == VQA_BF16)) {
    VQA_ARG(x && w && y && B > 0 && T_in > 0, "conv1d_fwd: bad arguments");
    VQA_ARG(!(flags & VQA_ADD_RESIDUAL) || residual, "VQA_ADD_RESIDUAL without residual");
    return co1_fwd(x, w, bias, residual, y, B, T_in, C_in, K, dilation, pad_left,
                   flags & (VQA_PRE_RELU | VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32), dtype, (hipStream_t)stream);
  }
  GatherArgs a{x, w, bias, residual, nullptr, y, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad_left,
               W_DIRECT, K, 0, T_out, flags & (VQA_PRE_RELU | VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32)};
  return run_gather(a, dtype, (hipStream_t)stream);
}

// flags for the data-gradient gather: the gather input is dy (y side), output dx (x side)
static int swap_xy_flags(int flags) {
  int f = flags & (VQA_POST_MASK | VQA_ADD_RESIDUAL);
  if (flags & VQA_X_F32) f |= VQA_Y_F32;
  if (flags & VQA_Y_F32) f |= VQA_X_F32;
  return f;
}

extern "C" int vqa_conv1d_bwd_data(const void* dy, const float* w, const void* mask, const void* residual, void* dx,
                                   int B, int T_in, int T_out, int C_in, int C_out, int K, int stride, int dilation,
                                   int pad_left, int flags, int dtype, vqa_stream_t stream) {
  VQA_ARG(stride >= 1 && dilation >= 1 && K >= 1, "conv1d_bwd_data: stride %d, dilation %d, K %d must be >= 1", stride,
          dilation, K);
  VQA_ARG(T_out == (T_in + stride - 1) / stride, "conv1d_bwd_data: T_out %d != ceil(T_in/stride)", T_out);
  if (co1_supported(C_in, C_out, K, stride, dilation, dtype, flags) && (dtype == VQA_F32 || dtype == VQA_BF16)) {
    VQA_ARG(dy && w && dx && B > 0 && T_in > 0, "conv1d_bwd_data: bad arguments");
    VQA_ARG(!(flags & VQA_POST_MASK) || mask, "VQA_POST_MASK without mask");
    VQA_ARG(!(flags & VQA_ADD_RESIDUAL) || residual, "VQA_ADD_RESIDUAL without residual");
    // same kernel (and dx arithmetic) as the fused data + weight gradient, without the weight partials
    const int f = ((flags & VQA_POST_MASK) ? VQA_PRE_RELU : 0) | (flags & (VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32));
    return co1_bwd(dy, w, (flags & VQA_POST_MASK) ? mask : nullptr, residual, dx, B, T_in, C_in, K, dilation,
                   pad_left, f, dtype, nullptr, nullptr, (hipStream_t)stream);
  }
  const int f = swap_xy_flags(flags);
  if (stride == 1) {
    GatherArgs a{dy, w, nullptr, residual, mask, dx, B, T_out, T_in, C_out, C_in, K, 1, dilation,
                 (K - 1) * dilation - pad_left, W_FLIP_T, K, 0, T_in, f};
    return run_gather(a, dtype, (hipStream_t)stream);
  }
  VQA_REQUIRE(stride == 2 && K == 4 && dilation == 1 && pad_left == 1, VQA_E_UNSUPPORTED,
              "conv1d_bwd_data: strided data-gradient supports stride 2, K 4, pad_left 1 (got s=%d K=%d d=%d p=%d)",
              stride, K, dilation, pad_left);
  GatherArgs a{dy, w, nullptr, residual, mask, dx, B, T_out, T_out, C_out, 2 * C_in, 3, 1, 1, 1,
               W_PAIR, K, pad_left, T_in, f};
  return run_gather(a, dtype, (hipStream_t)stream);
}

extern "C" size_t vqa_conv1d_bwd_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                                  int dilation, int pad_left, int flags, int dtype) {
  (void)pad_left;
  return wgrad_ws(dtype, B, T_in, T_out, C_in, C_out, K, stride, dilation, flags);
}

extern "C" int vqa_conv1d_bwd_weight(const void* x, const void* dy, float* dw, float* db, int B, int T_in, int T_out,
                                     int C_in, int C_out, int K, int stride, int dilation, int pad_left, int flags,
                                     int dtype, void* workspace, size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(stride >= 1 && dilation >= 1 && K >= 1, "conv1d_bwd_weight: stride %d, dilation %d, K %d must be >= 1", stride,
          dilation, K);
  VQA_ARG(T_out == (T_in + stride - 1) / stride, "conv1d_bwd_weight: T_out %d != ceil(T_in/stride)", T_out);
  return run_wgrad(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad_left,
                   flags & (VQA_PRE_RELU | VQA_X_F32 | VQA_Y_F32), dtype, workspace, ws_bytes, (hipStream_t)stream,
                   nullptr);
}

extern "C" int vqa_conv1d_transpose_fwd(const void* x, const float* w, const float* bias, const void* residual,
                                        void* y, int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                        int pad_left, int flags, int dtype, vqa_stream_t stream) {
  VQA_REQUIRE(stride == 2 && K == 4 && pad_left == 1, VQA_E_UNSUPPORTED,
              "conv1d_transpose: supports stride 2, K 4, pad_left 1 (got s=%d K=%d p=%d)", stride, K, pad_left);
  VQA_ARG(T_out == stride * T_in, "conv1d_transpose_fwd: T_out %d != stride*T_in", T_out);
  GatherArgs a{x, w, bias, residual, nullptr, y, B, T_in, T_in, C_in, 2 * C_out, 3, 1, 1, 1,
               W_PAIR, K, pad_left, T_out, flags & (VQA_PRE_RELU | VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32)};
  return run_gather(a, dtype, (hipStream_t)stream);
}

extern "C" int vqa_conv1d_transpose_bwd_data(const void* dy, const float* w, const void* mask, const void* residual,
                                             void* dx, int B, int T_in, int T_out, int C_in, int C_out, int K,
                                             int stride, int pad_left, int flags, int dtype, vqa_stream_t stream) {
  VQA_REQUIRE(stride == 2 && K == 4 && pad_left == 1, VQA_E_UNSUPPORTED,
              "conv1d_transpose: supports stride 2, K 4, pad_left 1");
  VQA_ARG(T_out == stride * T_in, "conv1d_transpose_bwd_data: T_out %d != stride*T_in", T_out);
  GatherArgs a{dy, w, nullptr, residual, mask, dx, B, T_out, T_in, C_out, C_in, K, stride, 1, pad_left,
               W_DIRECT, K, 0, T_in, swap_xy_flags(flags)};
  return run_gather(a, dtype, (hipStream_t)stream);
}

extern "C" size_t vqa_conv1d_transpose_bwd_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K,
                                                            int stride, int pad_left, int flags, int dtype) {
  (void)pad_left;
  const int f = (swap_xy_flags(flags) & (VQA_X_F32 | VQA_Y_F32)) | WG_DB_FROM_X;
  return wgrad_ws(dtype, B, T_out, T_in, C_out, C_in, K, stride, 1, f);
}

extern "C" int vqa_conv1d_transpose_bwd_weight(const void* x, const void* dy, float* dw, float* db, int B, int T_in,
                                               int T_out, int C_in, int C_out, int K, int stride, int pad_left,
                                               int flags, int dtype, void* workspace, size_t ws_bytes,
                                               vqa_stream_t stream) {
  VQA_REQUIRE(stride == 2 && K == 4 && pad_left == 1, VQA_E_UNSUPPORTED,
              "conv1d_transpose: supports stride 2, K 4, pad_left 1");
  VQA_ARG(T_out == stride * T_in, "conv1d_transpose_bwd_weight: T_out %d != stride*T_in", T_out);
  // dW[k][co][ci] = sum_i dy[2i + k - 1][co] * x[i][ci]: the gather weight-gradient with dy as its input;
  // db[co] = column sums of dy, taken from the same staged rows (WG_DB_FROM_X)
  const int f = (swap_xy_flags(flags) & (VQA_X_F32 | VQA_Y_F32)) | WG_DB_FROM_X;
  return run_wgrad(dy, x, dw, db, B, T_out, T_in, C_out, C_in, K, stride, 1, pad_left, f, dtype, workspace, ws_bytes,
                   (hipStream_t)stream, nullptr);
}

extern "C" int vqa_conv1d_bwd_weight_partials(const void* x, const void* dy, float* dw, float* db, int B, int T_in,
                                              int T_out, int C_in, int C_out, int K, int stride, int dilation,
                                              int pad_left, int flags, int dtype, void* workspace, size_t ws_bytes,
                                              vqa_partials_desc* desc, vqa_stream_t stream) {
  VQA_ARG(desc, "bwd_weight_partials: NULL descriptor");
  VQA_ARG(stride >= 1 && dilation >= 1 && K >= 1, "conv1d_bwd_weight: stride %d, dilation %d, K %d must be >= 1", stride,
          dilation, K);
  VQA_ARG(T_out == (T_in + stride - 1) / stride, "conv1d_bwd_weight: T_out %d != ceil(T_in/stride)", T_out);
  return run_wgrad(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad_left,
                   flags & (VQA_PRE_RELU | VQA_X_F32 | VQA_Y_F32), dtype, workspace, ws_bytes, (hipStream_t)stream,
                   desc);
}

extern "C" int vqa_conv1d_transpose_bwd_weight_partials(const void* x, const void* dy, float* dw, float* db, int B,
                                                        int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                                        int pad_left, int flags, int dtype, void* workspace,
                                                        size_t ws_bytes, vqa_partials_desc* desc,
                                                        vqa_stream_t stream) {
  VQA_ARG(desc, "bwd_weight_partials: NULL descriptor");
  VQA_REQUIRE(stride == 2 && K == 4 && pad_left == 1, VQA_E_UNSUPPORTED,
              "conv1d_transpose: supports stride 2, K 4, pad_left 1");
  VQA_ARG(T_out == stride * T_in, "conv1d_transpose_bwd_weight: T_out %d != stride*T_in", T_out);
  const int f = (swap_xy_flags(flags) & (VQA_X_F32 | VQA_Y_F32)) | WG_DB_FROM_X;
  return run_wgrad(dy, x, dw, db, B, T_out, T_in, C_out, C_in, K, stride, 1, pad_left, f, dtype, workspace, ws_bytes,
                   (hipStream_t)stream, desc);
}

// ---- fused data + weight gradient of a stride-1 conv whose input u feeds it through an optional ReLU
static size_t fused_bwd_ws(int C_in, int C_out, int K) {
  return (size_t)num_cus() * kMaxGatherPerCU * (size_t)(K * C_in * C_out + C_out) * sizeof(float);
}

static GatherArgs fused_bwd_args(const void* dy, const float* w, const void* x, const void* residual, void* dx, int B,
                                 int T_in, int T_out, int C_in, int C_out, int K, int dilation, int pad_left,
                                 int flags) {
  const bool relu = flags & VQA_PRE_RELU;
  const int f = swap_xy_flags(flags & (VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32)) | (relu ? VQA_POST_MASK : 0);
  GatherArgs a{dy, w, nullptr, residual, x, dx, B, T_out, T_in, C_out, C_in, K, 1, dilation,
               (K - 1) * dilation - pad_left, W_FLIP_T, K, 0, T_in, f};
  a.wrelu = relu ? 1 : 0;
  return a;
}

extern "C" size_t vqa_conv1d_bwd_data_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K,
                                                       int stride, int dilation, int pad_left, int flags, int dtype) {
  if (B < 1 || T_in < 1 || T_out < 1 || C_in < 1 || C_out < 1 || K < 1 || stride < 1 || dilation < 1) return 0;
  size_t need = wgrad_ws(dtype, B, T_in, T_out, C_in, C_out, K, stride, dilation,
                         flags & (VQA_PRE_RELU | VQA_X_F32 | VQA_Y_F32));
  if (co1_supported(C_in, C_out, K, stride, dilation, dtype, flags)) need = std::max(need, co1_bwd_workspace(C_in, K));
  if (stride == 1) {
    const GatherArgs a = fused_bwd_args(nullptr, nullptr, nullptr, nullptr, nullptr, B, T_in, T_out, C_in, C_out, K,
                                        dilation, pad_left, flags);
    if (conv32_pvx(a, dtype, true)) need = std::max(need, fused_bwd_ws(C_in, C_out, K));
  }
  return need;
}

extern "C" int vqa_conv1d_bwd_data_weight(const void* dy, const float* w, const void* x, const void* residual,
                                          void* dx, float* dw, float* db, int B, int T_in, int T_out, int C_in,
                                          int C_out, int K, int stride, int dilation, int pad_left, int flags,
                                          int dtype, void* workspace, size_t ws_bytes, vqa_partials_desc* desc,
                                          vqa_stream_t stream) {
  VQA_ARG(stride >= 1 && dilation >= 1 && K >= 1, "conv1d_bwd_data_weight: stride %d, dilation %d, K %d must be >= 1", stride,
          dilation, K);
  VQA_ARG(T_out == (T_in + stride - 1) / stride, "conv1d_bwd_data_weight: T_out %d != ceil(T_in/stride)", T_out);
  VQA_ARG(dy && w && x && dx && dw, "conv1d_bwd_data_weight: null tensor pointer");
  VQA_ARG(dtype == VQA_F32 || dtype == VQA_BF16, "unknown dtype %d", dtype);
  const hipStream_t s = (hipStream_t)stream;
  if (co1_supported(C_in, C_out, K, stride, dilation, dtype, flags)) {
    const size_t need = co1_bwd_workspace(C_in, K);
    VQA_ARG(workspace && ws_bytes >= need, "workspace too small: need %zu bytes, got %zu", need, ws_bytes);
    VQA_ARG(!(flags & VQA_ADD_RESIDUAL) || residual, "VQA_ADD_RESIDUAL without residual");
    int nparts = 0;
    const int rc = co1_bwd(dy, w, x, residual, dx, B, T_in, C_in, K, dilation, pad_left,
                           flags & (VQA_PRE_RELU | VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32), dtype, workspace,
                           &nparts, s);
    if (rc != VQA_OK) return rc;
    const int KCO = K * C_in, E = KCO + 1;
    if (desc) {
      *desc = vqa_partials_desc{(const float*)workspace, dw, db, nparts, E, KCO, 0};
      return VQA_OK;
    }
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((E + kRedCols - 1) / kRedCols), dim3(256), 0, s, (const float*)workspace, nparts, E,
                       KCO, dw, db);
    VQA_LAUNCHED("reduce_partials_kernel");
    return VQA_OK;
  }
  if (stride == 1) {
    GatherArgs a = fused_bwd_args(dy, w, x, residual, dx, B, T_in, T_out, C_in, C_out, K, dilation, pad_left, flags);
    if (const int pvx = conv32_pvx(a, dtype, true)) {
      const size_t need = fused_bwd_ws(C_in, C_out, K);
      VQA_ARG(workspace && ws_bytes >= need, "workspace too small: need %zu bytes, got %zu", need, ws_bytes);
      a.wpart = (float*)workspace;
      int nwg = 0;
      const int rc = dtype == VQA_BF16 ? launch_conv32<bf16, true>(a, pvx, s, &nwg)
                                       : launch_conv32<float, true>(a, pvx, s, &nwg);
      if (rc != VQA_OK) return rc;
      const int KCO = K * C_in * C_out, E = KCO + C_out;
      if (desc) {
        *desc = vqa_partials_desc{(const float*)workspace, dw, db, nwg, E, KCO, 0};
        return VQA_OK;
      }
      hipLaunchKernelGGL(reduce_partials_kernel, dim3((E + kRedCols - 1) / kRedCols), dim3(256), 0, s, (const float*)workspace, nwg, E,
                         KCO, dw, db);
      VQA_LAUNCHED("reduce_partials_kernel");
      return VQA_OK;
    }
  }
  // not fusable here: data gradient, then the weight gradient from the same operands
  const bool relu = flags & VQA_PRE_RELU;
  int rc = vqa_conv1d_bwd_data(dy, w, relu ? x : nullptr, residual, dx, B, T_in, T_out, C_in, C_out, K, stride,
                               dilation, pad_left,
                               (relu ? VQA_POST_MASK : 0) | (flags & (VQA_ADD_RESIDUAL | VQA_X_F32 | VQA_Y_F32)),
                               dtype, stream);
  if (rc != VQA_OK) return rc;
  return run_wgrad(x, dy, dw, db, B, T_in, T_out, C_in, C_out, K, stride, dilation, pad_left,
                   flags & (VQA_PRE_RELU | VQA_X_F32 | VQA_Y_F32), dtype, workspace, ws_bytes, s, desc);
}

extern "C" int vqa_reduce_partials(const vqa_partials_desc* descs, int count, vqa_stream_t stream) {
  VQA_ARG(count >= 0 && (count == 0 || descs), "reduce_partials: bad descriptor list");
  for (int base = 0; base < count; base += kMaxDescs) {
    ReduceBatch rb{};
    rb.count = count - base < kMaxDescs ? count - base : kMaxDescs;
    int blocks = 0;
    for (int i = 0; i < rb.count; ++i) {
      const vqa_partials_desc& d = descs[base + i];
      VQA_ARG(d.partials && d.n > 0 && d.nparts > 0 && d.n_w <= d.n, "reduce_partials: bad descriptor %d", base + i);
      rb.d[i] = d;
      rb.start[i] = blocks;
      rb.vec4[i] = desc_vec4(d) ? 1 : 0;
#ifdef VQA_REDUCE_COL64
      blocks += rb.vec4[i] ? (d.n + 63) / 64 : (d.n + kRedCols - 1) / kRedCols;
#else
      blocks += rb.vec4[i] ? (d.n + kRedCols256 - 1) / kRedCols256 : (d.n + kRedCols - 1) / kRedCols;
#endif
    }
    rb.start[rb.count] = blocks;
    hipLaunchKernelGGL(reduce_partials_batched_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rb);
    VQA_LAUNCHED("reduce_partials_batched_kernel");
  }
  return VQA_OK;
}
