// vqa_prior.hip — the factorized-attention prior (gfx950): sequence-linear layers, embeddings, factorized
// attention, the fused output head + cross entropy, and the autoregressive decode step.
//
// Replaces (reference file:line):
//   src/autoregressive/autoregressive_fmha.py:119-158   FMHABasedAutoregressiveModel.call
//       x_embedding * sqrt(d_model) + PositionalEmbedding, dropout, (+ x_cond)   -> prior_embed_fwd
//       out = layers.Dense(bins)                                                 -> head_* (fused with the loss)
//   src/transformer/factorized_attention.py:36          Conv1D(3w, 3, padding="causal") -> seqlin (3 taps)
//   keras MultiHeadAttention query/key/value/output EinsumDense, proj / mlp Dense      -> seqlin (1 tap)
//   src/transformer/factorized_attention.py:74-388      row / col / prev-row attention -> attn_*
//   autoregressive.py:189-212, prior.py:272-300          loss / accuracy / teacher forcing -> head_*, tf_mix
//   src/autoregressive/autoregressive_fmha.py:162-240    sample (Gumbel-max per step)      -> vqa_prior_decode
// Activations are channels-last (rows = N*T, C) in the compute dtype; weights fp32 (Keras layouts); every
// reduction runs in a fixed order (weight gradients as per-workgroup partial rows for vqa_reduce_partials).
#include "vqa_common.h"
#include "vqa_mfma.h"
#include <algorithm>
#include <math.h>
#include <type_traits>

namespace vqa {

static int pr_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

// counter-based uniform in (0, 1): splitmix64 chain over (seed, a, b, c), 24 high bits (oracle/prior_ref.py
// gumbel_uniform restates it)
__host__ __device__ inline float prior_uniform(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = splitmix64(seed);
  h = splitmix64(h ^ a);
  h = splitmix64(h ^ b);
  h = splitmix64(h ^ c);
  return ((float)(uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float wave_sum_f(float v) { return warp_sum(v); }
__device__ __forceinline__ float wave_max_f(float v) { return warp_max(v); }

// ---------------------------------------------------------------------------------------------------
// Sequence-linear layer (MFMA): Y[r][n] = sum_tap sum_k X[src(r, tap)][k] * Wv[tap][k][n] + b[n] (+ R[r][n])
//   src(r, tap) = the row of the same sequence at time t + dir * (taps - 1 - tap); rows outside [0, T) are zero.
//   dir = -1, taps = 3: Conv1D(k=3, padding="causal") forward; dir = +1 with the transposed weight view: its
//   data gradient. taps = 1: Dense / EinsumDense (and their data gradients with wtrans = 1).
//   Wv[tap][k][n] = wtrans ? w[(tap*N + n)*K + k] : w[(tap*K + k)*N + n]
// Workgroup = 128 rows of one sequence; wave w owns rows 32w .. 32w+31 (two 16-row MFMA column tiles) and
// every 16-wide output tile. Operands: A = Wv^T (staged in LDS per tap, output channel rows), B = X^T (row
// tile in LDS); the output D[n][row] gives each lane 4 consecutive channels of one row.
struct SeqLinArgs {
  const void* x;
  const float* w;
  const void* wp;  // optional: weights prepared by vqa_seqlin_prep as [taps][N][K] in the activation dtype
  const float* b;
  const void* r;
  void* y;
  long long ldx, ldr, ldy;
  int nseq, T, K, N, taps, dir, wtrans, accumulate, tiles_per_seq;
  const float* lng;  // optional (seqlin_d, bf16, K = 128): LayerNorm(gamma, beta, eps) of each input row first
  const float* lnb;
  float lneps;
};

constexpr int kSlRows = 128;

template <class T, int NT>
__global__ __launch_bounds__(256) void seqlin_kernel(SeqLinArgs a) {
  typedef Mfma<T> M;
  constexpr int PAD = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KS = a.K + PAD;  // LDS row stride (elements) of both tiles
  T* Wt = (T*)smem;          // [N][K + PAD]
  const int halo = a.taps - 1, lo = a.dir < 0 ? halo : 0;
  T* X = Wt + a.N * KS;      // [kSlRows + halo][K + PAD]; row j <-> time t0 - lo + j
  const int seq = blockIdx.x / a.tiles_per_seq, t0 = (blockIdx.x - seq * a.tiles_per_seq) * kSlRows;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // stage the row tile (16-byte chunks; zeros outside the sequence)
  {
    constexpr int VEC = 16 / (int)sizeof(T);
    const int cpr = a.K / VEC, rows = kSlRows + halo;
    for (int e = threadIdx.x; e < rows * cpr; e += 256) {
      const int j = e / cpr, q = e - j * cpr, t = t0 - lo + j;
      uint4 v = {0u, 0u, 0u, 0u};
      if (t >= 0 && t < a.T) v = *(const uint4*)((const T*)a.x + ((long long)seq * a.T + t) * a.ldx + q * VEC);
      *(uint4*)(X + j * KS + q * VEC) = v;
    }
  }
  f32x4 acc[2][NT];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[s][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kof = M::koff(lane), col = lane & 15;
  for (int tap = 0; tap < a.taps; ++tap) {
    if (tap) __syncthreads();  // every read of the previous tap's weights is done
    if (a.wp) {  // prepared image rows: straight 16-byte copies
      constexpr int VEC = 16 / (int)sizeof(T);
      const T* wp = (const T*)a.wp + (size_t)tap * a.K * a.N;
      const int cpr = a.K / VEC;
      for (int e = threadIdx.x; e < a.N * cpr; e += 256) {
        const int n = e / cpr, q = e - n * cpr;
        *(uint4*)(Wt + n * KS + q * VEC) = *(const uint4*)(wp + (size_t)n * a.K + q * VEC);
      }
    } else {
    const float* w = a.w + (size_t)tap * a.K * a.N;
    // 16-byte coalesced weight reads (4 consecutive elements of the contiguous axis)
    for (int e4 = threadIdx.x; e4 < a.K * a.N / 4; e4 += 256) {
      const f32x4 v = *(const f32x4*)(w + 4 * e4);
      if (a.wtrans) {  // w[n][k]: 4 consecutive k of one n
        const int n = 4 * e4 / a.K, k = 4 * e4 - n * a.K;
        st4(Wt + n * KS + k, v);
      } else {         // w[k][n]: 4 consecutive n of one k
        const int k = 4 * e4 / a.N, n = 4 * e4 - k * a.N;
#pragma unroll
        for (int i = 0; i < 4; ++i) Wt[(n + i) * KS + k] = (T)v[i];
      }
    }
    }
    __syncthreads();
    // row j of X for output row i: i + dir * (taps - 1 - tap) + lo
    const int sh = a.dir * (a.taps - 1 - tap) + lo;
    const T* xb0 = X + (wave * 32 + col + sh) * KS + kof;
    const T* wb = Wt + col * KS + kof;
    for (int kc = 0; kc < a.K; kc += M::KS) {
      const typename M::frag b0 = M::load(xb0 + kc), b1 = M::load(xb0 + 16 * KS + kc);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if (nt * 16 >= a.N) break;
        const typename M::frag af = M::load(wb + nt * 16 * KS + kc);
        acc[0][nt] = M::mma(af, b0, acc[0][nt]);
        acc[1][nt] = M::mma(af, b1, acc[1][nt]);
      }
    }
  }
  // epilogue: lane (row = col, g) holds channels nt*16 + 4g .. +3
  const int g4 = 4 * (lane >> 4);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int t = t0 + wave * 32 + s * 16 + col;
    if (t >= a.T) continue;
    const long long row = (long long)seq * a.T + t;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (nt * 16 >= a.N) break;
      const int c = nt * 16 + g4;
      f32x4 v = acc[s][nt];
      if (a.b) v = v + f32x4{a.b[c], a.b[c + 1], a.b[c + 2], a.b[c + 3]};
      if (a.r) v = v + ld4((const T*)a.r + row * a.ldr + c);
      T* yp = (T*)a.y + row * a.ldy + c;
      if (a.accumulate) v = v + ld4((const T*)yp);
      st4(yp, v);
    }
  }
}

// 4 consecutive activation elements kept raw (bf16: 8 bytes, fp32: 16 bytes) and widened when used
template <class T> struct RawR4;
template <> struct RawR4<bf16> {
  typedef uint2 type;
  type v;
  __device__ __forceinline__ f32x4 f() const {
    const bf16x4 b = __builtin_bit_cast(bf16x4, v);
    return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
  }
};
template <> struct RawR4<float> {
  typedef uint4 type;
  type v;
  __device__ __forceinline__ f32x4 f() const { return __builtin_bit_cast(f32x4, v); }
};

// Persistent direct form for prepared weights (the prior's shapes, K and taps compile-time): the weight images
// of every tap staged ONCE per workgroup in LDS; each wave takes 16 rows of a 64-row tile and loads its B
// fragments (X^T: lane (row, g) <- 8 consecutive channels of its row) straight from global memory into
// registers — no LDS copy of X, no barrier per tile — with the NEXT tile's fragments and residual rows
// loaded while the current tile's MFMAs and stores run. The 1-tap epilogue goes through a per-wave fp32 LDS tile
// (16 rows x N) so that bias, residual and the store run on row-contiguous 16-byte chunks (whole rows per
// store instruction) instead of 4-channel pieces of 16 rows.
constexpr int kSdEpad = 4;

// 16 bytes of activations <-> VEC / 4 groups of 4 fp32
template <class T> __device__ __forceinline__ void chunk_widen(const uint4& u, f32x4* v) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 b = __builtin_bit_cast(bf16x8, u);
    v[0] = f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
    v[1] = f32x4{(float)b[4], (float)b[5], (float)b[6], (float)b[7]};
  } else {
    v[0] = __builtin_bit_cast(f32x4, u);
  }
}
template <class T> __device__ __forceinline__ uint4 chunk_narrow(const f32x4* v) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 b = {(bf16)v[0][0], (bf16)v[0][1], (bf16)v[0][2], (bf16)v[0][3],
                      (bf16)v[1][0], (bf16)v[1][1], (bf16)v[1][2], (bf16)v[1][3]};
    return __builtin_bit_cast(uint4, b);
  } else {
    return __builtin_bit_cast(uint4, v[0]);
  }
}

// LayerNorm of one row held as the B fragments of a 128-channel row (bf16, lane (row, g) holds channels
// 32 kc + 8 g .. +7 in fragment kc): the same arithmetic as layernorm8_fwd_kernel<bf16, 16> (vqa_cond.hip) —
// per-chunk sequential sums, then its pairwise sums over the 16 chunks, chunk bit 0 first (xl::grp_sum<16>; chunk
// bits 1, 0 are lane bits 5, 4 here, chunk bits 3, 2 the fragment index bits 1, 0) — so the fused and the unfused
// forms are bit-identical.
__device__ __forceinline__ void ln_row_frags(bf16x8 (&x)[4], const float* gs, const float* bs, int g8, float eps) {
  // the bf16 inputs are re-widened per pass (cheap) rather than held as 32 fp32 registers
  auto bfly = [](const float (&c)[4]) {
    float t[4];
#pragma unroll
    for (int kc = 0; kc < 4; ++kc) t[kc] = xl::sum32(xl::sum16(c[kc]));  // chunk bits 0, 1
    return (t[0] + t[1]) + (t[2] + t[3]);                                 // chunk bits 2, 3
  };
  float s[4];
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    s[kc] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[kc] += (float)x[kc][i];
  }
  const float mean = bfly(s) / 128.f;
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
    s[kc] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float d = (float)x[kc][i] - mean;
      s[kc] += d * d;
    }
  }
  const float inv = 1.0f / sqrtf(bfly(s) / 128.f + eps);
#pragma unroll
  for (int kc = 0; kc < 4; ++kc) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
      x[kc][i] = (bf16)(((float)x[kc][i] - mean) * inv * gs[32 * kc + g8 + i] + bs[32 * kc + g8 + i]);
  }
}

template <class T, int K, int TAPS, int NT, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void seqlin_d_kernel(SeqLinArgs a, int ntiles) {
  typedef Mfma<T> M;
  typedef typename M::frag F;
  constexpr int PAD = 16 / (int)sizeof(T), VEC = 16 / (int)sizeof(T), KS = K + PAD, NKC = K / M::KS;
  constexpr int NG = VEC / 4, IT = 16 * 16 * NT / VEC / 64;  // fp32 groups per chunk, chunks per lane (max)
  // the LDS epilogue only where its tile keeps two workgroups per CU (the 3-tap images take ~80 KB already)
  constexpr bool LE = TAPS == 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Wt = (T*)smem;  // [TAPS * N][K + PAD]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), col = lane & 15, kof = M::koff(lane),
            g4 = 4 * (lane >> 4);
  const int ES = a.N + kSdEpad, cpr = a.N / VEC, nch = 16 * cpr;
  float* E = (float*)(Wt + TAPS * a.N * KS) + wave * 16 * ES;  // this wave's [16][N + pad] fp32 tile (LE)
  // LayerNorm parameters (LN form): after the image and the epilogue tiles
  float* Lg = (float*)(Wt + TAPS * a.N * KS) + (LE ? WAVES * 16 * ES : 0);
  constexpr bool LNF = sizeof(T) == 2 && K == 128;
  if constexpr (LNF)
    if (a.lng)
      for (int e = threadIdx.x; e < 2 * K; e += 64 * WAVES) Lg[e] = e < K ? a.lng[e] : a.lnb[e - K];
  // the bias, staged once (after the LayerNorm parameters' slots): the epilogue reads it from LDS (a global load
  // per output block, each used at once, was waited for in turn: NT round trips per tile)
  float* Lb = Lg + 2 * K;
  if (a.b)
    for (int e = threadIdx.x; e < a.N; e += 64 * WAVES) Lb[e] = a.b[e];
  constexpr int CPR = K / VEC;
  for (int e = threadIdx.x; e < TAPS * a.N * CPR; e += 64 * WAVES) {
    const int n = e / CPR, q = e % CPR;
    *(uint4*)(Wt + n * KS + q * VEC) = *(const uint4*)((const T*)a.wp + (size_t)n * K + q * VEC);
  }
  constexpr int kSdRows = 16 * WAVES;
  F bf[2][TAPS][NKC];
  uint4 rr[2][IT];      // LE: residual chunks of the lane's output chunks
  RawR4<T> r4[2][NT];   // otherwise: residual channels (4) of the lane's row per output tile
  // register double buffer: the slot is a compile-time constant (runtime-indexed register arrays spill)
  auto load_tile = [&](int tile, auto S) {
    constexpr int slot = decltype(S)::value;
    const int seq = tile / a.tiles_per_seq, tb = (tile - seq * a.tiles_per_seq) * kSdRows + wave * 16,
              t = tb + col;
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int src = t + a.dir * (TAPS - 1 - tap);
      const bool ok = src >= 0 && src < a.T && t < a.T;
      const T* p = (const T*)a.x + ((long long)seq * a.T + (ok ? src : 0)) * a.ldx + kof;
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        F v = M::load(p + kc * M::KS);
        if (!ok) v = F{};
        bf[slot][tap][kc] = v;
      }
    }
    if (a.r) {
      if constexpr (LE) {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
          const int e = lane + 64 * i, row = e / cpr, q = e - row * cpr;
          if (e < nch && tb + row < a.T)
            rr[slot][i] = *(const uint4*)((const T*)a.r + ((long long)seq * a.T + tb + row) * a.ldr + q * VEC);
        }
      } else {
        const bool ok = t < a.T;
        const T* rp = (const T*)a.r + ((long long)seq * a.T + (ok ? t : 0)) * a.ldr + g4;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          if (nt * 16 < a.N) r4[slot][nt].v = *(const typename RawR4<T>::type*)(rp + nt * 16);
      }
    }
  };
  auto compute = [&](int tile, auto S) {
    constexpr int slot = decltype(S)::value;
    if constexpr (LNF) {
      if (a.lng) {  // normalise the rows now (their loads have landed); rows outside [0, T) stay zero
        const int seq = tile / a.tiles_per_seq, t = (tile - seq * a.tiles_per_seq) * kSdRows + wave * 16 + col;
#pragma unroll
        for (int tap = 0; tap < TAPS; ++tap) {
          const int src = t + a.dir * (TAPS - 1 - tap);
          ln_row_frags(bf[slot][tap], Lg, Lg + K, kof, a.lneps);
          if (!(src >= 0 && src < a.T && t < a.T))
#pragma unroll
            for (int kc = 0; kc < NKC; ++kc) bf[slot][tap][kc] = F{};
          __builtin_amdgcn_sched_barrier(0);  // one row set at a time (register pressure)
        }
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap)
#pragma unroll
      for (int kc = 0; kc < NKC; ++kc) {
        const F b = bf[slot][tap][kc];
        const T* wb = Wt + (tap * a.N + col) * KS + kof + kc * M::KS;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if (nt * 16 >= a.N) break;
          acc[nt] = M::mma(M::load(wb + nt * 16 * KS), b, acc[nt]);
        }
      }
    if constexpr (!LE) {  // lane (row = col, g): channels nt*16 + 4g .. +3 of its row straight to memory
      const int seq = tile / a.tiles_per_seq, t = (tile - seq * a.tiles_per_seq) * kSdRows + wave * 16 + col;
      if (t < a.T) {
        const long long row = (long long)seq * a.T + t;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if (nt * 16 >= a.N) break;
          const int c = nt * 16 + g4;
          f32x4 v = acc[nt];
          if (a.b) v = v + *(const f32x4*)(Lb + c);
          if (a.r) v = v + r4[slot][nt].f();
          T* yp = (T*)a.y + row * a.ldy + c;
          if (a.accumulate) v = v + ld4((const T*)yp);
          st4(yp, v);
        }
      }
      return;
    }
    // lane (row = col, g) holds channels nt*16 + 4g .. +3 -> the wave's fp32 tile; LDS traffic of one wave
    // is processed in order, so its reads below see these writes
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (nt * 16 >= a.N) break;
      *(f32x4*)(E + col * ES + nt * 16 + g4) = acc[nt];
    }
    __builtin_amdgcn_wave_barrier();
    const int seq = tile / a.tiles_per_seq, tb = (tile - seq * a.tiles_per_seq) * kSdRows + wave * 16;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int e = lane + 64 * i, row = e / cpr, q = e - row * cpr;
      if (e >= nch || tb + row >= a.T) continue;
      const long long grow = (long long)seq * a.T + tb + row;
      f32x4 v[NG], u[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) v[g] = *(const f32x4*)(E + row * ES + q * VEC + 4 * g);
      if (a.b)
#pragma unroll
        for (int g = 0; g < NG; ++g) v[g] = v[g] + *(const f32x4*)(Lb + q * VEC + 4 * g);
      if (a.r) {
        chunk_widen<T>(rr[slot][i], u);
#pragma unroll
        for (int g = 0; g < NG; ++g) v[g] = v[g] + u[g];
      }
      uint4* yp = (uint4*)((T*)a.y + grow * a.ldy + q * VEC);
      if (a.accumulate) {
        chunk_widen<T>(*yp, u);
#pragma unroll
        for (int g = 0; g < NG; ++g) v[g] = v[g] + u[g];
      }
      *yp = chunk_narrow<T>(v);
    }
    __builtin_amdgcn_wave_barrier();
  };
  typedef std::integral_constant<int, 0> S0;
  typedef std::integral_constant<int, 1> S1;
  const int G = gridDim.x;
  int tile = blockIdx.x;
  if (tile < ntiles) load_tile(tile, S0());
  __syncthreads();  // weight images staged
  for (; tile < ntiles; tile += 2 * G) {
    if (tile + G < ntiles) load_tile(tile + G, S1());
    compute(tile, S0());
    if (tile + G >= ntiles) break;
    if (tile + 2 * G < ntiles) load_tile(tile + 2 * G, S0());
    compute(tile + G, S1());
  }
}

// Weight preparation for seqlin: out[tap][n][k] = Wv[tap][k][n] in the activation dtype, for a batch of layers in
// one launch (blockIdx.y = descriptor). Run once per step; the forward passes and the data gradients then stage
// their weights with plain 16-byte copies.
constexpr int kMaxPrep = 48;
struct PrepBatch {
  vqa_seqlin_prep_desc d[kMaxPrep];
};

template <class T>
__global__ __launch_bounds__(256) void seqlin_prep_kernel(PrepBatch b) {
  const vqa_seqlin_prep_desc& d = b.d[blockIdx.y];
  const int total = d.taps * d.K * d.N;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int tap = e / (d.N * d.K), rem = e - tap * d.N * d.K, n = rem / d.K, k = rem - n * d.K;
    const float v = d.wtrans ? d.w[((size_t)tap * d.N + n) * d.K + k] : d.w[((size_t)tap * d.K + k) * d.N + n];
    ((T*)d.out)[e] = (T)v;
  }
}

// Weight gradient of the sequence-linear layer (forward direction dir = -1 or taps = 1):
//   dW[tap][k][n] = sum_t X[t - (taps-1-tap)][k] dY[t][n],  db[n] = sum_t dY[t][n]
// Workgroup = one row segment of one sequence, 64-row chunks staged in LDS; MFMA K = rows via transposed
// fragment reads (Mfma::rows). Wave w owns the (tap, k-tile) pairs p = w, w+4, ... and every n-tile: per
// 32-row step it reads NT dY fragments and one X fragment per pair. One fp32 partial row per workgroup:
// [dW (taps*K*N) | db (N)].
struct SeqWgArgs {
  const void* x;
  const void* dy;
  float* part;
  long long ldx, lddy;
  int nseq, T, K, N, taps, seg_rows, segs_per_seq;
};

template <class T, int PPW, int NT>
__global__ __launch_bounds__(256) void seqlin_wgrad_kernel(SeqWgArgs a) {
  typedef Mfma<T> M;
  constexpr int PAD = 16 / (int)sizeof(T), CH = 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int XS = a.K + PAD, YS = a.N + PAD, halo = a.taps - 1;
  T* X = (T*)smem;               // [CH + halo][K + PAD]; row j <-> time c0 - halo + j
  T* Y = X + (CH + halo) * XS;   // [CH][N + PAD]
  const int seq = blockIdx.x / a.segs_per_seq, seg = blockIdx.x - seq * a.segs_per_seq;
  const int tb = seg * a.seg_rows, te = std::min(a.T, tb + a.seg_rows);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int npairs = a.taps * (a.K / 16);
  f32x4 acc[PPW][NT], accb[NT];
#pragma unroll
  for (int p = 0; p < PPW; ++p)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[p][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) accb[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool bias_wave = wave == 3;  // the wave with the fewest pairs also sums the bias
  constexpr int VEC = 16 / (int)sizeof(T);
  for (int c0 = tb; c0 < te; c0 += CH) {
    __syncthreads();
    const int cx = a.K / VEC, cy = a.N / VEC;
    for (int e = threadIdx.x; e < (CH + halo) * cx; e += 256) {
      const int j = e / cx, q = e - j * cx, t = c0 - halo + j;
      uint4 v = {0u, 0u, 0u, 0u};
      // source rows of this segment's outputs only: t < te (rows past the segment belong to the next one)
      if (t >= 0 && t < te) v = *(const uint4*)((const T*)a.x + ((long long)seq * a.T + t) * a.ldx + q * VEC);
      *(uint4*)(X + j * XS + q * VEC) = v;
    }
    for (int e = threadIdx.x; e < CH * cy; e += 256) {
      const int j = e / cy, q = e - j * cy, t = c0 + j;
      uint4 v = {0u, 0u, 0u, 0u};
      if (t < te) v = *(const uint4*)((const T*)a.dy + ((long long)seq * a.T + t) * a.lddy + q * VEC);
      *(uint4*)(Y + j * YS + q * VEC) = v;
    }
    __syncthreads();
    for (int kk = 0; kk < CH; kk += M::KS) {
      typename M::frag bf[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bf[nt] = nt * 16 < a.N ? M::rows(Y + kk * YS + nt * 16, YS) : bf[0];
#pragma unroll
      for (int p = 0; p < PPW; ++p) {
        const int pr = wave + 4 * p;
        if (pr >= npairs) break;
        const int tap = pr / (a.K / 16), kt = pr - tap * (a.K / 16);
        const typename M::frag af = M::rows(X + (kk + tap) * XS + kt * 16, XS);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          if (nt * 16 < a.N) acc[p][nt] = M::mma(af, bf[nt], acc[p][nt]);
      }
      if (bias_wave) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          if (nt * 16 < a.N) accb[nt] = M::mma(M::ones(), bf[nt], accb[nt]);
      }
    }
  }
  float* part = a.part + (size_t)blockIdx.x * ((size_t)a.taps * a.K * a.N + a.N);
  const int n = lane & 15, g4 = 4 * (lane >> 4);
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int pr = wave + 4 * p;
    if (pr >= npairs) break;
    const int tap = pr / (a.K / 16), kt = pr - tap * (a.K / 16);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (nt * 16 >= a.N) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) part[((size_t)tap * a.K + kt * 16 + g4 + i) * a.N + nt * 16 + n] = acc[p][nt][i];
    }
  }
  if (bias_wave && lane < 16) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      if (nt * 16 < a.N) part[(size_t)a.taps * a.K * a.N + nt * 16 + n] = accb[nt][0];
  }
}

// ---------------------------------------------------------------------------------------------------
// embeddings (autoregressive_fmha.py:119-151): x = table[tok] (row 0 replaced by y_cond when given) * scale
// + pos[t]; dropout; + x_cond. One thread per 4 channels.
constexpr unsigned long long kEmbDropSalt = 0x454d42ull;  // VQA_EMB_DROPOUT_SALT (vqa.h)

struct EmbArgs {
  const float* table;
  const float* pos;
  const int64_t* tok;
  const float* ycond;  // (N, W) or null
  const void* xcond;   // (N, T, W) activation dtype or null
  void* out;
  long long rows;
  int T, W, bins;
  float scale, rate;
  unsigned long long seed;
  const int64_t* ctr;  // optional device step counter mixed into the seed (advances under graph replay)
  long long off;       // global flat index of out[0] (data parallel: rank * N*T*W) — the dropout mask's key
};

__device__ __forceinline__ unsigned long long seed_at(unsigned long long seed, const int64_t* ctr) {
  return ctr ? seed ^ splitmix64((uint64_t)*ctr) : seed;
}

template <class T>
__global__ __launch_bounds__(256) void prior_embed_kernel(EmbArgs a) {
  const long long total = a.rows * (a.W / 4);
  const unsigned long long seed = seed_at(a.seed, a.ctr);
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long r = e / (a.W / 4);
    const int c = (int)(e - r * (a.W / 4)) * 4, t = (int)(r % a.T);
    const long long n = r / a.T;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (a.ycond && t == 0) {
      v = *(const f32x4*)(a.ycond + n * a.W + c);
    } else {
      const int64_t k = a.tok[r];
      if (k >= 0 && k < a.bins) v = *(const f32x4*)(a.table + k * a.W + c);
    }
    v = v * a.scale;
    v = v + *(const f32x4*)(a.pos + (long long)t * a.W + c);
    if (a.rate > 0.f) {
      // the mask of dropout_kernel over the flat (N, T, W) index with salt kEmbDropSalt: the backward is
      // vqa_dropout on the gradient with the same (seed, salt, counter)
      const float ks = 1.0f / (1.0f - a.rate);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = prior_uniform(seed, kEmbDropSalt, (uint64_t)(a.off + r * a.W + c + i), 0) >= a.rate ? v[i] * ks : 0.f;
    }
    if (a.xcond) v = v + ld4((const T*)a.xcond + r * a.W + c);
    st4((T*)a.out + r * a.W + c, v);
  }
}

// out[r][c] (+)= sum_{n < nout} x[n * ostride + r * C + c], fixed order over n (fp32 out)
template <class T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* x, float* out, int nout, long long ostride, long long inner,
                                                    int accumulate) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < inner; e += (long long)gridDim.x * 256) {
    float s = 0.f;
    for (int n = 0; n < nout; ++n) s += ld(x + n * ostride + e);
    out[e] = accumulate ? out[e] + s : s;
  }
}

template <class T>
__global__ __launch_bounds__(256) void axpy_kernel(const T* x, const T* y, T* z, long long n) {
  for (long long e = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; e < n; e += (long long)gridDim.x * 1024) {
    if (e + 4 <= n) {
      st4(z + e, ld4(x + e) + ld4(y + e));
    } else {
      for (long long i = e; i < n; ++i) st(z + i, ld(x + i) + ld(y + i));
    }
  }
}

// keras Dropout(rate): x * (1 / (1 - rate)) where u >= rate, else 0 (the same mask on the gradient); the mask
// is keyed on the global flat index off + e (data parallel: each rank passes its shard's first index)
template <class T>
__global__ __launch_bounds__(256) void dropout_kernel(T* x, long long n, float rate, unsigned long long seed0,
                                                     unsigned long long salt, long long off, const int64_t* ctr) {
  const float ks = 1.0f / (1.0f - rate);
  const unsigned long long seed = seed_at(seed0, ctr);
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256)
    st(x + e, prior_uniform(seed, salt, (uint64_t)(off + e), 0) >= rate ? ld(x + e) * ks : 0.f);
}

__global__ __launch_bounds__(256) void scale_f32_kernel(float* x, long long n, float s) {
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) x[e] *= s;
}

// prior.py:262-290: latent_input = [start, codes[:-1]]; pred = [start, argmax[:-1]];
// out = mask ? pred : latent_input with mask = explicit (uint8) or uniform(seed, step, row) < rate
__global__ __launch_bounds__(256) void tf_mix_kernel(const int64_t* codes, const int64_t* amax, const uint8_t* mask,
                                                    int64_t* out, long long rows, int T, int64_t start, float rate,
                                                    unsigned long long seed, unsigned long long step0,
                                                    long long row_offset, const int64_t* ctr) {
  const unsigned long long step = step0 + (ctr ? (unsigned long long)*ctr : 0ull);
  for (long long r = (long long)blockIdx.x * 256 + threadIdx.x; r < rows; r += (long long)gridDim.x * 256) {
    const int t = (int)(r % T);
    const int64_t latent = t == 0 ? start : codes[r - 1];
    bool m = false;
    if (amax) m = mask ? mask[r] != 0 : prior_uniform(seed, 0x5446ull, step, (uint64_t)(r + row_offset)) < rate;
    out[r] = m ? (t == 0 ? start : amax[r - 1]) : latent;
  }
}


// ---------------------------------------------------------------------------------------------------
// Factorized attention (keras MultiHeadAttention core after the query/key/value EinsumDense; head dim 16).
// Q, K, V, O: (N, T, H*16) in the activation dtype; lse: (N, T, H) fp32 in the log2 domain (x = s*scale*log2e).
//   mode 0 row      (factorized_attention.py:74-141): causal inside each block of l positions
//   mode 1 col      (:210-286): position j of block b attends positions j of blocks 0..b (causal over blocks)
//   mode 2 prev-row (:308-388): block b attends every position of block b-1; block 0 sees the zero block,
//                   i.e. keys = key bias, values = value bias: O = value bias exactly
// Modes 0 and 2: flash attention on MFMA. A workgroup = 64 queries (wave w: 16); key tiles of 64 in LDS.
// S^T = K Q^T (K = head dim) leaves each lane 16 scores of ONE query (lane & 15), so softmax statistics are
// per-lane plus two cross-group shuffles; O^T = V^T P^T (K = keys) reads V^T by transposed LDS reads.
constexpr int AHD = 16;  // head dim
constexpr float kLog2e = 1.4426950408889634f;

template <class T> struct Att;
template <> struct Att<bf16> {
  typedef short s4 __attribute__((ext_vector_type(4)));
  typedef s4 dfrag;  // head dims 4g .. 4g+3 of one row (g = lane >> 4)
  static __device__ __forceinline__ dfrag ld_d(const bf16* row) {
    return *(const s4*)(row + 4 * ((threadIdx.x & 63) >> 4));
  }
  static __device__ __forceinline__ f32x4 mm_d(dfrag a, dfrag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  }
  // sum over 32 rows of a row-major tile window (16 columns from `tile`, row stride `stride`): the A operand
  // is the window transposed (lane (col, g) reads rows r0+4g..+3 and r0+16+4g..+3 by ds_read_b64_tr_b16),
  // the B operand the caller's 8 values for the same rows
  static __device__ __forceinline__ f32x4 mm_rows(const bf16* tile, int stride, int r0, const float (&p)[8], f32x4 c) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef short v8s __attribute__((ext_vector_type(8)));
    const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
    const bf16* a0 = tile + (r0 + 4 * g + (li >> 2)) * stride + 4 * (li & 3);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0 + 16 * stride));
    const bf16x8 A = __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    const bf16x8 B = {(bf16)p[0], (bf16)p[1], (bf16)p[2], (bf16)p[3], (bf16)p[4], (bf16)p[5], (bf16)p[6], (bf16)p[7]};
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B, c, 0, 0, 0);
  }
};
template <> struct Att<float> {
  typedef f32x4 dfrag;  // element c = head dim 4c + g
  static __device__ __forceinline__ dfrag ld_d(const float* row) {
    const int g = (threadIdx.x & 63) >> 4;
    return f32x4{row[g], row[4 + g], row[8 + g], row[12 + g]};
  }
  static __device__ __forceinline__ f32x4 mm_d(dfrag a, dfrag b, f32x4 c) {
#pragma unroll
    for (int i = 0; i < 4; ++i) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], c, 0, 0, 0);
    return c;
  }
  // MFMA j takes rows r0 + 16*(j>>2) + 4g + (j&3) in its K slots g = 0..3
  static __device__ __forceinline__ f32x4 mm_rows(const float* tile, int stride, int r0, const float (&p)[8], f32x4 c) {
    const int l = threadIdx.x & 63, li = l & 15, g = l >> 4;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(tile[(r0 + 16 * (j >> 2) + 4 * g + (j & 3)) * stride + li], p[j], c, 0, 0, 0);
    return c;
  }
};

struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  const void* dout;
  float* dsum;  // D = rowsum(dO * O), written by attn_bwd_q, read by attn_bwd_kv
  void* dq;
  void* dk;
  void* dv;
  const float* vbias;  // mode 2: value bias (H*16), the block-0 output
  int N, T, H, l;
  float scale;
};

// raw v_exp_f32 (no denormal range handling: probabilities below 2^-126 flush to zero, as in any softmax)
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ float grp_max(float v) { return xl::max32(xl::max16(v)); }
__device__ __forceinline__ float grp_sum(float v) { return xl::sum32(xl::sum16(v)); }

constexpr int AKS = AHD + 4;  // LDS row stride of a 64 x 16 tile (elements)

// 64 rows x 16 of (N, T, H*16) rows [r0, r0+64) of head h -> LDS tile [64][AKS]
template <class T>
__device__ __forceinline__ void stage64(T* dst, const T* src, long long row0, int H, int h) {
  const int r = threadIdx.x >> 2, q = (threadIdx.x & 3) * 4;
  const T* p = src + ((row0 + r) * H + h) * AHD + q;
  if constexpr (sizeof(T) == 2) *(uint2*)(dst + r * AKS + q) = *(const uint2*)p;
  else *(uint4*)(dst + r * AKS + q) = *(const uint4*)p;
}

// the calling thread's 4-element chunk of a 64 x 16 tile, held in registers between the global load (issued one
// tile ahead) and the LDS store
template <class T> struct Chunk64 {
  typedef typename std::conditional<sizeof(T) == 2, uint2, uint4>::type V;
  V v;
  __device__ __forceinline__ void load(const T* src, long long row0, int H, int h) {
    const int r = threadIdx.x >> 2, q = (threadIdx.x & 3) * 4;
    v = *(const V*)(src + ((row0 + r) * H + h) * AHD + q);
  }
  __device__ __forceinline__ void store(T* dst) const {
    const int r = threadIdx.x >> 2, q = (threadIdx.x & 3) * 4;
    *(V*)(dst + r * AKS + q) = v;
  }
};

// Ceiling (row attention at SMALL_PRIOR, B = 8, ctx 8192, 2 heads, blocks of 2048): 134 M causal scores, each
// one v_exp_f32 (8 issue cycles per 64 lanes) plus ~4 other VALU (scale FMA, max, sum, bf16 pack) -> about
// 20 us on 256 CUs; the QK / PV MFMAs (head dim 16, K = 16) are < 10 % of that. Measured 64 us (r2g/r3). A
// single-wave-per-64-queries form without workgroup barriers (4 query groups per staged key tile) measured
// 69.5 us: at 8 waves per CU the per-wave serial chain of the online softmax is not hidden, where this form
// keeps 32 waves per CU.
template <class T, int MODE>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  typedef Att<T> A;
  __shared__ __attribute__((aligned(16))) T Ks[64 * AKS];
  __shared__ __attribute__((aligned(16))) T Vs[64 * AKS];
  const int qt = blockIdx.x, h = blockIdx.y, n = blockIdx.z, q0 = qt * 64, b = q0 / a.l;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  const int qi = q0 + wave * 16 + li;
  const long long qrow = (long long)n * a.T + qi;
  T* orow = (T*)a.o + (qrow * a.H + h) * AHD + 4 * g;
  if (MODE == 2 && b == 0) {  // the zero block: uniform weights over identical (bias) values
    f32x4 v = *(const f32x4*)(a.vbias + h * AHD + 4 * g);
    st4(orow, v);
    if (g == 0) a.lse[qrow * a.H + h] = 0.f;
    return;
  }
  const typename A::dfrag qf = A::ld_d((const T*)a.q + (qrow * a.H + h) * AHD);
  const int kt0 = MODE == 0 ? b * a.l / 64 : (b - 1) * a.l / 64, kt1 = MODE == 0 ? qt : b * a.l / 64 - 1;
  const float c = a.scale * kLog2e;
  float m = -INFINITY, lsum = 0.f;
  f32x4 oacc = {0.f, 0.f, 0.f, 0.f};
  Chunk64<T> ck, cv;
  ck.load((const T*)a.k, (long long)n * a.T + kt0 * 64, a.H, h);
  cv.load((const T*)a.v, (long long)n * a.T + kt0 * 64, a.H, h);
  for (int kt = kt0; kt <= kt1; ++kt) {
    __syncthreads();
    ck.store(Ks);
    cv.store(Vs);
    __syncthreads();
    if (kt < kt1) {  // next tile in flight while this one computes
      ck.load((const T*)a.k, (long long)n * a.T + (kt + 1) * 64, a.H, h);
      cv.load((const T*)a.v, (long long)n * a.T + (kt + 1) * 64, a.H, h);
    }
    // raw scores; the scale (> 0) is applied inside the exponent: p = 2^(s*c - m), m = max(s)*c
    float x[4][4];
    float mt = -INFINITY;
    const bool diag = MODE == 0 && kt == qt;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const f32x4 s = A::mm_d(A::ld_d(Ks + (st * 16 + li) * AKS), qf, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i) x[st][i] = s[i];
    }
    if (diag) {
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (st * 16 + 4 * g + i > wave * 16 + li) x[st][i] = -INFINITY;
    }
#pragma unroll
    for (int st = 0; st < 4; ++st)
      mt = fmaxf(fmaxf(fmaxf(mt, x[st][0]), fmaxf(x[st][1], x[st][2])), x[st][3]);
    mt = grp_max(mt) * c;
    const float mn = fmaxf(m, mt), alpha = fexp2(m - mn);
    m = mn;
    float p[4][4], ps = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[st][i] = fexp2(__builtin_fmaf(x[st][i], c, -mn));
        ps += p[st][i];
      }
    lsum = lsum * alpha + ps;
    oacc = oacc * alpha;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const float p8[8] = {p[2 * cc][0], p[2 * cc][1], p[2 * cc][2], p[2 * cc][3],
                           p[2 * cc + 1][0], p[2 * cc + 1][1], p[2 * cc + 1][2], p[2 * cc + 1][3]};
      oacc = A::mm_rows(Vs, AKS, 32 * cc, p8, oacc);
    }
  }
  const float lt = grp_sum(lsum), inv = 1.0f / lt;
  st4(orow, oacc * inv);
  if (g == 0) a.lse[qrow * a.H + h] = m + log2f(lt);
}

template <class T, int MODE>
__global__ __launch_bounds__(256) void attn_bwd_q_kernel(AttnArgs a) {
  typedef Att<T> A;
  __shared__ __attribute__((aligned(16))) T Ks[64 * AKS];
  __shared__ __attribute__((aligned(16))) T Vs[64 * AKS];
  const int qt = blockIdx.x, h = blockIdx.y, n = blockIdx.z, q0 = qt * 64, b = q0 / a.l;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  const int qi = q0 + wave * 16 + li;
  const long long qrow = (long long)n * a.T + qi, off = (qrow * a.H + h) * AHD;
  // D = rowsum(dO * O)
  const f32x4 dov = ld4((const T*)a.dout + off + 4 * g), ov = ld4((const T*)a.o + off + 4 * g);
  const float D = grp_sum(dov[0] * ov[0] + dov[1] * ov[1] + dov[2] * ov[2] + dov[3] * ov[3]);
  if (g == 0) a.dsum[qrow * a.H + h] = D;
  T* dqrow = (T*)a.dq + off + 4 * g;
  if (MODE == 2 && b == 0) {  // constant scores: no gradient reaches the queries
    st4(dqrow, f32x4{0.f, 0.f, 0.f, 0.f});
    return;
  }
  const typename A::dfrag qf = A::ld_d((const T*)a.q + off), dof = A::ld_d((const T*)a.dout + off);
  const float lse = a.lse[qrow * a.H + h];
  const int kt0 = MODE == 0 ? b * a.l / 64 : (b - 1) * a.l / 64, kt1 = MODE == 0 ? qt : b * a.l / 64 - 1;
  const float c = a.scale * kLog2e;
  f32x4 dqacc = {0.f, 0.f, 0.f, 0.f};
  Chunk64<T> ck, cv;
  ck.load((const T*)a.k, (long long)n * a.T + kt0 * 64, a.H, h);
  cv.load((const T*)a.v, (long long)n * a.T + kt0 * 64, a.H, h);
  for (int kt = kt0; kt <= kt1; ++kt) {
    __syncthreads();
    ck.store(Ks);
    cv.store(Vs);
    __syncthreads();
    if (kt < kt1) {
      ck.load((const T*)a.k, (long long)n * a.T + (kt + 1) * 64, a.H, h);
      cv.load((const T*)a.v, (long long)n * a.T + (kt + 1) * 64, a.H, h);
    }
    float ds[4][4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const f32x4 s = A::mm_d(A::ld_d(Ks + (st * 16 + li) * AKS), qf, f32x4{0.f, 0.f, 0.f, 0.f});
      const f32x4 dp = A::mm_d(A::ld_d(Vs + (st * 16 + li) * AKS), dof, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float p = fexp2(__builtin_fmaf(s[i], c, -lse));
        if (MODE == 0 && kt == qt && st * 16 + 4 * g + i > wave * 16 + li) p = 0.f;
        ds[st][i] = p * (dp[i] - D);
      }
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const float p8[8] = {ds[2 * cc][0], ds[2 * cc][1], ds[2 * cc][2], ds[2 * cc][3],
                           ds[2 * cc + 1][0], ds[2 * cc + 1][1], ds[2 * cc + 1][2], ds[2 * cc + 1][3]};
      dqacc = A::mm_rows(Ks, AKS, 32 * cc, p8, dqacc);
    }
  }
  st4(dqrow, dqacc * a.scale);
}

template <class T, int MODE>
__global__ __launch_bounds__(256) void attn_bwd_kv_kernel(AttnArgs a) {
  typedef Att<T> A;
  __shared__ __attribute__((aligned(16))) T Qs[64 * AKS];
  __shared__ __attribute__((aligned(16))) T Ds[64 * AKS];  // dO tile
  __shared__ __attribute__((aligned(16))) float Ls[64];
  __shared__ __attribute__((aligned(16))) float Dd[64];
  const int kt = blockIdx.x, h = blockIdx.y, n = blockIdx.z, k0 = kt * 64, b = k0 / a.l;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  const int ki = k0 + wave * 16 + li;
  const long long krow = (long long)n * a.T + ki, off = (krow * a.H + h) * AHD;
  T* dkrow = (T*)a.dk + off + 4 * g;
  T* dvrow = (T*)a.dv + off + 4 * g;
  const int nblk = a.T / a.l;
  int qt0, qt1;
  if (MODE == 0) {
    qt0 = kt;
    qt1 = (b + 1) * a.l / 64 - 1;
  } else {
    qt0 = (b + 1) * a.l / 64;
    qt1 = b + 1 < nblk ? (b + 2) * a.l / 64 - 1 : qt0 - 1;
  }
  const typename A::dfrag kf = A::ld_d((const T*)a.k + off), vf = A::ld_d((const T*)a.v + off);
  const float c = a.scale * kLog2e;
  f32x4 dkacc = {0.f, 0.f, 0.f, 0.f}, dvacc = {0.f, 0.f, 0.f, 0.f};
  Chunk64<T> cq, cd;
  float pl = 0.f, pd = 0.f;
  auto load_q = [&](int qt) {
    const long long r0 = (long long)n * a.T + qt * 64;
    cq.load((const T*)a.q, r0, a.H, h);
    cd.load((const T*)a.dout, r0, a.H, h);
    if (threadIdx.x < 64) {
      pl = a.lse[(r0 + threadIdx.x) * a.H + h];
      pd = a.dsum[(r0 + threadIdx.x) * a.H + h];
    }
  };
  if (qt0 <= qt1) load_q(qt0);
  for (int qt = qt0; qt <= qt1; ++qt) {
    __syncthreads();
    cq.store(Qs);
    cd.store(Ds);
    if (threadIdx.x < 64) {
      Ls[threadIdx.x] = pl;
      Dd[threadIdx.x] = pd;
    }
    __syncthreads();
    if (qt < qt1) load_q(qt + 1);
    float p[4][4], ds[4][4];
#pragma unroll
    for (int qs = 0; qs < 4; ++qs) {
      const f32x4 s = A::mm_d(A::ld_d(Qs + (qs * 16 + li) * AKS), kf, f32x4{0.f, 0.f, 0.f, 0.f});
      const f32x4 dp = A::mm_d(A::ld_d(Ds + (qs * 16 + li) * AKS), vf, f32x4{0.f, 0.f, 0.f, 0.f});
      // the 4 query rows' lse and D: one 16-byte LDS read each
      const f32x4 lq = *(const f32x4*)(Ls + qs * 16 + 4 * g), dq = *(const f32x4*)(Dd + qs * 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ql = qs * 16 + 4 * g + i;
        float pv = fexp2(__builtin_fmaf(s[i], c, -lq[i]));
        if (MODE == 0 && qt == kt && wave * 16 + li > ql) pv = 0.f;
        p[qs][i] = pv;
        ds[qs][i] = pv * (dp[i] - dq[i]);
      }
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const float p8[8] = {p[2 * cc][0], p[2 * cc][1], p[2 * cc][2], p[2 * cc][3],
                           p[2 * cc + 1][0], p[2 * cc + 1][1], p[2 * cc + 1][2], p[2 * cc + 1][3]};
      const float d8[8] = {ds[2 * cc][0], ds[2 * cc][1], ds[2 * cc][2], ds[2 * cc][3],
                           ds[2 * cc + 1][0], ds[2 * cc + 1][1], ds[2 * cc + 1][2], ds[2 * cc + 1][3]};
      dvacc = A::mm_rows(Ds, AKS, 32 * cc, p8, dvacc);
      dkacc = A::mm_rows(Qs, AKS, 32 * cc, d8, dkacc);
    }
  }
  st4(dkrow, dkacc * a.scale);
  st4(dvrow, dvacc);
}

// mode 1 (column attention, blocks <= 8): one thread per (item, position in block, head); all NB rows of the
// column in registers. Forward writes O and lse; backward writes dQ, dK, dV of the whole column (no atomics).
template <class T, int NB>
__global__ __launch_bounds__(256) void attn_col_fwd_kernel(AttnArgs a) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)a.N * a.l * a.H) return;
  const int h = (int)(e % a.H), j = (int)((e / a.H) % a.l);
  const long long n = e / ((long long)a.H * a.l);
  auto off = [&](int b) { return (((long long)n * a.T + (long long)b * a.l + j) * a.H + h) * AHD; };
  float kk[NB][AHD];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int d = 0; d < AHD; d += 4) {
      const f32x4 v = ld4((const T*)a.k + off(b) + d);
      kk[b][d] = v[0]; kk[b][d + 1] = v[1]; kk[b][d + 2] = v[2]; kk[b][d + 3] = v[3];
    }
  const float c = a.scale * kLog2e;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float q[AHD];
#pragma unroll
    for (int d = 0; d < AHD; d += 4) {
      const f32x4 v = ld4((const T*)a.q + off(b) + d);
      q[d] = v[0]; q[d + 1] = v[1]; q[d + 2] = v[2]; q[d + 3] = v[3];
    }
    float x[NB], m = -INFINITY;
#pragma unroll
    for (int bb = 0; bb <= b; ++bb) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < AHD; ++d) s += q[d] * kk[bb][d];
      x[bb] = s * c;
      m = fmaxf(m, x[bb]);
    }
    float l = 0.f, o[AHD];
#pragma unroll
    for (int d = 0; d < AHD; ++d) o[d] = 0.f;
#pragma unroll
    for (int bb = 0; bb <= b; ++bb) {
      const float p = exp2f(x[bb] - m);
      l += p;
#pragma unroll
      for (int d = 0; d < AHD; d += 4) {
        const f32x4 v = ld4((const T*)a.v + off(bb) + d);
        o[d] += p * v[0]; o[d + 1] += p * v[1]; o[d + 2] += p * v[2]; o[d + 3] += p * v[3];
      }
    }
    const float inv = 1.0f / l;
#pragma unroll
    for (int d = 0; d < AHD; d += 4)
      st4((T*)a.o + off(b) + d, f32x4{o[d] * inv, o[d + 1] * inv, o[d + 2] * inv, o[d + 3] * inv});
    a.lse[(off(b) / AHD)] = m + log2f(l);
  }
}

template <class T, int NB>
__global__ __launch_bounds__(256) void attn_col_bwd_kernel(AttnArgs a) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)a.N * a.l * a.H) return;
  const int h = (int)(e % a.H), j = (int)((e / a.H) % a.l);
  const long long n = e / ((long long)a.H * a.l);
  auto off = [&](int b) { return (((long long)n * a.T + (long long)b * a.l + j) * a.H + h) * AHD; };
  auto ldrow = [&](const void* base, int b, float (&r)[AHD]) {
#pragma unroll
    for (int d = 0; d < AHD; d += 4) {
      const f32x4 v = ld4((const T*)base + off(b) + d);
      r[d] = v[0]; r[d + 1] = v[1]; r[d + 2] = v[2]; r[d + 3] = v[3];
    }
  };
  const float c = a.scale * kLog2e;
  // P and dS for the column (lower triangle)
  float P[NB][NB], dS[NB][NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float q[AHD], go[AHD];
    ldrow(a.q, b, q);
    ldrow(a.dout, b, go);
    const float lse = a.lse[off(b) / AHD];
    float D = 0.f;
#pragma unroll
    for (int bb = 0; bb <= b; ++bb) {
      float kr[AHD], vr[AHD];
      ldrow(a.k, bb, kr);
      ldrow(a.v, bb, vr);
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < AHD; ++d) {
        s += q[d] * kr[d];
        dp += go[d] * vr[d];
      }
      P[b][bb] = exp2f(s * c - lse);
      dS[b][bb] = dp;
      D += P[b][bb] * dp;
    }
#pragma unroll
    for (int bb = 0; bb <= b; ++bb) dS[b][bb] = P[b][bb] * (dS[b][bb] - D);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    // dQ_b = scale * sum_{bb <= b} dS[b][bb] k_bb ; dK_b = scale * sum_{bq >= b} dS[bq][b] q_bq ;
    // dV_b = sum_{bq >= b} P[bq][b] dO_bq
    float dq[AHD], dk[AHD], dv[AHD];
#pragma unroll
    for (int d = 0; d < AHD; ++d) dq[d] = dk[d] = dv[d] = 0.f;
#pragma unroll
    for (int bb = 0; bb <= b; ++bb) {
      float kr[AHD];
      ldrow(a.k, bb, kr);
#pragma unroll
      for (int d = 0; d < AHD; ++d) dq[d] += dS[b][bb] * kr[d];
    }
#pragma unroll
    for (int bq = b; bq < NB; ++bq) {
      float q[AHD], go[AHD];
      ldrow(a.q, bq, q);
      ldrow(a.dout, bq, go);
#pragma unroll
      for (int d = 0; d < AHD; ++d) {
        dk[d] += dS[bq][b] * q[d];
        dv[d] += P[bq][b] * go[d];
      }
    }
#pragma unroll
    for (int d = 0; d < AHD; d += 4) {
      st4((T*)a.dq + off(b) + d, f32x4{dq[d], dq[d + 1], dq[d + 2], dq[d + 3]} * a.scale);
      st4((T*)a.dk + off(b) + d, f32x4{dk[d], dk[d + 1], dk[d + 2], dk[d + 3]} * a.scale);
      st4((T*)a.dv + off(b) + d, f32x4{dv[d], dv[d + 1], dv[d + 2], dv[d + 3]});
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Output head fused with the loss (autoregressive_fmha.py:80,158 Dense(bins); autoregressive.py:189-212):
// logits = X W + b are never written. Wt = W^T in the activation dtype, (V, 128), prepared once per step.
//   head_fwd:    per row lse, argmax (first maximum, tf.argmax), and with targets the row loss lse - logit[t]
//                and correctness
//   head_bwd_dx: dX = dlogits W^T, dlogits = (softmax - onehot) * inv_count (logits recomputed per vocab tile)
//   head_bwd_dw: dW = X^T dlogits, db = sum dlogits per (vocab tile, row segment) partial
constexpr int HK = 128;            // model width (the head's K)
template <class T> constexpr int hstride() { return HK + 16 / (int)sizeof(T); }

struct HeadArgs {
  const void* x;
  const void* wt;  // (V, HK)
  const float* bias;
  const int64_t* tgt;
  float* lse;
  int64_t* amax;
  float* loss_row;
  float* correct;
  void* dx;
  float* part;  // dW partials: [segment][HK * V + V]
  long long M;
  int V, seg_rows;
  float inv_count;
};

// logits^T of a 16-vocab subtile for one 16-row subtile: lane (row = lane & 15, g) gets vocab 4g .. 4g+3
template <class T>
__device__ __forceinline__ f32x4 head_tile(const T* wtl, const T* xl, int stride) {
  typedef Mfma<T> M;
  const int lane = threadIdx.x & 63, kof = M::koff(lane), col = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < HK; kc += M::KS)
    acc = M::mma(M::load(wtl + col * stride + kof + kc), M::load(xl + col * stride + kof + kc), acc);
  return acc;
}

template <class T>
__device__ __forceinline__ void stage_rows128(T* dst, const T* src, long long row0, long long nrows_avail, int nrows) {
  constexpr int VEC = 16 / (int)sizeof(T), CPR = HK / VEC, S = hstride<T>();
  for (int e = threadIdx.x; e < nrows * CPR; e += 256) {
    const int j = e / CPR, q = e - j * CPR;
    uint4 v = {0u, 0u, 0u, 0u};
    if (row0 + j < nrows_avail) v = *(const uint4*)(src + (row0 + j) * HK + q * VEC);
    *(uint4*)(dst + j * S + q * VEC) = v;
  }
}

// 64 rows of HK channels staged HBM -> registers -> LDS: the next tile's loads are issued before the current
// tile's MFMAs, so their latency hides behind them (rows past `avail` are zeros)
template <class T>
struct Rows64Regs {
  static constexpr int VEC = 16 / (int)sizeof(T), CPR = HK / VEC, PER = 64 * CPR / 256, S = hstride<T>();
  uint4 v[PER];
  __device__ __forceinline__ void load(const T* src, long long row0, long long avail) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * 256, j = e / CPR, q = e - j * CPR;
      v[i] = row0 + j < avail ? *(const uint4*)(src + (row0 + j) * HK + q * VEC) : uint4{0u, 0u, 0u, 0u};
    }
  }
  __device__ __forceinline__ void store(T* dst) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = threadIdx.x + i * 256, j = e / CPR, q = e - j * CPR;
      *(uint4*)(dst + j * S + q * VEC) = v[i];
    }
  }
};

// logits^T of a 16-vocab subtile with the 16 rows' fragments held in registers (xf[kc] = rows' K slice kc)
template <class T>
__device__ __forceinline__ f32x4 head_tile_x(const T* wtl, const typename Mfma<T>::frag (&xf)[HK / Mfma<T>::KS],
                                             int stride) {
  typedef Mfma<T> M;
  const int lane = threadIdx.x & 63, kof = M::koff(lane), col = lane & 15;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < HK / M::KS; ++kc) acc = M::mma(M::load(wtl + col * stride + kof + kc * M::KS), xf[kc], acc);
  return acc;
}

// this lane's share of dot(row, w) for a row held as B fragments (xf[kc]: channels kc*KS + koff ..) and a
// (HK) row w of Wt in the activation dtype; grp_sum over the four lane groups completes it
template <class T>
__device__ __forceinline__ float head_dot_row(const typename Mfma<T>::frag (&xf)[HK / Mfma<T>::KS], const T* w) {
  typedef Mfma<T> M;
  const int kof = M::koff(threadIdx.x & 63);
  float acc = 0.f;
#pragma unroll
  for (int kc = 0; kc < HK / M::KS; ++kc) {
    if constexpr (sizeof(T) == 2) {
      const bf16x8 wv = *(const bf16x8*)(w + kc * M::KS + kof);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = __builtin_fmaf((float)xf[kc][j], (float)wv[j], acc);
    } else {
      acc = __builtin_fmaf(xf[kc], w[kc * M::KS + kof], acc);
    }
  }
  return acc;
}

// the B fragments of a workgroup's rows (wave w: rows 32w + 16s + (lane & 15)) for every K slice
template <class T>
__device__ __forceinline__ void head_xfrags(typename Mfma<T>::frag (&xf)[2][HK / Mfma<T>::KS], const T* X, int stride) {
  typedef Mfma<T> M;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), kof = M::koff(lane), col = lane & 15;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int kc = 0; kc < HK / M::KS; ++kc) xf[s][kc] = M::load(X + (wave * 32 + s * 16 + col) * stride + kof + kc * M::KS);
}

// workgroup = 128 rows (wave w: rows 32w .. 32w+31 as two 16-row subtiles, their fragments in registers);
// vocab tiles of 64 through LDS, the next one prefetched into registers
template <class T>
__global__ __launch_bounds__(256) void head_fwd_kernel(HeadArgs a) {
  constexpr int S = hstride<T>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* X = (T*)smem;     // [128][S]
  T* W = X + 128 * S;  // [64][S]
  const long long r0 = (long long)blockIdx.x * 128;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  stage_rows128<T>(X, (const T*)a.x, r0, a.M, 128);
  Rows64Regs<T> wn;
  wn.load((const T*)a.wt, 0, a.V);
  __syncthreads();
  typename Mfma<T>::frag xf[2][HK / Mfma<T>::KS];
  head_xfrags<T>(xf, X, S);
  long long rows[2];
  int64_t tg[2];
  float m[2], l[2], bv[2], tl[2];
  int bi[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    rows[s] = r0 + wave * 32 + s * 16 + li;
    tg[s] = (a.tgt && rows[s] < a.M) ? a.tgt[rows[s]] : -1;
    m[s] = -INFINITY; l[s] = 0.f; bv[s] = -INFINITY; bi[s] = 0; tl[s] = -INFINITY;
  }
  constexpr float L2E = 1.4426950408889634f;
  // the tile's bias (slots past V: -inf) through LDS, loaded one tile ahead by wave 0 with the weight rows (read
  // straight from global memory after the barrier, each tile waited for its bias loads there)
  __shared__ __attribute__((aligned(16))) float Bt[64];
  float bn = threadIdx.x < 64 && (int)threadIdx.x < a.V ? a.bias[threadIdx.x] : -INFINITY;
  for (int v0 = 0; v0 < a.V; v0 += 64) {
    __syncthreads();
    wn.store(W);
    if (threadIdx.x < 64) Bt[threadIdx.x] = bn;
    if (v0 + 64 < a.V) {
      wn.load((const T*)a.wt, v0 + 64, a.V);
      if (threadIdx.x < 64) bn = v0 + 64 + (int)threadIdx.x < a.V ? a.bias[v0 + 64 + threadIdx.x] : -INFINITY;
    }
    __syncthreads();
    // this lane's 16 vocab slots of the tile: v0 + 16 st + 4 g + i (slots past V: -inf)
    f32x4 bq[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) bq[st] = *(const f32x4*)(Bt + st * 16 + 4 * g);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float x[16];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const f32x4 acc = head_tile_x<T>(W + st * 16 * S, xf[s], S);
#pragma unroll
        for (int i = 0; i < 4; ++i) x[4 * st + i] = acc[i] + bq[st][i];  // -inf past V
      }
      float mt = x[0];
#pragma unroll
      for (int k = 1; k < 16; ++k) mt = fmaxf(mt, x[k]);
      // the first slot holding the tile maximum (slots ascend in vocab within the lane): tf.argmax's first max
      int ti = 15;
#pragma unroll
      for (int k = 14; k >= 0; --k) ti = x[k] == mt ? k : ti;
      if (mt > bv[s]) {
        bv[s] = mt;
        bi[s] = v0 + (ti >> 2) * 16 + 4 * g + (ti & 3);
      }
      const float mn = fmaxf(m[s], mt);
      if (mn == -INFINITY) continue;  // only vocab slots past V in this lane so far
      const float nm = -mn * L2E;
      float ps = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) ps += __builtin_amdgcn_exp2f(__builtin_fmaf(x[k], L2E, nm));
      l[s] = l[s] * __builtin_amdgcn_exp2f((m[s] - mn) * L2E) + ps;
      m[s] = mn;
    }
  }
  // the target's logit, once per row: the row's fragments (registers) . Wt[target] + bias[target]
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bool tin = tg[s] >= 0 && tg[s] < a.V;
    const float part = tin ? head_dot_row<T>(xf[s], (const T*)a.wt + tg[s] * HK) : 0.f;
    const float dot = grp_sum(part);
    tl[s] = tin ? dot + a.bias[tg[s]] : -INFINITY;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float mx = grp_max(m[s]);
    const float lt = grp_sum(l[s] * __expf(m[s] - mx));
    // argmax across the four lane groups: larger value, then the lower index
    // (the two lanes of each pair, in the same order for the values and the indices; the pick is symmetric)
    auto pick = [](float av, int ai, float bv2, int bi2, float& v, int& i) {
      const bool b_wins = bv2 > av || (bv2 == av && bi2 < ai);
      v = b_wins ? bv2 : av;
      i = b_wins ? bi2 : ai;
    };
    {
      float av, bv2;
      int ai, bi2;
      xl::pair16(bv[s], av, bv2);
      xl::pair16(bi[s], ai, bi2);
      pick(av, ai, bv2, bi2, bv[s], bi[s]);
      xl::pair32(bv[s], av, bv2);
      xl::pair32(bi[s], ai, bi2);
      pick(av, ai, bv2, bi2, bv[s], bi[s]);
    }
    const float t = tl[s];
    if (g == 0 && rows[s] < a.M) {
      const float lse = mx + logf(lt);
      a.lse[rows[s]] = lse;
      if (a.amax) a.amax[rows[s]] = bi[s];
      if (a.loss_row) a.loss_row[rows[s]] = lse - t;
      if (a.correct) a.correct[rows[s]] = (int64_t)bi[s] == tg[s] ? 1.f : 0.f;
    }
  }
}

template <class T>
__global__ __launch_bounds__(256) void head_bwd_dx_kernel(HeadArgs a) {
  typedef Att<T> A;
  constexpr int S = hstride<T>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* X = (T*)smem;
  T* W = X + 128 * S;
  const long long r0 = (long long)blockIdx.x * 128;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  stage_rows128<T>(X, (const T*)a.x, r0, a.M, 128);
  Rows64Regs<T> wn;
  wn.load((const T*)a.wt, 0, a.V);
  __syncthreads();
  typename Mfma<T>::frag xf[2][HK / Mfma<T>::KS];
  head_xfrags<T>(xf, X, S);
  long long rows[2];
  int64_t tg[2];
  float lse[2];
  f32x4 acc[2][HK / 16];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    rows[s] = r0 + wave * 32 + s * 16 + li;
    const bool in = rows[s] < a.M;
    tg[s] = in ? a.tgt[rows[s]] : -1;
    lse[s] = in ? a.lse[rows[s]] : INFINITY;  // rows past M: softmax 0, no target -> dlogits 0
#pragma unroll
    for (int kt = 0; kt < HK / 16; ++kt) acc[s][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // softmax * inv_count = exp2((z + b) log2e - (lse log2e - log2 inv_count)); the target's -inv_count is added
  // once per row after the loop (dX -= inv_count Wt[target])
  constexpr float L2E = 1.4426950408889634f;
  float nl[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) nl[s] = -(lse[s] * L2E - __log2f(a.inv_count));
  // the tile's bias through LDS, loaded one tile ahead (as head_fwd_kernel)
  __shared__ __attribute__((aligned(16))) float Bt[64];
  float bn = threadIdx.x < 64 && (int)threadIdx.x < a.V ? a.bias[threadIdx.x] : -INFINITY;
  for (int v0 = 0; v0 < a.V; v0 += 64) {
    __syncthreads();
    wn.store(W);
    if (threadIdx.x < 64) Bt[threadIdx.x] = bn;
    if (v0 + 64 < a.V) {
      wn.load((const T*)a.wt, v0 + 64, a.V);
      if (threadIdx.x < 64) bn = v0 + 64 + (int)threadIdx.x < a.V ? a.bias[v0 + 64 + threadIdx.x] : -INFINITY;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float dl[4][4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const f32x4 z = head_tile_x<T>(W + st * 16 * S, xf[s], S);
        const f32x4 bq = *(const f32x4*)(Bt + st * 16 + 4 * g);  // slots past V: -inf (probability 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) dl[st][i] = __builtin_amdgcn_exp2f(__builtin_fmaf(z[i] + bq[i], L2E, nl[s]));
      }
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const float p8[8] = {dl[2 * cc][0], dl[2 * cc][1], dl[2 * cc][2], dl[2 * cc][3],
                             dl[2 * cc + 1][0], dl[2 * cc + 1][1], dl[2 * cc + 1][2], dl[2 * cc + 1][3]};
#pragma unroll
        for (int kt = 0; kt < HK / 16; ++kt) acc[s][kt] = A::mm_rows(W + kt * 16, S, 32 * cc, p8, acc[s][kt]);
      }
      __builtin_amdgcn_sched_barrier(0);  // one row subtile at a time (register pressure)
    }
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (rows[s] >= a.M) continue;
    const bool tin = tg[s] >= 0 && tg[s] < a.V;
    const T* wtg = (const T*)a.wt + (tin ? tg[s] : 0) * HK;
#pragma unroll
    for (int kt = 0; kt < HK / 16; ++kt) {
      f32x4 o = acc[s][kt];
      if (tin) o = o - ld4(wtg + kt * 16 + 4 * g) * a.inv_count;  // the one-hot term of dlogits
      st4((T*)a.dx + rows[s] * HK + kt * 16 + 4 * g, o);
    }
  }
}

// workgroup = (vocab tile of 64: wave w owns vocab v0 + 16w .. +15, row segment); logits in the layout
// lane (vocab, g) <- rows 4g .. 4g+3 so that dW = X^T dlogits takes dlogits as the B operand directly
template <class T>
__global__ __launch_bounds__(256) void head_bwd_dw_kernel(HeadArgs a) {
  typedef Mfma<T> M;
  typedef Att<T> A;
  constexpr int S = hstride<T>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* W = (T*)smem;     // [64][S]
  T* X = W + 64 * S;   // [64][S]
  __shared__ __attribute__((aligned(16))) float Ls[64];  // lse log2e - log2 inv_count (+inf past the segment)
  __shared__ __attribute__((aligned(16))) int Tg[64];     // targets (-1 past the segment)
  const int nvt = (a.V + 63) / 64, vt = blockIdx.x % nvt, seg = blockIdx.x / nvt, v0 = vt * 64;
  const long long rb = (long long)seg * a.seg_rows, re = std::min<long long>(a.M, rb + a.seg_rows);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), li = lane & 15, g = lane >> 4;
  const int v = v0 + wave * 16 + li;
  constexpr float L2E = 1.4426950408889634f;
  const float bl = v < a.V ? a.bias[v] * L2E : -INFINITY;  // vocab slots past V: probability 0
  const float l2inv = __log2f(a.inv_count);
  stage_rows128<T>(W, (const T*)a.wt, v0, a.V, 64);
  f32x4 acc[HK / 16];
#pragma unroll
  for (int kt = 0; kt < HK / 16; ++kt) acc[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  const int kof = M::koff(lane);
  // the next row tile (and its lse / targets) prefetched into registers during the current one's MFMAs
  Rows64Regs<T> xn;
  float ln = INFINITY;
  int tn = -1;
  auto fetch = [&](long long c0) {
    xn.load((const T*)a.x, c0, re);
    if (threadIdx.x < 64) {
      const bool in = c0 + threadIdx.x < re;
      ln = in ? a.lse[c0 + threadIdx.x] * L2E - l2inv : INFINITY;
      tn = in ? (int)a.tgt[c0 + threadIdx.x] : -1;
    }
  };
  if (rb < re) fetch(rb);
  __syncthreads();
  typename M::frag wf[HK / M::KS];  // this wave's 16 vocab columns, every K slice
#pragma unroll
  for (int kc = 0; kc < HK / M::KS; ++kc) wf[kc] = M::load(W + (wave * 16 + li) * S + kof + kc * M::KS);
  for (long long c0 = rb; c0 < re; c0 += 64) {
    __syncthreads();
    xn.store(X);
    if (threadIdx.x < 64) {
      Ls[threadIdx.x] = ln;
      Tg[threadIdx.x] = tn;
    }
    if (c0 + 64 < re) fetch(c0 + 64);
    __syncthreads();
    float dl[4][4];
#pragma unroll
    for (int rs = 0; rs < 4; ++rs) {
      // logits[row][v]: A = X rows (rs*16 + col), B = W^T (vocab col)
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < HK / M::KS; ++kc) z = M::mma(M::load(X + (rs * 16 + li) * S + kof + kc * M::KS), wf[kc], z);
      // rows rs*16 + 4g + i: softmax * inv_count, minus inv_count at the target
      const f32x4 lq = *(const f32x4*)(Ls + rs * 16 + 4 * g);
      const int4 tq = *(const int4*)(Tg + rs * 16 + 4 * g);
      const int tqa[4] = {tq.x, tq.y, tq.z, tq.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float d = __builtin_amdgcn_exp2f(__builtin_fmaf(z[i], L2E, bl - lq[i]));
        if (v == tqa[i]) d -= a.inv_count;
        dl[rs][i] = d;
        db += d;
      }
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const float p8[8] = {dl[2 * cc][0], dl[2 * cc][1], dl[2 * cc][2], dl[2 * cc][3],
                           dl[2 * cc + 1][0], dl[2 * cc + 1][1], dl[2 * cc + 1][2], dl[2 * cc + 1][3]};
#pragma unroll
      for (int kt = 0; kt < HK / 16; ++kt) acc[kt] = A::mm_rows(X + kt * 16, S, 32 * cc, p8, acc[kt]);
    }
  }
  // partial row of this segment: dW (HK x V, Keras layout) | db (V); lane (vocab col, g) holds k = kt*16+4g+i
  float* part = a.part + (size_t)seg * ((size_t)HK * a.V + a.V);
  if (v < a.V) {
#pragma unroll
    for (int kt = 0; kt < HK / 16; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(size_t)(kt * 16 + 4 * g + i) * a.V + v] = acc[kt][i];
  }
  db = grp_sum(db);
  if (g == 0 && v < a.V) part[(size_t)HK * a.V + v] = db;
}

// W (HK, V) fp32 -> Wt (V, HK) in the activation dtype
template <class T>
__global__ __launch_bounds__(256) void head_wt_kernel(const float* w, T* wt, int V) {
  const long long total = (long long)HK * V;
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int k = (int)(e / V), v = (int)(e - (long long)k * V);
    st(wt + (long long)v * HK + k, w[e]);
  }
}

// out[i] = scale * sum_j x[i * n + j]: stage 1 sums fixed chunks of 4096 per workgroup, stage 2 sums the chunk
// results in order (deterministic)
constexpr int kRowsumChunk = 4096;
__global__ __launch_bounds__(256) void rowsum_part_kernel(const float* x, long long n, int nch, float* part) {
  __shared__ float red[4];
  const int row = blockIdx.x / nch, ch = blockIdx.x - row * nch;
  const float* p = x + (long long)row * n;
  const long long j0 = (long long)ch * kRowsumChunk, j1 = std::min<long long>(n, j0 + kRowsumChunk);
  float s = 0.f;
  for (long long j = j0 + threadIdx.x; j < j1; j += 256) s += p[j];
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ __launch_bounds__(256) void rowsum_final_kernel(const float* part, int nch, float scale, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int j = threadIdx.x; j < nch; j += 256) s += part[(long long)blockIdx.x * nch + j];
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s * scale;
}

// ---------------------------------------------------------------------------------------------------
// Autoregressive decode (autoregressive_fmha.py:162-240 sample()): the reference re-runs the whole model on
// the prefix at every step; here ONE persistent workgroup per sample walks the steps with a key/value cache
// (the factorized attention of position i only needs keys <= i, keys of the same column, or the previous
// block) and keeps the causal conv's last two LayerNorm outputs per layer in LDS. Per step: embedding, the
// depth residual-attention blocks, the output head, z = logits + Gumbel(seed, sample, step, bin) and
// next token = argmax z (RelaxedOneHotCategorical(1).sample() then argmax). fp32 throughout, weights fp32
// from L2. Optional: forced input tokens (teacher-forced check) and per-step logits output.
constexpr int kDecMaxLayers = 8;
constexpr int kDecW = 128;   // model width
constexpr int kDecAW = 32;   // attention width (m_attn 0.25)
constexpr int kDecMaxL = 2048;

struct DecLayer {
  const float *ln1g, *ln1b, *qkvw, *qkvb, *qw, *qb, *kw, *kb, *vw, *vb, *ow, *ob, *pw, *pb, *ln2g, *ln2b, *mw, *mb;
  int type;
  // composed once per decode (prior_decode_prep_kernel): the causal conv followed by the query/key/value
  // EinsumDense (one 384 x 96 map straight to the heads) and the output EinsumDense followed by proj (32 x 128)
  float *cw, *cb, *opw, *opb;
};

struct DecArgs {
  DecLayer L[kDecMaxLayers];
  const float *emb, *pos, *hw, *hb;
  const float* ycond;     // (N, W) or null
  const float* xcond;     // (N, T, W) fp32 or null
  const int64_t* forced;  // (N, steps + 1) or null
  float* logits;          // (N, steps, bins) or null
  int64_t* tokens;        // (N, steps + 1)
  float* kc;              // (N, depth, T, 32) key cache
  float* vc;              // (N, depth, T, 32) value cache
  int N, steps, T, depth, H, l, bins, ldo;  // ldo: head weight row stride (>= bins, % 4 == 0)
  long long start;
  unsigned long long seed;
  float scale, emb_scale, eps;
};

// y[o] = b[o] + sum_k x[k] W[k][o] (W row-major (K, O), O % 4 == 0): thread (4-output chunk c, k-group kg) sums
// its rows with 16-byte weight loads (many loads in flight per thread), then the k-groups are combined in a
// fixed order. scr holds >= 256 * 4 floats.
__device__ void dec_matvec(const float* x, int K, const float* W, const float* b, float* y, int O, float* scr) {
  const int tid = threadIdx.x, nc = O / 4;
  if (nc <= 256) {
    const int G = 256 / nc, kg = tid / nc, c = tid - kg * nc;
    if (kg < G) {
      const int k0 = kg * K / G, k1 = (kg + 1) * K / G;
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int k = k0; k < k1; ++k) s = s + x[k] * *(const f32x4*)(W + (size_t)k * O + 4 * c);
      *(f32x4*)(scr + (kg * nc + c) * 4) = s;
    }
    __syncthreads();
    if (tid < nc) {
      f32x4 s = *(const f32x4*)(scr + tid * 4);
      for (int g = 1; g < G; ++g) s = s + *(const f32x4*)(scr + (g * nc + tid) * 4);
      if (b) s = s + *(const f32x4*)(b + 4 * tid);
      *(f32x4*)(y + 4 * tid) = s;
    }
    __syncthreads();
  } else {
    for (int c = tid; c < nc; c += 256) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 16
      for (int k = 0; k < K; ++k) s = s + x[k] * *(const f32x4*)(W + (size_t)k * O + 4 * c);
      if (b) s = s + *(const f32x4*)(b + 4 * c);
      *(f32x4*)(y + 4 * c) = s;
    }
    __syncthreads();
  }
}

// LayerNorm of a 128-vector in LDS (wave 0 computes the statistics; fixed butterfly order)
__device__ void dec_layernorm(const float* x, const float* gm, const float* bt, float* y, float eps, float* stat) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    const float a0 = x[tid], a1 = x[tid + 64];
    const float mean = wave_sum_f(a0 + a1) / (float)kDecW;
    const float d0 = a0 - mean, d1 = a1 - mean;
    const float var = wave_sum_f(d0 * d0 + d1 * d1) / (float)kDecW;
    if (tid == 0) { stat[0] = mean; stat[1] = 1.0f / sqrtf(var + eps); }
  }
  __syncthreads();
  if (tid < kDecW) y[tid] = (x[tid] - stat[0]) * stat[1] * gm[tid] + bt[tid];
  __syncthreads();
}

// Linear maps of a layer composed in fp32 (the decode step then does 3 mat-vecs per layer instead of 7):
//   cw[tap*128 + k][j*32 + n] = sum_m qkvw[tap][k][j*32 + m] * Wj[m][n]   (j = query, key, value)
//   cb[j*32 + n] = sum_m qkvb[j*32 + m] * Wj[m][n] + bj[n]
//   opw[k][n] = sum_m ow[k][m] * pw[m][n],  opb[n] = sum_m ob[m] * pw[m][n] + pb[n]
__global__ __launch_bounds__(256) void prior_decode_prep_kernel(DecArgs a) {
  const DecLayer& ly = a.L[blockIdx.y];
  const int nc = 3 * kDecW * 3 * kDecAW, nb = 3 * kDecAW, no = kDecAW * kDecW;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < nc + nb + no + kDecW; e += gridDim.x * 256) {
    if (e < nc) {
      const int row = e / (3 * kDecAW), col = e - row * (3 * kDecAW), j = col / kDecAW, n = col - j * kDecAW;
      const float* Wj = j == 0 ? ly.qw : j == 1 ? ly.kw : ly.vw;
      float s = 0.f;
      for (int m = 0; m < kDecAW; ++m) s += ly.qkvw[row * 3 * kDecAW + j * kDecAW + m] * Wj[m * kDecAW + n];
      ly.cw[e] = s;
    } else if (e < nc + nb) {
      const int col = e - nc, j = col / kDecAW, n = col - j * kDecAW;
      const float* Wj = j == 0 ? ly.qw : j == 1 ? ly.kw : ly.vw;
      const float* bj = j == 0 ? ly.qb : j == 1 ? ly.kb : ly.vb;
      float s = 0.f;
      for (int m = 0; m < kDecAW; ++m) s += ly.qkvb[j * kDecAW + m] * Wj[m * kDecAW + n];
      ly.cb[col] = s + bj[n];
    } else if (e < nc + nb + no) {
      const int q = e - nc - nb, k = q / kDecW, n = q - k * kDecW;
      float s = 0.f;
      for (int m = 0; m < kDecAW; ++m) s += ly.ow[k * kDecAW + m] * ly.pw[m * kDecW + n];
      ly.opw[q] = s;
    } else {
      const int n = e - nc - nb - no;
      float s = 0.f;
      for (int m = 0; m < kDecAW; ++m) s += ly.ob[m] * ly.pw[m * kDecW + n];
      ly.opb[n] = s + ly.pb[n];
    }
  }
}

__global__ __launch_bounds__(256) void prior_decode_kernel(DecArgs a) {
  __shared__ __attribute__((aligned(16))) float x[kDecW], x1[kDecW], hb[kDecW], r1[kDecW];
  __shared__ float ring[kDecMaxLayers][3][kDecW];
  __shared__ __attribute__((aligned(16))) float cat[3 * kDecW], qkv[3 * kDecAW], oh[kDecAW];
  __shared__ float sc[2][kDecMaxL];
  __shared__ __attribute__((aligned(16))) float scr[2048];
  __shared__ __attribute__((aligned(16))) float red[32][kDecAW];
  __shared__ float stat[4];
  __shared__ __attribute__((aligned(16))) float bestv[1024];
  __shared__ int besti[256];
  const int n = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < kDecMaxLayers * 3 * kDecW; e += 256) (&ring[0][0][0])[e] = 0.f;
  int64_t tok = a.start;
  if (tid == 0) a.tokens[(size_t)n * (a.steps + 1)] = a.start;
  __syncthreads();
  for (int i = 0; i < a.steps; ++i) {
    // embedding (autoregressive_fmha.py:119-151)
    if (tid < kDecW) {
      float e = (a.ycond && i == 0) ? a.ycond[(size_t)n * kDecW + tid]
                                    : ((tok >= 0 && tok < a.bins) ? a.emb[(size_t)tok * kDecW + tid] : 0.f);
      e = e * a.emb_scale;
      e = e + a.pos[(size_t)i * kDecW + tid];
      if (a.xcond) e = e + a.xcond[((size_t)n * a.T + i) * kDecW + tid];
      x[tid] = e;
    }
    __syncthreads();
    const int b = i / a.l, p = i - b * a.l;
    for (int L = 0; L < a.depth; ++L) {
      const DecLayer& ly = a.L[L];
      float* aring = &ring[L][0][0];
      dec_layernorm(x, ly.ln1g, ly.ln1b, aring + (i % 3) * kDecW, a.eps, stat);
      // causal conv input [a_{i-2}, a_{i-1}, a_i] (zeros before the sequence start)
      if (tid < kDecW) {
#pragma unroll
        for (int tp = 0; tp < 3; ++tp) {
          const int j = i - 2 + tp;
          cat[tp * kDecW + tid] = j >= 0 ? aring[(j % 3) * kDecW + tid] : 0.f;
        }
      }
      __syncthreads();
      dec_matvec(cat, 3 * kDecW, ly.cw, ly.cb, qkv, 3 * kDecAW, scr);  // [q heads | k heads | v heads]
      const float* qh = qkv;
      const float* kh = qkv + kDecAW;
      const float* vh = qkv + 2 * kDecAW;
      float* kcL = a.kc + (((size_t)n * a.depth + L) * a.T) * kDecAW;
      float* vcL = a.vc + (((size_t)n * a.depth + L) * a.T) * kDecAW;
      if (tid < kDecAW) {
        kcL[(size_t)i * kDecAW + tid] = kh[tid];
        vcL[(size_t)i * kDecAW + tid] = vh[tid];
      }
      __threadfence_block();
      __syncthreads();
      // keys of this position: row: [b*l, i]; col: (b', p) for b' <= b; prev-row: block b-1 (b = 0: value bias)
      int cnt, j0, jstep;
      if (ly.type == 0) { cnt = p + 1; j0 = b * a.l; jstep = 1; }
      else if (ly.type == 1) { cnt = b + 1; j0 = p; jstep = a.l; }
      else { cnt = b > 0 ? a.l : 0; j0 = (b - 1) * a.l; jstep = 1; }
      if (cnt == 0) {
        if (tid < kDecAW) oh[tid] = ly.vb[tid];
        __syncthreads();
      } else {
        const int hd = kDecAW / a.H;
        for (int idx = tid; idx < cnt; idx += 256) {
          const f32x4* kr = (const f32x4*)(kcL + (size_t)(j0 + idx * jstep) * kDecAW);
          const f32x4* qv = (const f32x4*)qh;
          f32x4 kv[kDecAW / 4];
#pragma unroll
          for (int c = 0; c < kDecAW / 4; ++c) kv[c] = kr[c];
          for (int h = 0; h < a.H; ++h) {
            float s = 0.f;
            for (int c = h * hd / 4; c < (h + 1) * hd / 4; ++c) {
              const f32x4 pq = qv[c] * kv[c];
              s += (pq[0] + pq[1]) + (pq[2] + pq[3]);
            }
            sc[h][idx] = s * a.scale;
          }
        }
        __syncthreads();
        // per head max and sum (wave h reduces head h)
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        if (wave < a.H) {
          float m = -INFINITY;
          for (int idx = lane; idx < cnt; idx += 64) m = fmaxf(m, sc[wave][idx]);
          m = wave_max_f(m);
          float su = 0.f;
          for (int idx = lane; idx < cnt; idx += 64) {
            const float e = __expf(sc[wave][idx] - m);
            sc[wave][idx] = e;
            su += e;
          }
          su = wave_sum_f(su);
          if (lane == 0) stat[wave] = 1.0f / su;
        }
        __syncthreads();
        // o[h][d] = sum_j p_j v_j[h][d]: thread (4-channel chunk c4 = tid & 7, key slice sl = tid >> 3) over keys
        // sl, sl + 32, ... with 16-byte loads; slices combined in a fixed order
        {
          const int c4 = tid & 7, sl = tid >> 3, h = 4 * c4 / hd;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
          for (int idx = sl; idx < cnt; idx += 32)
            acc = acc + sc[h][idx] * *(const f32x4*)(vcL + (size_t)(j0 + idx * jstep) * kDecAW + 4 * c4);
          *(f32x4*)(&red[sl][4 * c4]) = acc;
        }
        __syncthreads();
        if (tid < kDecAW) {
          float o = red[0][tid];
          for (int sl = 1; sl < 32; ++sl) o += red[sl][tid];
          oh[tid] = o * stat[tid / hd];
        }
        __syncthreads();
      }
      dec_matvec(oh, kDecAW, ly.opw, ly.opb, r1, kDecW, scr);  // output EinsumDense o proj
      if (tid < kDecW) x1[tid] = x[tid] + r1[tid];
      __syncthreads();
      dec_layernorm(x1, ly.ln2g, ly.ln2b, hb, a.eps, stat);
      dec_matvec(hb, kDecW, ly.mw, ly.mb, cat, kDecW, scr);  // res2 (cat reused)
      if (tid < kDecW) x[tid] = cat[tid] + x1[tid];
      __syncthreads();
    }
    // output head + Gumbel-max
    dec_matvec(x, kDecW, a.hw, a.hb, scr, a.ldo, bestv);  // scr holds the logits (ldo >= bins columns)
    float bv = -INFINITY;
    int bi = 0;
    for (int v = tid; v < a.bins; v += 256) {
      const float lg = scr[v];
      if (a.logits) a.logits[((size_t)n * a.steps + i) * a.bins + v] = lg;
      const float u = prior_uniform(a.seed, (uint64_t)n, (uint64_t)i, (uint64_t)v);
      const float z = lg + (-logf(-logf(u)));
      if (z > bv) { bv = z; bi = v; }
    }
    __syncthreads();
    bestv[tid] = bv;
    besti[tid] = bi;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (tid < w) {
        const float ov = bestv[tid + w];
        const int oi = besti[tid + w];
        if (ov > bestv[tid] || (ov == bestv[tid] && oi < besti[tid])) { bestv[tid] = ov; besti[tid] = oi; }
      }
      __syncthreads();
    }
    const int64_t samp = besti[0];
    if (tid == 0) a.tokens[(size_t)n * (a.steps + 1) + i + 1] = samp;
    tok = a.forced ? a.forced[(size_t)n * (a.steps + 1) + i + 1] : samp;
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------------
static int pr_grid(long long work, int per = 256, int cap = 8192) {
  return (int)std::max<long long>(1, std::min<long long>((work + per - 1) / per, cap));
}
static bool pr_dt(int dtype) { return dtype == VQA_F32 || dtype == VQA_BF16; }

static size_t seqlin_lds(int K, int N, int taps, int esz) {
  const int ks = K + 16 / esz;
  return ((size_t)N * ks + (size_t)(kSlRows + taps - 1) * ks) * esz;
}
static size_t wgrad_lds(int K, int N, int taps, int esz) {
  return ((size_t)(64 + taps - 1) * (K + 16 / esz) + (size_t)64 * (N + 16 / esz)) * esz;
}
static int set_lds_attr(const void* fn, size_t bytes) {
  if (bytes <= 65536) return VQA_OK;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) != hipSuccess) {
    (void)hipGetLastError();
    set_error("prior: cannot reserve %zu B of LDS", bytes);
    return VQA_E_UNSUPPORTED;
  }
  return VQA_OK;
}

template <class T>
static int launch_seqlin(const SeqLinArgs& a, hipStream_t s) {
  if (a.wp) {
    // wide outputs: 8 waves per workgroup share one staged weight image (one workgroup per CU); narrow ones:
    // 4 waves, two workgroups per CU (measured per shape, tools/seqlin_time.py)
    const bool n2 = a.N <= 32, w8 = a.N >= 96;
    const int waves = w8 ? 8 : 4, max_per_cu = w8 ? 1 : 2;
    const int KS = a.K + 16 / (int)sizeof(T);
    const size_t lds = (size_t)a.taps * a.N * KS * sizeof(T) +
                       (a.taps == 1 ? (size_t)waves * 16 * (a.N + kSdEpad) * sizeof(float) : 0) +
                       (size_t)(2 * a.K + a.N) * sizeof(float);  // LayerNorm slots (used or not) + the bias
    const void* fn = nullptr;
#define VQA_SD(KK, TT)                                                                                         \
    if (a.K == KK && a.taps == TT)                                                                           \
      fn = n2 ? (const void*)seqlin_d_kernel<T, KK, TT, 2, 4>                                                \
              : w8 ? (const void*)seqlin_d_kernel<T, KK, TT, 8, 8> : (const void*)seqlin_d_kernel<T, KK, TT, 8, 4>;
    VQA_SD(32, 1) VQA_SD(128, 1) VQA_SD(96, 3) VQA_SD(128, 3)
#undef VQA_SD
    // the 1-tap epilogue stores (and reads the residual) in whole 16-byte chunks
    const int vec = 16 / (int)sizeof(T);
    const bool chunks = a.taps != 1 || (a.ldy % vec == 0 && ((uintptr_t)a.y & 15) == 0 &&
                                        (!a.r || (a.ldr % vec == 0 && ((uintptr_t)a.r & 15) == 0)));
    if (fn && chunks && lds <= 160 * 1024) {
      if (int rc = set_lds_attr(fn, lds)) return rc;
      SeqLinArgs c = a;
      c.tiles_per_seq = (a.T + 16 * waves - 1) / (16 * waves);
      int ntiles = a.nseq * c.tiles_per_seq;
      const int per_cu = std::max(1, std::min<int>(max_per_cu, (int)(160 * 1024 / lds)));
      const int nwg = std::min(ntiles, pr_cus() * per_cu);
      void* args[] = {&c, &ntiles};
      (void)hipLaunchKernel(fn, dim3(nwg), dim3(64 * waves), args, lds, s);
      VQA_LAUNCHED("seqlin_d_kernel");
      return VQA_OK;
    }
    // weights too large for one LDS image: stage per tap from the prepared image
  }
  VQA_REQUIRE(!a.lng, VQA_E_UNSUPPORTED, "seqlin_fwd_ln_prepped: K=%d N=%d taps=%d has no fused form", a.K, a.N,
              a.taps);
  const void* fn = a.N <= 32 ? (const void*)seqlin_kernel<T, 2> : (const void*)seqlin_kernel<T, 8>;
  const size_t lds = seqlin_lds(a.K, a.N, a.taps, sizeof(T));
  if (int rc = set_lds_attr(fn, lds)) return rc;
  SeqLinArgs c = a;
  void* args[] = {&c};
  (void)hipLaunchKernel(fn, dim3(a.nseq * a.tiles_per_seq), dim3(256), args, lds, s);
  VQA_LAUNCHED("seqlin_kernel");
  return VQA_OK;
}

template <class T>
static const void* wgrad_fn(int ppw, int N) {
  const bool n2 = N <= 32;
  if (ppw <= 1) return n2 ? (const void*)seqlin_wgrad_kernel<T, 1, 2> : (const void*)seqlin_wgrad_kernel<T, 1, 8>;
  if (ppw <= 2) return n2 ? (const void*)seqlin_wgrad_kernel<T, 2, 2> : (const void*)seqlin_wgrad_kernel<T, 2, 8>;
  return n2 ? (const void*)seqlin_wgrad_kernel<T, 6, 2> : (const void*)seqlin_wgrad_kernel<T, 6, 8>;
}

static void wgrad_plan(int nseq, int T, int& seg_rows, int& segs) {
  // about 2 workgroups per CU in total, segments a multiple of the 64-row chunk
  const long long target = std::max<long long>(1, (long long)2 * pr_cus() / std::max(1, nseq));
  seg_rows = (int)std::max<long long>(64, ((T + target - 1) / target + 63) / 64 * 64);
  segs = (T + seg_rows - 1) / seg_rows;
}

}  // namespace vqa

using namespace vqa;

extern "C" int vqa_seqlin_prep(const vqa_seqlin_prep_desc* descs, int count, int dtype, vqa_stream_t stream) {
  VQA_ARG(descs && count > 0 && pr_dt(dtype), "seqlin_prep: bad arguments");
  for (int i0 = 0; i0 < count; i0 += kMaxPrep) {
    PrepBatch b;
    const int n = std::min(kMaxPrep, count - i0);
    for (int i = 0; i < n; ++i) {
      b.d[i] = descs[i0 + i];
      VQA_ARG(b.d[i].w && b.d[i].out && b.d[i].taps > 0 && b.d[i].K > 0 && b.d[i].N > 0, "seqlin_prep: descriptor %d",
              i0 + i);
    }
    if (dtype == VQA_BF16)
      hipLaunchKernelGGL(seqlin_prep_kernel<bf16>, dim3(16, n), dim3(256), 0, (hipStream_t)stream, b);
    else
      hipLaunchKernelGGL(seqlin_prep_kernel<float>, dim3(16, n), dim3(256), 0, (hipStream_t)stream, b);
    VQA_LAUNCHED("seqlin_prep_kernel");
  }
  return VQA_OK;
}

static int seqlin_launch(const void* x, int64_t ldx, const float* w, const void* wp, const float* bias,
                         const void* residual, int64_t ldr, void* y, int64_t ldy, int nseq, int T, int K, int N,
                         int taps, int dir, int wtrans, int accumulate, int dtype, hipStream_t s) {
  VQA_ARG(x && (w || wp) && y && nseq > 0 && T > 0 && (taps == 1 || taps == 3) && (dir == -1 || dir == 1),
          "seqlin_fwd: bad arguments");
  VQA_ARG(pr_dt(dtype), "seqlin_fwd: unknown dtype %d", dtype);
  const int esz = dtype == VQA_BF16 ? 2 : 4, vec = 16 / esz;
  VQA_REQUIRE(K > 0 && K <= 256 && K % (dtype == VQA_BF16 ? 32 : 4) == 0 && N > 0 && N <= 128 && N % 16 == 0,
              VQA_E_UNSUPPORTED, "seqlin_fwd: K=%d N=%d unsupported", K, N);
  VQA_ARG(ldx % vec == 0 && ldy % 4 == 0 && (!residual || ldr % 4 == 0) && ldx >= K && ldy >= N,
          "seqlin_fwd: strides must keep 16-byte rows");
  VQA_ARG(((uintptr_t)(w ? (const void*)w : wp) & 15) == 0, "seqlin_fwd: weights must be 16-byte aligned");
  SeqLinArgs a{x, w, wp, bias, residual, y, ldx, ldr, ldy, nseq, T, K, N, taps, dir, wtrans, accumulate,
               (T + kSlRows - 1) / kSlRows};
  return dtype == VQA_BF16 ? launch_seqlin<bf16>(a, s) : launch_seqlin<float>(a, s);
}

extern "C" int vqa_seqlin_fwd(const void* x, int64_t ldx, const float* w, const float* bias, const void* residual,
                              int64_t ldr, void* y, int64_t ldy, int nseq, int T, int K, int N, int taps, int dir,
                              int wtrans, int accumulate, int dtype, vqa_stream_t stream) {
  VQA_ARG(w, "seqlin_fwd: no weights");
  return seqlin_launch(x, ldx, w, nullptr, bias, residual, ldr, y, ldy, nseq, T, K, N, taps, dir, wtrans, accumulate,
                       dtype, (hipStream_t)stream);
}

extern "C" int vqa_seqlin_fwd_prepped(const void* x, int64_t ldx, const void* wp, const float* bias,
                                      const void* residual, int64_t ldr, void* y, int64_t ldy, int nseq, int T, int K,
                                      int N, int taps, int dir, int accumulate, int dtype, vqa_stream_t stream) {
  VQA_ARG(wp, "seqlin_fwd_prepped: no weights");
  return seqlin_launch(x, ldx, nullptr, wp, bias, residual, ldr, y, ldy, nseq, T, K, N, taps, dir, 0, accumulate,
                       dtype, (hipStream_t)stream);
}

extern "C" int vqa_seqlin_fwd_ln_prepped(const void* x, int64_t ldx, const float* gamma, const float* beta,
                                         float eps, const void* wp, const float* bias, const void* residual,
                                         int64_t ldr, void* y, int64_t ldy, int nseq, int T, int K, int N, int taps,
                                         int dir, int dtype, vqa_stream_t stream) {
  VQA_ARG(x && wp && y && gamma && beta && nseq > 0 && T > 0 && (taps == 1 || taps == 3) && (dir == -1 || dir == 1),
          "seqlin_fwd_ln_prepped: bad arguments");
  VQA_REQUIRE(dtype == VQA_BF16 && K == 128 && N > 0 && N <= 128 && N % 16 == 0, VQA_E_UNSUPPORTED,
              "seqlin_fwd_ln_prepped: dtype %d K=%d N=%d unsupported (bf16, K = 128)", dtype, K, N);
  VQA_ARG(ldx % 8 == 0 && ldx >= K && ldy >= N && ldy % 4 == 0 && (!residual || ldr % 4 == 0),
          "seqlin_fwd_ln_prepped: strides must keep 16-byte rows");
  VQA_ARG(((uintptr_t)wp & 15) == 0, "seqlin_fwd_ln_prepped: weights must be 16-byte aligned");
  SeqLinArgs a{x, nullptr, wp, bias, residual, y, ldx, ldr, ldy, nseq, T, K, N, taps, dir, 0, 0,
               (T + kSlRows - 1) / kSlRows, gamma, beta, eps};
  return launch_seqlin<bf16>(a, (hipStream_t)stream);
}

extern "C" size_t vqa_seqlin_wgrad_workspace(int nseq, int T, int K, int N, int taps) {
  if (nseq < 1 || T < 1 || K < 1 || N < 1 || taps < 1) return 0;
  int seg_rows, segs;
  wgrad_plan(nseq, T, seg_rows, segs);
  return (size_t)nseq * segs * ((size_t)taps * K * N + N) * sizeof(float);
}

extern "C" int vqa_seqlin_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dw, float* db,
                                int nseq, int T, int K, int N, int taps, int dtype, void* workspace, size_t ws_bytes,
                                vqa_partials_desc* desc, vqa_stream_t stream) {
  VQA_ARG(x && dy && dw && nseq > 0 && T > 0 && (taps == 1 || taps == 3), "seqlin_wgrad: bad arguments");
  VQA_ARG(pr_dt(dtype), "seqlin_wgrad: unknown dtype %d", dtype);
  const int esz = dtype == VQA_BF16 ? 2 : 4, vec = 16 / esz;
  VQA_REQUIRE(K % 16 == 0 && K <= 128 && N % 16 == 0 && N <= 128 && (taps * K / 16 + 3) / 4 <= 6, VQA_E_UNSUPPORTED,
              "seqlin_wgrad: K=%d N=%d taps=%d unsupported", K, N, taps);
  VQA_ARG(ldx % vec == 0 && lddy % vec == 0, "seqlin_wgrad: strides must keep 16-byte rows");
  const size_t need = vqa_seqlin_wgrad_workspace(nseq, T, K, N, taps);
  VQA_ARG(workspace && ws_bytes >= need, "seqlin_wgrad: workspace %zu < %zu", ws_bytes, need);
  int seg_rows, segs;
  wgrad_plan(nseq, T, seg_rows, segs);
  SeqWgArgs a{x, dy, (float*)workspace, ldx, lddy, nseq, T, K, N, taps, seg_rows, segs};
  const int ppw = (taps * K / 16 + 3) / 4;
  const void* fn = dtype == VQA_BF16 ? wgrad_fn<bf16>(ppw, N) : wgrad_fn<float>(ppw, N);
  const size_t lds = wgrad_lds(K, N, taps, esz);
  if (int rc = set_lds_attr(fn, lds)) return rc;
  void* args[] = {&a};
  (void)hipLaunchKernel(fn, dim3(nseq * segs), dim3(256), args, lds, (hipStream_t)stream);
  VQA_LAUNCHED("seqlin_wgrad_kernel");
  const int E = taps * K * N + N;
  const vqa_partials_desc d{(const float*)workspace, dw, db, nseq * segs, E, taps * K * N, 0};
  if (desc) {
    *desc = d;
    return VQA_OK;
  }
  return vqa_reduce_partials(&d, 1, stream);
}

extern "C" int vqa_prior_embed_fwd(const float* table, const float* pos, const int64_t* tokens, const float* ycond,
                                   const void* xcond, void* out, int N, int T, int W, int bins, float scale, float rate,
                                   uint64_t seed, int64_t elem_offset, const int64_t* counter, int dtype,
                                   vqa_stream_t stream) {
  VQA_ARG(table && pos && tokens && out && N > 0 && T > 0 && W > 0 && W % 4 == 0 && bins > 0 && rate >= 0.f &&
              rate < 1.f && elem_offset >= 0, "prior_embed_fwd: bad arguments");
  VQA_ARG(pr_dt(dtype), "prior_embed_fwd: unknown dtype %d", dtype);
  EmbArgs a{table, pos, tokens, ycond, xcond, out, (long long)N * T, T, W, bins, scale, rate, seed, counter,
            (long long)elem_offset};
  const unsigned g = pr_grid(a.rows * (W / 4));
  if (dtype == VQA_BF16) hipLaunchKernelGGL(prior_embed_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(prior_embed_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, a);
  VQA_LAUNCHED("prior_embed_kernel");
  return VQA_OK;
}

extern "C" int vqa_colsum(const void* x, float* out, int nout, int64_t ostride, int64_t inner, int accumulate,
                          int dtype, vqa_stream_t stream) {
  VQA_ARG(x && out && nout > 0 && inner > 0 && pr_dt(dtype), "colsum: bad arguments");
  const unsigned g = pr_grid(inner);
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, out, nout,
                       (long long)ostride, (long long)inner, accumulate);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)x, out, nout,
                       (long long)ostride, (long long)inner, accumulate);
  VQA_LAUNCHED("colsum_kernel");
  return VQA_OK;
}

extern "C" int vqa_axpy(const void* x, const void* y, void* z, int64_t n, int dtype, vqa_stream_t stream) {
  VQA_ARG(x && y && z && n > 0 && pr_dt(dtype), "axpy: bad arguments");
  const unsigned g = pr_grid((n + 3) / 4);
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(axpy_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (const bf16*)y,
                       (bf16*)z, (long long)n);
  else
    hipLaunchKernelGGL(axpy_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       (const float*)y, (float*)z, (long long)n);
  VQA_LAUNCHED("axpy_kernel");
  return VQA_OK;
}

extern "C" int vqa_dropout(void* x, int64_t n, float rate, uint64_t seed, uint64_t salt, int64_t elem_offset,
                           const int64_t* counter, int dtype, vqa_stream_t stream) {
  VQA_ARG(x && n > 0 && rate >= 0.f && rate < 1.f && elem_offset >= 0 && pr_dt(dtype), "dropout: bad arguments");
  if (rate == 0.f) return VQA_OK;
  const unsigned g = pr_grid(n);
  if (dtype == VQA_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, (bf16*)x, (long long)n, rate,
                       (unsigned long long)seed, (unsigned long long)salt, (long long)elem_offset, counter);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, (float*)x, (long long)n,
                       rate, (unsigned long long)seed, (unsigned long long)salt, (long long)elem_offset, counter);
  VQA_LAUNCHED("dropout_kernel");
  return VQA_OK;
}

extern "C" int vqa_scale_f32(float* x, int64_t n, float s, vqa_stream_t stream) {
  VQA_ARG(x && n > 0, "scale_f32: bad arguments");
  hipLaunchKernelGGL(scale_f32_kernel, dim3(pr_grid(n)), dim3(256), 0, (hipStream_t)stream, x, (long long)n, s);
  VQA_LAUNCHED("scale_f32_kernel");
  return VQA_OK;
}

extern "C" int vqa_tf_mix(const int64_t* codes, const int64_t* amax, const uint8_t* mask, int64_t* out, int N, int T,
                          int64_t start, float rate, uint64_t seed, uint64_t step, int64_t row_offset,
                          const int64_t* counter, vqa_stream_t stream) {
  VQA_ARG(codes && out && N > 0 && T > 0 && (!mask || amax), "tf_mix: bad arguments");
  const long long rows = (long long)N * T;
  hipLaunchKernelGGL(tf_mix_kernel, dim3(pr_grid(rows)), dim3(256), 0, (hipStream_t)stream, codes, amax, mask, out,
                     rows, T, start, rate, (unsigned long long)seed, (unsigned long long)step, (long long)row_offset, counter);
  VQA_LAUNCHED("tf_mix_kernel");
  return VQA_OK;
}

template <class T>
static int launch_attn(bool fwd, int mode, const AttnArgs& a, hipStream_t s) {
  const int nb = a.T / a.l;
  if (mode == 1) {
    const unsigned g = pr_grid((long long)a.N * a.l * a.H, 256, 1 << 30);
#define VQA_COL(NB)                                                                                         \
  case NB:                                                                                                  \
    if (fwd) hipLaunchKernelGGL((attn_col_fwd_kernel<T, NB>), dim3(g), dim3(256), 0, s, a);                 \
    else hipLaunchKernelGGL((attn_col_bwd_kernel<T, NB>), dim3(g), dim3(256), 0, s, a);                     \
    break;
    switch (nb) {
      VQA_COL(1) VQA_COL(2) VQA_COL(3) VQA_COL(4) VQA_COL(5) VQA_COL(6) VQA_COL(7) VQA_COL(8)
      default: set_error("attn: column attention supports 1..8 blocks (got %d)", nb); return VQA_E_UNSUPPORTED;
    }
#undef VQA_COL
    VQA_LAUNCHED("attn_col_kernel");
    return VQA_OK;
  }
  const dim3 grid(a.T / 64, a.H, a.N);
  if (fwd) {
    if (mode == 0) hipLaunchKernelGGL((attn_fwd_kernel<T, 0>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<T, 2>), grid, dim3(256), 0, s, a);
    VQA_LAUNCHED("attn_fwd_kernel");
  } else {
    if (mode == 0) {
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, 0>), grid, dim3(256), 0, s, a);
      hipLaunchKernelGGL((attn_bwd_kv_kernel<T, 0>), grid, dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((attn_bwd_q_kernel<T, 2>), grid, dim3(256), 0, s, a);
      hipLaunchKernelGGL((attn_bwd_kv_kernel<T, 2>), grid, dim3(256), 0, s, a);
    }
    VQA_LAUNCHED("attn_bwd_kernel");
  }
  return VQA_OK;
}

static int attn_check(int N, int T, int H, int head_dim, int l, int mode) {
  VQA_ARG(N > 0 && T > 0 && H > 0 && l > 0 && T % l == 0 && mode >= 0 && mode <= 2, "attn: bad shape");
  VQA_REQUIRE(head_dim == AHD, VQA_E_UNSUPPORTED, "attn: head_dim %d unsupported (16)", head_dim);
  VQA_REQUIRE(mode == 1 || l % 64 == 0, VQA_E_UNSUPPORTED, "attn: block length %d not a multiple of 64", l);
  return VQA_OK;
}

extern "C" int vqa_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const float* vbias, int N,
                            int T, int H, int head_dim, int l, int mode, float scale, int dtype, vqa_stream_t stream) {
  VQA_ARG(q && k && v && o && lse && pr_dt(dtype) && (mode != 2 || vbias), "attn_fwd: bad arguments");
  if (int rc = attn_check(N, T, H, head_dim, l, mode)) return rc;
  AttnArgs a{q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, vbias, N, T, H, l, scale};
  hipStream_t s = (hipStream_t)stream;
  return dtype == VQA_BF16 ? launch_attn<bf16>(true, mode, a, s) : launch_attn<float>(true, mode, a, s);
}

extern "C" int vqa_attn_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse,
                            const void* dout, float* dsum, void* dq, void* dk, void* dv, int N, int T, int H,
                            int head_dim, int l, int mode, float scale, int dtype, vqa_stream_t stream) {
  VQA_ARG(q && k && v && o && lse && dout && dq && dk && dv && pr_dt(dtype) && (mode == 1 || dsum),
          "attn_bwd: bad arguments");
  if (int rc = attn_check(N, T, H, head_dim, l, mode)) return rc;
  AttnArgs a{q, k, v, (void*)o, (float*)lse, dout, dsum, dq, dk, dv, nullptr, N, T, H, l, scale};
  hipStream_t s = (hipStream_t)stream;
  return dtype == VQA_BF16 ? launch_attn<bf16>(false, mode, a, s) : launch_attn<float>(false, mode, a, s);
}

extern "C" int vqa_head_wt(const float* w, void* wt, int K, int V, int dtype, vqa_stream_t stream) {
  VQA_ARG(w && wt && K == HK && V > 0 && pr_dt(dtype), "head_wt: bad arguments (K must be %d)", HK);
  const unsigned g = pr_grid((long long)K * V);
  if (dtype == VQA_BF16) hipLaunchKernelGGL(head_wt_kernel<bf16>, dim3(g), dim3(256), 0, (hipStream_t)stream, w, (bf16*)wt, V);
  else hipLaunchKernelGGL(head_wt_kernel<float>, dim3(g), dim3(256), 0, (hipStream_t)stream, w, (float*)wt, V);
  VQA_LAUNCHED("head_wt_kernel");
  return VQA_OK;
}

template <class T>
static int launch_head(int which, const HeadArgs& a, unsigned grid, size_t lds, hipStream_t s) {
  const void* fn = which == 0 ? (const void*)head_fwd_kernel<T>
                              : which == 1 ? (const void*)head_bwd_dx_kernel<T> : (const void*)head_bwd_dw_kernel<T>;
  if (int rc = set_lds_attr(fn, lds)) return rc;
  HeadArgs c = a;
  void* args[] = {&c};
  (void)hipLaunchKernel(fn, dim3(grid), dim3(256), args, lds, s);
  VQA_LAUNCHED("head_kernel");
  return VQA_OK;
}

extern "C" int vqa_head_fwd(const void* x, const void* wt, const float* bias, const int64_t* targets, float* lse,
                            int64_t* amax, float* loss_row, float* correct, int64_t M, int K, int V, int dtype,
                            vqa_stream_t stream) {
  VQA_ARG(x && wt && bias && lse && M > 0 && K == HK && V > 0 && pr_dt(dtype), "head_fwd: bad arguments");
  VQA_ARG(!(loss_row || correct) || targets, "head_fwd: loss / correctness need targets");
  HeadArgs a{x, wt, bias, targets, lse, amax, loss_row, correct, nullptr, nullptr, (long long)M, V, 0, 0.f};
  const int esz = dtype == VQA_BF16 ? 2 : 4, S = HK + 16 / esz;
  const size_t lds = (size_t)(128 + 64) * S * esz;
  const unsigned g = (unsigned)((M + 127) / 128);
  hipStream_t s = (hipStream_t)stream;
  return dtype == VQA_BF16 ? launch_head<bf16>(0, a, g, lds, s) : launch_head<float>(0, a, g, lds, s);
}

static int head_segs(int64_t M, int V) {
  const int nvt = (V + 63) / 64;
  const long long want = std::max<long long>(1, (long long)2 * pr_cus() / nvt);
  return (int)std::min<long long>(want, (M + 63) / 64);
}

extern "C" size_t vqa_head_bwd_workspace(int64_t M, int K, int V) {
  if (M < 1 || K < 1 || V < 1) return 0;
  return (size_t)head_segs(M, V) * ((size_t)K * V + V) * sizeof(float);
}

extern "C" int vqa_head_bwd(const void* x, const void* wt, const float* bias, const int64_t* targets, const float* lse,
                            float inv_count, void* dx, float* dw, float* db, int64_t M, int K, int V, int dtype,
                            void* workspace, size_t ws_bytes, vqa_partials_desc* desc, vqa_stream_t stream) {
  VQA_ARG(x && wt && bias && targets && lse && dx && dw && db && M > 0 && K == HK && V > 0 && pr_dt(dtype),
          "head_bwd: bad arguments");
  const size_t need = vqa_head_bwd_workspace(M, K, V);
  VQA_ARG(workspace && ws_bytes >= need, "head_bwd: workspace %zu < %zu", ws_bytes, need);
  const int segs = head_segs(M, V), nvt = (V + 63) / 64;
  const long long seg_rows = ((M + segs - 1) / segs + 63) / 64 * 64;
  HeadArgs a{x, wt, bias, targets, (float*)lse, nullptr, nullptr, nullptr, dx, (float*)workspace, (long long)M, V,
             (int)seg_rows, inv_count};
  const int esz = dtype == VQA_BF16 ? 2 : 4, S = HK + 16 / esz;
  hipStream_t s = (hipStream_t)stream;
  int rc = dtype == VQA_BF16 ? launch_head<bf16>(1, a, (unsigned)((M + 127) / 128), (size_t)(128 + 64) * S * esz, s)
                             : launch_head<float>(1, a, (unsigned)((M + 127) / 128), (size_t)(128 + 64) * S * esz, s);
  if (rc) return rc;
  const int nseg = (int)((M + seg_rows - 1) / seg_rows);
  rc = dtype == VQA_BF16 ? launch_head<bf16>(2, a, (unsigned)(nseg * nvt), (size_t)128 * S * esz, s)
                         : launch_head<float>(2, a, (unsigned)(nseg * nvt), (size_t)128 * S * esz, s);
  if (rc) return rc;
  const vqa_partials_desc d{(const float*)workspace, dw, db, nseg, K * V + V, K * V, 0};
  if (desc) {
    *desc = d;
    return VQA_OK;
  }
  return vqa_reduce_partials(&d, 1, stream);
}

extern "C" size_t vqa_rowsum_workspace(int64_t rows, int64_t n) {
  if (rows < 1 || n < 1) return 0;
  return (size_t)rows * ((n + kRowsumChunk - 1) / kRowsumChunk) * sizeof(float);
}

extern "C" int vqa_rowsum(const float* x, int64_t rows, int64_t n, float scale, float* out, void* workspace,
                          size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(x && out && rows > 0 && n > 0 && rows < (1 << 20), "rowsum: bad arguments");
  VQA_ARG(workspace && ws_bytes >= vqa_rowsum_workspace(rows, n), "rowsum: workspace too small");
  const int nch = (int)((n + kRowsumChunk - 1) / kRowsumChunk);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(rowsum_part_kernel, dim3((unsigned)(rows * nch)), dim3(256), 0, s, x, (long long)n, nch,
                     (float*)workspace);
  hipLaunchKernelGGL(rowsum_final_kernel, dim3((unsigned)rows), dim3(256), 0, s, (const float*)workspace, nch, scale,
                     out);
  VQA_LAUNCHED("rowsum_kernel");
  return VQA_OK;
}

constexpr size_t kDecComposed = (size_t)3 * kDecW * 3 * kDecAW + 3 * kDecAW + kDecAW * kDecW + kDecW;  // floats/layer

extern "C" size_t vqa_prior_decode_cache_bytes(int N, int depth, int ctx) {
  if (N < 1 || depth < 1 || ctx < 1) return 0;
  return ((size_t)2 * N * depth * ctx * kDecAW + (size_t)depth * kDecComposed) * sizeof(float);
}

extern "C" int vqa_prior_decode(const vqa_prior_layer* layers, int depth, const float* x_embedding,
                                const float* pos_embedding, const float* out_kernel, const float* out_bias,
                                const float* ycond, const float* xcond, const int64_t* forced, float* logits,
                                int64_t* tokens, void* cache, size_t cache_bytes, int N, int steps, int ctx, int width,
                                int heads, int blocks, int bins, int out_ld, int64_t start, uint64_t seed,
                                vqa_stream_t stream) {
  VQA_ARG(layers && x_embedding && pos_embedding && out_kernel && out_bias && tokens && cache && N > 0 && steps > 0 &&
              steps <= ctx && blocks > 0 && ctx % blocks == 0 && bins > 0 && out_ld >= bins && out_ld % 4 == 0 &&
              out_ld <= 2048,
          "prior_decode: bad arguments (bins %d, out_ld %d)", bins, out_ld);
  VQA_REQUIRE(depth > 0 && depth <= kDecMaxLayers && width == kDecW && heads > 0 && kDecAW % heads == 0 &&
                  kDecAW / heads <= 32 && ctx / blocks <= kDecMaxL && heads <= 4,
              VQA_E_UNSUPPORTED, "prior_decode: depth %d width %d heads %d block %d unsupported", depth, width, heads,
              ctx / blocks);
  VQA_ARG(cache_bytes >= vqa_prior_decode_cache_bytes(N, depth, ctx), "prior_decode: cache too small");
  DecArgs a;
  float* comp = (float*)cache + (size_t)2 * N * depth * ctx * kDecAW;
  for (int L = 0; L < depth; ++L) {
    const vqa_prior_layer& s = layers[L];
    VQA_ARG(s.attn_type >= 0 && s.attn_type <= 2, "prior_decode: layer %d attention type %d", L, s.attn_type);
    float* c = comp + (size_t)L * kDecComposed;
    a.L[L] = DecLayer{s.ln1_gamma, s.ln1_beta, s.qkv_kernel, s.qkv_bias, s.query_kernel, s.query_bias, s.key_kernel,
                      s.key_bias, s.value_kernel, s.value_bias, s.out_kernel, s.out_bias, s.proj_kernel, s.proj_bias,
                      s.ln2_gamma, s.ln2_beta, s.mlp_kernel, s.mlp_bias, s.attn_type,
                      c, c + 3 * kDecW * 3 * kDecAW, c + 3 * kDecW * 3 * kDecAW + 3 * kDecAW,
                      c + 3 * kDecW * 3 * kDecAW + 3 * kDecAW + kDecAW * kDecW};
  }
  a.emb = x_embedding; a.pos = pos_embedding; a.hw = out_kernel; a.hb = out_bias;
  a.ycond = ycond; a.xcond = xcond; a.forced = forced; a.logits = logits; a.tokens = tokens;
  a.kc = (float*)cache;
  a.vc = (float*)cache + (size_t)N * depth * ctx * kDecAW;
  a.N = N; a.steps = steps; a.T = ctx; a.depth = depth; a.H = heads; a.l = ctx / blocks; a.bins = bins; a.ldo = out_ld;
  a.start = start; a.seed = seed;
  a.scale = 1.0f / sqrtf((float)(kDecAW / heads));
  a.emb_scale = sqrtf((float)width);
  a.eps = 1e-6f;
  hipLaunchKernelGGL(prior_decode_prep_kernel, dim3(64, depth), dim3(256), 0, (hipStream_t)stream, a);
  VQA_LAUNCHED("prior_decode_prep_kernel");
  hipLaunchKernelGGL(prior_decode_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, a);
  VQA_LAUNCHED("prior_decode_kernel");
  return VQA_OK;
}
