// vqa_spectral.hip — multi-resolution spectral loss and its gradient (gfx950).
//
// Replaces the reference's per-level
//   data_utils.py:25-30  spectral(x) = |tf.signal.stft(x, frame_length=win, frame_step=hop, fft_length=n_fft)|
//   data_utils.py:33-40  norm(x)     = tf.norm(x, 'fro', axis=[-2, -1])
//   vqvae.py:309-326     _multispectral_loss = mean_b mean_res norm(S_x - S_r) / norm(S_x)
// and the GradientTape backward of that expression w.r.t. the reconstruction (vqvae.py:143).
//
// A workgroup holds 256/TPF STFT frames at a time (TPF = N/4 threads per frame, at most 256), persistent
// over the frames: the windowed target and reconstruction frames are transformed by an in-LDS radix-4
// Stockham FFT (fp32; twiddles and window evaluated once per call in fp64 by spec_tables_kernel), the
// per-bin magnitudes |X_k|, |R_k| give the frame's partial sums sum (|X|-|R|)^2 and sum |X|^2, and — for the
// gradient — the bin gradient G_k = (|R_k| - |X_k|) R_k / |R_k| (0 where |R_k| = 0, TF's abs'(0)) is mapped
// back to the time domain by the adjoint of the one-sided rfft (an inverse FFT of the Hermitian extension
// of G), windowed, and written unscaled per frame. The per-item scale 1 / (nres * B * ||S_x - S_r|| *
// ||S_x||) is known only after every frame of the item is done, so a second kernel reduces the partial sums
// per (item, resolution) and a third overlap-adds the frame gradients (fixed summation order:
// deterministic) and applies the scales. No atomics, no host sync, graph-capturable.
#include "vqa_common.h"
#include <utility>
#include <algorithm>

namespace vqa {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// complex product with fused multiply-adds (4 VALU instead of 6; one rounding less per component)
__device__ __forceinline__ f32x2 cmul(f32x2 a, f32x2 b) {
  return f32x2{__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x)};
}
__device__ __forceinline__ f32x2 conj2(f32x2 a) { return f32x2{a.x, -a.y}; }
__device__ __forceinline__ float cabs2(f32x2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
// |z| by the hardware square root (v_sqrt_f32, 1 ulp; the pair kernels): the correctly rounded sqrtf expands to a
// scaling sequence (class test, selects, two multiplies) per value
__device__ __forceinline__ float cabs_hw(f32x2 a) { return __builtin_amdgcn_sqrtf(a.x * a.x + a.y * a.y); }

// Mixed-radix Stockham FFT in LDS: radix-8 stages while 8 divides the remaining length, then one radix-4 or
// radix-2 stage (2048 = 8.8.8.4, 1024 = 8.8.8.2, 512 = 8.8.8: 4 / 4 / 3 passes through LDS instead of the
// 6 / 5 / 5 of radix 4). Buffers are PADDED: element i lives at pidx(i) = i + i/8, which makes the stride-8
// writes of the first stage (and the 64-element jumps of the second) bank-conflict-free.
// tw[k] = exp(-2 pi i k / N) (conjugated for the inverse); TPF threads (local id lt) work on one frame.
__device__ __forceinline__ int pidx(int i) { return i + (i >> 3); }
template <int N> constexpr int fpad() { return N + N / 8; }  // padded buffer length (elements)

// y[q + S*(8p + k)] = tw^(k p S) * DFT8_k(x[q + S*(p + r m)], r = 0..7)
template <int N, int S, bool INV, int TPF>
__device__ __forceinline__ void fft_stage8(const f32x2* x, f32x2* y, const f32x2* tw, int lt) {
  constexpr int n = N / S, m = n / 8;
  constexpr float R2 = 0.70710678118654752f;
  for (int j = lt; j < N / 8; j += TPF) {
    const int p = j / S, q = j % S;
    f32x2 a[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) a[r] = x[pidx(q + S * (p + r * m))];
    // layer 1 (span 4): u = a_r + a_{r+4}, v = (a_r - a_{r+4}) w8^r
    f32x2 u[4], v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      u[r] = a[r] + a[r + 4];
      v[r] = a[r] - a[r + 4];
    }
    // w8^1 = (1 -+ i)/sqrt2, w8^2 = -+ i, w8^3 = (-1 -+ i)/sqrt2 (forward / inverse)
    if (INV) {
      v[1] = f32x2{R2 * (v[1].x - v[1].y), R2 * (v[1].x + v[1].y)};
      v[2] = f32x2{-v[2].y, v[2].x};
      v[3] = f32x2{-R2 * (v[3].x + v[3].y), R2 * (v[3].x - v[3].y)};
    } else {
      v[1] = f32x2{R2 * (v[1].x + v[1].y), R2 * (v[1].y - v[1].x)};
      v[2] = f32x2{v[2].y, -v[2].x};
      v[3] = f32x2{R2 * (v[3].y - v[3].x), -R2 * (v[3].x + v[3].y)};
    }
    // two 4-point DFTs: X[2k'] from u, X[2k'+1] from v
    f32x2 X[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x2* w = h ? v : u;
      const f32x2 b0 = w[0] + w[2], b1 = w[0] - w[2], b2 = w[1] + w[3], d = w[1] - w[3];
      const f32x2 jd = INV ? f32x2{-d.y, d.x} : f32x2{d.y, -d.x};
      X[h] = b0 + b2;
      X[2 + h] = b1 + jd;
      X[4 + h] = b0 - b2;
      X[6 + h] = b1 - jd;
    }
    y[pidx(q + S * (8 * p))] = X[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      f32x2 w = tw[k * p * S];
      if (INV) w = conj2(w);
      y[pidx(q + S * (8 * p + k))] = cmul(X[k], w);
    }
  }
}

// radix-4 stage (the last one when the remaining length is 4)
template <int N, int S, bool INV, int TPF>
__device__ __forceinline__ void fft_stage4(const f32x2* x, f32x2* y, const f32x2* tw, int lt) {
  constexpr int n = N / S, m = n / 4;
  for (int j = lt; j < N / 4; j += TPF) {
    const int p = j / S, q = j % S;
    const f32x2 a0 = x[pidx(q + S * p)], a1 = x[pidx(q + S * (p + m))], a2 = x[pidx(q + S * (p + 2 * m))],
                a3 = x[pidx(q + S * (p + 3 * m))];
    f32x2 w1 = tw[p * S], w2 = tw[2 * p * S], w3 = tw[3 * p * S];
    if (INV) {
      w1 = conj2(w1);
      w2 = conj2(w2);
      w3 = conj2(w3);
    }
    const f32x2 b0 = a0 + a2, b1 = a0 - a2, b2 = a1 + a3, d = a1 - a3;
    const f32x2 jd = INV ? f32x2{-d.y, d.x} : f32x2{d.y, -d.x};  // +i d (inverse) / -i d (forward)
    y[pidx(q + S * (4 * p))] = b0 + b2;
    y[pidx(q + S * (4 * p + 1))] = cmul(b1 + jd, w1);
    y[pidx(q + S * (4 * p + 2))] = cmul(b0 - b2, w2);
    y[pidx(q + S * (4 * p + 3))] = cmul(b1 - jd, w3);
  }
}

// the last stage when the remaining length is 2: n = 2, S = N/2
template <int N, int TPF>
__device__ __forceinline__ void fft_stage2(const f32x2* x, f32x2* y, int lt) {
  for (int q = lt; q < N / 2; q += TPF) {
    const f32x2 a = x[pidx(q)], b = x[pidx(q + N / 2)];
    y[pidx(q)] = a + b;
    y[pidx(q + N / 2)] = a - b;
  }
}

template <int N, int S, bool INV, int TPF>
__device__ __forceinline__ void fft_rec(f32x2* x, f32x2* y, const f32x2* tw, int lt) {
  constexpr int n = N / S;
  if constexpr (n >= 8) {
    fft_stage8<N, S, INV, TPF>(x, y, tw, lt);
    __syncthreads();
    fft_rec<N, S * 8, INV, TPF>(y, x, tw, lt);
  } else if constexpr (n == 4) {
    fft_stage4<N, S, INV, TPF>(x, y, tw, lt);
    __syncthreads();
  } else if constexpr (n == 2) {
    fft_stage2<N, TPF>(x, y, lt);
    __syncthreads();
  }
}

template <int N> constexpr int fft_stages() {
  int s = 0, n = N;
  while (n >= 8) {
    n /= 8;
    ++s;
  }
  return s + (n > 1 ? 1 : 0);
}

// In-place (logically) N-point FFT of a[] in LDS (padded layout); b[] is scratch. All frame slots of the
// workgroup run in lockstep (workgroup barriers). Returns the buffer holding the result (natural order,
// padded). Unnormalised in both directions. Caller syncs before (a written) — ends with a sync.
template <int N, bool INV, int TPF>
__device__ __forceinline__ f32x2* fft(f32x2* a, f32x2* b, const f32x2* tw, int lt) {
  fft_rec<N, 1, INV, TPF>(a, b, tw, lt);
  return (fft_stages<N>() & 1) ? b : a;
}

constexpr int SPEC_MAX_RES = 8;

// |STFT| of a signal (vqa_stft_magnitude: no workspace, so the twiddles and window are evaluated in the
// kernel when tw is null)
struct SpecFrameArgs {
  const float* x;   // signal (B, T) fp32
  float* mag;       // |X| (B*F, N/2+1)
  const float* tw;  // N twiddles (re, im) from spec_tables_kernel, or null: evaluated in the kernel
  const float* wn;  // periodic Hann window of length win (null with tw)
  int B, T, F, hop, win;
};

// threads per frame: N/8 butterflies per radix-8 stage, at most the whole workgroup
template <int N> constexpr int spec_tpf() { return N / 8 < 256 ? N / 8 : 256; }

template <int N>
__global__ __launch_bounds__(256) void spec_frame_kernel(SpecFrameArgs a) {
  constexpr int TPF = spec_tpf<N>(), FPI = 256 / TPF;  // frame slots per workgroup
  constexpr int KB = N / 2 + 1, NB = (KB + TPF - 1) / TPF;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x2* tw = (f32x2*)smem;
  float* wn = (float*)(tw + N);
  f32x2* slots = (f32x2*)(wn + ((a.win + 3) & ~3));
  const int tid = threadIdx.x, sl = tid / TPF, lt = tid - sl * TPF;
  f32x2* buf0 = slots + (size_t)sl * 2 * fpad<N>();
  f32x2* buf1 = buf0 + fpad<N>();

  if (a.tw) {
    for (int e = tid; e < N / 2; e += 256) ((float4*)tw)[e] = ((const float4*)a.tw)[e];
    for (int e = tid; e < a.win; e += 256) wn[e] = a.wn[e];
  } else {
    for (int k = tid; k < N; k += 256) {
      double sn, cs;
      sincospi(2.0 * (double)k / (double)N, &sn, &cs);
      tw[k] = f32x2{(float)cs, (float)-sn};
    }
    for (int n = tid; n < a.win; n += 256) wn[n] = (float)(0.5 - 0.5 * cospi(2.0 * (double)n / (double)a.win));
  }
  __syncthreads();

  const int nframes = a.B * a.F;
  constexpr int NL = N / TPF;
  float xv[NL];
  auto load_frame = [&](int f0_) {
    const int fc = min(f0_ + sl, nframes - 1);  // an idle slot recomputes a valid frame and stores nothing
    const int bb = fc / a.F, f = fc - bb * a.F;
    const size_t off = (size_t)bb * a.T + (size_t)f * a.hop;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int n = lt + i * TPF;
      xv[i] = a.x[off + (n < a.win ? n : 0)];
    }
  };
  if (blockIdx.x * FPI < nframes) load_frame(blockIdx.x * FPI);
  for (int f0 = blockIdx.x * FPI; f0 < nframes; f0 += gridDim.x * FPI) {
    const int fi = f0 + sl;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int n = lt + i * TPF;
      buf0[pidx(n)] = n < a.win ? f32x2{xv[i] * wn[n], 0.f} : f32x2{0.f, 0.f};
    }
    if (f0 + gridDim.x * FPI < nframes) load_frame(f0 + gridDim.x * FPI);  // lands during this frame's FFT
    __syncthreads();
    const f32x2* X = fft<N, false, TPF>(buf0, buf1, tw, lt);
    if (fi < nframes) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int k = lt + TPF * j;
        if (k < KB) a.mag[(size_t)fi * KB + k] = cabs2(X[pidx(k)]);
      }
    }
    __syncthreads();
  }
}

// Frames in PAIRS (a, b): ONE complex FFT of z = w*s_a + i w*s_b gives both real frames' spectra
// (S_a[k] = (Z[k] + conj Z[N-k]) / 2, S_b[k] = (Z[k] - conj Z[N-k]) / 2i). MAG writes |S| (the target's
// spectrograms, once per step); LOSS / GRAD compare |S| of the reconstruction against the precomputed
// target magnitudes and GRAD runs ONE inverse FFT of H_a + i H_b (both adjoint outputs are real, so
// y_a = Re, y_b = Im). One FFT per frame (two with the gradient) instead of the three of a direct form.
//
// ONE WAVE PER FRAME PAIR (no workgroup barrier after the table load): each wave owns an LDS buffer of N
// complex values and runs the Stockham FFT in it with register-resident radix-16 / 8 / 4 / 2 butterflies
// (2048 = 16.16.8, 1024 = 16.16.4, 512 = 8.8.8, 256 = 16.16: three passes instead of the four to six of a
// radix-8 / radix-4 plan). A pass loads every input of the lane's butterflies before it stores an output, and
// all lanes of a wave execute each LDS instruction together (in order), so the passes run IN PLACE in one
// buffer with no barrier between them. The first forward pass reads the windowed samples straight from HBM
// (lane j of butterfly j takes samples j + r N/R: coalesced), the last inverse pass writes the windowed frame
// gradients straight to HBM (samples q + S k: coalesced); the next pair's samples and target magnitudes are
// prefetched into registers while the current pair is transformed.
enum { PAIR_LOSS = 0, PAIR_GRAD = 1, PAIR_MAG = 2 };
struct SpecPairArgs {
  const float* r;   // signal (B, T) fp32: reconstruction (LOSS, GRAD) or target (MAG)
  const float* tm;  // LOSS / GRAD: target magnitudes (B*F, N/2+1)
  float* out;       // GRAD: unscaled frame gradients (B*F, win); MAG: magnitudes (B*F, N/2+1)
  float* part;      // LOSS / GRAD: per-frame (sum (|X|-|R|)^2, sum |X|^2)
  const float* tw;  // N twiddles (re, im)
  const float* wn;  // window
  int B, T, F, hop, win;
};

// cos / sin (2 pi e / 16), e = 0..15 (the radix-16 butterfly's internal twiddles)
__device__ constexpr float kC16[16] = {1.f, 0.92387953251128676f, 0.70710678118654752f, 0.38268343236508977f, 0.f,
                                       -0.38268343236508977f, -0.70710678118654752f, -0.92387953251128676f, -1.f,
                                       -0.92387953251128676f, -0.70710678118654752f, -0.38268343236508977f, 0.f,
                                       0.38268343236508977f, 0.70710678118654752f, 0.92387953251128676f};
template <int E, bool INV> __device__ __forceinline__ f32x2 w16mul(f32x2 a) {
  constexpr int e = E & 15;
  if constexpr (e == 0) return a;
  else if constexpr (e == 4) return INV ? f32x2{-a.y, a.x} : f32x2{a.y, -a.x};  // +-i
  else if constexpr (e == 8) return f32x2{-a.x, -a.y};
  else if constexpr (e == 12) return INV ? f32x2{a.y, -a.x} : f32x2{-a.y, a.x};
  else {
    const float c = kC16[e], sn = kC16[(e + 12) & 15];  // sin(2 pi e/16) = cos(2 pi (e - 4)/16)
    const f32x2 w = INV ? f32x2{c, sn} : f32x2{c, -sn};
    return cmul(a, w);
  }
}

// X[k] = sum_r a[r] W_R^{rk} in place (W_R = exp(-+2 pi i / R)), natural order
template <bool INV> __device__ __forceinline__ void dft4(f32x2& a0, f32x2& a1, f32x2& a2, f32x2& a3) {
  const f32x2 b0 = a0 + a2, b1 = a0 - a2, b2 = a1 + a3, d = a1 - a3;
  const f32x2 jd = INV ? f32x2{-d.y, d.x} : f32x2{d.y, -d.x};
  a0 = b0 + b2;
  a1 = b1 + jd;
  a2 = b0 - b2;
  a3 = b1 - jd;
}
template <int R, bool INV> __device__ __forceinline__ void dft(f32x2 (&a)[R]) {
  if constexpr (R == 2) {
    const f32x2 t = a[0] - a[1];
    a[0] = a[0] + a[1];
    a[1] = t;
  } else if constexpr (R == 4) {
    dft4<INV>(a[0], a[1], a[2], a[3]);
  } else if constexpr (R == 8) {
    // r = r1 + 2 r2 (r1 < 2, r2 < 4): 4-point DFTs over r2, W8^{r1 k2}, 2-point DFTs over r1
    dft4<INV>(a[0], a[2], a[4], a[6]);
    dft4<INV>(a[1], a[3], a[5], a[7]);
    a[3] = w16mul<2, INV>(a[3]);
    a[5] = w16mul<4, INV>(a[5]);
    a[7] = w16mul<6, INV>(a[7]);
    f32x2 o[8];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      o[k2] = a[2 * k2] + a[2 * k2 + 1];
      o[k2 + 4] = a[2 * k2] - a[2 * k2 + 1];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = o[k];
  } else if constexpr (R == 16) {
    // r = r1 + 4 r2: 4-point DFTs over r2 (B[r1][k2] lands in a[r1 + 4 k2]), W16^{r1 k2}, 4-point DFTs over r1
#pragma unroll
    for (int r1 = 0; r1 < 4; ++r1) dft4<INV>(a[r1], a[r1 + 4], a[r1 + 8], a[r1 + 12]);
    a[5] = w16mul<1, INV>(a[5]);
    a[9] = w16mul<2, INV>(a[9]);
    a[13] = w16mul<3, INV>(a[13]);
    a[6] = w16mul<2, INV>(a[6]);
    a[10] = w16mul<4, INV>(a[10]);
    a[14] = w16mul<6, INV>(a[14]);
    a[7] = w16mul<3, INV>(a[7]);
    a[11] = w16mul<6, INV>(a[11]);
    a[15] = w16mul<9, INV>(a[15]);
    f32x2 o[16];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      f32x2 c0 = a[4 * k2], c1 = a[4 * k2 + 1], c2 = a[4 * k2 + 2], c3 = a[4 * k2 + 3];
      dft4<INV>(c0, c1, c2, c3);
      o[k2] = c0;
      o[k2 + 4] = c1;
      o[k2 + 8] = c2;
      o[k2 + 12] = c3;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = o[k];
  }
}

// the radix plan of an N-point FFT: radix of pass s (0 when there is no such pass)
template <int N, int P> constexpr int wradix() {
  if constexpr (N == 2048) return P < 2 ? 16 : (P == 2 ? 8 : 0);
  else if constexpr (N == 1024) return P < 2 ? 16 : (P == 2 ? 4 : 0);
  else if constexpr (N == 512) return P < 3 ? 8 : 0;
  else return P < 2 ? 16 : 0;  // 256
}
template <int N, int P> constexpr int wstride() { return P == 0 ? 1 : wstride<N, (P > 0 ? P - 1 : 0)>() * wradix<N, (P > 0 ? P - 1 : 0)>(); }

constexpr int kSpecWaves = 4;  // waves (frame pairs in flight) per workgroup

// the pass twiddles W_N^{k e}, k < R (conjugated for the inverse), from the fp64-rounded table; VQA_SPEC_TWD:
// only k = 1, 2, 4, 8 from the table, the others one complex product away (fewer LDS reads, +1 ulp)
template <int R, bool INV> __device__ __forceinline__ void pass_twiddles(f32x2 (&w)[R], const f32x2* tw, int e) {
  w[0] = f32x2{1.f, 0.f};
#ifdef VQA_SPEC_TWD
#pragma unroll
  for (int k = 1; k < R; k <<= 1) w[k] = tw[k * e];
#pragma unroll
  for (int k = 3; k < R; ++k)
    if (k & (k - 1)) w[k] = cmul(w[k & -k], w[k - (k & -k)]);
#else
#pragma unroll
  for (int k = 1; k < R; ++k) w[k] = tw[k * e];
#endif
  if (INV) {
#pragma unroll
    for (int k = 1; k < R; ++k) w[k] = conj2(w[k]);
  }
}

// one Stockham pass of radix R at stride S over the wave's buffer z (in place): butterfly j = q + S p reads
// z[q + S (p + r m)] and writes z[q + S (R p + k)] = W_N^{k p S} DFT_R(...)_k. Every load of the lane precedes
// its first store (all lanes of the wave execute each LDS instruction together).
template <int N, int R, int S, bool INV>
__device__ __forceinline__ void wpass(f32x2* z, const f32x2* tw, int lane) {
  constexpr int m = N / (S * R), NBF = N / R, IT = (NBF + 63) / 64;
  f32x2 v[IT][R];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (NBF % 64 == 0 || j < NBF) {
      const int p = j / S, q = j - p * S;
#pragma unroll
      for (int r = 0; r < R; ++r) v[it][r] = z[pidx(q + S * (p + r * m))];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int j = lane + 64 * it;
    if (NBF % 64 == 0 || j < NBF) {
      const int p = j / S, q = j - p * S;
      dft<R, INV>(v[it]);
      if constexpr (m == 1) {
        // the last pass (p = 0): every twiddle is W^0
#pragma unroll
        for (int k = 0; k < R; ++k) z[pidx(q + S * k)] = v[it][k];
      } else {
        f32x2 w[R];
        pass_twiddles<R, INV>(w, tw, p * S);
#pragma unroll
        for (int k = 0; k < R; ++k) z[pidx(q + S * (R * p + k))] = k ? cmul(v[it][k], w[k]) : v[it][k];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// the target-magnitude launches (PAIR_MAG, no gradient half) at 5 / 3 waves per SIMD for N = 512 / 1024: their few
// spilled registers cost less than the third round of pairs they save (512: 25.1 -> 21.6 us, 1024: 29.3 -> 26.5 us;
// the gradient launches spill inside their passes at that occupancy and took twice as long, so they keep theirs;
// profiles/r6_spectral_occ.txt)
template <int N, int MODE> constexpr int spec_pair_min_waves() {
  return MODE == PAIR_MAG ? (N == 512 ? 5 : (N == 1024 ? 3 : 1)) : 1;
}
template <int N, int MODE>
__global__ __launch_bounds__(64 * kSpecWaves) __attribute__((amdgpu_waves_per_eu(spec_pair_min_waves<N, MODE>(), 8)))
void spec_pair_kernel(SpecPairArgs a) {
  constexpr bool GRAD = MODE == PAIR_GRAD, MAG = MODE == PAIR_MAG;
  constexpr int KB = N / 2 + 1, NB = (KB + 63) / 64;
  constexpr int R0 = wradix<N, 0>(), R1 = wradix<N, 1>(), R2 = wradix<N, 2>();
  constexpr int S1 = wstride<N, 1>(), S2 = wstride<N, 2>();
  constexpr int NBF0 = N / R0, IT0 = (NBF0 + 63) / 64, M0 = N / R0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x2* tw = (f32x2*)smem;
  float* wn = (float*)(tw + N);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  f32x2* z = (f32x2*)(wn + N) + (size_t)wave * fpad<N>();

  // twiddles, and the window zero-padded to N (the FFT's zero padding without a per-sample branch)
  for (int e = threadIdx.x; e < N / 2; e += 64 * kSpecWaves) ((float4*)tw)[e] = ((const float4*)a.tw)[e];
  for (int e = threadIdx.x; e < N; e += 64 * kSpecWaves) wn[e] = e < a.win ? a.wn[e] : 0.f;
  __syncthreads();

  const int nframes = a.B * a.F, npairs = (nframes + 1) / 2;
  const int gw = blockIdx.x * kSpecWaves + wave, nw = gridDim.x * kSpecWaves;
  // the pair's raw samples in pass-0 order (butterfly j = lane + 64 it, input r: sample j + r M0), loaded one
  // pair ahead; its target magnitudes (bin lane + 64 j) are requested when the pair starts and land during its
  // forward passes
  float ra[IT0][R0], rb[IT0][R0], ta[MAG ? 1 : NB], tb[MAG ? 1 : NB];
  auto frame_base = [&](int f) {
    const int bb_ = f / a.F;
    return a.r + (size_t)bb_ * a.T + (size_t)(f - bb_ * a.F) * a.hop;
  };
  auto load_samples = [&](int pp) {
    const float* sa = frame_base(min(2 * pp, nframes - 1));
    const float* sb = frame_base(min(2 * pp + 1, nframes - 1));
#pragma unroll
    for (int it = 0; it < IT0; ++it)
#pragma unroll
      for (int r = 0; r < R0; ++r) {
        const int n = lane + 64 * it + r * M0, nc = n < a.win ? n : 0;
        ra[it][r] = sa[nc];
        rb[it][r] = sb[nc];
      }
  };
  if (gw < npairs) load_samples(gw);
  for (int pp = gw; pp < npairs; pp += nw) {
    const int fa = 2 * pp, fb = fa + 1;
    const bool acta = fa < nframes, actb = fb < nframes;
    if constexpr (!MAG) {
      const int pa = min(fa, nframes - 1), pb = min(fb, nframes - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int k = lane + 64 * j, kc = k < KB ? k : 0;
        ta[j] = a.tm[(size_t)pa * KB + kc];
        tb[j] = a.tm[(size_t)pb * KB + kc];
      }
    }
    // pass 0 from the registers: windowed samples (n >= win: the FFT's zero padding), one butterfly at a time
#pragma unroll
    for (int it = 0; it < IT0; ++it) {
      const int p = lane + 64 * it;  // S = 1: q = 0
      if (NBF0 % 64 == 0 || p < NBF0) {
        f32x2 v[R0];
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          const float w = wn[p + r * M0];
          v[r] = f32x2{ra[it][r] * w, rb[it][r] * w};
        }
        dft<R0, false>(v);
        f32x2 w[R0];
        pass_twiddles<R0, false>(w, tw, p);
#pragma unroll
        for (int k = 0; k < R0; ++k) z[pidx(R0 * p + k)] = k ? cmul(v[k], w[k]) : v[k];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
    if (pp + nw < npairs) load_samples(pp + nw);  // lands during this pair's remaining passes
    wpass<N, R1, S1, false>(z, tw, lane);
    if constexpr (R2 > 0) wpass<N, R2, S2, false>(z, tw, lane);
    // bins: |S_a|, |S_b|, the loss partials and (GRAD) H = H_a + i H_b in place
    float sda = 0.f, sxa = 0.f, sdb = 0.f, sxb = 0.f;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int k = lane + 64 * j;
      if (k < KB) {
        // bins k and N-k are read and (GRAD) rewritten by this lane only
        const int km = (N - k) & (N - 1);
        const f32x2 zk = z[pidx(k)], zm = z[pidx(km)];
        const f32x2 rka = f32x2{0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y)};
        const f32x2 rkb = f32x2{0.5f * (zk.y + zm.y), 0.5f * (zm.x - zk.x)};
        const float mra = cabs_hw(rka), mrb = cabs_hw(rkb);
        if constexpr (MAG) {
          if (acta) a.out[(size_t)fa * KB + k] = mra;
          if (actb) a.out[(size_t)fb * KB + k] = mrb;
        } else {
          const float da = ta[j] - mra, db = tb[j] - mrb;
          sda += da * da;
          sxa += ta[j] * ta[j];
          sdb += db * db;
          sxb += tb[j] * tb[j];
          if constexpr (GRAD) {
            // dL/d(Re,Im)R_k = (|R|-|X|) R/|R| (0 at |R| = 0); H = H_a + i H_b, each the Hermitian extension of
            // G/2 (G at k = 0, N/2)
            // 1/|R| by v_rcp_f32 (1 ulp): the gradient's tolerance is 1e-4 of its max, the loss does not use it
            const float ga = mra > 0.f ? (mra - ta[j]) * __builtin_amdgcn_rcpf(mra) : 0.f;
            const float gb = mrb > 0.f ? (mrb - tb[j]) * __builtin_amdgcn_rcpf(mrb) : 0.f;
            const f32x2 Ga = f32x2{ga * rka.x, ga * rka.y}, Gb = f32x2{gb * rkb.x, gb * rkb.y};
            if (k == 0 || k == N / 2) {
              z[pidx(k)] = f32x2{Ga.x, Gb.x};
            } else {
              z[pidx(k)] = f32x2{0.5f * Ga.x - 0.5f * Gb.y, 0.5f * Ga.y + 0.5f * Gb.x};
              z[pidx(km)] = f32x2{0.5f * Ga.x + 0.5f * Gb.y, 0.5f * Gb.x - 0.5f * Ga.y};
            }
          }
        }
      }
    }
    if constexpr (!MAG) {
      sda = warp_sum(sda);
      sxa = warp_sum(sxa);
      sdb = warp_sum(sdb);
      sxb = warp_sum(sxb);
      if (lane == 0) {
        if (acta) {
          a.part[2 * (size_t)fa] = sda;
          a.part[2 * (size_t)fa + 1] = sxa;
        }
        if (actb) {
          a.part[2 * (size_t)fb] = sdb;
          a.part[2 * (size_t)fb + 1] = sxb;
        }
      }
    }
    if constexpr (GRAD) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
      // inverse FFT: passes 0 .. P-2 in LDS, the last pass straight to the frame gradients (windowed)
      constexpr int RL = R2 > 0 ? R2 : R1, SL = R2 > 0 ? S2 : S1, NBFL = N / RL, ITL = (NBFL + 63) / 64;
      wpass<N, R0, 1, true>(z, tw, lane);
      if constexpr (R2 > 0) wpass<N, R1, S1, true>(z, tw, lane);
      f32x2 v[ITL][RL];
#pragma unroll
      for (int it = 0; it < ITL; ++it) {
        const int q = lane + 64 * it;  // the last pass: m = 1, p = 0, butterfly j = q < S
        if (NBFL % 64 == 0 || q < NBFL) {
#pragma unroll
          for (int r = 0; r < RL; ++r) v[it][r] = z[pidx(q + SL * r)];
        }
      }
      float* oa = a.out + (size_t)fa * a.win;
      float* ob = a.out + (size_t)fb * a.win;
#pragma unroll
      for (int it = 0; it < ITL; ++it) {
        const int q = lane + 64 * it;
        if (NBFL % 64 == 0 || q < NBFL) {
          dft<RL, true>(v[it]);
#pragma unroll
          for (int k = 0; k < RL; ++k) {
            const int n = q + SL * k;
            if (n < a.win) {
              if (acta) oa[n] = v[it][k].x * wn[n];
              if (actb) ob[n] = v[it][k].y * wn[n];
            }
          }
        }
      }
    }
    // the next pair's pass 0 rewrites z: every read of it above precedes those stores in the wave's order
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------------------------------
// Frame pairs by a FOUR-STEP FFT held in registers (round 6; N = 512, 1024, 2048): N = P x 64, P = N / 64 points per
// lane, one wave per frame pair as above. Forward, with n = 64 n1 + n2, k = k1 + P k2:
//   lane n2 loads z[64 n1 + n2] (n1 < P), P-point DFT over n1 in registers, times W_N^{n2 k1}
//   -> ONE transpose through the wave's LDS buffer: the 64-point DFT of index k1 goes to the G = 64 / P lanes
//      (k1, g), lane g holding n2 = g + G m (m < P)
//   P-point DFT over m in registers, times W_64^{g q}, then a G-point DFT across the G lanes (radix-2 DPP stages:
//      quad_perm / half-row mirror exchanges, no LDS) -> lane (k1, g) holds Z[k1 + P (q + P bitrev(g))], q < P
//   the pair separation needs Z[N - k] beside Z[k]: ONE exchange through the LDS buffer (every lane writes its bins
//      at their natural index, reads the mirror bins)
// and the inverse (GRAD) runs the same steps backwards (cross-lane DIT, P-point DFT, W_N^{-n2 k1}, transpose,
// P-point DFT, windowed stores of the frame gradients at n = lane + 64 n1). Three passes through LDS per pair where
// the Stockham form makes five to seven, and its per-butterfly twiddle reads are replaced by one table row per
// lane (W_N^{n2 k1} laid out [k1][n2] at a padded pitch) and compile-time constants. LDS layouts (8-byte slots):
// the transpose rows have pitch 64 + G (the strided side hits 32 distinct slots per half wave) and the bin exchange
// puts bin k at k + (k / P^2) 32 / G (both the own and the mirror accesses conflict-free, tools/spec4_banks.py).
// Same loss / gradient definition and the same fp64-rounded twiddle and window tables as spec_pair_kernel.
__device__ constexpr float kC32[32] = {
    1.f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f,
    0.55557023301960229f, 0.38268343236508984f, 0.19509032201612833f, 0.f, -0.19509032201612819f,
    -0.38268343236508973f, -0.55557023301960196f, -0.70710678118654746f, -0.83146961230254535f,
    -0.92387953251128674f, -0.98078528040323043f, -1.f, -0.98078528040323043f, -0.92387953251128685f,
    -0.83146961230254546f, -0.70710678118654768f, -0.55557023301960218f, -0.38268343236509034f,
    -0.19509032201612866f, 0.f, 0.1950903220161283f, 0.38268343236509f, 0.55557023301960184f,
    0.70710678118654735f, 0.83146961230254524f, 0.92387953251128652f, 0.98078528040323032f};
template <int E, bool INV> __device__ __forceinline__ f32x2 w32mul(f32x2 a) {
  constexpr int e = E & 31;
  if constexpr ((e & 1) == 0) {
    return w16mul<e / 2, INV>(a);
  } else {
    const float c = kC32[e], sn = kC32[(e + 24) & 31];  // sin(2 pi e/32) = cos(2 pi (e - 8)/32)
    return cmul(a, INV ? f32x2{c, sn} : f32x2{c, -sn});
  }
}
template <bool INV, int... K>
__device__ __forceinline__ void dft32_combine(f32x2 (&a)[32], const f32x2 (&ev)[16], const f32x2 (&od)[16],
                                              std::integer_sequence<int, K...>) {
  ((a[K] = ev[K] + w32mul<K, INV>(od[K]), a[K + 16] = ev[K] - w32mul<K, INV>(od[K])), ...);
}
// natural-order P-point DFT in registers (P = 32: two 16-point DFTs of the even / odd inputs and one combine)
template <int P, bool INV> __device__ __forceinline__ void dftp(f32x2 (&a)[P]) {
  if constexpr (P == 32) {
    f32x2 ev[16], od[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ev[i] = a[2 * i];
      od[i] = a[2 * i + 1];
    }
    dft<16, INV>(ev);
    dft<16, INV>(od);
    dft32_combine<INV>(a, ev, od, std::make_integer_sequence<int, 16>{});
  } else {
    dft<P, INV>(a);
  }
}
// v of lane (lane ^ S) within groups of G <= 8 lanes (DPP: xor 1 / 2 by quad_perm, xor 4 by half-row mirror then
// quad reverse)
template <int S> __device__ __forceinline__ float xlane(float v) {
  if constexpr (S == 1) return xl::xor1(v);
  else if constexpr (S == 2) return xl::xor2(v);
  else return xl::dpp<0x1B>(xl::hmirror(v));
}
template <int N> struct Spec4 {
  static constexpr int P = N / 64, G = 64 / P, GB = G == 2 ? 1 : G == 4 ? 2 : 3, PITCH = 64 + G, BUF = N + 64;
  static_assert(P * PITCH <= BUF && N + 32 <= BUF, "buffer plan");
  // LDS slot of natural bin k in the exchange
  static __device__ __forceinline__ int slot(int k) { return k + (k / (P * P)) * (32 / G); }
};
__device__ __forceinline__ int bitrev_n(int g, int bits) {
  return bits == 1 ? g : bits == 2 ? (((g & 1) << 1) | (g >> 1)) : (((g & 1) << 2) | (g & 2) | (g >> 2));
}
// waves (frame pairs in flight) per workgroup, and whether the next pair's samples are prefetched into registers:
// N = 2048 runs 8 waves (two per SIMD: a lone wave issues a VALU instruction every 4 cycles, two every 2) within
// 256 VGPRs, which leaves no room for the 64-register prefetch; the smaller transforms prefetch and reach two or
// more waves per SIMD through several 4-wave workgroups per CU
template <int N> constexpr int spec4_waves() { return N == 2048 ? 8 : 4; }
template <int N> constexpr bool spec4_prefetch() { return N != 2048; }

// the G-point DFT across the lane group, forward (DIF: natural in, lane g holds output bitrev(g)) or inverse (DIT:
// bitrev in, natural out); stage twiddles W_{2s}^{g mod s} from W_64 (tw64), upper lanes only (1 for the others)
template <int N, bool INV>
__device__ __forceinline__ void xlane_dft(f32x2 (&c)[N / 64], int g, const f32x2* tw64) {
  typedef Spec4<N> S4;
  constexpr int P = S4::P, G = S4::G;
  auto stage = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    const bool up = (g & s) != 0;
    const float sg = up ? -1.f : 1.f;
    f32x2 w = f32x2{1.f, 0.f};
    if constexpr (s > 1) {
      if (up) w = tw64[(g & (s - 1)) * (32 / s)];
      if (INV) w = conj2(w);
    }
#pragma unroll
    for (int q = 0; q < P; ++q) {
      f32x2 u = c[q];
      if constexpr (INV && s > 1) u = cmul(u, w);  // DIT: the upper input twiddled before the exchange
      const f32x2 pv = f32x2{xlane<s>(u.x), xlane<s>(u.y)};
      f32x2 r = f32x2{__builtin_fmaf(sg, u.x, pv.x), __builtin_fmaf(sg, u.y, pv.y)};  // lower u + p, upper p - u
      if constexpr (!INV && s > 1) r = cmul(r, w);  // DIF: the upper output twiddled after it
      c[q] = r;
    }
  };
  if constexpr (!INV) {
    if constexpr (G >= 8) stage(std::integral_constant<int, 4>{});
    if constexpr (G >= 4) stage(std::integral_constant<int, 2>{});
    stage(std::integral_constant<int, 1>{});
  } else {
    stage(std::integral_constant<int, 1>{});
    if constexpr (G >= 4) stage(std::integral_constant<int, 2>{});
    if constexpr (G >= 8) stage(std::integral_constant<int, 4>{});
  }
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <int N, int MODE>
__global__ __launch_bounds__(64 * spec4_waves<N>()) void spec_pair4_kernel(SpecPairArgs a) {
  typedef Spec4<N> S4;
  constexpr bool GRAD = MODE == PAIR_GRAD, MAG = MODE == PAIR_MAG, PREF = spec4_prefetch<N>();
  constexpr int W = spec4_waves<N>();
  constexpr int P = S4::P, G = S4::G, PITCH = S4::PITCH, KB = N / 2 + 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x2* T = (f32x2*)smem;       // T[k1 PITCH + n2] = W_N^{n2 k1}
  f32x2* tw64 = T + P * PITCH;   // W_64^e = W_N^{e P}
  float* wn = (float*)(tw64 + 64);  // window, zero-padded to N
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  f32x2* buf = (f32x2*)(wn + N) + (size_t)wave * S4::BUF;
  const f32x2* twg = (const f32x2*)a.tw;
  for (int e = threadIdx.x; e < P * 64; e += 64 * W) {
    const int k1 = e >> 6, n2 = e & 63;
    T[k1 * PITCH + n2] = twg[n2 * k1];
  }
  for (int e = threadIdx.x; e < 64; e += 64 * W) tw64[e] = twg[e * P];
  for (int e = threadIdx.x; e < N; e += 64 * W) wn[e] = e < a.win ? a.wn[e] : 0.f;
  __syncthreads();

  const int k1s = lane / G, g = lane & (G - 1), h = bitrev_n(g, S4::GB);
  const int kbase = k1s + P * P * h;  // own bin of register q: kbase + P q
  const int nframes = a.B * a.F, npairs = (nframes + 1) / 2;
  const int gw = blockIdx.x * W + wave, nw = gridDim.x * W;
  constexpr int NB = (KB + 63) / 64;
  float ra[P], rb[P], ta[MAG ? 1 : NB], tb[MAG ? 1 : NB];
  auto frame_base = [&](int f) {
    const int bb_ = f / a.F;
    return a.r + (size_t)bb_ * a.T + (size_t)(f - bb_ * a.F) * a.hop;
  };
  auto load_samples = [&](int pp) {
    const float* sa = frame_base(min(2 * pp, nframes - 1));
    const float* sb = frame_base(min(2 * pp + 1, nframes - 1));
#pragma unroll
    for (int n1 = 0; n1 < P; ++n1) {
      const int n = lane + 64 * n1, nc = n < a.win ? n : 0;
      ra[n1] = sa[nc];
      rb[n1] = sb[nc];
    }
  };
  if (PREF && gw < npairs) load_samples(gw);
  for (int pp = gw; pp < npairs; pp += nw) {
    const int fa = 2 * pp, fb = fa + 1;
    const bool acta = fa < nframes, actb = fb < nframes;
    if (!PREF) load_samples(pp);  // no prefetch: the other wave of the SIMD works meanwhile
    if constexpr (!MAG) {
      // target magnitudes of the lane's canonical bins lane + 64 j, requested now, used after the forward transform
      const int pa = min(fa, nframes - 1), pb = min(fb, nframes - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int k = lane + 64 * j, kc = k < KB ? k : 0;
        ta[j] = a.tm[(size_t)pa * KB + kc];
        tb[j] = a.tm[(size_t)pb * KB + kc];
      }
    }
    f32x2 c[P];
#pragma unroll
    for (int n1 = 0; n1 < P; ++n1) {
      const float w = wn[lane + 64 * n1];
      c[n1] = f32x2{ra[n1] * w, rb[n1] * w};
    }
    // the next pair's samples: requested here for MAG (its bins are short), after the bins for LOSS / GRAD (their
    // live range then spans only the inverse transform: fewer registers held through the forward one and the bins)
    if (PREF && MAG && pp + nw < npairs) load_samples(pp + nw);
    dftp<P, false>(c);  // over n1 -> k1
#pragma unroll
    for (int k1 = 1; k1 < P; ++k1) c[k1] = cmul(c[k1], T[k1 * PITCH + lane]);
#pragma unroll
    for (int k1 = 0; k1 < P; ++k1) buf[k1 * PITCH + lane] = c[k1];
    wave_sync_lds();
#pragma unroll
    for (int m = 0; m < P; ++m) c[m] = buf[k1s * PITCH + g + G * m];
    wave_sync_lds();
    dftp<P, false>(c);  // over m -> q
#pragma unroll
    for (int q = 1; q < P; ++q) c[q] = cmul(c[q], tw64[g * q]);  // g = 0: W^0 = 1 exactly
    xlane_dft<N, false>(c, g, tw64);  // lane (k1s, g): Z[kbase + P q]
    // the bins: every lane writes its Z values at their natural slots, then takes canonical bins k = lane + 64 j
    // (k <= N / 2: each once, as spec_pair_kernel) with their mirrors N - k; GRAD writes H at k and N - k back and
    // every lane reads its own bins' H for the inverse
#pragma unroll
    for (int q = 0; q < P; ++q) buf[S4::slot(kbase + P * q)] = c[q];
    wave_sync_lds();
    float sda = 0.f, sxa = 0.f, sdb = 0.f, sxb = 0.f;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int k = lane + 64 * j;
      if (NB * 64 == KB || k < KB) {
        const int km = (N - k) & (N - 1);
        const f32x2 zk = buf[S4::slot(k)], zm = buf[S4::slot(km)];
        const f32x2 rka = f32x2{0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y)};
        const f32x2 rkb = f32x2{0.5f * (zk.y + zm.y), 0.5f * (zm.x - zk.x)};
        const float mra = cabs_hw(rka), mrb = cabs_hw(rkb);
        if constexpr (MAG) {
          if (acta) a.out[(size_t)fa * KB + k] = mra;
          if (actb) a.out[(size_t)fb * KB + k] = mrb;
        } else {
          const float da = ta[j] - mra, db = tb[j] - mrb;
          sda += da * da;
          sxa += ta[j] * ta[j];
          sdb += db * db;
          sxb += tb[j] * tb[j];
          if constexpr (GRAD) {
            // dL/d(Re,Im)R_k = (|R|-|X|) R/|R| (0 at |R| = 0); H = H_a + i H_b, each the Hermitian extension of
            // G/2 (G at k = 0, N/2) — spec_pair_kernel's values, written over Z at k and N - k at once: no later
            // iteration reads those slots (its k and N - k lie in other 64-bin bands)
            const float ga = mra > 0.f ? (mra - ta[j]) * __builtin_amdgcn_rcpf(mra) : 0.f;
            const float gb = mrb > 0.f ? (mrb - tb[j]) * __builtin_amdgcn_rcpf(mrb) : 0.f;
            const f32x2 Ga = f32x2{ga * rka.x, ga * rka.y}, Gb = f32x2{gb * rkb.x, gb * rkb.y};
            if (k == 0 || k == N / 2) {
              buf[S4::slot(k)] = f32x2{Ga.x, Gb.x};
            } else {
              buf[S4::slot(k)] = f32x2{0.5f * Ga.x - 0.5f * Gb.y, 0.5f * Ga.y + 0.5f * Gb.x};
              buf[S4::slot(km)] = f32x2{0.5f * Ga.x + 0.5f * Gb.y, 0.5f * Gb.x - 0.5f * Ga.y};
            }
          }
        }
      }
    }
    if constexpr (GRAD) {
      wave_sync_lds();
#pragma unroll
      for (int q = 0; q < P; ++q) c[q] = buf[S4::slot(kbase + P * q)];
    }
    wave_sync_lds();  // every read of buf precedes the next writes
    if (PREF && !MAG && pp + nw < npairs) load_samples(pp + nw);
    if constexpr (!MAG) {
      sda = warp_sum(sda);
      sxa = warp_sum(sxa);
      sdb = warp_sum(sdb);
      sxb = warp_sum(sxb);
      if (lane == 0) {
        if (acta) {
          a.part[2 * (size_t)fa] = sda;
          a.part[2 * (size_t)fa + 1] = sxa;
        }
        if (actb) {
          a.part[2 * (size_t)fb] = sdb;
          a.part[2 * (size_t)fb + 1] = sxb;
        }
      }
    }
    if constexpr (GRAD) {
      xlane_dft<N, true>(c, g, tw64);  // lane (k1s, g): index g of the 64-point inverse, times W_64^{-g q}
#pragma unroll
      for (int q = 1; q < P; ++q) c[q] = cmul(c[q], conj2(tw64[g * q]));
      dftp<P, true>(c);  // over q -> m: n2 = g + G m
#pragma unroll
      for (int m = 0; m < P; ++m) {
        const int e = k1s * PITCH + g + G * m;
        c[m] = cmul(c[m], conj2(T[e]));
        buf[e] = c[m];
      }
      wave_sync_lds();
#pragma unroll
      for (int k1 = 0; k1 < P; ++k1) c[k1] = buf[k1 * PITCH + lane];
      wave_sync_lds();
      dftp<P, true>(c);  // over k1 -> n1: h[lane + 64 n1]
      float* oa = a.out + (size_t)fa * a.win;
      float* ob = a.out + (size_t)fb * a.win;
#pragma unroll
      for (int n1 = 0; n1 < P; ++n1) {
        const int n = lane + 64 * n1;
        if (n < a.win) {
          const float w = wn[n];
          if (acta) oa[n] = c[n1].x * w;
          if (actb) ob[n] = c[n1].y * w;
        }
      }
    }
  }
}

// twiddles exp(-2 pi i k / N) (N complex per resolution) and periodic Hann windows
// (tf.signal.hann_window(win, periodic=True)), evaluated in fp64 and rounded once
struct SpecTables {
  float* tw[SPEC_MAX_RES];
  float* wn[SPEC_MAX_RES];
  int N[SPEC_MAX_RES], win[SPEC_MAX_RES];
  int nres;
};

__global__ __launch_bounds__(256) void spec_tables_kernel(SpecTables t) {
  const int res = blockIdx.y;
  const int N = t.N[res], W = t.win[res];
  for (int k = blockIdx.x * 256 + threadIdx.x; k < N; k += gridDim.x * 256) {
    double sn, cs;
    sincospi(2.0 * (double)k / (double)N, &sn, &cs);
    t.tw[res][2 * k] = (float)cs;
    t.tw[res][2 * k + 1] = (float)-sn;
  }
  for (int n = blockIdx.x * 256 + threadIdx.x; n < W; n += gridDim.x * 256)
    t.wn[res][n] = (float)(0.5 - 0.5 * cospi(2.0 * (double)n / (double)W));
}

struct SpecScaleArgs {
  const float* part[SPEC_MAX_RES];
  int F[SPEC_MAX_RES];
  float* lossbr;  // (B, nres) per item and resolution: ||S_x - S_r|| / ||S_x||
  float* scale;   // (B, nres): inv / (||S_x - S_r|| * ||S_x||)
  int nres;
  float inv;  // 1 / (nres * B)
};

__global__ __launch_bounds__(256) void spec_scale_kernel(SpecScaleArgs a) {
  __shared__ float red[4];
  const int b = blockIdx.x / a.nres, res = blockIdx.x - b * a.nres;
  const int F = a.F[res];
  const float* p = a.part[res] + (size_t)b * F * 2;
  float sd = 0.f, sx = 0.f;
  for (int f = threadIdx.x; f < F; f += 256) {
    sd += p[2 * f];
    sx += p[2 * f + 1];
  }
  sd = block_sum_256(sd, red);
  __syncthreads();
  sx = block_sum_256(sx, red);
  if (threadIdx.x == 0) {
    const float nd = sqrtf(sd), nx = sqrtf(sx);
    a.lossbr[blockIdx.x] = nd / nx;
    a.scale[blockIdx.x] = a.inv / (nd * nx);
  }
}

struct SpecGatherArgs {
  const float* fg[SPEC_MAX_RES];
  int F[SPEC_MAX_RES], hop[SPEC_MAX_RES], win[SPEC_MAX_RES];
  const float* lossbr;
  const float* scale;
  float* dr;         // (B, T) or null (loss only)
  float* loss_out;   // [1]: mean_b mean_res lossbr
  float* item_loss;  // (B) or null: mean_res lossbr
  int B, T, nres;
};

__global__ __launch_bounds__(256) void spec_gather_kernel(SpecGatherArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float tot = 0.f;
    for (int b = 0; b < a.B; ++b) {
      float s = 0.f;
      for (int r = 0; r < a.nres; ++r) s += a.lossbr[b * a.nres + r];
      s = s / (float)a.nres;
      if (a.item_loss) a.item_loss[b] = s;
      tot += s;
    }
    a.loss_out[0] = tot / (float)a.B;
  }
  if (!a.dr) return;
  const long long n = (long long)a.B * a.T;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int b = (int)(i / a.T), t = (int)(i - (long long)b * a.T);
    float acc = 0.f;
    for (int r = 0; r < a.nres; ++r) {
      const int hop = a.hop[r], win = a.win[r], F = a.F[r];
      const int f_hi = min(F - 1, t / hop);
      const int f_lo = t >= win ? (t - win) / hop + 1 : 0;
      const float* g = a.fg[r] + (size_t)b * F * win;
      float s = 0.f;
      for (int f = f_lo; f <= f_hi; ++f) s += g[(size_t)f * win + (t - f * hop)];
      acc += a.scale[b * a.nres + r] * s;
    }
    a.dr[i] = acc;
  }
}

// The same overlap-add for the usual shapes (<= 4 resolutions, <= 8 frames over a sample, T < 2^24): item =
// blockIdx.y (no 64-bit division per sample), and every frame read of every resolution is issued before the
// sums (clamped addresses; a frame past the sample's range is loaded and not added), so a thread's 15-odd
// loads are in flight together instead of one trip-count-dependent loop iteration at a time. Same sums in the
// same order: bit-identical to spec_gather_kernel.
constexpr int kGatherMaxRes = 4, kGatherMaxF = 8;
__global__ __launch_bounds__(256) void spec_gather8_kernel(SpecGatherArgs a) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    float tot = 0.f;
    for (int b = 0; b < a.B; ++b) {
      float s = 0.f;
      for (int r = 0; r < a.nres; ++r) s += a.lossbr[b * a.nres + r];
      s = s / (float)a.nres;
      if (a.item_loss) a.item_loss[b] = s;
      tot += s;
    }
    a.loss_out[0] = tot / (float)a.B;
  }
  const int b = blockIdx.y;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < a.T; t += gridDim.x * 256) {
    float v[kGatherMaxRes][kGatherMaxF];
    int nf[kGatherMaxRes];
#pragma unroll
    for (int r = 0; r < kGatherMaxRes; ++r) {
      if (r >= a.nres) break;  // uniform
      const int hop = a.hop[r], win = a.win[r], F = a.F[r];
      const int f_hi = min(F - 1, t / hop);
      const int f_lo = t >= win ? (t - win) / hop + 1 : 0;
      nf[r] = f_hi - f_lo + 1;
      const float* g = a.fg[r] + (size_t)b * F * win;
#pragma unroll
      for (int j = 0; j < kGatherMaxF; ++j) {
        const int f = min(f_lo + j, f_hi);
        v[r][j] = g[(size_t)f * win + min(t - f * hop, win - 1)];
      }
    }
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < kGatherMaxRes; ++r) {
      if (r >= a.nres) break;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < kGatherMaxF; ++j)
        if (j < nf[r]) s += v[r][j];
      acc += a.scale[b * a.nres + r] * s;
    }
    a.dr[(size_t)b * a.T + t] = acc;
  }
}

static bool spec_gather8_ok(const SpecGatherArgs& a) {
  if (!a.dr || a.nres > kGatherMaxRes || a.T >= (1 << 24) || a.B > 65535) return false;  // items = grid rows
  for (int r = 0; r < a.nres; ++r)
    if ((a.win[r] + a.hop[r] - 1) / a.hop[r] > kGatherMaxF) return false;
  return true;
}

template <int N>
static int launch_frames(const SpecFrameArgs& fa, hipStream_t s) {
  constexpr int FPI = 256 / spec_tpf<N>();
  const size_t lds = (size_t)N * sizeof(f32x2) + (size_t)((fa.win + 3) & ~3) * sizeof(float) +
                     (size_t)FPI * 2 * fpad<N>() * sizeof(f32x2);
  const int nframes = fa.B * fa.F;
  const int groups = (nframes + FPI - 1) / FPI;
  const int grid = groups < 2048 ? groups : 2048;
  hipLaunchKernelGGL((spec_frame_kernel<N>), dim3(grid), dim3(256), lds, s, fa);
  VQA_LAUNCHED("spec_frame_kernel");
  return VQA_OK;
}

static bool spec_n_ok(int n) { return n == 256 || n == 512 || n == 1024 || n == 2048; }

static int dispatch_frames(int n_fft, const SpecFrameArgs& fa, hipStream_t s) {
  switch (n_fft) {
    case 256: return launch_frames<256>(fa, s);
    case 512: return launch_frames<512>(fa, s);
    case 1024: return launch_frames<1024>(fa, s);
    case 2048: return launch_frames<2048>(fa, s);
    default: set_error("spectral: n_fft %d unsupported (256, 512, 1024, 2048)", n_fft); return VQA_E_UNSUPPORTED;
  }
}

template <int N, int MODE>
static int launch_pairs(const SpecPairArgs& pa, hipStream_t s) {
  constexpr int FPI = kSpecWaves;  // frame pairs (one per wave) in flight per workgroup
  const size_t lds = (size_t)N * sizeof(f32x2) + (size_t)N * sizeof(float) + (size_t)FPI * fpad<N>() * sizeof(f32x2);
  static size_t lds_set = 0;
  if (lds > 65536 && lds > lds_set) {
    if (hipFuncSetAttribute((const void*)spec_pair_kernel<N, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess) {
      (void)hipGetLastError();
      set_error("spectral: cannot reserve %zu B of LDS", lds);
      return VQA_E_UNSUPPORTED;
    }
    lds_set = lds;
  }
  // persistent: as many workgroups as fit on the chip at once (LDS-bound), each wave walking its pairs with the
  // next pair's samples prefetched; the tables are loaded once per workgroup
  const int npairs = (pa.B * pa.F + 1) / 2;
  const int groups = (npairs + FPI - 1) / FPI;
  static int cus = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  static size_t occ_lds = 0;  // resident workgroups per CU (LDS and registers), queried once per LDS size
  static int per_cu = 1;
  if (occ_lds != lds) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)spec_pair_kernel<N, MODE>, 64 * kSpecWaves,
                                                     lds) != hipSuccess || per_cu <= 0) {
      (void)hipGetLastError();
      per_cu = 1;
    }
    occ_lds = lds;
  }
  const int grid = std::min(groups, cus * per_cu);
  hipLaunchKernelGGL((spec_pair_kernel<N, MODE>), dim3(grid), dim3(64 * kSpecWaves), lds, s, pa);
  VQA_LAUNCHED("spec_pair_kernel");
  return VQA_OK;
}

// the four-step kernel: persistent, sized by the occupancy API as launch_pairs
template <int N, int MODE>
static int launch_pairs4(const SpecPairArgs& pa, hipStream_t s) {
  typedef Spec4<N> S4;
  const void* fn = (const void*)spec_pair4_kernel<N, MODE>;
  constexpr int W = spec4_waves<N>();
  const size_t lds = (size_t)(S4::P * S4::PITCH + 64) * sizeof(f32x2) + (size_t)N * sizeof(float) +
                     (size_t)W * S4::BUF * sizeof(f32x2);
  static size_t lds_set = 0;
  if (lds > 65536 && lds > lds_set) {
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
      (void)hipGetLastError();
      set_error("spectral: cannot reserve %zu B of LDS", lds);
      return VQA_E_UNSUPPORTED;
    }
    lds_set = lds;
  }
  const int npairs = (pa.B * pa.F + 1) / 2;
  const int groups = (npairs + W - 1) / W;
  static int cus = [] {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  static size_t occ_lds = 0;
  static int per_cu = 1;
  if (occ_lds != lds) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * W, lds) != hipSuccess || per_cu <= 0) {
      (void)hipGetLastError();
      per_cu = 1;
    }
    occ_lds = lds;
  }
  const int grid = std::min(groups, cus * per_cu);
  hipLaunchKernelGGL((spec_pair4_kernel<N, MODE>), dim3(grid), dim3(64 * W), lds, s, pa);
  VQA_LAUNCHED("spec_pair4_kernel");
  return VQA_OK;
}

template <int MODE>
static int dispatch_pairs(int n_fft, const SpecPairArgs& pa, hipStream_t s) {
  switch (n_fft) {
    // the four-step form where it is faster (2048: 8 waves, two per SIMD, 84 -> 58 us per gradient launch at config 2);
    // the Stockham form (one radix-8 / 16 / 4 pass per LDS round trip) keeps fewer VALU instructions per pair for
    // the shorter transforms, which run at several waves per SIMD either way (round 6, profiles/r6_spectral.txt)
    case 256: return launch_pairs<256, MODE>(pa, s);
    case 512: return launch_pairs<512, MODE>(pa, s);
    case 1024: return launch_pairs<1024, MODE>(pa, s);
    case 2048: return launch_pairs4<2048, MODE>(pa, s);
    default: set_error("spectral: n_fft %d unsupported (256, 512, 1024, 2048)", n_fft); return VQA_E_UNSUPPORTED;
  }
}

static size_t align64(size_t n) { return (n + 63) & ~(size_t)63; }

// Target region (floats; per resolution: twiddles 2N | window | |S_x| (B*F, N/2+1)) and loss workspace
// (per resolution: frame gradients (grad only) | per-frame partials; then per-item losses | scales).
struct SpecLayout {
  size_t tw[SPEC_MAX_RES], wn[SPEC_MAX_RES], tm[SPEC_MAX_RES], target;
  size_t fg[SPEC_MAX_RES], part[SPEC_MAX_RES], tail, loss;
  int F[SPEC_MAX_RES];
};

static int spec_layout(int B, int T, const int* n_fft, const int* hop, const int* win, int nres, bool grad,
                       SpecLayout* L) {
  if (B <= 0 || T <= 0 || nres <= 0 || nres > SPEC_MAX_RES || !n_fft || !hop || !win) return VQA_E_INVALID_ARG;
  size_t o = 0;
  for (int r = 0; r < nres; ++r) {
    if (hop[r] <= 0 || win[r] <= 0 || win[r] > n_fft[r] || win[r] > T || !spec_n_ok(n_fft[r])) return VQA_E_INVALID_ARG;
    L->F[r] = 1 + (T - win[r]) / hop[r];
    L->tw[r] = o;
    o += align64((size_t)2 * n_fft[r]);
    L->wn[r] = o;
    o += align64((size_t)win[r]);
    L->tm[r] = o;
    o += align64((size_t)B * L->F[r] * (n_fft[r] / 2 + 1));
  }
  L->target = o * sizeof(float);
  o = 0;
  for (int r = 0; r < nres; ++r) {
    L->fg[r] = o;
    if (grad) o += align64((size_t)B * L->F[r] * win[r]);
    L->part[r] = o;
    o += align64((size_t)B * L->F[r] * 2);
  }
  L->tail = o;
  o += align64((size_t)B * nres * 2);
  L->loss = o * sizeof(float);
  return VQA_OK;
}

static int spec_target(const float* x, float* tg, const SpecLayout& L, int B, int T, const int* n_fft, const int* hop,
                       const int* win, int nres, hipStream_t s) {
  SpecTables tb{};
  int maxn = 0;
  for (int i = 0; i < nres; ++i) {
    tb.tw[i] = tg + L.tw[i];
    tb.wn[i] = tg + L.wn[i];
    tb.N[i] = n_fft[i];
    tb.win[i] = win[i];
    maxn = n_fft[i] > maxn ? n_fft[i] : maxn;
  }
  tb.nres = nres;
  hipLaunchKernelGGL(spec_tables_kernel, dim3((maxn + 255) / 256, nres), dim3(256), 0, s, tb);
  VQA_LAUNCHED("spec_tables_kernel");
  for (int i = 0; i < nres; ++i) {
    SpecPairArgs pa{x, nullptr, tg + L.tm[i], nullptr, tg + L.tw[i], tg + L.wn[i], B, T, L.F[i], hop[i], win[i]};
    if (int rc = dispatch_pairs<PAIR_MAG>(n_fft[i], pa, s)) return rc;
  }
  return VQA_OK;
}

static int spec_loss(const float* tg, const float* r, float* loss_out, float* dr, float* item_loss, float* ws,
                     const SpecLayout& L, int B, int T, const int* n_fft, const int* hop, const int* win, int nres,
                     hipStream_t s) {
  const bool grad = dr != nullptr;
  SpecScaleArgs sa{};
  SpecGatherArgs ga{};
  for (int i = 0; i < nres; ++i) {
    SpecPairArgs pa{r, tg + L.tm[i], ws + L.fg[i], ws + L.part[i], tg + L.tw[i], tg + L.wn[i], B, T, L.F[i], hop[i],
                    win[i]};
    const int rc = grad ? dispatch_pairs<PAIR_GRAD>(n_fft[i], pa, s) : dispatch_pairs<PAIR_LOSS>(n_fft[i], pa, s);
    if (rc != VQA_OK) return rc;
    sa.part[i] = ws + L.part[i];
    sa.F[i] = L.F[i];
    ga.fg[i] = ws + L.fg[i];
    ga.F[i] = L.F[i];
    ga.hop[i] = hop[i];
    ga.win[i] = win[i];
  }
  sa.lossbr = ws + L.tail;
  sa.scale = ws + L.tail + (size_t)B * nres;
  sa.nres = nres;
  sa.inv = (float)(1.0 / ((double)nres * (double)B));
  hipLaunchKernelGGL(spec_scale_kernel, dim3(B * nres), dim3(256), 0, s, sa);
  VQA_LAUNCHED("spec_scale_kernel");
  ga.lossbr = sa.lossbr;
  ga.scale = sa.scale;
  ga.dr = dr;
  ga.loss_out = loss_out;
  ga.item_loss = item_loss;
  ga.B = B;
  ga.T = T;
  ga.nres = nres;
  if (spec_gather8_ok(ga)) {
    int nx = (T + 255) / 256;
    if (nx > 1024) nx = 1024;
    hipLaunchKernelGGL(spec_gather8_kernel, dim3(nx, B), dim3(256), 0, s, ga);
    VQA_LAUNCHED("spec_gather8_kernel");
    return VQA_OK;
  }
  long long nb = grad ? ((long long)B * T + 255) / 256 : 1;
  if (nb > 8192) nb = 8192;
  hipLaunchKernelGGL(spec_gather_kernel, dim3((int)nb), dim3(256), 0, s, ga);
  VQA_LAUNCHED("spec_gather_kernel");
  return VQA_OK;
}

}  // namespace vqa

using namespace vqa;

#define SPEC_SHAPE_ERR "spectral: bad shape (B=%d T=%d nres=%d; need 0 < win <= n_fft, win <= T, hop > 0, " \
                       "n_fft in {256, 512, 1024, 2048})"

extern "C" size_t vqa_spectral_target_workspace(int B, int T, const int* n_fft, const int* hop, const int* win,
                                                int nres) {
  SpecLayout L;
  return spec_layout(B, T, n_fft, hop, win, nres, false, &L) == VQA_OK ? L.target : 0;
}

extern "C" int vqa_spectral_target(const float* x, void* target, size_t target_bytes, int B, int T, const int* n_fft,
                                   const int* hop, const int* win, int nres, vqa_stream_t stream) {
  VQA_ARG(x && target, "spectral_target: null pointer");
  SpecLayout L;
  VQA_ARG(spec_layout(B, T, n_fft, hop, win, nres, false, &L) == VQA_OK, SPEC_SHAPE_ERR, B, T, nres);
  VQA_ARG(target_bytes >= L.target, "spectral_target: buffer %zu < %zu bytes", target_bytes, L.target);
  return spec_target(x, (float*)target, L, B, T, n_fft, hop, win, nres, (hipStream_t)stream);
}

extern "C" size_t vqa_spectral_loss_target_workspace(int B, int T, const int* n_fft, const int* hop, const int* win,
                                                     int nres, int with_grad) {
  SpecLayout L;
  return spec_layout(B, T, n_fft, hop, win, nres, with_grad != 0, &L) == VQA_OK ? L.loss : 0;
}

extern "C" int vqa_spectral_loss_target(const void* target, const float* r, float* loss_out, float* dr,
                                        float* item_loss, int B, int T, const int* n_fft, const int* hop,
                                        const int* win, int nres, void* workspace, size_t ws_bytes,
                                        vqa_stream_t stream) {
  VQA_ARG(target && r && loss_out, "spectral_loss_target: null pointer");
  SpecLayout L;
  VQA_ARG(spec_layout(B, T, n_fft, hop, win, nres, dr != nullptr, &L) == VQA_OK, SPEC_SHAPE_ERR, B, T, nres);
  VQA_ARG(workspace && ws_bytes >= L.loss, "spectral_loss_target: workspace %zu < %zu bytes", ws_bytes, L.loss);
  return spec_loss((const float*)target, r, loss_out, dr, item_loss, (float*)workspace, L, B, T, n_fft, hop, win, nres,
                   (hipStream_t)stream);
}

extern "C" size_t vqa_spectral_loss_workspace(int B, int T, const int* n_fft, const int* hop, const int* win,
                                              int nres, int with_grad) {
  SpecLayout L;
  if (spec_layout(B, T, n_fft, hop, win, nres, with_grad != 0, &L) != VQA_OK) return 0;
  return L.target + L.loss;
}

extern "C" int vqa_spectral_loss(const float* x, const float* r, float* loss_out, float* dr, float* item_loss, int B,
                                 int T, const int* n_fft, const int* hop, const int* win, int nres, void* workspace,
                                 size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(x && r && loss_out, "spectral_loss: null pointer");
  SpecLayout L;
  VQA_ARG(spec_layout(B, T, n_fft, hop, win, nres, dr != nullptr, &L) == VQA_OK, SPEC_SHAPE_ERR, B, T, nres);
  VQA_ARG(workspace && ws_bytes >= L.target + L.loss, "spectral_loss: workspace %zu < %zu bytes", ws_bytes,
          L.target + L.loss);
  hipStream_t s = (hipStream_t)stream;
  float* tg = (float*)workspace;
  if (int rc = spec_target(x, tg, L, B, T, n_fft, hop, win, nres, s)) return rc;
  return spec_loss(tg, r, loss_out, dr, item_loss, tg + L.target / sizeof(float), L, B, T, n_fft, hop, win, nres, s);
}

extern "C" int vqa_stft_magnitude(const float* x, float* mag, int B, int T, int n_fft, int hop, int win,
                                  vqa_stream_t stream) {
  VQA_ARG(x && mag && B > 0 && hop > 0 && win > 0 && win <= n_fft && win <= T,
          "stft_magnitude: bad arguments (B=%d T=%d n_fft=%d hop=%d win=%d)", B, T, n_fft, hop, win);
  const int F = 1 + (T - win) / hop;
  // no workspace in this entry point: the kernel evaluates its twiddles and window itself
  SpecFrameArgs fa{x, mag, nullptr, nullptr, B, T, F, hop, win};
  return dispatch_frames(n_fft, fa, (hipStream_t)stream);
}
