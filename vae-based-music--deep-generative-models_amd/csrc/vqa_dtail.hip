// vqa_dtail.hip — the decoder tail: the last Conv1DTranspose of the last decoder block followed by the
// decoder's output Conv1D (encdec.py:67-68 then :148), as ONE thin convolution (gfx950).
//
// Nothing sits between the two layers, so the composition is linear in h (the transposed conv's input,
// C = 32 channels at T rows per item):
//     u[s]  = b_up + sum_{kb, j: s = 2j + kb - 1} W_up[kb] h[j]            (K=4, stride 2, SAME: pad 1)
//     y[t]  = b_out + sum_k W_out[k] . u[t + k - 1]                        (K=3, SAME, u[-1] = u[2T] = 0)
//  => y[2j + p] = bias + sum_{a=-1..1} sum_c V[a][c][p] h[j + a][c]        (p = 0, 1: the two output phases)
// with V[a][c][p] = sum_k sum_o W_out[k][o] W_up[p + k - 2a][o][c] (terms with p + k - 2a outside 0..3
// vanish) and two edge corrections per item (the out conv's zero padding at t = 0 and t = 2T - 1 drops
// tap k = 0 resp. k = 2). The 64-channel full-rate tensor u is never formed: the forward reads h and
// writes y, the backward reads h and dy and writes dh, and the parameter gradients follow from
// dV = sum h (x) dy by the chain rule through the (bilinear) composition. Same function as the reference's
// two layers; only the association of the sums differs (u is not rounded to the activation dtype).
//
// Lanes: 4 lanes per row, each owning 8 consecutive channels (one 16-byte bf16 chunk), 16 rows per wave
// instruction. The forward loads every h row once (per-row tap dots, neighbours' terms exchanged across lanes); the
// backward reads each row's dy window (6 values) per lane.
#include "vqa_common.h"

namespace vqa {

constexpr int DT_C = 32;   // transposed-conv input channels the lane map covers
constexpr int DT_NV = 192; // V[3][32][2]
// composite workspace: V | edge0[32] | edge1[32] | bias_int, b0, b2, (pad)
constexpr int DT_COMP = DT_NV + 2 * DT_C + 4;
// backward partial row: dV[3][32][2] | Eh[32] | Et[32] | S, F, L, (pad)
constexpr int DT_PART = DT_NV + 2 * DT_C + 4;

// 8 channels held packed until use (bf16: one 16-byte load), so several rows' loads can be in flight
template <class T> struct Raw8;
template <> struct Raw8<bf16> {
  uint4 w;
  __device__ __forceinline__ void load(const bf16* p, bool ok) { w = ok ? *(const uint4*)p : uint4{0u, 0u, 0u, 0u}; }
  // unconditional load (p must be valid), zeros selected when !ok
  __device__ __forceinline__ void load_sel(const bf16* p, bool ok) {
    const uint4 x = *(const uint4*)p;
    w = uint4{ok ? x.x : 0u, ok ? x.y : 0u, ok ? x.z : 0u, ok ? x.w : 0u};
  }
  __device__ __forceinline__ void get(float (&v)[8]) const {
    const unsigned u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
    }
  }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p, bool ok) {
    a = b = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok) {
      a = *(const f32x4*)p;
      b = *(const f32x4*)(p + 4);
    }
  }
  __device__ __forceinline__ void load_sel(const float* p, bool ok) {
    const f32x4 x = *(const f32x4*)p, y = *(const f32x4*)(p + 4), z = {0.f, 0.f, 0.f, 0.f};
    a = ok ? x : z;
    b = ok ? y : z;
  }
  __device__ __forceinline__ void get(float (&v)[8]) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = a[i];
      v[i + 4] = b[i];
    }
  }
};

template <class T> __device__ __forceinline__ void dt_store8(T* p, const float (&v)[8]);
template <> __device__ __forceinline__ void dt_store8<bf16>(bf16* p, const float (&v)[8]) {
  bf16x8 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = (bf16)v[i];
  *(bf16x8*)p = x;
}
template <> __device__ __forceinline__ void dt_store8<float>(float* p, const float (&v)[8]) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

// V, edge vectors and bias terms from the two layers' weights: one wave per output (the sum over the Cu
// channels split across the lanes, then a fixed-order wave reduction); DT_COMP_WAVES waves in all
constexpr int DT_COMP_WAVES = DT_NV + 2 * DT_C + 1;
__global__ __launch_bounds__(256) void dtail_compose_kernel(const float* w_up, const float* b_up, const float* w_out,
                                                            const float* b_out, int Cu, float* comp) {
  const int e = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (e >= DT_COMP_WAVES) return;
  if (e < DT_NV + 2 * DT_C) {
    float s = 0.f;
    if (e < DT_NV) {
      const int a = e / (2 * DT_C) - 1, c = (e >> 1) % DT_C, p = e & 1;
      if (Cu <= 64) {
        // one channel per lane: the six loads issued together (clamped indices, unused terms skipped), the
        // same products added in the same order as the loop below
        const int o = min(lane, Cu - 1);
        float wo[3], wu[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int kb = min(max(p + k - 2 * a, 0), 3);
          wo[k] = w_out[k * Cu + o];
          wu[k] = w_up[((size_t)kb * Cu + o) * DT_C + c];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int kb = p + k - 2 * a;
          if (kb >= 0 && kb <= 3 && lane < Cu) s += wo[k] * wu[k];
        }
      } else {
        for (int k = 0; k < 3; ++k) {
          const int kb = p + k - 2 * a;
          if (kb < 0 || kb > 3) continue;
          for (int o = lane; o < Cu; o += 64) s += w_out[k * Cu + o] * w_up[((size_t)kb * Cu + o) * DT_C + c];
        }
      }
    } else {
      const int c = (e - DT_NV) % DT_C, edge = (e - DT_NV) / DT_C;  // edge 0: (k=0, kb=0); 1: (k=2, kb=3)
      const int k = edge ? 2 : 0, kb = edge ? 3 : 0;
      for (int o = lane; o < Cu; o += 64) s += w_out[k * Cu + o] * w_up[((size_t)kb * Cu + o) * DT_C + c];
    }
    s = warp_sum(s);
    if (lane == 0) comp[e] = s;
  } else {
    float bk[3] = {0.f, 0.f, 0.f};
    for (int o = lane; o < Cu; o += 64) {
      const float bu = b_up ? b_up[o] : 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) bk[k] += w_out[k * Cu + o] * bu;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) bk[k] = warp_sum(bk[k]);
    if (lane == 0) {
      const float bo = b_out ? b_out[0] : 0.f;
      comp[DT_NV + 2 * DT_C] = bo + bk[0] + bk[1] + bk[2];
      comp[DT_NV + 2 * DT_C + 1] = bk[0];
      comp[DT_NV + 2 * DT_C + 2] = bk[2];
      comp[DT_NV + 2 * DT_C + 3] = 0.f;
    }
  }
}

struct DtArgs {
  const void* h;    // (B, T, 32)
  const float* dy;  // backward: (B, 2T) fp32
  float* y;         // forward: (B, 2T) fp32
  void* dh;         // backward: (B, T, 32)
  const float* comp;
  float* part;      // backward: one DT_PART row per workgroup (row order: dt_part_row)
  int B, T;
  int pgroups;      // backward: > 0 -> partial rows laid out [rows / pgroups][pgroups] for the two-stage reduction
};

// Partial row of workgroup p among P: with G = pgroups > 0 the rows are stored [P / G][G] (row p at (p mod R) G +
// p / R, R = P / G), so that reducing the buffer as R rows of G DT_PART-wide rows sums each group g's workgroups
// g R .. g R + R - 1 in order (stage 1, R-deep instead of P-deep), and the G group sums are then reduced in order.
__device__ __forceinline__ int dt_part_row(int p, int P, int G) {
  if (G <= 0) return p;
  const int R = P / G;
  return (p % R) * G + p / R;
}

// y[n, 2j + p], row-dot form: with A_a[p](i) = sum_c V[a][c][p] h[i][c] (three taps a = -1, 0, 1 -> index 0..2),
//     y[2j + p] = bias + A_0[p](j - 1) + A_1[p](j) + A_2[p](j + 1)
// so every h row is loaded ONCE. A lane quad owns kDtU consecutive rows (a wave 16 kDtU rows per pass); each lane
// forms the six tap dots of its 8-channel slice per row, the neighbour rows' terms come from the same lane (inside the
// quad's rows) or from the quads either side (ds_bpermute), and the wave's two halo rows (J0 - 1, J0 + 16 kDtU) are
// loaded by the first / last quad; the 4 slices are then added in the quad (DPP) and lane q of the quad stores row q.
// The next pass's loads are issued before this pass's arithmetic. Grid (row blocks, items), grid-stride over rows.
constexpr int kDtU = 4;  // rows per lane quad and pass (= the quad's 4 lanes: one stored row each)
__device__ __forceinline__ float dt_from_lane(float v, int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
template <class T>
__global__ __launch_bounds__(256) void dtail_fwd_kernel(DtArgs a) {
  constexpr int U = kDtU;
  const int lane = threadIdx.x & 63, r = lane >> 2, q = lane & 3, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float v[3][8][2];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) v[t][i][p] = a.comp[(t * DT_C + 8 * q + i) * 2 + p];
  const float bias = a.comp[DT_NV + 2 * DT_C], b0 = a.comp[DT_NV + 2 * DT_C + 1], b2 = a.comp[DT_NV + 2 * DT_C + 2];
  const T* H = (const T*)a.h + (size_t)blockIdx.y * a.T * DT_C;  // item n = blockIdx.y
  float* Y = a.y + (size_t)blockIdx.y * a.T * 2;
  const int step = gridDim.x * 64 * U;
  // loads from clamped addresses, zeros selected afterwards (no load in a branch: the wait before the arithmetic
  // then counts only the previous pass's loads); the extra row is the halo (r = 0: J - 1, r = 15: J + 16U)
  auto fetch = [&](int J, Raw8<T>(&raw)[U], Raw8<T>& rx) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = J + U * r + u;
      const bool ok = j < a.T;
      raw[u].load_sel(H + (size_t)(ok ? j : a.T - 1) * DT_C + 8 * q, ok);
    }
    const int jx = r == 0 ? J - 1 : J + 16 * U;
    const bool okx = (r == 0 || r == 15) && jx >= 0 && jx < a.T;
    rx.load_sel(H + (size_t)(okx ? jx : 0) * DT_C + 8 * q, okx);
  };
  int J0 = blockIdx.x * 64 * U + wave * 16 * U;
  Raw8<T> raw[U], rx;
  fetch(J0, raw, rx);
  for (; J0 < a.T; J0 += step) {
    Raw8<T> rawn[U], rxn;
    fetch(J0 + step, rawn, rxn);  // past the item: clamped addresses, zeros
    float A[U][3][2];  // this lane's slice of the three tap dots of its U rows
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float h[8];
      raw[u].get(h);
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          float s = v[t][0][p] * h[0];
#pragma unroll
          for (int i = 1; i < 8; ++i) s += v[t][i][p] * h[i];
          A[u][t][p] = s;
        }
    }
    // halo row: tap 0 of row J0 - 1 (first quad) or tap 2 of row J0 + 16U (last quad)
    float X[2];
    {
      float h[8];
      rx.get(h);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        float s = (r == 0 ? v[0][0][p] : v[2][0][p]) * h[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) s += (r == 0 ? v[0][i][p] : v[2][i][p]) * h[i];
        X[p] = s;
      }
    }
    float pm[2], pp[2];  // the previous row's tap-0 and the next row's tap-2 slices for rows u = 0 and U - 1
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      pm[p] = dt_from_lane(A[U - 1][0][p], (lane - 4) & 63);
      pp[p] = dt_from_lane(A[0][2][p], (lane + 4) & 63);
      if (r == 0) pm[p] = X[p];
      if (r == 15) pp[p] = X[p];
    }
    float y[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        y[u][p] = ((u == 0 ? pm[p] : A[u - 1][0][p]) + A[u][1][p]) + (u == U - 1 ? pp[p] : A[u + 1][2][p]);
      const int j = J0 + U * r + u;
      if (j == 0 || j == a.T - 1) {
        // the out conv's padding at t = 0 drops tap k = 0, at t = 2T - 1 tap k = 2 (edge vectors of comp)
        float h[8];
        raw[u].get(h);
        const int p = j == 0 ? 0 : 1;
        const float* e = a.comp + DT_NV + p * DT_C + 8 * q;
        float c = e[0] * h[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) c += e[i] * h[i];
        if (j == 0) y[u][0] -= c;
        if (j == a.T - 1) {
          if (j == 0) {  // T = 1: both corrections on the same row
            const float* e1 = a.comp + DT_NV + DT_C + 8 * q;
            float c1 = e1[0] * h[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) c1 += e1[i] * h[i];
            y[u][1] -= c1;
          } else {
            y[u][1] -= c;
          }
        }
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        y[u][p] += xl::xor1(y[u][p]);
        y[u][p] += xl::xor2(y[u][p]);
      }
    }
    // lane q of the quad stores row U r + q: 64 consecutive rows' (y[2j], y[2j+1]) per wave store
    float o0 = y[0][0], o1 = y[0][1];
#pragma unroll
    for (int u = 1; u < U; ++u) {
      o0 = q == u ? y[u][0] : o0;
      o1 = q == u ? y[u][1] : o1;
    }
    const int j = J0 + U * r + q;
    if (j < a.T) {
      o0 += bias - (j == 0 ? b0 : 0.f);
      o1 += bias - (j == a.T - 1 ? b2 : 0.f);
      *(float2*)(Y + (size_t)j * 2) = make_float2(o0, o1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) raw[u] = rawn[u];
    rx = rxn;
  }
}

// dh (adjoint of the composite) and the per-workgroup partial row of dV / edge sums / dy sums
template <class T>
__global__ __launch_bounds__(256) void dtail_bwd_kernel(DtArgs a) {
  __shared__ float red[4][4][68];  // [wave][q][element of the lane's slice]
  const int lane = threadIdx.x & 63, r = lane >> 2, q = lane & 3, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float v[3][8][2], e0[8], e1[8];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) v[t][i][p] = a.comp[(t * DT_C + 8 * q + i) * 2 + p];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    e0[i] = a.comp[DT_NV + 8 * q + i];
    e1[i] = a.comp[DT_NV + DT_C + 8 * q + i];
  }
  float dv[3][8][2], eh[8], et[8], sS = 0.f, sF = 0.f, sL = 0.f;
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i) dv[t][i][0] = dv[t][i][1] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) eh[i] = et[i] = 0.f;
  const T* H = (const T*)a.h + (size_t)blockIdx.y * a.T * DT_C;  // item n = blockIdx.y
  T* DH = (T*)a.dh + (size_t)blockIdx.y * a.T * DT_C;
  const float* dyn = a.dy + (size_t)blockIdx.y * 2 * a.T;
  const int T2 = 2 * a.T;
  constexpr int U = 2;
  const int step = gridDim.x * 64 * U;
  // the next iteration's h / dy loads are issued before this iteration's arithmetic (software pipelining: at two
  // waves per SIMD the loads of one iteration alone cannot cover the HBM latency)
  auto fetch = [&](int J, Raw8<T>(&raw)[U], float (&g)[U][6]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional loads from clamped addresses, zeros selected afterwards: no load sits in a branch, so the
      // compiler's wait before the arithmetic counts only the previous iteration's loads, not these
      const int j = J + 16 * u + r;
      const bool lv = j < a.T;
      const int jc = lv ? j : a.T - 1;
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int t = 2 * j - 2 + 2 * m;
        const bool ok = lv && t >= 0 && t < T2;
        const float2 w = *(const float2*)(dyn + min(max(t, 0), T2 - 2));
        g[u][2 * m] = ok ? w.x : 0.f;
        g[u][2 * m + 1] = ok ? w.y : 0.f;
      }
      raw[u].load_sel(H + (size_t)jc * DT_C + 8 * q, lv);
    }
  };
  int J0 = blockIdx.x * 64 * U + wave * 16 * U;
  Raw8<T> raw[U];
  float g[U][6];  // dy[2j - 2 .. 2j + 3] (zero outside the item)
  fetch(J0, raw, g);
  for (; J0 < a.T; J0 += step) {
    Raw8<T> rawn[U];
    float gn[U][6];
    fetch(J0 + step, rawn, gn);  // past the item: every lane's loads are predicated off (zeros)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = J0 + 16 * u + r;
      const bool lv = j < a.T;
      const float* gg = g[u];
      float h0[8];
      raw[u].get(h0);
      // dh[j][c] = sum_{a,p} V[a][c][p] dy[2(j - a) + p]: a = -1 -> gg[4 + p], a = 0 -> gg[2 + p], a = 1 -> gg[p]
      float d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        d[i] = v[0][i][0] * gg[4] + v[0][i][1] * gg[5] + v[1][i][0] * gg[2] + v[1][i][1] * gg[3] +
               v[2][i][0] * gg[0] + v[2][i][1] * gg[1];
        if (j == 0) d[i] -= e0[i] * gg[2];
        if (j == a.T - 1) d[i] -= e1[i] * gg[3];
      }
      if (lv) dt_store8<T>(DH + (size_t)j * DT_C + 8 * q, d);
      // dV[a][c][p] = sum_j h[j + a][c] dy[2j + p] = sum_j h[j][c] dy[2(j - a) + p]: row j's own h against the
      // same dy window (out-of-item dy reads are zero); edge sums; dy sums (q == 0 lanes only)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dv[0][i][0] += h0[i] * gg[4];
        dv[0][i][1] += h0[i] * gg[5];
        dv[1][i][0] += h0[i] * gg[2];
        dv[1][i][1] += h0[i] * gg[3];
        dv[2][i][0] += h0[i] * gg[0];
        dv[2][i][1] += h0[i] * gg[1];
        if (j == 0) eh[i] += h0[i] * gg[2];
        if (j == a.T - 1) et[i] += h0[i] * gg[3];
      }
      if (q == 0 && lv) {
        sS += gg[2] + gg[3];
        if (j == 0) sF += gg[2];
        if (j == a.T - 1) sL += gg[3];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      raw[u] = rawn[u];
#pragma unroll
      for (int k = 0; k < 6; ++k) g[u][k] = gn[u][k];
    }
  }
  // per-lane slice (64 values: dv 48 | eh 8 | et 8; q == 0 adds S, F, L) -> sum over the 16 rows of the
  // wave (lanes with equal q), then over the 4 waves, in a fixed order
  float s[67];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s[(t * 8 + i) * 2] = dv[t][i][0];
      s[(t * 8 + i) * 2 + 1] = dv[t][i][1];
    }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s[48 + i] = eh[i];
    s[56 + i] = et[i];
  }
  s[64] = sS;
  s[65] = sF;
  s[66] = sL;
#pragma unroll
  for (int e = 0; e < 67; ++e) {
    // over the lanes of equal q: the row's 4 (rotations by 4 and 8 keep q), then the 4 rows
    float x = s[e];
    x += xl::ror4(x);
    x += xl::ror8(x);
    x = xl::sum32(xl::sum16(x));
    s[e] = x;
  }
  if (r == 0) {
#pragma unroll
    for (int e = 0; e < 67; ++e) red[wave][q][e] = s[e];
  }
  __syncthreads();
  float* out = a.part + (size_t)dt_part_row(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, a.pgroups) *
                           DT_PART;
  for (int e = threadIdx.x; e < DT_PART; e += 256) {
    // element e of the partial row -> (q, slice index)
    int qq, si;
    if (e < DT_NV) {
      const int t = e / (2 * DT_C), c = (e >> 1) % DT_C, p = e & 1;
      qq = c >> 3;
      si = (t * 8 + (c & 7)) * 2 + p;
    } else if (e < DT_NV + 2 * DT_C) {
      const int c = (e - DT_NV) % DT_C, which = (e - DT_NV) / DT_C;
      qq = c >> 3;
      si = 48 + 8 * which + (c & 7);
    } else {
      qq = 0;
      si = 64 + (e - DT_NV - 2 * DT_C);
    }
    float x = 0.f;
    if (si < 67)
      for (int w = 0; w < 4; ++w) x += red[w][qq][si];
    out[e] = x;
  }
}

// parameter gradients from the reduced partial row. Blocks [0, nbo): one wave per dW_out element (the
// 192-term sum split across the lanes); blocks [nbo, ...): one thread per dW_up element, then db_up, db_out
__global__ __launch_bounds__(256) void dtail_chain_kernel(const float* red, const float* w_up, const float* b_up,
                                                          const float* w_out, int Cu, int nbo, float* dw_up,
                                                          float* db_up, float* dw_out, float* db_out) {
  const float* dV = red;
  const float* Eh = red + DT_NV;
  const float* Et = red + DT_NV + DT_C;
  const float S = red[DT_NV + 2 * DT_C], F = red[DT_NV + 2 * DT_C + 1], L = red[DT_NV + 2 * DT_C + 2];
  // gradient of the per-tap composite V_k: the shared dV plus the edge terms of taps 0 and 2
  auto dvk = [&](int k, int a, int c, int p) {
    float x = dV[((a + 1) * DT_C + c) * 2 + p];
    if (k == 0 && a == 0 && p == 0) x -= Eh[c];
    if (k == 2 && a == 0 && p == 1) x -= Et[c];
    return x;
  };
  auto sk = [&](int k) { return S - (k == 0 ? F : 0.f) - (k == 2 ? L : 0.f); };
  if ((int)blockIdx.x < nbo) {
    // dW_out[k][o] = sum_{a, p, c} dV_k[a][c][p] W_up[p + k - 2a][o][c] + b_up[o] S_k
    const int e = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (e >= 3 * Cu) return;
    const int k = e / Cu, o = e % Cu;
    float x = 0.f;
    for (int t = lane; t < DT_NV; t += 64) {
      const int a = t / (2 * DT_C) - 1, c = (t >> 1) % DT_C, p = t & 1, kb = p + k - 2 * a;
      if (kb >= 0 && kb <= 3) x += dvk(k, a, c, p) * w_up[((size_t)kb * Cu + o) * DT_C + c];
    }
    x = warp_sum(x);
    if (lane == 0) dw_out[e] = x + (b_up ? b_up[o] : 0.f) * sk(k);
    return;
  }
  const int e = (blockIdx.x - nbo) * 256 + threadIdx.x;
  if (e < 4 * Cu * DT_C) {
    // dW_up[kb][o][c] = sum_{k, a, p: p + k - 2a = kb} dV_k[a][c][p] W_out[k][o]
    const int kb = e / (Cu * DT_C), o = (e / DT_C) % Cu, c = e % DT_C;
    float x = 0.f;
    for (int k = 0; k < 3; ++k)
      for (int p = 0; p < 2; ++p) {
        const int t2 = p + k - kb;  // = 2a
        if (t2 & 1) continue;
        const int a = t2 / 2;
        if (a < -1 || a > 1) continue;
        x += dvk(k, a, c, p) * w_out[k * Cu + o];
      }
    dw_up[e] = x;
  } else if (e < 4 * Cu * DT_C + Cu) {
    const int o = e - 4 * Cu * DT_C;
    float x = 0.f;
    for (int k = 0; k < 3; ++k) x += w_out[k * Cu + o] * sk(k);
    if (db_up) db_up[o] = x;
  } else if (e == 4 * Cu * DT_C + Cu) {
    if (db_out) db_out[0] = S;
  }
}

// grid (gx, B): gx row blocks per item (rows_per_block rows per block and iteration: the forward's 4 waves x 16 x
// U = 3 = 192, the backward's 4 x 16 x U = 2 = 128), about 1024 workgroups in all (4 resident per CU); one partial
// row per workgroup in the backward
constexpr int kDtGroups = 16;  // stage-1 groups of the backward's partial-row reduction
// backward workgroups over all items: one round of 2 per CU (205 VGPRs: 2 waves per SIMD). 1024 (two rounds) took
// 41.8 us per launch at B = 32, T = 32768, 512 38.3 us (768 forward / 512 backward A/B, profiles/r6_dtail.txt)
constexpr int kDtBwdWgs = 512;
// forward workgroups over all items: one round of 3 per CU (154 VGPRs); 1024 took 19.8 us, 768 18.7 us (the
// neighbour-load form before: 24.8 us)
constexpr int kDtFwdWgs = 768;

static int dt_gx(int B, int T, int rows_per_block, int total) {
  const int per_item = (T + rows_per_block - 1) / rows_per_block;
  int gx = total / B;
  if (gx > per_item) gx = per_item;
  return gx > 0 ? gx : 1;
}

}  // namespace vqa

using namespace vqa;

extern "C" int vqa_dtail_supported(int C, int Cu, int K_up, int stride_up, int K_out, int C_out, int dtype) {
  return C == DT_C && Cu >= 1 && Cu <= 1024 && K_up == 4 && stride_up == 2 && K_out == 3 && C_out == 1 &&
         (dtype == VQA_BF16 || dtype == VQA_F32);
}

extern "C" size_t vqa_dtail_workspace(int B, int T, int C, int Cu, int dtype) {
  if (B < 1 || T < 1) return 0;
  (void)C;
  (void)Cu;
  (void)dtype;
  const size_t g = (size_t)dt_gx(B, T, 128, kDtBwdWgs) * B;  // the backward's partial rows (+ the stage-1 group sums)
  return ((size_t)DT_COMP + (size_t)DT_PART + (g + kDtGroups) * DT_PART) * sizeof(float);
}

extern "C" int vqa_dtail_fwd(const void* h, const float* w_up, const float* b_up, const float* w_out,
                             const float* b_out, float* y, int B, int T, int C, int Cu, int dtype, void* workspace,
                             size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(h && w_up && w_out && y && B > 0 && T > 0, "dtail_fwd: bad arguments");
  VQA_REQUIRE(vqa_dtail_supported(C, Cu, 4, 2, 3, 1, dtype), VQA_E_UNSUPPORTED, "dtail_fwd: unsupported C=%d Cu=%d",
              C, Cu);
  VQA_ARG(workspace && ws_bytes >= vqa_dtail_workspace(B, T, C, Cu, dtype), "dtail_fwd: workspace too small");
  VQA_ARG(B <= 65535, "dtail_fwd: B=%d items exceed the grid's item rows (65535)", B);
  const hipStream_t s = (hipStream_t)stream;
  float* comp = (float*)workspace;
  hipLaunchKernelGGL(dtail_compose_kernel, dim3((DT_COMP_WAVES + 3) / 4), dim3(256), 0, s, w_up, b_up, w_out, b_out,
                     Cu, comp);
  VQA_LAUNCHED("dtail_compose_kernel");
  DtArgs a{h, nullptr, y, nullptr, comp, nullptr, B, T, 0};
  const dim3 g(dt_gx(B, T, 64 * kDtU, kDtFwdWgs), B);
  if (dtype == VQA_BF16) hipLaunchKernelGGL(dtail_fwd_kernel<bf16>, g, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dtail_fwd_kernel<float>, g, dim3(256), 0, s, a);
  VQA_LAUNCHED("dtail_fwd_kernel");
  return VQA_OK;
}

extern "C" int vqa_dtail_bwd(const float* dy, const void* h, const float* w_up, const float* b_up,
                             const float* w_out, const float* b_out, void* dh, float* dw_up, float* db_up,
                             float* dw_out, float* db_out, int B, int T, int C, int Cu, int dtype, void* workspace,
                             size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(dy && h && w_up && w_out && dh && dw_up && dw_out && B > 0 && T > 0, "dtail_bwd: bad arguments");
  VQA_REQUIRE(vqa_dtail_supported(C, Cu, 4, 2, 3, 1, dtype), VQA_E_UNSUPPORTED, "dtail_bwd: unsupported C=%d Cu=%d",
              C, Cu);
  VQA_ARG(workspace && ws_bytes >= vqa_dtail_workspace(B, T, C, Cu, dtype), "dtail_bwd: workspace too small");
  VQA_ARG(B <= 65535, "dtail_bwd: B=%d items exceed the grid's item rows (65535)", B);
  const hipStream_t s = (hipStream_t)stream;
  float* comp = (float*)workspace;
  float* red = comp + DT_COMP;
  float* part = red + DT_PART;
  hipLaunchKernelGGL(dtail_compose_kernel, dim3((DT_COMP_WAVES + 3) / 4), dim3(256), 0, s, w_up, b_up, w_out, b_out,
                     Cu, comp);
  VQA_LAUNCHED("dtail_compose_kernel");
  const dim3 g(dt_gx(B, T, 128, kDtBwdWgs), B);
  // many partial rows of few columns: reduced in two fixed-order stages (a single 1024-deep pass over 2 column
  // blocks was a 23 us serial chain of row loads at the head of every level's backward)
  const int P = (int)(g.x * g.y), G = (P >= 4 * kDtGroups && P % kDtGroups == 0) ? kDtGroups : 0;
  float* stage1 = part + (size_t)P * DT_PART;
  DtArgs a{h, dy, nullptr, dh, comp, part, B, T, G};
  if (dtype == VQA_BF16) hipLaunchKernelGGL(dtail_bwd_kernel<bf16>, g, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dtail_bwd_kernel<float>, g, dim3(256), 0, s, a);
  VQA_LAUNCHED("dtail_bwd_kernel");
  if (G > 0) {
    const vqa_partials_desc d1{part, stage1, nullptr, P / G, G * DT_PART, G * DT_PART, 0};
    if (int rc = vqa_reduce_partials(&d1, 1, stream)) return rc;
    const vqa_partials_desc d2{stage1, red, nullptr, G, DT_PART, DT_PART, 0};
    if (int rc = vqa_reduce_partials(&d2, 1, stream)) return rc;
  } else {
    const vqa_partials_desc d{part, red, nullptr, P, DT_PART, DT_PART, 0};
    if (int rc = vqa_reduce_partials(&d, 1, stream)) return rc;
  }
  const int nbo = (3 * Cu + 3) / 4, nbu = (4 * Cu * DT_C + Cu + 1 + 255) / 256;
  hipLaunchKernelGGL(dtail_chain_kernel, dim3(nbo + nbu), dim3(256), 0, s, red, w_up, b_up, w_out, Cu, nbo, dw_up,
                     db_up, dw_out, db_out);
  VQA_LAUNCHED("dtail_chain_kernel");
  return VQA_OK;
}
