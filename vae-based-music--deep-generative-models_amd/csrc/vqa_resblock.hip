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
#include <algorithm>
#include <type_traits>

namespace vqa {

constexpr int RC = 32;    // block width (residual_width of the SMALL_VQ_VAE configs)
constexpr int RTM = 128;  // output rows per tile (runtime-dilation kernels; see rs_fwd_rt / rs_bwd_rt)
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
  int ntm, ntiles, tpw, textra;  // workgroup w owns tiles [w tpw + min(w, textra), +tpw + (w < textra))
  int nwg;
};

template <class T> constexpr int rs_stride() { return RC + lds_pad<T>(); }
constexpr int round16(int v) { return (v + 15) & ~15; }
// s_waitcnt immediate (gfx9 layout: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]): vmcnt(0) only
constexpr int kVmcnt0 = 0x0F70;

// Phase stamps of the backward (dev builds only, -DVQA_RS_STAMPS): s_memtime per wave at 8 points of one tile
// (the workgroup's 5th), read back by vqa_rs_stamps (tools/rs_stamps.py)
#ifdef VQA_RS_STAMPS
constexpr int kRsStampWgs = 1024;
__device__ unsigned long long g_rs_stamps[kRsStampWgs * 4 * 8];
#define RS_STAMP(i)                                                                                      \
  do {                                                                                                   \
    if (stamp_on && lane == 0 && blockIdx.x < kRsStampWgs)                                               \
      g_rs_stamps[(blockIdx.x * 4 + wave) * 8 + (i)] = __builtin_amdgcn_s_memtime();                     \
  } while (0)
#else
#define RS_STAMP(i) \
  do {              \
  } while (0)
#endif

// ---------------------------------------------------------------------------------------------------
// Lane maps. Every tile lives in LDS as [row][32 channels] at an 80-byte row stride (bf16). The maps below
// choose which lane handles which row / channel so that the kernels' LDS instructions are free of bank
// conflicts (MI355X_MICROARCH.md "LDS": ds_read_b128 serves lane groups {0-3,12-15,20-27}, ... on 64
// banks, ds_write_b128 groups of 8 contiguous lanes on 32 banks, ds_read_b64_tr_b16 32-lane halves):
//   rs_pi(n)   tile row of MFMA column n = lane & 15: {0-3, 12-15} -> the odd rows, {4-11} -> the even rows
//   rs_sig(g)  16-byte channel chunk of lane group g = lane >> 4: 0, 2, 1, 3. Used for the 8 output
//              channels a lane holds after an MFMA pair (row m of output tile mt = channel
//              8 sig(m >> 2) + 4 mt + (m & 3)), and — KPERM, backward only — for the K slice of the bf16
//              A/B fragments. Without KPERM every output is the same MFMA sum in the same K order as the
//              unfused gather kernels (the forward stays bit-identical to them).
//   rs_rows    the transposed (K = rows) fragment of the weight-gradient products takes its 32 rows as
//              even rows in lanes 0-31 and odd rows in lanes 32-63 (same K map for both operands).
__device__ __forceinline__ int rs_pi(int n) {
  return 2 * ((n & 3) | ((n >> 1) & 4)) + (((n >> 3) ^ (n >> 2) ^ 1) & 1);
}
__device__ __forceinline__ int rs_sig(int g) { return ((g & 1) << 1) | (g >> 1); }
template <class T, bool KPERM> __device__ __forceinline__ int rs_kcol(int lane) {
  if constexpr (sizeof(T) == 2) return 8 * (KPERM ? rs_sig(lane >> 4) : (lane >> 4));
  else return lane >> 4;
}
// first of the 8 consecutive output channels a lane holds after the MFMAs of tiles mt = 0, 1
__device__ __forceinline__ int rs_ocol(int lane) { return 8 * rs_sig(lane >> 4); }
// A-operand row (within one tap's 32 rows) that produces output channel oc
__device__ __forceinline__ int rs_arow(int oc) { return ((oc >> 2) & 1) * 16 + rs_pi(4 * rs_sig(oc >> 3) + (oc & 3)); }

template <class T> __device__ __forceinline__ typename Mfma<T>::frag rs_rows(const T* o, int stride);
template <> __device__ __forceinline__ bf16x8 rs_rows<bf16>(const bf16* o, int stride) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
  const bf16* a0 = o + (2 * (4 * (g & 1) + (i >> 2)) + (g >> 1)) * stride + 4 * (i & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0 + 16 * stride));
  return __builtin_bit_cast(bf16x8, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
template <> __device__ __forceinline__ float rs_rows<float>(const float* o, int stride) {
  return Mfma<float>::rows(o, stride);
}

// the lane's 8 consecutive channels (lo: tile mt = 0, hi: mt = 1) <-> memory (one 16-byte access for bf16)
template <class T> __device__ __forceinline__ void ld8(const T* p, f32x4& lo, f32x4& hi);
template <> __device__ __forceinline__ void ld8<float>(const float* p, f32x4& lo, f32x4& hi) {
  lo = *(const f32x4*)p;
  hi = *(const f32x4*)(p + 4);
}
template <> __device__ __forceinline__ void ld8<bf16>(const bf16* p, f32x4& lo, f32x4& hi) {
  const bf16x8 v = *(const bf16x8*)p;
  lo = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  hi = f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
}
template <class T> __device__ __forceinline__ void st8(T* p, f32x4 lo, f32x4 hi);
template <> __device__ __forceinline__ void st8<float>(float* p, f32x4 lo, f32x4 hi) {
  *(f32x4*)p = lo;
  *(f32x4*)(p + 4) = hi;
}
__device__ __forceinline__ uint4 bf16_bits(f32x4 lo, f32x4 hi);
template <> __device__ __forceinline__ void st8<bf16>(bf16* p, f32x4 lo, f32x4 hi) {
  *(uint4*)p = bf16_bits(lo, hi);
}

// store of the lane's 8 channels through a buffer descriptor: rows past the item's end are dropped by the
// hardware range check (no per-lane branch)
template <class T>
__device__ __forceinline__ void st8_buf(__amdgpu_buffer_rsrc_t r, int byte_off, f32x4 lo, f32x4 hi) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  if constexpr (sizeof(T) == 2) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, bf16_bits(lo, hi)), r, byte_off, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, lo), r, byte_off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, hi), r, byte_off + 16, 0, 0);
  }
}

// the lane's 8 channels kept as raw activation bits (4 or 8 dwords) and widened when used
template <class T> struct Raw8 {
  uint4 v[sizeof(T) / 2];
  __device__ __forceinline__ void load(const T* p) {
#pragma unroll
    for (int i = 0; i < (int)sizeof(T) / 2; ++i) v[i] = ((const uint4*)p)[i];
  }
  __device__ __forceinline__ void unpack(f32x4& lo, f32x4& hi) const {
    if constexpr (sizeof(T) == 2) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, v[0]);
      lo = f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
      hi = f32x4{(float)b[4], (float)b[5], (float)b[6], (float)b[7]};
    } else {
      lo = __builtin_bit_cast(f32x4, v[0]);
      hi = __builtin_bit_cast(f32x4, v[1]);
    }
  }
};

// (value > 0) for the lane's 8 channels read from LDS (bf16: signed 16-bit compares on the raw bits, so
// -0 counts as not positive)
template <class T> __device__ __forceinline__ void pos8(const T* p, bool (&m)[8]);
template <> __device__ __forceinline__ void pos8<bf16>(const bf16* p, bool (&m)[8]) {
  const uint4 u = *(const uint4*)p;
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[2 * i] = (short)(w[i] & 0xFFFFu) > 0;
    m[2 * i + 1] = (int)w[i] > 0xFFFF;
  }
}
template <> __device__ __forceinline__ void pos8<float>(const float* p, bool (&m)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = p[i] > 0.f;
}

// bf16 epilogue helpers on packed bits (two bf16 per dword, packed integer ops: one instruction per pair)
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
// two floats rounded to bf16 by ONE v_cvt_pk_bf16_f32 (a vector conversion; element-wise casts of a bf16x8
// were emitted as one cvt per value plus a v_perm per pair)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, b2));
}
// the 8 channels rounded to bf16, as raw bits
__device__ __forceinline__ uint4 bf16_bits(f32x4 lo, f32x4 hi) {
  return uint4{pk_bf16(lo[0], lo[1]), pk_bf16(lo[2], lo[3]), pk_bf16(hi[0], hi[1]), pk_bf16(hi[2], hi[3])};
}
// d * (r > 0) per bf16 where r >= 0 (a relu'd tensor): d's bits times min(r's bits, 1) (v_pk_min_u16 + v_pk_mul_lo_u16).
// Written as two asm statements: from the builtin form the compiler re-derived a per-half compare + select
// (v_cmp_ne_u16 / v_cndmask / v_lshrrev / v_perm and hazard s_nops: ~6 instructions per dword instead of 2).
// Plain VALU operands: no memory operation and no wait state inside the strings (cdna_hip_programming.md §5.7).
__device__ __forceinline__ unsigned mask_pos_pk(unsigned d, unsigned r) {
  unsigned m, o;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(r), "s"(0x00010001u));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(o) : "v"(d), "v"(m));
  return o;
}
__device__ __forceinline__ uint4 mask_pos8(uint4 d, uint4 r) {
  return uint4{mask_pos_pk(d.x, r.x), mask_pos_pk(d.y, r.y), mask_pos_pk(d.z, r.z), mask_pos_pk(d.w, r.w)};
}

// bf16 weight images in LDS, built once per workgroup from coalesced 16-byte loads of the fp32 Keras kernel
// (3, 32, 32) (round 6): every lane of every wave then reads each A fragment as ONE 16-byte LDS read, where each wave
// used to gather its fragments itself by strided scalar global loads (48 per 6 fragments, repeated by all four
// waves) — the same bf16 values, so the same MFMA operands and bit-identical results.
//   NAT = true:  img[(k*32 + r) * kImgP + c] = w[k][r][c]  (rows = Keras dim 1: the transposed conv's A rows)
//   NAT = false: img[(k*32 + c) * kImgP + r] = w[k][r][c]  (rows = Keras dim 2, the output channel: a conv's A rows)
constexpr int kImgP = RC + 8;          // bf16 per image row (80 bytes, the tiles' pitch)
constexpr int kImgRows = 3 * RC;      // rows per image
template <bool NAT>
__device__ __forceinline__ void stage_img(bf16* img, const f32x4 (&v)[3 * RC * RC / 4 / 256]) {
#pragma unroll
  for (int i = 0; i < 3 * RC * RC / 4 / 256; ++i) {
    const int e = 4 * (threadIdx.x + 256 * i), k = e / (RC * RC), r = (e / RC) % RC, c = e % RC;  // c .. c + 3
    if constexpr (NAT) {
      *(uint2*)(img + (k * RC + r) * kImgP + c) =
          uint2{pk_bf16(v[i][0], v[i][1]), pk_bf16(v[i][2], v[i][3])};
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) img[(k * RC + c + q) * kImgP + r] = (bf16)v[i][q];
    }
  }
}
__device__ __forceinline__ void load_w4(f32x4 (&v)[3 * RC * RC / 4 / 256], const float* w) {
#pragma unroll
  for (int i = 0; i < 3 * RC * RC / 4 / 256; ++i) v[i] = ((const f32x4*)w)[threadIdx.x + 256 * i];
}
// the lane's A fragments from an image: row = the output channel of (mt, m) (the map of load_wfrags), K slice kc
template <bool KPERM>
__device__ __forceinline__ void frags_from_img(bf16x8 (&wf)[3][2][1], const bf16* img) {
  const int lane = threadIdx.x & 63, m = lane & 15, kc = rs_kcol<bf16, KPERM>(lane);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int o = 8 * rs_sig(m >> 2) + 4 * mt + (m & 3);
      wf[k][mt][0] = *(const bf16x8*)(img + (k * RC + o) * kImgP + kc);
    }
}

// The tile loads go through a per-item buffer descriptor: the hardware range check returns zeros for rows
// outside [0, T) (SAME padding; negative offsets wrap past num_records), so a chunk costs one add and one
// buffer_load, and the per-thread chunk offsets are fixed for the launch.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs_rsrc(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int kRsOOB = -0x40000000;  // chunk offset that stays out of range for any row base

// Rows of a tile staged HBM -> registers -> LDS, 16 B per chunk. bf16 rows are 4 chunks; the 8 contiguous
// lanes of one ds_write_b128 bank group take rows r and r + 4 (disjoint 16-dword windows at 80-byte rows).
template <class T, int PV, int NTH = 256>
struct Rows32Buf {
  static constexpr int VEC = 16 / (int)sizeof(T), CPR = RC / VEC, ROWB = RC * (int)sizeof(T);
  uint4 v[PV];
  int goff[PV], loff[PV];  // byte offset from the tile's first row; LDS element offset from the buffer
  // chunks past the tile's rows load zeros (out-of-range offset) and store them to a trash slot `trash`
  // elements from the buffer: every lane stores, so the staging needs no EXEC-masked branches
  __device__ __forceinline__ void init(int nrows, int trash, int tid = -1) {
    constexpr int XS = RC + 16 / (int)sizeof(T);
    if (tid < 0) tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = tid + i * NTH;
      int rr, q;
      if constexpr (CPR == 4) {
        const int G = e >> 3;
        rr = 8 * (G >> 2) + (G & 3) + 4 * ((e >> 2) & 1);
        q = e & 3;
      } else {
        rr = e / CPR;
        q = e - rr * CPR;
      }
      const bool in = rr < nrows;
      goff[i] = in ? rr * ROWB + q * 16 : kRsOOB;
      loff[i] = in ? rr * XS + q * VEC : trash;
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, int row0) {
    const int base = row0 * ROWB;
#pragma unroll
    for (int i = 0; i < PV; ++i)
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, goff[i] + base, 0, 0));
  }
  template <bool RELU>
  __device__ __forceinline__ void store(T* dst) const {
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      uint4 w = v[i];
      if constexpr (RELU) {
        if constexpr (sizeof(T) == 2) w = __builtin_bit_cast(uint4, relu_frag(__builtin_bit_cast(bf16x8, w)));
        else relu_bits<T>(w);
      }
      *(uint4*)(dst + loff[i]) = w;
    }
  }
};

// (item, tile-in-item) of a workgroup's current tile, advanced without a division per tile
struct RsCursor {
  int n, tm;
  __device__ __forceinline__ void set(int tile, int ntm) {
    n = tile / ntm;
    tm = tile - n * ntm;
  }
  __device__ __forceinline__ void next(int ntm) {
    if (++tm == ntm) {
      tm = 0;
      ++n;
    }
  }
};

// chunks per thread for the largest tile of a launch (rows <= 256 at RMAXD)
template <class T> constexpr int rs_pv() { return sizeof(T) == 2 ? 4 : 8; }

template <class T> constexpr int rs_ncc() { return RC / Mfma<T>::KS; }

// A fragments of a forward conv held in registers: wf[k][mt][cc-step] (A[m][K] = W[k][c][och(mt, m)],
// Keras layout), loaded once per workgroup
template <class T, bool KPERM>
__device__ __forceinline__ void load_wfrags(typename Mfma<T>::frag (&wf)[3][2][rs_ncc<T>()], const float* w) {
  const int lane = threadIdx.x & 63, m = lane & 15, kc = rs_kcol<T, KPERM>(lane);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < rs_ncc<T>(); ++s) {
        const int o = 8 * rs_sig(m >> 2) + 4 * mt + (m & 3);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) wf[k][mt][s][j] = (bf16)w[(k * RC + s * 32 + kc + j) * RC + o];
        } else {
          wf[k][mt][s] = w[(k * RC + s * 4 + kc) * RC + o];
        }
      }
}

// A fragments of a TRANSPOSED conv (output = Keras input channel, input = Keras output channel) held in
// registers: the same lane -> channel map as load_wfrags, read from the kernel transposed (no LDS image)
template <class T>
__device__ __forceinline__ void load_wfrags_t(typename Mfma<T>::frag (&wf)[3][2][rs_ncc<T>()], const float* w) {
  const int lane = threadIdx.x & 63, m = lane & 15, kc = rs_kcol<T, true>(lane);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < rs_ncc<T>(); ++s) {
        const int o = 8 * rs_sig(m >> 2) + 4 * mt + (m & 3);
        if constexpr (sizeof(T) == 2) {
          // the 8 inputs are contiguous in the Keras kernel: two 16-byte loads
          const f32x4* src = (const f32x4*)(w + (k * RC + o) * RC + s * 32 + kc);
          const f32x4 lo = src[0], hi = src[1];
          wf[k][mt][s] = bf16x8{(bf16)lo[0], (bf16)lo[1], (bf16)lo[2], (bf16)lo[3],
                                (bf16)hi[0], (bf16)hi[1], (bf16)hi[2], (bf16)hi[3]};
        } else {
          wf[k][mt][s] = w[(k * RC + o) * RC + s * 4 + kc];
        }
      }
}

// NJ 16-row n-tiles at once: every B fragment is loaded before the first MFMA, then the MFMAs run tap-major
// over the n-tiles (2*NJ independent accumulator chains), so the LDS latency and the MFMA dependency chain
// are hidden inside the wave. Output acc[j][mt]: rows rb[j] + rs_pi(lane & 15), channels rs_ocol(lane) +
// 4 mt + 0..3. afrag(k, mt, s) supplies the A fragment (registers or an LDS image). Tap order k = 0, 1, 2,
// then channel blocks — the accumulation order of the unfused gather kernels.
template <class T, bool RELU_IN, bool KPERM, bool ALDS, int NJ, class AFrag>
__device__ __forceinline__ void conv_multi(f32x4 (&acc)[NJ][2], AFrag afrag, const T* in, const int (&rb)[NJ],
                                           int tap_step, f32x4 init0 = f32x4{0.f, 0.f, 0.f, 0.f},
                                           f32x4 init1 = f32x4{0.f, 0.f, 0.f, 0.f}) {
  typedef Mfma<T> M;
  constexpr int XS = rs_stride<T>(), NCC = rs_ncc<T>();
  const int lane = threadIdx.x & 63;
  const T* base = in + rs_pi(lane & 15) * XS + rs_kcol<T, KPERM>(lane);
  typename M::frag b[NJ][3][NCC];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int s = 0; s < NCC; ++s) {
        b[j][k][s] = M::load(base + (rb[j] + k * tap_step) * XS + s * M::KS);
        if (RELU_IN) b[j][k][s] = relu_frag(b[j][k][s]);
      }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    acc[j][0] = init0;
    acc[j][1] = init1;
  }
  typename M::frag af[3][NCC][2];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int s = 0; s < NCC; ++s) {
      af[k][s][0] = afrag(k, 0, s);
      af[k][s][1] = afrag(k, 1, s);
    }
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int s = 0; s < NCC; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[j][0] = M::mma(af[k][s][0], b[j][k][s], acc[j][0]);
        acc[j][1] = M::mma(af[k][s][1], b[j][k][s], acc[j][1]);
      }
  if constexpr (sizeof(T) == 2) {
    // issue order: every LDS fragment read (B and, from an image, A), then the MFMAs — the reads overlap
    // each other instead of one read -> wait -> MFMA pair at a time
    __builtin_amdgcn_sched_group_barrier(0x100, NJ * 3 * NCC + (ALDS ? 6 * NCC : 0), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, NJ * 6 * NCC, 0);
  }
}

__device__ __forceinline__ f32x4 bias4(const float* b, int o) { return f32x4{b[o], b[o + 1], b[o + 2], b[o + 3]}; }

// ---------------------------------------------------------------------------------------------------
// 3 waves/SIMD for bf16 (<= 168 VGPRs without spilling); the fp32 parity build needs more registers
// forward K order: natural (false) keeps it bit-identical to the unfused gather kernels
// (the conflict-free K order here — the PMC shows 5.2 M LDS bank-conflict cycles per 3 launches at T = 32768
// without it — was measured 2-4 % faster per launch and equal on the step, so bit-identity stays)
constexpr bool kRsFwdKperm = false;

template <class T> constexpr int rs_fwd_waves() { return sizeof(T) == 2 ? 3 : 2; }

// Rows per tile: chosen so that the recomputed rows fill whole 16-row MFMA tiles over the 4 waves
// (forward: RT + 16 = 192 = 12 tiles; backward: round16(RT + 2d) <= 192 with RT a multiple of 32 for the
// K = rows weight-gradient products)
constexpr int rs_fwd_rt(int dt) { return dt > 0 ? 176 : RTM; }
// (192-row tiles for d <= 9 and 160 for d = 27 — fewer recomputed halo rows per output row — measured slower
// on the step: 7.59 / 7.53 vs 7.51 ms)
constexpr int rs_bwd_rt(int dt) { return (dt > 0 && dt <= 9) ? 160 : RTM; }

template <class T, int DT, int RT = rs_fwd_rt(DT)>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(rs_fwd_waves<T>(), 8)))
void resblock_fwd_kernel(ResArgs a) {
  constexpr int XS = rs_stride<T>(), HR = RT + 16, NT = RT / 16, NJ = (NT + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* X = (T*)smem;  // local j <-> row t0 - 1 - d + j, XR = HR + 2d rows (raw x)
  const int d = DT > 0 ? DT : a.d, XR = HR + 2 * d;
  T* H = X + XR * XS;  // local i <-> row t0 - 1 + i, relu(h)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tbeg = blockIdx.x * a.tpw + min((int)blockIdx.x, a.textra),
            tend = tbeg + a.tpw + ((int)blockIdx.x < a.textra);
  if (tbeg >= tend) return;
  typename Mfma<T>::frag wfa[3][2][rs_ncc<T>()], wfb[3][2][rs_ncc<T>()];
  if constexpr (sizeof(T) == 2 && DT > 0) {
    // the two conv images in the H region (2 x 96 rows of the tile's HR = 192), read before the prologue's barrier;
    // H is first written after it
    bf16* img = (bf16*)(X + (HR + 2 * DT) * XS);
    f32x4 va[3 * RC * RC / 4 / 256], vb[3 * RC * RC / 4 / 256];
    load_w4(va, a.wa);
    load_w4(vb, a.wb);
    stage_img<false>(img, va);
    stage_img<false>(img + kImgRows * kImgP, vb);
    __syncthreads();
    frags_from_img<kRsFwdKperm>(wfa, img);
    frags_from_img<kRsFwdKperm>(wfb, img + kImgRows * kImgP);
  } else {
    load_wfrags<T, kRsFwdKperm>(wfa, a.wa);
    load_wfrags<T, kRsFwdKperm>(wfb, a.wb);
  }
  const int pn = rs_pi(lane & 15), oc = rs_ocol(lane);
  f32x4 bav[2], bbv[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    bav[mt] = a.ba ? bias4(a.ba, oc + 4 * mt) : f32x4{0.f, 0.f, 0.f, 0.f};
    bbv[mt] = a.bb ? bias4(a.bb, oc + 4 * mt) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const unsigned ibytes = (unsigned)a.T * RC * (unsigned)sizeof(T);
  auto load_x = [&](Rows32Buf<T, rs_pv<T>()>& bx, const RsCursor& c) {
    bx.load(rs_rsrc((const T*)a.x + (size_t)c.n * a.T * RC, ibytes), c.tm * RT - 1 - d);
  };
  Rows32Buf<T, rs_pv<T>()> nx;
  nx.init(XR, (XR + HR) * XS);  // trash row after H
  RsCursor cur, ldc;  // the tile being computed; the tile being loaded (cur + 1 or + 2)
  cur.set(tbeg, a.ntm);
  ldc = cur;
  load_x(nx, ldc);
  nx.template store<false>(X);
  if (tbeg + 1 < tend) {
    ldc.next(a.ntm);
    load_x(nx, ldc);
  }
  __syncthreads();
  for (int tile = tbeg; tile < tend; ++tile, cur.next(a.ntm)) {
    const int n = cur.n, t0 = cur.tm * RT;
#ifdef VQA_RS_STAMPS
    const bool stamp_on = tile == tbeg + 4;
#endif
    RS_STAMP(0);
    // h rows t0-1 .. t0+RT+14 (conv_b reads t0-1 .. t0+RT); rows outside the item are conv_b's SAME zeros
    const bool interior = t0 - 1 >= 0 && t0 - 1 + HR <= a.T;  // uniform: no SAME-padding rows in h
    // y rows of this lane: n-tiles wave, wave+4, ... of RT/16; their residual x rows are read from X now, so
    // X is free for the next tile as soon as conv_a is done
    int ry[NJ];
    Raw8<T> xres[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      ry[j] = min(wave + 4 * j, NT - 1) * 16;
      xres[j].load(X + (ry[j] + pn + 1 + d) * XS + oc);
    }
    auto wa_frag = [&](int k, int mt, int sc) { return wfa[k][mt][sc]; };
    auto wb_frag = [&](int k, int mt, int sc) { return wfb[k][mt][sc]; };
    {
      // h n-tiles wave, wave+4, wave+8 of HR/16 (an out-of-range slot computes a valid tile, unstored)
      int rb[3];
      f32x4 acc[3][2];
#pragma unroll
      for (int j = 0; j < 3; ++j) rb[j] = min(wave + 4 * j, HR / 16 - 1) * 16;
      conv_multi<T, true, kRsFwdKperm, false, 3>(acc, wa_frag, X, rb, d, bav[0], bav[1]);  // bias-initialised
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (wave + 4 * j >= HR / 16) continue;
        const int i = rb[j] + pn, r = t0 - 1 + i;
        const bool live = interior || (r >= 0 && r < a.T);
        if constexpr (sizeof(T) == 2) {
          // round, then ReLU on the bf16 bits (identical to ReLU then round): 4 cvt + 4 packed max per 8
          uint4 u = __builtin_bit_cast(uint4, relu_frag(__builtin_bit_cast(bf16x8, bf16_bits(acc[j][0], acc[j][1]))));
          if (!interior && !live) u = uint4{0u, 0u, 0u, 0u};
          *(uint4*)(H + i * XS + oc) = u;
          // the tile's own rows 1..RT (rows >= T dropped by the range check)
          if (a.h && i >= 1 && i <= RT)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, u),
                                                   rs_rsrc((T*)a.h + (size_t)n * a.T * RC, ibytes),
                                                   (r * RC + oc) * (int)sizeof(T), 0, 0);
        } else {
          f32x4 v[2];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            v[mt] = acc[j][mt];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[mt][q] = live ? fmaxf(v[mt][q], 0.f) : 0.f;
          }
          st8(H + i * XS + oc, v[0], v[1]);
          if (a.h && i >= 1 && i <= RT)
            st8_buf<T>(rs_rsrc((T*)a.h + (size_t)n * a.T * RC, ibytes), (r * RC + oc) * (int)sizeof(T), v[0], v[1]);
        }
      }
    }
    RS_STAMP(1);
    __syncthreads();  // H complete; every read of X for this tile is done
    RS_STAMP(2);
    if (tile + 1 < tend) {
      nx.template store<false>(X);
      if (tile + 2 < tend) {
        ldc.next(a.ntm);
        load_x(nx, ldc);
      }
    }
    RS_STAMP(3);
    {
      const __amdgpu_buffer_rsrc_t yr = rs_rsrc((T*)a.y + (size_t)n * a.T * RC, ibytes);
      f32x4 acc[NJ][2];
      conv_multi<T, false, kRsFwdKperm, false, NJ>(acc, wb_frag, H, ry, 1, bbv[0], bbv[1]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (wave + 4 * j >= NT) continue;
        const int tl = ry[j] + pn;
        f32x4 x0, x1;
        xres[j].unpack(x0, x1);
        st8_buf<T>(yr, ((t0 + tl) * RC + oc) * (int)sizeof(T), x0 + acc[j][0], x1 + acc[j][1]);
      }
    }
    RS_STAMP(4);
    if (tile + 1 < tend) __syncthreads();  // every read of H done; the next tile's X is in LDS
    RS_STAMP(5);
  }
}

// ---------------------------------------------------------------------------------------------------
// Backward (h recomputed). DT > 0: the dilation as a compile-time constant (every LDS offset of the tile
// becomes an immediate); DT = 0: any dilation <= RMAXD from the arguments. The work between two barriers is
// split over two wave PAIRS ("teams"), so each weight gradient is accumulated by one pair over all 32 output
// channels: every transposed K = rows fragment read for a weight-gradient product feeds 2 MFMAs instead of 1
// (50 instead of 80 ds_read_b64_tr_b16 pairs per wave per tile), each wave holds two of the three
// weight-fragment sets, and dh has an LDS buffer of its own (the single-team form with dh written over relu(h)
// took 61.0 us where this takes 55.3, T = 32768, d = 9, bf16).
//   all waves      h = relu(conv_a(relu x))            -> H                (rows t0-d .. t0+RT+d)
//   team W (0, 1)  dW_b (input-channel tile = pair index, both output tiles) from H, Y;  then dx -> HBM
//   team H (2, 3)  dh = conv_b^T(dy) * (h > 0) -> D (its own buffer);                then dW_a from X, D
// Barriers per tile: H ready, D ready, every read done (then the next tile's staged rows are stored), the
// stored rows visible: four (the one-buffer form needs five).
// HALVES = 2 (not instantiated; measured 4 % slower on the step): a 512-thread workgroup whose two
// 4-wave halves run the same pipeline on their own tiles (even / odd offsets of the workgroup's range, each half its
// own LDS region) and add their weight gradients through LDS at the end in a fixed order. The product launches
// HALVES = 1, whose code the half logic compiles out of. (The LDS-DMA staged form measured in round 5 is in git
// history at 8432c5f.)
template <class T, int DT, int RT = rs_bwd_rt(DT), int HALVES = 1>
__global__ __launch_bounds__(256 * HALVES) void resblock_bwd_kernel(ResArgs a) {
  typedef Mfma<T> M;
  constexpr int NW = 4;
  constexpr int XS = rs_stride<T>(), NT = RT / 16;
  // dx n-tiles per team-W wave (interleaved), in batches NA1 + NA2 (a team-H share measured slower)
  constexpr int NA = (NT + 1) / 2, NA1 = NA < 3 ? NA : 3, NA2 = NA - NA1;
  static_assert(NA2 >= 1 && NA2 <= 3, "dx: two batches per team-W wave");
  constexpr int DM = DT > 0 ? DT : RMAXD, HRM = round16(RT + 2 * DM);
  // recomputed 16-row tiles: NP1 per wave for h (batches P1A + P1B), NDH per team-H wave for dh (DH1 + DH2 + DH3)
  constexpr int NHT = HRM / 16, NP1 = (NHT + 3) / 4, P1A = NP1 < 3 ? NP1 : 3, P1B = NP1 - P1A;
  constexpr int NDH = (NHT + 1) / 2, DH1 = NDH < 3 ? NDH : 3, DH2 = NDH - DH1 < 3 ? NDH - DH1 : 3,
                DH3 = NDH - DH1 - DH2;
  static_assert(P1B <= 3 && DH3 <= 3, "recomputed rows: at most 24 16-row tiles");
  constexpr int PVX = ((HRM + 2 * DM) * RC * (int)sizeof(T) / 16 + 64 * NW - 1) / (64 * NW);
  constexpr int PVY = ((HRM + 2) * RC * (int)sizeof(T) / 16 + 64 * NW - 1) / (64 * NW);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int d = DT > 0 ? DT : a.d, HR = round16(RT + 2 * d), XR = HR + 2 * d, YR = HR + 2;
  const int wave_g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = HALVES > 1 ? wave_g >> 2 : 0;
  // each half's LDS region: X, Y, H, D and the trash row (bwd_lds), 16-byte aligned
  const int half_elems = ((XR + YR + 2 * HR + 1) * XS * (int)sizeof(T) + 15) / 16 * 16 / (int)sizeof(T);
  T* X = (T*)smem + half * half_elems;  // local j <-> row t0 - 2d + j: relu(x)
  T* Y = X + XR * XS;  // local m <-> row t0 - d - 1 + m (dy)
  T* H = Y + YR * XS;  // local i <-> row t0 - d + i: relu(h)
  T* D = H + HR * XS;  // local i <-> row t0 - d + i: dh
  const int wave = wave_g & 3, lane = threadIdx.x & 63;  // wave within the half's pipeline
  const int team = wave >> 1, tw = wave & 1;  // team 0 = W, 1 = H; tw = the pair's input-channel tile
  const int tbeg = blockIdx.x * a.tpw + min((int)blockIdx.x, a.textra),
            tend = tbeg + a.tpw + ((int)blockIdx.x < a.textra);
  if (tbeg >= tend) return;
  // this half's tiles: tbeg + half, + HALVES, ...; every half runs niter iterations (barriers are workgroup-wide),
  // computing only while its tile exists
  const int niter = (tend - tbeg + HALVES - 1) / HALVES;
  auto adv = [&](RsCursor& c) {
#pragma unroll
    for (int h = 0; h < HALVES; ++h) c.next(a.ntm);
  };
  // conv_a's forward fragments (recompute h) on every wave; team W: conv_a^T (dx), team H: conv_b^T (dh)
  typename M::frag wfa[3][2][rs_ncc<T>()], wt[3][2][rs_ncc<T>()];
  if constexpr (sizeof(T) == 2) {
    // three images in the H and D regions (3 x 96 rows of their 2 HR >= 288): conv_a (every wave's wfa), conv_a and
    // conv_b transposed (team W's / team H's wt); read before the prologue's barrier, H / D first written after it
    bf16* img = (bf16*)H;
    f32x4 va[3 * RC * RC / 4 / 256], vb[3 * RC * RC / 4 / 256];
    load_w4(va, a.wa);
    load_w4(vb, a.wb);
    stage_img<false>(img, va);
    stage_img<true>(img + kImgRows * kImgP, va);
    stage_img<true>(img + 2 * kImgRows * kImgP, vb);
    __syncthreads();
    frags_from_img<true>(wfa, img);
    frags_from_img<true>(wt, img + (team == 0 ? 1 : 2) * kImgRows * kImgP);
  } else {
    load_wfrags<T, true>(wfa, a.wa);
    load_wfrags_t<T>(wt, team == 0 ? a.wa : a.wb);
  }
  const int pn = rs_pi(lane & 15), oc = rs_ocol(lane);
  f32x4 bav[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) bav[mt] = a.ba ? bias4(a.ba, oc + 4 * mt) : f32x4{0.f, 0.f, 0.f, 0.f};
  // this pair's weight gradient: [output tile][tap] for input-channel tile tw, and the bias of output tile tw
  f32x4 gw[2][3], gb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int k = 0; k < 3; ++k) gw[o][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nht = HR / 16;

  const unsigned ibytes = (unsigned)a.T * RC * (unsigned)sizeof(T);
  auto load_tile = [&](Rows32Buf<T, PVX>& bx, Rows32Buf<T, PVY>& by, const RsCursor& c) {
    const size_t o = (size_t)c.n * a.T * RC;
    bx.load(rs_rsrc((const T*)a.x + o, ibytes), c.tm * RT - 2 * d);
    by.load(rs_rsrc((const T*)a.dy + o, ibytes), c.tm * RT - d - 1);
  };
  Rows32Buf<T, PVX> nx;
  Rows32Buf<T, PVY> ny;
  nx.init(XR, (XR + YR + 2 * HR) * XS, (int)(threadIdx.x & 255));  // trash row after D
  ny.init(YR, (YR + 2 * HR) * XS, (int)(threadIdx.x & 255));
  RsCursor cur, ldc;
  cur.set(min(tbeg + half, tend - 1), a.ntm);
  ldc = cur;
  if (tbeg + half < tend) {
    load_tile(nx, ny, ldc);
    nx.template store<true>(X);
    ny.template store<false>(Y);
  }
  if (tbeg + half + HALVES < tend) {
    adv(ldc);
    load_tile(nx, ny, ldc);
  }
  __syncthreads();
  auto wt_frag = [&](int k, int mt, int sc) { return wt[k][mt][sc]; };
  for (int it = 0; it < niter; ++it, adv(cur)) {
    const int tile = tbeg + half + HALVES * it;
    const bool valid = HALVES == 1 || tile < tend;  // wave-uniform: this half has a tile this iteration
    const int n = cur.n, t0 = cur.tm * RT;
    const bool interior = t0 - d >= 0 && t0 - d + HR <= a.T;  // uniform: no SAME-padding rows
#ifdef VQA_RS_STAMPS
    const bool stamp_on = tile == tbeg + 4;
#endif
    RS_STAMP(0);
    // 1. relu(h) over the dh rows (zero outside the item): n-tiles wave + 4 (j0 + j)
    auto h_batch = [&](auto nj, int j0) {
      constexpr int NJB = decltype(nj)::value;
      int rh[NJB];
#pragma unroll
      for (int j = 0; j < NJB; ++j) rh[j] = min(wave + 4 * (j0 + j), nht - 1) * 16;
      f32x4 acc[NJB][2];
      conv_multi<T, false, true, false, NJB>(acc, [&](int k, int mt, int sc) { return wfa[k][mt][sc]; }, X, rh, d,
                                             bav[0], bav[1]);  // bias-initialised, as the forward
      if constexpr (sizeof(T) == 2) {
        // round, then ReLU on the bf16 bits (identical to ReLU then round): 4 cvt + 4 packed max per 8; the
        // SAME-padding rows of an edge tile are zeroed on a separate (wave-uniform) path
        auto store_h = [&](auto edge) {
#pragma unroll
          for (int j = 0; j < NJB; ++j) {
            if (wave + 4 * (j0 + j) >= nht) continue;
            const int i = rh[j] + pn;
            uint4 u = __builtin_bit_cast(uint4, relu_frag(__builtin_bit_cast(bf16x8, bf16_bits(acc[j][0], acc[j][1]))));
            if constexpr (decltype(edge)::value) {
              const int r = t0 - d + i;
              if (r < 0 || r >= a.T) u = uint4{0u, 0u, 0u, 0u};
            }
            *(uint4*)(H + i * XS + oc) = u;
          }
        };
        if (interior) store_h(std::false_type{});
        else store_h(std::true_type{});
      } else {
#pragma unroll
        for (int j = 0; j < NJB; ++j) {
          if (wave + 4 * (j0 + j) >= nht) continue;
          const int i = rh[j] + pn, r = t0 - d + i;
          const bool live = interior || (r >= 0 && r < a.T);
          f32x4 v[2];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            v[mt] = acc[j][mt];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[mt][q] = live ? fmaxf(v[mt][q], 0.f) : 0.f;
          }
          st8(H + i * XS + oc, v[0], v[1]);
        }
      }
    };
    if (valid) {
      h_batch(std::integral_constant<int, P1A>{}, 0);
      if constexpr (P1B > 0) h_batch(std::integral_constant<int, P1B>{}, P1A);
    }
    RS_STAMP(1);
    __syncthreads();
    RS_STAMP(2);
    if (!valid) {
    } else if (team == 0) {
      // 2W. dW_b[k][c][o] += sum_t relu(h)[t+k-1][c] dy[t][o] (c in tile tw, every o), db_b[o in tile tw]
#pragma unroll
      for (int kk = 0; kk < RT; kk += M::KS) {
        const typename M::frag b0 = rs_rows(Y + (d + 1 + kk) * XS, XS);
        const typename M::frag b1 = rs_rows(Y + (d + 1 + kk) * XS + 16, XS);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const typename M::frag af = rs_rows(H + (d + k - 1 + kk) * XS + tw * 16, XS);
          gw[0][k] = M::mma(af, b0, gw[0][k]);
          gw[1][k] = M::mma(af, b1, gw[1][k]);
        }
        gb = M::mma(M::ones(), tw ? b1 : b0, gb);
      }
    } else {
      // 2H. dh = conv_b^T(dy) * (h > 0) -> D: n-tiles tw + 2 (j0 + j)
      auto dh_batch = [&](auto nj, int j0) {
        constexpr int NJB = decltype(nj)::value;
        int rh[NJB], rb[NJB];
#pragma unroll
        for (int j = 0; j < NJB; ++j) {
          rh[j] = min(tw + 2 * (j0 + j), nht - 1) * 16;
          rb[j] = rh[j] + 2;
        }
        f32x4 dh[NJB][2];
        conv_multi<T, false, true, false, NJB>(dh, wt_frag, Y, rb, -1);
#pragma unroll
        for (int j = 0; j < NJB; ++j) {
          if (tw + 2 * (j0 + j) >= nht) continue;
          const int i = rh[j] + pn;
          if constexpr (sizeof(T) == 2) {
            // the mask on the rounded values: the same result as masking first
            *(uint4*)(D + i * XS + oc) = mask_pos8(bf16_bits(dh[j][0], dh[j][1]), *(const uint4*)(H + i * XS + oc));
          } else {
            bool hp[8];
            pos8(H + i * XS + oc, hp);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              dh[j][0][q] = hp[q] ? dh[j][0][q] : 0.f;
              dh[j][1][q] = hp[4 + q] ? dh[j][1][q] : 0.f;
            }
            st8(D + i * XS + oc, dh[j][0], dh[j][1]);
          }
        }
      };
      dh_batch(std::integral_constant<int, DH1>{}, 0);
      if constexpr (DH2 > 0) dh_batch(std::integral_constant<int, DH2>{}, DH1);
      if constexpr (DH3 > 0) dh_batch(std::integral_constant<int, DH3>{}, DH1 + DH2);
    }
    RS_STAMP(3);
    __syncthreads();
    RS_STAMP(4);
    // The next tile's staged rows (loaded a tile ago) are waited for HERE, before this tile's dx stores are issued.
    // vmcnt counts loads and stores in one queue: left to the compiler, the wait sits at the rows' register use at the
    // end of the tile — after team W's dx stores — and, its count merged over both teams' paths, also waits for
    // those stores' write acknowledgements (s_waitcnt vmcnt(0) there; every wave then idles at the next barrier).
    // A real s_waitcnt here (the builtin: the compiler's wait pass accounts for it) leaves the later use waitless.
    __builtin_amdgcn_s_waitcnt(kVmcnt0);
    RS_STAMP(5);
    // 3. dx = dy + conv_a^T(dh) * (x > 0) on the tile's rows, NJB n-tiles nt(j) at a time (nt(j) >= NT: none)
    const __amdgpu_buffer_rsrc_t dxr = rs_rsrc((T*)a.y + (size_t)n * a.T * RC, ibytes);
    auto dx_batch = [&](auto nj, auto nt, auto frag) {
      constexpr int NJB = decltype(nj)::value;
      int rb[NJB];
      f32x4 acc[NJB][2];
#pragma unroll
      for (int j = 0; j < NJB; ++j) rb[j] = min(nt(j), NT - 1) * 16 + 2 * d;
      conv_multi<T, false, true, false, NJB>(acc, frag, D, rb, -d);
#pragma unroll
      for (int j = 0; j < NJB; ++j) {
        if (nt(j) >= NT) continue;
        const int tl = nt(j) * 16 + pn;
        bool xp[8];
        f32x4 y0, y1;
        pos8(X + (tl + 2 * d) * XS + oc, xp);
        ld8(Y + (tl + d + 1) * XS + oc, y0, y1);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          y0[q] += xp[q] ? acc[j][0][q] : 0.f;
          y1[q] += xp[4 + q] ? acc[j][1][q] : 0.f;
        }
        st8_buf<T>(dxr, ((t0 + tl) * RC + oc) * (int)sizeof(T), y0, y1);  // rows >= T dropped
      }
    };
    if (!valid) {
    } else if (team == 0) {
      // 3W. n-tiles tw, tw + 2, ...
      dx_batch(std::integral_constant<int, NA1>{}, [&](int j) { return tw + 2 * j; }, wt_frag);
      dx_batch(std::integral_constant<int, NA2>{}, [&](int j) { return tw + 2 * (NA1 + j); }, wt_frag);
    } else {
      // 4H. dW_a[k][c][o] += sum_t relu(x)[t+(k-1)d][c] dh[t][o] (c in tile tw, every o), db_a[o in tile tw]
#pragma unroll
      for (int kk = 0; kk < RT; kk += M::KS) {
        const typename M::frag b0 = rs_rows(D + (d + kk) * XS, XS);
        const typename M::frag b1 = rs_rows(D + (d + kk) * XS + 16, XS);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const typename M::frag af = rs_rows(X + ((k + 1) * d + kk) * XS + tw * 16, XS);
          gw[0][k] = M::mma(af, b0, gw[0][k]);
          gw[1][k] = M::mma(af, b1, gw[1][k]);
        }
        gb = M::mma(M::ones(), tw ? b1 : b0, gb);
      }
    }
    RS_STAMP(6);
    if (it + 1 < niter) {
      __syncthreads();  // every read of X, Y, H and D for this tile is done
      if (tile + HALVES < tend) {
        nx.template store<true>(X);
        ny.template store<false>(Y);
      }
      if (tile + 2 * HALVES < tend) {
        adv(ldc);
        load_tile(nx, ny, ldc);
      }
      __syncthreads();
    }
    RS_STAMP(7);
  }
  if constexpr (HALVES > 1) {
    // the two halves' sums of the same gradient slice (same wave index) add in a fixed order: half 0 + half 1
    __syncthreads();  // every LDS read of the last tiles is done
    float* xch = (float*)smem + ((wave * 64 + lane) * 28);
    if (half == 1) {
#pragma unroll
      for (int o = 0; o < 2; ++o)
#pragma unroll
        for (int k = 0; k < 3; ++k) *(f32x4*)(xch + 4 * (3 * o + k)) = gw[o][k];
      *(f32x4*)(xch + 24) = gb;
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int k = 0; k < 3; ++k) gw[o][k] = gw[o][k] + *(const f32x4*)(xch + 4 * (3 * o + k));
    gb = gb + *(const f32x4*)(xch + 24);
  }
  // partial rows (team W: dW_b | db_b into part_b; team H: dW_a | db_a into part_a), Keras dW[k][c][o]
  float* pr = (team == 0 ? a.part_b : a.part_a) + (size_t)blockIdx.x * (3 * RC * RC + RC);
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pr[(k * RC + tw * 16 + 4 * (lane >> 4) + r) * RC + o * 16 + (lane & 15)] = gw[o][k][r];
  if (lane < 16) pr[3 * RC * RC + tw * 16 + lane] = gb[0];
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
// backward: tiles per workgroup at least (bounds the partial rows of short launches). 2 against 4, 3 and 1 in
// alternating same-box runs: 7.316 ms/step (5 runs) vs 7.363 (4), 7.355 (3), 7.369 (1): level 2's short launches
// (T <= 4096) are latency-bound chains of tiles per workgroup
constexpr int kResMinTiles = 2;

// + one trash row for the staging chunks past a tile's rows (Rows32Buf)
static size_t fwd_lds(int d, int esz, int rt) {
  const int s = RC + 16 / esz, HR = rt + 16;
  return ((size_t)(HR + 2 * d) * s + (size_t)HR * s + s) * esz;
}
// X (HR + 2d rows), Y (HR + 2), relu(h) and dh (HR each), the trash row
static size_t bwd_lds(int d, int esz, int rt) {
  const int s = RC + 16 / esz, HR = round16(rt + 2 * d);
  return ((size_t)(HR + 2 * d) * s + (size_t)(HR + 2) * s + (size_t)2 * HR * s + s) * esz;
}

static int set_lds(const void* fn, size_t bytes) {
  constexpr int NS = 32;
  static size_t done[NS] = {};
  static const void* fns[NS] = {};
  if (bytes <= 65536) return VQA_OK;
  int slot = 0;
  while (slot < NS - 1 && fns[slot] && fns[slot] != fn) ++slot;
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

// kernel instance for a dilation: the model's dilations (3^i, i < 4) are compiled constants
template <class T> struct RsFwd {
  template <int D> static const void* fn() { return (const void*)resblock_fwd_kernel<T, D>; }
};
template <class T> struct RsBwd {
  template <int D> static const void* fn() { return (const void*)resblock_bwd_kernel<T, D>; }
};
// the 128-row tile plan of d <= 9 (shorter launches: whole rounds of tiles per workgroup, see bwd_rt_for)
template <class T> struct RsBwd128 {
  template <int D> static const void* fn() { return (const void*)resblock_bwd_kernel<T, D, (D > 0 && D <= 9) ? 128 : rs_bwd_rt(D)>; }
};


template <class F> static const void* rs_pick(int d) {
  switch (d) {
    case 1: return F::template fn<1>();
    case 3: return F::template fn<3>();
    case 9: return F::template fn<9>();
    case 27: return F::template fn<27>();
    default: return F::template fn<0>();
  }
}

static int fwd_rt_of(int d) { return (d == 1 || d == 3 || d == 9 || d == 27) ? rs_fwd_rt(d) : RTM; }
static int bwd_rt_of(int d) { return (d == 1 || d == 3 || d == 9 || d == 27) ? rs_bwd_rt(d) : RTM; }
// rows per backward tile for a launch: d <= 9 items shorter than 8192 rows use 128-row tiles (whole
// 2-tile rounds per workgroup: 0.4-1.0 us faster per launch at T = 1024-4096; slower from T = 8192, where
// 160-row tiles keep less halo per row; profiles/r5_resblock_dma.txt)
static int bwd_rt_for(int d, int T) {
  return (d == 1 || d == 3 || d == 9) && T < 8192 ? 128 : bwd_rt_of(d);
}

static void plan(ResArgs& a, int per_cu, int rt, int min_tiles = 1) {
  a.ntm = (a.T + rt - 1) / rt;
  a.ntiles = a.ntm * a.B;
  // every slot gets floor(ntiles / nwg) tiles and the first (ntiles mod nwg) one more: workgroups w and
  // w + #CUs (dispatched to the same CU) never both hold an extra tile while extras <= #CUs
  a.nwg = std::min(rs_cus() * per_cu, std::max(1, a.ntiles / min_tiles));
  a.tpw = a.ntiles / a.nwg;
  a.textra = a.ntiles - a.tpw * a.nwg;
}

}  // namespace vqa

using namespace vqa;

#ifdef VQA_RS_STAMPS
extern "C" int vqa_rs_stamps(unsigned long long* host, int n) {
  const int m = std::min(n, kRsStampWgs * 4 * 8);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rs_stamps), (size_t)m * 8) == hipSuccess ? m : -1;
}
#endif

extern "C" int vqa_resblock_supported(int C, int dilation, int dtype) {
  if (C != RC || dilation < 1 || dilation > RMAXD || !(dtype == VQA_F32 || dtype == VQA_BF16)) return 0;
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  return bwd_lds(dilation, esz, bwd_rt_of(dilation)) <= 160 * 1024 &&
         fwd_lds(dilation, esz, fwd_rt_of(dilation)) <= 160 * 1024;
}

extern "C" int vqa_resblock_fwd(const void* x, const float* wa, const float* ba, const float* wb, const float* bb,
                                void* y, void* h_out, int B, int T, int C, int dilation, int dtype,
                                vqa_stream_t stream) {
  VQA_ARG(x && wa && wb && y && B > 0 && T > 0, "resblock_fwd: bad arguments");
  VQA_REQUIRE(vqa_resblock_supported(C, dilation, dtype), VQA_E_UNSUPPORTED,
              "resblock_fwd: unsupported C=%d dilation=%d dtype=%d", C, dilation, dtype);
  VQA_ARG((long long)T * C * 4 < (1ll << 30), "resblock_fwd: item too long for 32-bit buffer offsets (T=%d)", T);
  ResArgs a{x, nullptr, y, h_out, wa, ba, wb, bb, nullptr, nullptr, B, T, dilation, 0, 0, 0, 0, 0};
  plan(a, 3, fwd_rt_of(dilation));
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  // one LDS reservation for every dilation (the largest plan)
  const size_t lds = std::max(fwd_lds(RMAXD, esz, RTM), fwd_lds(27, esz, rs_fwd_rt(27)));
  const hipStream_t s = (hipStream_t)stream;
  const dim3 grid(a.nwg);
  const void* fn = dtype == VQA_BF16 ? rs_pick<RsFwd<bf16>>(dilation) : rs_pick<RsFwd<float>>(dilation);
  if (int rc = set_lds(fn, lds)) return rc;
  void* args[] = {&a};
  (void)hipLaunchKernel(fn, grid, dim3(256), args, lds, s);
  VQA_LAUNCHED("resblock_fwd_kernel");
  return VQA_OK;
}

extern "C" size_t vqa_resblock_bwd_workspace(int B, int T, int C, int dilation, int dtype) {
  if (C < 1) return 0;
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
  ResArgs a{x, dy, dx, nullptr, wa, ba, wb, nullptr, (float*)workspace, nullptr, B, T, dilation, 0, 0, 0, 0, 0};
  // at least kResMinTiles tiles per workgroup: a workgroup's weight-gradient partial row (2 x 3,104 fp32) is
  // larger than a tile's activations, so short launches use fewer, longer-lived workgroups
  const int esz = dtype == VQA_BF16 ? 2 : 4;
  const hipStream_t s = (hipStream_t)stream;
  const int rt = bwd_rt_for(dilation, T);
  plan(a, kResPerCU, rt, kResMinTiles);
  a.part_b = a.part_a + (size_t)a.nwg * E;
  const size_t lds = bwd_lds(dilation, esz, rt);
  size_t lds_max = bwd_lds(RMAXD, esz, RTM);  // one reservation for every dilation (the largest plan)
  for (int dd : {1, 3, 9, 27}) lds_max = std::max(lds_max, bwd_lds(dd, esz, rs_bwd_rt(dd)));
  const void* fn = rt != bwd_rt_of(dilation)
                       ? (dtype == VQA_BF16 ? rs_pick<RsBwd128<bf16>>(dilation) : rs_pick<RsBwd128<float>>(dilation))
                       : (dtype == VQA_BF16 ? rs_pick<RsBwd<bf16>>(dilation) : rs_pick<RsBwd<float>>(dilation));
  if (int rc = set_lds(fn, lds_max)) return rc;
  void* args[] = {&a};
  (void)hipLaunchKernel(fn, dim3(a.nwg), dim3(256), args, lds, s);
  VQA_LAUNCHED("resblock_bwd_kernel");
  const int nwg = a.nwg;
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
