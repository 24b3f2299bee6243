// vqa_mfma.h — MFMA fragment traits and bit-level ReLU helpers shared by the conv kernels (gfx950).
#pragma once
#include "vqa_common.h"

namespace vqa {

// MFMA fragment traits. bf16: v_mfma_f32_16x16x32_bf16 (8 consecutive channels per lane, one
// 16-byte LDS read). fp32: v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain; used for parity runs).
template <class T> struct Mfma;
template <> struct Mfma<bf16> {
  static constexpr int KS = 32;
  typedef bf16x8 frag;
  static __device__ __forceinline__ int koff(int lane) { return 8 * (lane >> 4); }
  static __device__ __forceinline__ frag load(const bf16* p) { return *(const bf16x8*)p; }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // 8 elements with a row stride (strided LDS gather; used by the weight-gradient kernel)
  static __device__ __forceinline__ frag gather(const bf16* p, int stride) {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = p[j * stride];
    return f;
  }
  static __device__ __forceinline__ frag ones() {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (bf16)1.0f;
    return f;
  }
  // operand whose K index runs down the rows of a row-major LDS tile: lane l gets rows 8(l>>4) .. +7 of
  // column l&15 from `o` = &tile[row0][col0] — two ds_read_b64_tr_b16 (cdna_hip_programming.md T10);
  // the caller keeps EXEC full and the row stride a multiple of 8 bytes
  static __device__ __forceinline__ frag rows(const bf16* o, int stride) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    const int l = threadIdx.x & 63, i = l & 15;
    const bf16* a0 = o + (8 * (l >> 4) + (i >> 2)) * stride + 4 * (i & 3);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0 + 4 * stride));
    typedef short v8s __attribute__((ext_vector_type(8)));
    return __builtin_bit_cast(frag, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
  // the same 32 rows under another K order: lanes 0-31 take the even rows, lanes 32-63 the odd rows. Both
  // operands of a product must use the same order. With a row stride of 20 or 36 dwords (32 or 64 bf16
  // channels + 16 B of padding) each read is free of bank conflicts (rows() is 2-way there).
  static __device__ __forceinline__ frag rows_eo(const bf16* o, int stride) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const bf16* a0 = o + (2 * (4 * (g & 1) + (i >> 2)) + (g >> 1)) * stride + 4 * (i & 3);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a0);
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a0 + 16 * stride));
    typedef short v8s __attribute__((ext_vector_type(8)));
    return __builtin_bit_cast(frag, (v8s)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
};
template <> struct Mfma<float> {
  static constexpr int KS = 4;
  typedef float frag;
  static __device__ __forceinline__ int koff(int lane) { return lane >> 4; }
  static __device__ __forceinline__ frag load(const float* p) { return *p; }
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag gather(const float* p, int) { return *p; }
  static __device__ __forceinline__ frag ones() { return 1.0f; }
  static __device__ __forceinline__ frag rows(const float* o, int stride) {
    const int l = threadIdx.x & 63;
    return o[(l >> 4) * stride + (l & 15)];
  }
  static __device__ __forceinline__ frag rows_eo(const float* o, int stride) { return rows(o, stride); }
};

template <class T> __device__ __forceinline__ void relu_bits(uint4& v);
template <> __device__ __forceinline__ void relu_bits<bf16>(uint4& v) {
  uint32_t* w = (uint32_t*)&v;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] &= ~(((w[i] >> 15) & 0x00010001u) * 0xFFFFu);
}
template <> __device__ __forceinline__ void relu_bits<float>(uint4& v) {
  uint32_t* w = (uint32_t*)&v;
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] &= ~(uint32_t)((int32_t)w[i] >> 31);
}

template <class T> constexpr int lds_pad() { return 16 / (int)sizeof(T); }

// ReLU of 8 bf16 lanes: a bf16 is negative iff its int16 is — one packed integer max per dword
// (written per component: a subscripted vector element in an unrolled loop miscompiled to lane 0 only)
__device__ __forceinline__ unsigned relu_pk2_bf16(unsigned w) {
  typedef short v2s __attribute__((ext_vector_type(2)));
  const v2s z = {0, 0};
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(__builtin_bit_cast(v2s, w), z));
}
__device__ __forceinline__ bf16x8 relu_frag(bf16x8 f) {
  const uint4 u = __builtin_bit_cast(uint4, f);
  return __builtin_bit_cast(bf16x8, uint4{relu_pk2_bf16(u.x), relu_pk2_bf16(u.y), relu_pk2_bf16(u.z),
                                           relu_pk2_bf16(u.w)});
}
__device__ __forceinline__ float relu_frag(float f) {
  const int32_t b = __float_as_int(f);
  return __int_as_float(b & ~(b >> 31));
}

}  // namespace vqa
