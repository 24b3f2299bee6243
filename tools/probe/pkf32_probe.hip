// Do packed-FP32 VALU instructions (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) give different results from run
// to run while MFMA-heavy kernels of other queues share the CUs? (GPU dev tool, round 5)
//   pkf32_probe pk NSTREAMS_M REPS       (NSTREAMS_M = 0: P alone)
// P: every thread runs a long chain of float2 multiply-adds (ext_vector float2 arithmetic -> v_pk_*_f32); its first
// launch (alone) is the reference, every later launch (beside M on NSTREAMS_M streams) must equal it bitwise.
// M: bf16 MFMA chains (16x16x32) from an LDS tile. The control binary pkf32_probe_nopk is the same source built
// with -Xclang -target-feature -Xclang -packed-fp32-ops (the same arithmetic as v_fma_f32 / v_mul_f32 / v_add_f32).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096, BLOCKS = 4096, THREADS = 256;

template <bool PK>
__global__ __launch_bounds__(THREADS) void chain(float* out, float seed) {
  const int t = blockIdx.x * THREADS + threadIdx.x;
  const float a0 = seed + (float)(t & 1023) * 1e-3f, b0 = 1.f - (float)(t >> 10) * 1e-4f;
  if constexpr (PK) {
    f32x2 v = {a0, b0}, c = {0.999f, 1.0001f}, d = {1e-3f, -1e-3f};
    for (int i = 0; i < ITERS; ++i) {
      v = v * c + d;             // v_pk_fma_f32 (or mul + add)
      v = v * v * f32x2{0.5f, 0.5f} + f32x2{0.25f, 0.75f};
    }
    out[2 * t] = v.x;
    out[2 * t + 1] = v.y;
  } else {
    float x = a0, y = b0;
    for (int i = 0; i < ITERS; ++i) {
      x = __builtin_fmaf(x, 0.999f, 1e-3f);
      y = __builtin_fmaf(y, 1.0001f, -1e-3f);
      x = __builtin_fmaf(x * x, 0.5f, 0.25f);
      y = __builtin_fmaf(y * y, 0.5f, 0.75f);
    }
    out[2 * t] = x;
    out[2 * t + 1] = y;
  }
}

__global__ __launch_bounds__(256) void mfma_load(float* sink, int rounds) {
  __shared__ __attribute__((aligned(16))) __bf16 tile[64 * 40];
  const int lane = threadIdx.x & 63;
  for (int e = threadIdx.x; e < 64 * 40; e += 256) tile[e] = (__bf16)(float)((e * 7 + blockIdx.x) & 15);
  __syncthreads();
  f32x4 acc[4] = {};
  for (int r = 0; r < rounds; ++r) {
    const bf16x8 a = *(const bf16x8*)(tile + (lane & 15) * 40 + 8 * (lane >> 4));
    const bf16x8 b = *(const bf16x8*)(tile + (16 + (lane & 15)) * 40 + 8 * (lane >> 4));
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[k], 0, 0, 0);
  }
  if (acc[0][0] == 12345.f) sink[blockIdx.x] = acc[1][0] + acc[2][0] + acc[3][0];
}

int main(int argc, char** argv) {
  const bool pk = argc < 2 || !strcmp(argv[1], "pk");
  const int nm = argc > 2 ? atoi(argv[2]) : 2, reps = argc > 3 ? atoi(argv[3]) : 10;
  const size_t n = (size_t)BLOCKS * THREADS * 2;
  std::vector<hipStream_t> st(1 + nm);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  float *dp, *sink;
  (void)hipMalloc(&dp, n * 4);
  (void)hipMalloc(&sink, 1 << 16);
  auto launch = [&]() {
    if (pk) hipLaunchKernelGGL(chain<true>, dim3(BLOCKS), dim3(THREADS), 0, st[0], dp, 0.25f);
    else hipLaunchKernelGGL(chain<false>, dim3(BLOCKS), dim3(THREADS), 0, st[0], dp, 0.25f);
  };
  std::vector<float> ref(n), got(n);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(ref.data(), dp, n * 4, hipMemcpyDeviceToHost);
  long long bad = 0, runs = 0;
  for (int r = 0; r < reps; ++r) {
    for (int s = 1; s <= nm; ++s) hipLaunchKernelGGL(mfma_load, dim3(2048), dim3(256), 0, st[s], sink, 200000);
    for (int k = 0; k < 4; ++k) {
      launch();
      (void)hipStreamSynchronize(st[0]);
      (void)hipMemcpy(got.data(), dp, n * 4, hipMemcpyDeviceToHost);
      long long b = 0;
      for (size_t i = 0; i < n; ++i) b += memcmp(&got[i], &ref[i], 4) != 0;
      bad += b;
      ++runs;
      if (b) printf("rep %d launch %d: %lld of %zu values differ\n", r, k, b, n);
    }
    (void)hipDeviceSynchronize();
  }
  printf("pkf32_probe %s beside %d MFMA streams: %lld launches, %lld differing values\n", pk ? "pk" : "scalar", nm,
         runs, bad);
  return 0;
}
