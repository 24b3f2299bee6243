#include "vqa_mfma.h"
#include <cstdio>
using namespace vqa;
__global__ void k(const bf16* in, bf16* out) {
  bf16x8 f = *(const bf16x8*)(in + 8 * threadIdx.x);
  f = relu_frag(f);
  *(bf16x8*)(out + 8 * threadIdx.x) = f;
}
int main() {
  const int n = 64 * 8;
  bf16 h[n], o[n];
  for (int i = 0; i < n; ++i) h[i] = (bf16)((i % 7) - 3.0f + 0.25f * (i % 3));
  bf16 *din, *dout;
  hipMalloc(&din, n * 2); hipMalloc(&dout, n * 2);
  hipMemcpy(din, h, n * 2, hipMemcpyHostToDevice);
  k<<<1, 64>>>(din, dout);
  hipMemcpy(o, dout, n * 2, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) { float a = (float)h[i], b = (float)o[i]; if (b != (a > 0 ? a : 0)) { if (bad < 8) printf("i=%d in=%f out=%f\n", i, a, b); ++bad; } }
  printf("bad=%d\n", bad);
  return 0;
}
