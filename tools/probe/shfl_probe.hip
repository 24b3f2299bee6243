// Do cross-lane shuffles (ds_bpermute_b32, what __shfl_xor compiles to here) ever return wrong data when other
// work shares the GPU? (GPU dev tool.) Every thread runs a long chain of integer shuffles whose exact result is
// known on the host; the program launches it on NSTREAMS streams at once, REPS times, and counts threads whose
// result differs from the expected value. Integer arithmetic only: any difference is a wrong shuffle result.
//   shfl_probe NSTREAMS REPS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int ITERS = 4096, BLOCKS = 2048, THREADS = 256;

__device__ __forceinline__ unsigned mix(unsigned x) { x ^= x >> 15; x *= 0x2c1b3c6dU; x ^= x >> 12; return x; }

__global__ __launch_bounds__(THREADS) void chain(unsigned* out, unsigned seed) {
  const int lane = threadIdx.x & 63;
  unsigned v = mix(seed ^ (blockIdx.x * THREADS + threadIdx.x));
  for (int i = 0; i < ITERS; ++i) {
    const unsigned a = __shfl_xor(v, 1, 64), b = __shfl_xor(v, 2, 64), c = __shfl_xor(v, 16 + (i & 15), 64);
    v = mix(v + 3 * a + 5 * b + 7 * c + (unsigned)lane + (unsigned)i);
  }
  out[blockIdx.x * THREADS + threadIdx.x] = v;
}

static unsigned hmix(unsigned x) { x ^= x >> 15; x *= 0x2c1b3c6dU; x ^= x >> 12; return x; }

int main(int argc, char** argv) {
  const int ns = argc > 1 ? atoi(argv[1]) : 1, reps = argc > 2 ? atoi(argv[2]) : 10;
  const size_t n = (size_t)BLOCKS * THREADS;
  // expected results on the host, one wave of 64 lanes at a time
  std::vector<unsigned> want(n);
  for (size_t w = 0; w < n / 64; ++w) {
    unsigned v[64], nv[64];
    for (int l = 0; l < 64; ++l) v[l] = hmix(1234u ^ (unsigned)(w * 64 + l));
    for (int i = 0; i < ITERS; ++i) {
      for (int l = 0; l < 64; ++l) {
        const unsigned a = v[l ^ 1], b = v[l ^ 2], c = v[l ^ (16 + (i & 15))];
        nv[l] = hmix(v[l] + 3 * a + 5 * b + 7 * c + (unsigned)l + (unsigned)i);
      }
      for (int l = 0; l < 64; ++l) v[l] = nv[l];
    }
    for (int l = 0; l < 64; ++l) want[w * 64 + l] = v[l];
  }
  std::vector<hipStream_t> st(ns);
  std::vector<unsigned*> d(ns);
  for (int s = 0; s < ns; ++s) {
    (void)hipStreamCreate(&st[s]);
    (void)hipMalloc(&d[s], n * 4);
  }
  std::vector<unsigned> got(n);
  long long bad = 0, runs = 0;
  for (int r = 0; r < reps; ++r) {
    for (int s = 0; s < ns; ++s) hipLaunchKernelGGL(chain, dim3(BLOCKS), dim3(THREADS), 0, st[s], d[s], 1234u);
    for (int s = 0; s < ns; ++s) {
      (void)hipStreamSynchronize(st[s]);
      (void)hipMemcpy(got.data(), d[s], n * 4, hipMemcpyDeviceToHost);
      long long b = 0;
      for (size_t i = 0; i < n; ++i) b += got[i] != want[i];
      bad += b;
      ++runs;
      if (b) printf("rep %d stream %d: %lld of %zu threads wrong\n", r, s, b, n);
    }
  }
  printf("shfl_probe: %d streams x %d reps = %lld launches, %lld wrong thread results\n", ns, reps, runs, bad);
  return 0;
}
