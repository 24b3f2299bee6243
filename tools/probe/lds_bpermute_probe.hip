// Do cross-lane shuffles of a kernel WITHOUT an LDS allocation return wrong data — and does another kernel's LDS
// change under them — when both run at the same time on the GPU? (GPU dev tool, round 5)
//
// P kernels (one per variant) run a long chain of integer shuffles whose exact result the host computes:
//   bperm      __shfl_xor / __shfl (ds_bpermute_b32), no LDS allocation — what vqa_dtail_fwd does
//   bperm_lds  the same shuffles with 256 B of LDS allocated (and touched) by the workgroup
//   dpp        the same permutations by DPP (quad_perm, row_mirror): VALU, no LDS crossbar
// The L kernel fills 64 KiB of LDS per workgroup with a pattern, reads it back permuted, counts mismatches.
//   lds_bpermute_probe VARIANT NSTREAMS_L REPS [LDS_KIB]     (NSTREAMS_L = 0: P alone; VARIANT none: L only)
// LDS_KIB: the L kernel's LDS per workgroup (default 64; gfx950 allows up to 160 KiB per workgroup).
// P runs on one stream, L on NSTREAMS_L others, concurrently, REPS times; prints wrong P results and L mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr int ITERS = 2048, BLOCKS = 2048, THREADS = 256;
static int g_lwords = 16384;  // LDS words per L workgroup (power of two)

__device__ __forceinline__ unsigned mix(unsigned x) { x ^= x >> 15; x *= 0x2c1b3c6dU; x ^= x >> 12; return x; }
static unsigned hmix(unsigned x) { x ^= x >> 15; x *= 0x2c1b3c6dU; x ^= x >> 12; return x; }

template <int MODE>  // 0 bperm, 1 bperm_lds, 2 dpp
__global__ __launch_bounds__(THREADS) void chain(unsigned* out, unsigned seed) {
  const int lane = threadIdx.x & 63;
  __shared__ unsigned pad[MODE == 1 ? 64 : 1];
  if (MODE == 1) {
    pad[lane] = (unsigned)lane;
    __syncthreads();
  }
  unsigned v = mix(seed ^ (blockIdx.x * THREADS + threadIdx.x));
  for (int i = 0; i < ITERS; ++i) {
    unsigned a, b, c;
    if (MODE == 2) {
      a = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]: lane ^ 1
      b = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]: lane ^ 2
      c = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror: 15 - (lane & 15)
    } else {
      a = __shfl_xor(v, 1, 64);
      b = __shfl_xor(v, 2, 64);
      c = __shfl(v, (lane & ~15) | (15 - (lane & 15)), 64);
    }
    v = mix(v + 3 * a + 5 * b + 7 * c + (unsigned)lane + (unsigned)i);
  }
  if (MODE == 1) v += pad[lane] - (unsigned)lane;  // 0: keeps the allocation live
  out[blockIdx.x * THREADS + threadIdx.x] = v;
}

__global__ __launch_bounds__(256) void lds_check(unsigned* bad, int rounds, unsigned seed, int lwords) {
  extern __shared__ unsigned L[];
  unsigned miss = 0;
  for (int r = 0; r < rounds; ++r) {
    const unsigned key = seed * 0x9E3779B9u + blockIdx.x * 7919u + (unsigned)r;
    for (int w = threadIdx.x; w < lwords; w += 256) L[w] = mix(key ^ (unsigned)w);
    __syncthreads();
    for (int w = threadIdx.x; w < lwords; w += 256) {
      const int q = (w * 97 + r) % lwords;
      miss += L[q] != mix(key ^ (unsigned)q);
    }
    __syncthreads();
  }
  if (miss) atomicAdd(bad, miss);
}

int main(int argc, char** argv) {
  const char* var = argc > 1 ? argv[1] : "bperm";
  const int nl = argc > 2 ? atoi(argv[2]) : 2, reps = argc > 3 ? atoi(argv[3]) : 10;
  const int mode = !strcmp(var, "bperm") ? 0 : !strcmp(var, "bperm_lds") ? 1 : !strcmp(var, "dpp") ? 2 : 3;
  if (argc > 4) g_lwords = atoi(argv[4]) * 256;
  const size_t n = (size_t)BLOCKS * THREADS;
  std::vector<unsigned> want(n);
  for (size_t w = 0; w < n / 64; ++w) {
    unsigned v[64], nv[64];
    for (int l = 0; l < 64; ++l) v[l] = hmix(1234u ^ (unsigned)(w * 64 + l));
    for (int i = 0; i < ITERS; ++i) {
      for (int l = 0; l < 64; ++l) {
        const unsigned a = v[l ^ 1], b = v[l ^ 2], c = v[(l & ~15) | (15 - (l & 15))];
        nv[l] = hmix(v[l] + 3 * a + 5 * b + 7 * c + (unsigned)l + (unsigned)i);
      }
      for (int l = 0; l < 64; ++l) v[l] = nv[l];
    }
    for (int l = 0; l < 64; ++l) want[w * 64 + l] = v[l];
  }
  (void)hipFuncSetAttribute((const void*)lds_check, hipFuncAttributeMaxDynamicSharedMemorySize, g_lwords * 4);
  std::vector<hipStream_t> st(1 + nl);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  unsigned *dp, *dbad;
  (void)hipMalloc(&dp, n * 4);
  (void)hipMalloc(&dbad, 4);
  (void)hipMemset(dbad, 0, 4);
  std::vector<unsigned> got(n);
  long long pbad = 0, pruns = 0;
  for (int r = 0; r < reps; ++r) {
    for (int s = 1; s <= nl; ++s)
      hipLaunchKernelGGL(lds_check, dim3(1024), dim3(256), g_lwords * 4, st[s], dbad, 1500, (unsigned)(r * 16 + s),
                         g_lwords);
    for (int k = 0; k < (mode == 3 ? 0 : 4); ++k) {
      if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(BLOCKS), dim3(THREADS), 0, st[0], dp, 1234u);
      if (mode == 1) hipLaunchKernelGGL(chain<1>, dim3(BLOCKS), dim3(THREADS), 0, st[0], dp, 1234u);
      if (mode == 2) hipLaunchKernelGGL(chain<2>, dim3(BLOCKS), dim3(THREADS), 0, st[0], dp, 1234u);
      (void)hipStreamSynchronize(st[0]);
      (void)hipMemcpy(got.data(), dp, n * 4, hipMemcpyDeviceToHost);
      long long b = 0;
      for (size_t i = 0; i < n; ++i) b += got[i] != want[i];
      pbad += b;
      ++pruns;
      if (b) printf("rep %d launch %d: %lld of %zu P threads wrong\n", r, k, b, n);
    }
    (void)hipDeviceSynchronize();
  }
  unsigned lbad = 0;
  (void)hipMemcpy(&lbad, dbad, 4, hipMemcpyDeviceToHost);
  printf("lds_bpermute_probe %s beside %d LDS streams of %d KiB: %lld P launches, %lld wrong P thread results; "
         "L mismatches %u\n", var, nl, g_lwords / 256, pruns, pbad, lbad);
  return 0;
}
