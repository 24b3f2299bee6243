// Does hipOccupancyMaxActiveBlocksPerMultiprocessor(fn, 256, L) depend on the kernel's
// MaxDynamicSharedMemorySize attribute set earlier (process history), for the same L? (GPU dev tool)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(256) void dummy(float* o) {
  extern __shared__ float s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (o) o[threadIdx.x] = s[255 - threadIdx.x];
}
static int occ(size_t lds) {
  int nb = -1;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)dummy, 256, lds);
  if (e != hipSuccess) { (void)hipGetLastError(); return -100 - (int)e; }
  return nb;
}
int main() {
  const size_t Ls[] = {16384, 40960, 54000, 70000};
  printf("before any attribute:");
  for (size_t L : Ls) printf("  L=%zu -> %d", L, occ(L));
  printf("\n");
  for (int attr : {70000, 100000, 160000}) {
    hipError_t e = hipFuncSetAttribute((const void*)dummy, hipFuncAttributeMaxDynamicSharedMemorySize, attr);
    printf("attribute %d (%s):", attr, hipGetErrorString(e));
    for (size_t L : Ls) printf("  L=%zu -> %d", L, occ(L));
    printf("\n");
  }
  return 0;
}
