// Workgroups per CU the runtime reports for a 256-thread kernel by dynamic LDS
// size (is a tile at the 160 KiB / 5 edge really 5 per CU?).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) probe_kernel(int* out) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (out) out[threadIdx.x] = lds[255 - threadIdx.x];
}

int main() {
  const int sizes[] = {30000, 31000, 31232, 31744, 32000, 32256, 32512, 32768, 33000, 40960, 40961};
  for (int s : sizes) {
    int blocks = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, probe_kernel, 256, s);
    std::printf("{\"dynamic_lds\": %d, \"blocks_per_cu\": %d, \"err\": %d}\n", s, blocks, (int)e);
  }
  return 0;
}
