// Hardware/runtime probes used by tests and tools (not on the training hot path).
//  * lds_probe: every block fills `bytes` of dynamic LDS with a block-unique pattern, waits, then
//    re-reads it; any mismatch means the LDS range is not private to the block (e.g. a dynamic
//    allocation above the runtime's per-block limit aliasing a co-resident block).
#include <stdexcept>
#include <string>

#include "common.h"

namespace {
__global__ void lds_probe_kernel(int words, int* errors, int spin) {
  extern __shared__ __attribute__((aligned(16))) int lds_words[];
  const unsigned tag = (blockIdx.x * 2654435761u) ^ 0x5bd1e995u;
  for (int i = threadIdx.x; i < words; i += blockDim.x) lds_words[i] = (int)(tag + (unsigned)i);
  __syncthreads();
  long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  __syncthreads();
  int bad = 0;
  for (int i = threadIdx.x; i < words; i += blockDim.x)
    if (lds_words[i] != (int)(tag + (unsigned)i)) ++bad;
  if (bad) atomicAdd(errors, bad);
}
}  // namespace

void dtf_lds_probe(int bytes, int blocks, int* errors, int spin, hipStream_t st) {
  hipLaunchKernelGGL(lds_probe_kernel, dim3(blocks), dim3(256), (size_t)bytes, st, bytes / 4,
                     errors, spin);
}

int dtf_max_dynamic_lds(int dev) {
  int v = 0;
  hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
  return v;
}
