// Diagnostic (tools/ix_order.py): occupy `blocks` one-wave workgroup slots (with `lds` bytes of LDS
// each, like a resident warm-up wave) for `ticks` of the constant wall clock (100 MHz) while issuing
// almost nothing (s_sleep), to tell slot occupancy apart from issue contention.
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(64) occupy_kernel(long long ticks, int* sink) {
  extern __shared__ int lds[];
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
  if (threadIdx.x == 0 && ticks < 0) sink[blockIdx.x] = lds[0];  // never taken; keeps the LDS request
}

extern "C" int occupy(int blocks, int lds, long long ticks, int* sink, void* stream) {
  hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(64), lds, (hipStream_t)stream, ticks, sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
