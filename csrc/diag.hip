// Diagnostics: a CU-occupying stand-in for a concurrent collective kernel.
//
// In overlapped DP (sharetrade/trainer/engine.py::_overlap_step) RCCL's all-reduce kernel of step t
// runs beside step t+1's fused kernel; each of its workgroups holds a CU whose LDS the step kernel's
// one-workgroup-per-CU launch (~159 KiB) then cannot use.  `occupy_kernel` reproduces that on a
// single GPU: `grid` workgroups, each holding 4 KiB of LDS for `usec` microseconds (s_memrealtime,
// 100 MHz), so tools/overlap_rehearsal.py can time the static vs dynamic chunk schedule with k CUs
// taken away for T us per step.  Bounded: every wave exits after usec (or 2^24 polls).
#include "common.h"

namespace st {

__global__ void __launch_bounds__(64) occupy_kernel(int usec, int* sink) {
  __shared__ int hold[1024];   // 4 KiB: no co-residency with the step kernel's workgroup
  hold[threadIdx.x] = (int)threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long ticks = (unsigned long long)usec * 100ull;
  int polls = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks && polls < (1 << 24)) {
    __builtin_amdgcn_s_sleep(2);
    ++polls;
  }
  __syncthreads();
  if (threadIdx.x == 0 && hold[63] == -1) sink[blockIdx.x] = polls;   // keeps `hold` live
}

}  // namespace st

extern "C" hipError_t st_occupy(int grid, int usec, int* sink, hipStream_t stream) {
  if (grid < 1 || grid > 4096 || usec < 0 || usec > 100000) return hipErrorInvalidValue;
  hipLaunchKernelGGL(st::occupy_kernel, dim3(grid), dim3(64), 0, stream, usec, sink);
  return hipGetLastError();
}
