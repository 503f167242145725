// PMC calibration for the coder's access shapes: every launch reads or writes exactly
// n_chunks x 64 KiB.  Two families:
//  * per-lane ("lane B"): one 64 KiB chunk per lane, read or written in per-lane bursts of B
//    consecutive 16-B granules (B = 1: 16-B granules; B = 4: both coders' 64-B bursts; B = 8:
//    whole 128-B lines), with coder-like pacing between bursts;
//  * coalesced ("coal"): lane i of every wave-instruction touches 16 B at 16 i of a contiguous
//    1 KiB run, the streaming shape MI355X_MICROARCH.md calibrates FETCH_SIZE / WRITE_SIZE on
//    (the anchor: its reads are counted at 1/2 by FETCH_SIZE, its writes exactly by WRITE_SIZE).
// Run each counter pass under rocprofv3 --pmc (tools/profile.sh does) and divide the known byte
// count by the counted bytes: tools/pmc_calib.py prints the factor per shape and counter set.
// Build:  hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int B, bool WRITE>
__global__ __launch_bounds__(256) void k_calib(uint4* buf, uint64_t chunk16, uint32_t* sink) {
  const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint4* p = buf + k * chunk16;
  uint32_t acc = (uint32_t)k;
  for (uint64_t g = 0; g < chunk16; g += B) {
    if (WRITE) {
#pragma unroll
      for (int b = 0; b < B; ++b) p[g + b] = make_uint4(acc, (uint32_t)g, b, 7);
    } else {
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const uint4 v = p[g + b];
        acc ^= v.x + v.y * 3 + v.z * 5 + v.w;
      }
    }
    for (int i = 0; i < 4 * B; ++i) acc = acc * 1664525u + 1013904223u;  // coder-like pacing
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// coalesced: the grid sweeps the buffer in 1 KiB wave-instructions, 16 per wave per round
template <bool WRITE>
__global__ __launch_bounds__(256) void k_calib_coal(uint4* buf, uint64_t n16, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t acc = threadIdx.x;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
    if (WRITE) {
      buf[i] = make_uint4(acc, (uint32_t)i, 3, 7);
    } else {
      const uint4 v = buf[i];
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint64_t n = 1 << 18, chunk = 65536, chunk16 = chunk / 16;
  uint4* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, n * chunk) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
  if (hipMemset(buf, 1, n * chunk) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
#define RUN(B, W)                                                                          \
  hipLaunchKernelGGL((k_calib<B, W>), dim3(n / 256), dim3(256), 0, 0, buf, chunk16, sink); \
  if (hipDeviceSynchronize() != hipSuccess) return 2;
#define RUNC(W)                                                                              \
  hipLaunchKernelGGL((k_calib_coal<W>), dim3(256 * 16), dim3(256), 0, 0, buf, n * chunk16, \
                     sink);                                                                  \
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  RUN(1, false) RUN(4, false) RUN(8, false) RUN(1, true) RUN(4, true) RUN(8, true)
  RUNC(false) RUNC(true)
  printf("bytes_per_launch %llu\n", (unsigned long long)(n * chunk));
  return hipFree(buf) != hipSuccess || hipFree(sink) != hipSuccess;
}
