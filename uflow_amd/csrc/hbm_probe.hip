// hbm_probe.hip -- the read-only streaming ceiling the bench reports beside the gate's roofline
// ("also report a measured read-only streaming ceiling from a trivial kernel
// for context").  Not part of the CRC path: it reads a buffer as one contiguous stream -- each wave a
// contiguous range of 1-KB steps, 16 B per lane per step, 4 steps in flight, non-temporal loads --
// and XOR-folds the data so the loads stay live.  One workgroup of 8 waves per CU, like the gate.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "frame_crc_kernels.hpp"

namespace ufc_dev {

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kProbeWaves = 8;
constexpr int kProbeDepth = 4;

__global__ __launch_bounds__(kProbeWaves * 64) void read_stream_kernel(const uint8_t* bytes, uint64_t nsteps,
                                                                          uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t W = gridDim.x * kProbeWaves;
  const uint32_t w = blockIdx.x * kProbeWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t lo = nsteps * w / W, hi = nsteps * (w + 1) / W;
  uint32_t acc = 0;
  v4u data[kProbeDepth];
#pragma unroll
  for (int i = 0; i < kProbeDepth; i++) data[i] = (v4u){0, 0, 0, 0};
  for (uint64_t k = lo; k < hi; k += kProbeDepth) {
#pragma unroll
    for (int s = 0; s < kProbeDepth; s++) {
      const uint64_t kk = k + s < hi ? k + s : hi - 1;
      const v4u v = __builtin_nontemporal_load((const v4u*)(bytes + kk * 1024 + 16 * lane));
      acc ^= data[s].x ^ data[s].y ^ data[s].z ^ data[s].w;
      data[s] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < kProbeDepth; i++) acc ^= data[i].x ^ data[i].y ^ data[i].z ^ data[i].w;
  // one vector atomic per wave (lane 0 after a wave XOR): the result is never read, it only keeps
  // the loads from being dead code
  for (int off = 32; off > 0; off >>= 1) acc ^= __shfl_xor(acc, off);
  if (lane == 0) atomicXor(sink, acc);
}

}  // namespace

int read_stream(const uint8_t* bytes, uint64_t nbytes, uint32_t* sink, int ncu, void* stream) {
  const uint64_t nsteps = nbytes / 1024;
  if (nsteps == 0) return (int)hipSuccess;
  hipLaunchKernelGGL(read_stream_kernel, dim3((unsigned)ncu), dim3(kProbeWaves * 64), 0, (hipStream_t)stream, bytes,
                     nsteps, sink);
  return (int)hipGetLastError();
}

}  // namespace ufc_dev
