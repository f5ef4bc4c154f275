// trailer_probe.hip -- what does one trailer write per frame cost, by alignment?  (tuning probe for the
// variable-length seal; not product code)
//
// Config 3's batch shape (10M frames of U[64,1500] B, 7.8 GB, CSR; the lanes probe's offsets), one
// thread per frame writing 4 bytes at its trailer, in frame order, with nothing else running:
//   unaligned   a dword store at the trailer itself (the product's store; 3 in 4 trailers are not
//               4-byte aligned);
//   aligned     a dword store at the trailer rounded down to 4 B (wrong bytes: cost only);
//   aligned x2  the two aligned dwords covering the trailer (one dwordx2 store);
//   fixed       a dword store at every 1500th byte's trailer of a 1M-frame batch (config 2's pattern)
//               for the per-write rate of the fixed seal;
//   block B     the whole aligned B-byte block (B = 16, 32, 64, 128) holding the trailer's first byte,
//               B / 16 lanes per frame, one dwordx4 each (does a full-sector write skip the memory's
//               read-modify-write of a partial one?).
// Prints one line per variant (median of 9 launches; writes per second).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32_a1 __attribute__((aligned(1)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_a4 __attribute__((aligned(4)));

__global__ void w_unaligned(uint8_t* bytes, const uint64_t* off, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *(u32_a1*)(bytes + off[i + 1] - 4) = 0x11A6F2A3u ^ i;
}
__global__ void w_aligned(uint8_t* bytes, const uint64_t* off, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *(uint32_t*)(bytes + ((off[i + 1] - 4) & ~3ull)) = 0x11A6F2A3u ^ i;
}
__global__ void w_aligned2(uint8_t* bytes, const uint64_t* off, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    *(u32x2_a4*)(bytes + ((off[i + 1] - 4) & ~3ull)) = (u32x2){i, ~i};
  }
}
__global__ void w_fixed(uint8_t* bytes, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *(uint32_t*)(bytes + (uint64_t)i * 1500 + 1496) = 0x11A6F2A3u ^ i;
}

template <int B>
__global__ void w_block(uint8_t* bytes, const uint64_t* off, uint32_t n) {
  constexpr uint32_t T = B / 16;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x, i = g / T, c = g % T;
  if (i < n) {
    uint8_t* a = bytes + ((off[i + 1] - 4) & ~(uint64_t)(B - 1)) + 16 * c;
    *(uint4*)a = make_uint4(i, ~i, c, 0x11A6F2A3u);
  }
}

int main() {
  const uint32_t n = 10000000;
  std::vector<uint64_t> off(n + 1, 0);
  uint64_t x = 0x5EED0002;
  for (uint32_t i = 0; i < n; i++) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    off[i + 1] = off[i] + 64 + (x >> 33) % 1437;
  }
  const uint64_t total = off[n];
  uint8_t* bytes;
  uint64_t* doff;
  if (hipMalloc(&bytes, total + 4096) != hipSuccess || hipMalloc(&doff, 8 * (n + 1)) != hipSuccess) return 1;
  (void)hipMemset(bytes, 0x3C, total + 4096);
  (void)hipMemcpy(doff, off.data(), 8 * (n + 1), hipMemcpyHostToDevice);
  printf("trailer probe: %u frames, %.3f GB\n", n, total / 1e9);
  const uint32_t nf = 1000000;
  struct V {
    const char* name;
    uint32_t writes;
    int k;
  } vs[] = {{"unaligned", n, 0}, {"aligned", n, 1}, {"aligned x2", n, 2}, {"fixed 1M x 1500", nf, 3},
                {"block 16", n, 16}, {"block 32", n, 32}, {"block 64", n, 64}, {"block 128", n, 128}};
  auto launch = [&](int k) {
    switch (k) {
      case 0: hipLaunchKernelGGL(w_unaligned, dim3((n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      case 1: hipLaunchKernelGGL(w_aligned, dim3((n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      case 2: hipLaunchKernelGGL(w_aligned2, dim3((n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      case 3: hipLaunchKernelGGL(w_fixed, dim3((nf + 255) / 256), dim3(256), 0, 0, bytes, nf); break;
      case 16: hipLaunchKernelGGL(w_block<16>, dim3((n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      case 32: hipLaunchKernelGGL(w_block<32>, dim3((2 * n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      case 64: hipLaunchKernelGGL(w_block<64>, dim3((4 * n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
      default: hipLaunchKernelGGL(w_block<128>, dim3((8 * n + 255) / 256), dim3(256), 0, 0, bytes, doff, n); break;
    }
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int i = 0; i < 300; i++) launch(0);  // settle: clocks ramp up from idle
  (void)hipDeviceSynchronize();
  for (int round = 0; round < 2; round++)
    for (auto& v : vs) {
      for (int w = 0; w < 3; w++) launch(v.k);
      std::vector<float> t;
      for (int r = 0; r < 9; r++) {
        (void)hipEventRecord(e0, 0);
        launch(v.k);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
          printf("%s failed\n", v.name);
          return 1;
        }
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      const float med = t[t.size() / 2];
      printf("round %d  %-16s median %.4f ms  %.1f G writes/s\n", round, v.name, med, v.writes / med / 1e6);
      fflush(stdout);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
