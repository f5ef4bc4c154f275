// VALU / LDS issue-rate probe (not product code): independent v_perm/v_bitop3 streams, and
// ds_read_b32 streams with the lane-replicated table pattern, at 16 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void probe(unsigned* out, int iters) {
  __shared__ __attribute__((aligned(16))) unsigned lds[40960];
  for (int i = threadIdx.x; i < 40960; i += 1024) lds[i] = i * 2654435761u;
  __syncthreads();
  unsigned a = threadIdx.x, b = a * 7 + 1, c = a * 13 + 5, d = a ^ 0x55, e = a + 99, f = a * 3, g = a ^ 0xF0F0, h = ~a;
  const unsigned K = ((threadIdx.x & 31) * 4) | (((threadIdx.x & 31) * 4 + 128) << 8) | (1u << 24);
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {  // 8 independent v_bitop3 chains, 8 instrs per iteration
      a = __builtin_amdgcn_bitop3_b32(a, b, it, 0x96); b = __builtin_amdgcn_bitop3_b32(b, c, it, 0x96);
      c = __builtin_amdgcn_bitop3_b32(c, d, it, 0x96); d = __builtin_amdgcn_bitop3_b32(d, e, it, 0x96);
      e = __builtin_amdgcn_bitop3_b32(e, f, it, 0x96); f = __builtin_amdgcn_bitop3_b32(f, g, it, 0x96);
      g = __builtin_amdgcn_bitop3_b32(g, h, it, 0x96); h = __builtin_amdgcn_bitop3_b32(h, a, it, 0x96);
    } else if (MODE == 1) {  // 8 independent v_perm chains
      a = __builtin_amdgcn_perm(a, b, 0x01020304u + it); b = __builtin_amdgcn_perm(b, c, 0x01020304u + it);
      c = __builtin_amdgcn_perm(c, d, 0x01020304u + it); d = __builtin_amdgcn_perm(d, e, 0x01020304u + it);
      e = __builtin_amdgcn_perm(e, f, 0x01020304u + it); f = __builtin_amdgcn_perm(f, g, 0x01020304u + it);
      g = __builtin_amdgcn_perm(g, h, 0x01020304u + it); h = __builtin_amdgcn_perm(h, a, 0x01020304u + it);
    } else if (MODE == 2) {  // chain-step shape: 4 perm + 4 ds_read + 2 bitop3, 2 independent chains
      const char* t = (const char*)lds + 32768;
      unsigned r0 = *(const unsigned*)(t + __builtin_amdgcn_perm(a, K, 0x0C020400u));
      unsigned r1 = *(const unsigned*)(t + __builtin_amdgcn_perm(a, K, 0x0C020501u));
      unsigned r2 = *(const unsigned*)(t + __builtin_amdgcn_perm(a, K, 0x0C030600u));
      unsigned r3 = *(const unsigned*)(t + __builtin_amdgcn_perm(a, K, 0x0C030701u));
      unsigned s0 = *(const unsigned*)(t + __builtin_amdgcn_perm(b, K, 0x0C020400u));
      unsigned s1 = *(const unsigned*)(t + __builtin_amdgcn_perm(b, K, 0x0C020501u));
      unsigned s2 = *(const unsigned*)(t + __builtin_amdgcn_perm(b, K, 0x0C030600u));
      unsigned s3 = *(const unsigned*)(t + __builtin_amdgcn_perm(b, K, 0x0C030701u));
      a = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(r0, r1, r2, 0x96), r3, it, 0x96);
      b = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(s0, s1, s2, 0x96), s3, it, 0x96);
    } else {  // ds_read only: 8 independent reads per iteration, addresses from the lane copy pattern
      const char* t = (const char*)lds + 32768;
      unsigned x0 = *(const unsigned*)(t + ((a & 0xFF00u) | (K & 0xFF)));
      unsigned x1 = *(const unsigned*)(t + ((b & 0xFF00u) | (K & 0xFF)));
      unsigned x2 = *(const unsigned*)(t + ((c & 0xFF00u) | (K & 0xFF)));
      unsigned x3 = *(const unsigned*)(t + ((d & 0xFF00u) | (K & 0xFF)));
      unsigned x4 = *(const unsigned*)(t + ((e & 0xFF00u) | (K & 0xFF)));
      unsigned x5 = *(const unsigned*)(t + ((f & 0xFF00u) | (K & 0xFF)));
      unsigned x6 = *(const unsigned*)(t + ((g & 0xFF00u) | (K & 0xFF)));
      unsigned x7 = *(const unsigned*)(t + ((h & 0xFF00u) | (K & 0xFF)));
      a ^= x0; b ^= x1; c ^= x2; d ^= x3; e ^= x4; f ^= x5; g ^= x6; h ^= x7;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

int main() {
  unsigned* o; CK(hipMalloc(&o, 256 * 1024 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int dev; hipDeviceProp_t prop; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&prop, dev));
  printf("clock %d kHz, CUs %d\n", prop.clockRate, prop.multiProcessorCount);
  auto run = [&](const char* nm, auto k, int iters, double instr_per_iter) {
    k<<<256, 1024>>>(o, iters); CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 7; r++) { CK(hipEventRecord(e0)); k<<<256, 1024>>>(o, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms); }
    std::sort(ts.begin(), ts.end());
    double ms = ts[3];
    double winstr = instr_per_iter * iters * 16.0;  // wave-instructions per CU
    double cyc = ms * 1e-3 * 2.4e9;
    printf("%-34s %.3f ms  wave-instr/CU/cycle @2.4GHz = %.3f  (cycles per wave-instr per SIMD = %.2f)\n", nm, ms, winstr / cyc, 4.0 * cyc / winstr);
    fflush(stdout);
  };
  run("bitop3 x8 indep", probe<0>, 20000, 8);
  run("perm x8 indep", probe<1>, 20000, 8);
  run("chain-step x2 (8 ds_read, 10 valu)", probe<2>, 20000, 18);
  run("ds_read_b32 x8 (+8 valu)", probe<3>, 20000, 16);
  return 0;
}
