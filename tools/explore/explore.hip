// Design-space exploration for the frame-CRC kernel on gfx950 (not product code).
// Measures (a) HBM read efficiency of the candidate per-lane access patterns and
// (b) throughput of candidate CRC kernels, checked against a CPU bytewise CRC.
// Build: hipcc --offload-arch=gfx950 -O3 -o explore explore.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

static const uint32_t POLY_R = 0x9960034Cu;   // reflected 0x132c00699 (crc.rs:50)

// ---------------- host tables ----------------
static uint32_t T_ref[256];      // crc.rs PARTIAL_RESULTS semantics
static uint32_t L[4][256];       // linear (register-domain) slice-by-4 tables
static void build_tables() {
  for (int i = 0; i < 256; i++) {
    uint32_t r = ~0u ^ (uint32_t)i;               // extend_slow(0,[i]) : reg = !0 ^ byte
    for (int b = 0; b < 8; b++) r = (r & 1) ? (r >> 1) ^ POLY_R : (r >> 1);
    T_ref[i] = ~r;
    uint32_t v = (uint32_t)i;                     // linear table: step8 of byte with reg 0
    for (int b = 0; b < 8; b++) v = (v & 1) ? (v >> 1) ^ POLY_R : (v >> 1);
    L[0][i] = v;
  }
  for (int k = 1; k < 4; k++)
    for (int i = 0; i < 256; i++) { uint32_t v = L[k-1][i]; L[k][i] = (v >> 8) ^ L[0][v & 0xff]; }
}
static uint32_t crc_cpu(const uint8_t* d, size_t n) {
  uint32_t c = 0;
  for (size_t i = 0; i < n; i++) c = (c >> 8) ^ T_ref[(uint8_t)(c ^ d[i])];
  return c;
}

// ---------------- device helpers ----------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__global__ void fill_kernel(uint64_t* p, size_t nwords, uint64_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t st = (size_t)gridDim.x * blockDim.x;
  for (; i < nwords; i += st) p[i] = splitmix64(seed ^ (i * 0x2545F4914F6CDD1Dull));
}

// M1: fully coalesced dwordx4 stream (each wave-instruction reads 1 KiB contiguous).
__global__ __launch_bounds__(256) void m_coalesced(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t T = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  #pragma unroll 4
  for (size_t i = t; i < n16; i += T) { uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  out[t] = acc;
}

// Mk: lane reads a contiguous chunk of CHUNK16 x 16 B at byte offset frame*stride + part*chunkbytes.
template <int PARTS, int CHUNK16>
__global__ __launch_bounds__(256) void m_chunk(const uint8_t* __restrict__ base, size_t stride, int nframes, uint32_t* out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  int f = t / PARTS, part = t % PARTS;
  if (f >= nframes) return;
  const uint8_t* q = base + (size_t)f * stride + (size_t)part * (1496 / PARTS / 4 * 4);
  uint32_t acc = 0;
  #pragma unroll 8
  for (int i = 0; i < CHUNK16; i++) {
    const uint32_t* w = (const uint32_t*)(q + 16 * i);
    uint4 v = *(const uint4*)w;
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[t] = acc;
}

// ---------------- candidate CRC kernel C1 ----------------
// lane per frame, direct dwordx4 loads, slice-by-4 linear tables in LDS replicated 32x
// (entry e of table k for copy c at byte k*32768 + e*128 + c*4 -> conflict-free ds_read_b32).
__device__ __forceinline__ uint32_t lds_ld(const char* lds, uint32_t byteoff) {
  return *(const uint32_t*)(lds + byteoff);
}
__device__ __forceinline__ uint32_t step4(const char* lds, uint32_t r, uint32_t c4) {
  uint32_t a0 = ((r << 7) & 0x7F80u) | c4;
  uint32_t a1 = ((r >> 1) & 0x7F80u) | c4;
  uint32_t a2 = ((r >> 9) & 0x7F80u) | c4;
  uint32_t a3 = ((r >> 17) & 0x7F80u) | c4;
  return lds_ld(lds, a0 + 3 * 32768) ^ lds_ld(lds, a1 + 2 * 32768) ^ lds_ld(lds, a2 + 32768) ^ lds_ld(lds, a3);
}

template <int FPL>
__global__ __launch_bounds__(1024) void c1_lane_per_frame(const uint8_t* __restrict__ base, size_t stride,
    int nframes, const uint32_t* __restrict__ gtab, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  uint32_t* l32 = (uint32_t*)lds;
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    int k = i >> 13, e = (i >> 5) & 255;
    l32[i] = gtab[k * 256 + e];
  }
  __syncthreads();
  const uint32_t c4 = (threadIdx.x & 31) * 4;
  int T = gridDim.x * blockDim.x;
  for (int f0 = blockIdx.x * blockDim.x + threadIdx.x; f0 < nframes; f0 += T * FPL) {
    uint32_t r[FPL];
    const uint8_t* q[FPL];
    #pragma unroll
    for (int j = 0; j < FPL; j++) {
      int f = f0 + j * T; if (f >= nframes) f = nframes - 1;
      q[j] = base + (size_t)f * stride; r[j] = 0xFFFFFFFFu;
    }
    // 1496 bytes = 93 x 16 + 8
    #pragma unroll 2
    for (int i = 0; i < 93; i++) {
      uint4 v[FPL];
      #pragma unroll
      for (int j = 0; j < FPL; j++) v[j] = *(const uint4*)(q[j] + 16 * i);
      #pragma unroll
      for (int j = 0; j < FPL; j++) {
        r[j] = step4(lds, r[j] ^ v[j].x, c4);
        r[j] = step4(lds, r[j] ^ v[j].y, c4);
        r[j] = step4(lds, r[j] ^ v[j].z, c4);
        r[j] = step4(lds, r[j] ^ v[j].w, c4);
      }
    }
    #pragma unroll
    for (int j = 0; j < FPL; j++) {
      uint2 v = *(const uint2*)(q[j] + 16 * 93);
      r[j] = step4(lds, r[j] ^ v.x, c4);
      r[j] = step4(lds, r[j] ^ v.y, c4);
      int f = f0 + j * T;
      if (f < nframes) out[f] = ~r[j];
    }
  }
}

// C2: 4 lanes per frame (contiguous 376-byte chunks with an 8-byte zero front pad),
// combine across the 4 lanes by multiplying with A^376 (advance 376 zero bytes) using
// a second (unreplicated) set of 4 tables.
__device__ __forceinline__ uint32_t mulK(const uint32_t* K, uint32_t r) {
  return K[r & 0xff] ^ K[256 + ((r >> 8) & 0xff)] ^ K[512 + ((r >> 16) & 0xff)] ^ K[768 + (r >> 24)];
}
__global__ __launch_bounds__(1024) void c2_quad_per_frame(const uint8_t* __restrict__ base, size_t stride,
    int nframes, const uint32_t* __restrict__ gtab, const uint32_t* __restrict__ gK, uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  uint32_t* l32 = (uint32_t*)lds;
  uint32_t* K = (uint32_t*)(lds + 131072);
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    int k = i >> 13, e = (i >> 5) & 255;
    l32[i] = gtab[k * 256 + e];
  }
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) K[i] = gK[i];
  __syncthreads();
  const uint32_t c4 = (threadIdx.x & 31) * 4;
  int T = gridDim.x * blockDim.x;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < nframes * 4; t += T) {
    int f = t >> 2, part = t & 3;
    // virtual frame = 8 zero bytes || 1496 data bytes = 1504 = 4 x 376; part p covers virtual [376p, 376p+376)
    const uint8_t* q = base + (size_t)f * stride + 376 * part - 8;
    uint32_t r = 0;
    // 376 = 8 + 23 x 16; part 0's first 8 virtual bytes are the zero pad (skip: r stays 0)
    uint2 h = part ? *(const uint2*)q : make_uint2(0u, 0u);
    r = step4(lds, r ^ h.x, c4);
    r = step4(lds, r ^ h.y, c4);
    const uint32_t inj = part ? 0u : 0xFFFFFFFFu;   // init ~0 folded into the first data word
    #pragma unroll 4
    for (int i = 0; i < 23; i++) {
      uint4 v = *(const uint4*)(q + 8 + 16 * i);
      if (i == 0) v.x ^= inj;
      r = step4(lds, r ^ v.x, c4);
      r = step4(lds, r ^ v.y, c4);
      r = step4(lds, r ^ v.z, c4);
      r = step4(lds, r ^ v.w, c4);
    }
    // tree: level1 pairs (0,1),(2,3): v = r_even*K ^ r_odd ; level2: v01*K^2 ^ v23
    uint32_t up = __shfl_xor(r, 1, 4);
    uint32_t v1 = (part & 1) ? (mulK(K, up) ^ r) : 0;     // valid on odd lanes
    uint32_t up2 = __shfl_xor(v1, 2, 4);
    uint32_t v2 = mulK(K, mulK(K, up2)) ^ v1;             // valid on lane 3
    if (part == 3) out[f] = ~v2;
  }
}

static void fill(uint8_t* d, size_t bytes, uint64_t seed) {
  fill_kernel<<<4096, 256>>>((uint64_t*)d, bytes / 8, seed);
  CK(hipGetLastError());
}

int main(int argc, char** argv) {
  build_tables();
  // check KAT
  const char* kat = "123456789";
  printf("KAT crc(\"123456789\") = %08X (expect 11A6F2A3)\n", crc_cpu((const uint8_t*)kat, 9));
  const int N = argc > 1 ? atoi(argv[1]) : 1000000;
  const size_t STRIDE = 1500;
  const size_t bytes = (size_t)N * STRIDE + 4096;
  uint8_t* d; CK(hipMalloc(&d, bytes));
  fill(d, bytes, 0x5EED0001);
  uint32_t* dout; CK(hipMalloc(&dout, sizeof(uint32_t) * (size_t)N * 4 + (1 << 22)));
  uint32_t* dtab; CK(hipMalloc(&dtab, 4 * 256 * 4));
  CK(hipMemcpy(dtab, L, sizeof(L), hipMemcpyHostToDevice));
  // K = A^376 as 4 byte tables: K[k][e] = advance (e << 8k) by 376 zero bytes
  std::vector<uint32_t> Kt(1024);
  for (int k = 0; k < 4; k++) for (int e = 0; e < 256; e++) {
    uint32_t v = (uint32_t)e << (8 * k);
    for (int s = 0; s < 376; s++) v = (v >> 8) ^ L[0][v & 0xff];
    Kt[k * 256 + e] = v;
  }
  uint32_t* dK; CK(hipMalloc(&dK, 4096));
  CK(hipMemcpy(dK, Kt.data(), 4096, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)c1_lane_per_frame<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)c1_lane_per_frame<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)c2_quad_per_frame, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));

  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double algo_bytes, auto launch) {
    launch(); CK(hipGetLastError()); CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int rep = 0; rep < 15; rep++) {
      CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    float med = ts[ts.size() / 2];
    printf("%-40s median %8.3f ms  min %8.3f ms  %8.1f GB/s (%.3f of 8 TB/s)\n", name, med, ts[0],
           algo_bytes / med / 1e6, algo_bytes / med / 1e6 / 8000.0);
    fflush(stdout);
  };
  const double fb = (double)N * 1500.0;
  size_t n16 = (size_t)N * STRIDE / 16;
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64]; snprintf(nm, 64, "M1 coalesced grid=%d", g);
    timeit(nm, (double)n16 * 16, [&] { m_coalesced<<<g, 256>>>((const uint4*)d, n16, dout); });
  }
  timeit("M lane-per-frame (93x16B)", fb, [&] { m_chunk<1, 93><<<(N + 255) / 256, 256>>>(d, STRIDE, N, dout); });
  timeit("M 2 lanes/frame (47x16B)", fb, [&] { m_chunk<2, 47><<<(N * 2 + 255) / 256, 256>>>(d, STRIDE, N, dout); });
  timeit("M 4 lanes/frame (24x16B)", fb, [&] { m_chunk<4, 24><<<(N * 4 + 255) / 256, 256>>>(d, STRIDE, N, dout); });
  timeit("M 16 lanes/frame (6x16B)", fb, [&] { m_chunk<16, 6><<<(N * 16 + 255) / 256, 256>>>(d, STRIDE, N, dout); });

  int ncu = 256;
  std::vector<uint8_t> hframes((size_t)4096 * STRIDE);
  CK(hipMemcpy(hframes.data(), d, hframes.size(), hipMemcpyDeviceToHost));
  std::vector<uint32_t> hout(4096);
  auto check = [&](const char* name) {
    CK(hipMemcpy(hout.data(), dout, 4096 * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int f = 0; f < 4096; f++) if (hout[f] != crc_cpu(&hframes[(size_t)f * STRIDE], 1496)) bad++;
    printf("  check %s: %d/4096 mismatches\n", name, bad);
  };
  for (int thr : {512, 1024}) {
    char nm[64]; snprintf(nm, 64, "C1 lane/frame FPL1 thr=%d", thr);
    timeit(nm, fb, [&] { c1_lane_per_frame<1><<<ncu, thr, 131072>>>(d, STRIDE, N, dtab, dout); });
    check(nm);
    snprintf(nm, 64, "C1 lane/frame FPL2 thr=%d", thr);
    timeit(nm, fb, [&] { c1_lane_per_frame<2><<<ncu, thr, 131072>>>(d, STRIDE, N, dtab, dout); });
    check(nm);
  }
  for (int thr : {512, 1024}) {
    char nm[64]; snprintf(nm, 64, "C2 quad/frame thr=%d", thr);
    timeit(nm, fb, [&] { c2_quad_per_frame<<<ncu, thr, 131072 + 4096>>>(d, STRIDE, N, dtab, dK, dout); });
    check(nm);
  }
  printf("done\n");
  return 0;
}
