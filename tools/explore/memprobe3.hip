// Memory probe 3 (exploration, not product code): loads-only streaming over 1M x 1500-B frames with
// the lane->address patterns a frame-CRC kernel could use.  One 1024-thread workgroup per CU owning
// a contiguous range of 4-frame sets; wave w of a workgroup takes sets lo + w, lo + w + 16, ...
// (the order the lean kernel's claims produce); NBUF sets in flight per wave.
//   frame16  : 16 lanes per frame, 256-B runs right-aligned to the frame end (the lean kernel)
//   frame16a : the same, addresses rounded down to 16 B
//   frame16p : frame16 with lanes wholly in the pad reading a fixed L2-resident line
//   frame32  : 32 lanes per frame, 512-B runs right-aligned (2 frames per instruction)
//   contig   : the set's 6000 bytes as contiguous 1 KiB wave-instructions (6 per set, 16-B aligned)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s line %d\n", hipGetErrorString(e_), __LINE__);          \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 g_u32x4;

enum Pat { kFrame16 = 0, kFrame16a = 1, kFrame16p = 2, kFrame32 = 3, kContig = 4 };

template <int PAT, int NBUF, bool NT>
__global__ __launch_bounds__(1024) void probe(const uint8_t* __restrict__ base, int nsets, const uint8_t* safe,
                                              uint32_t* out) {
  constexpr int NI = 6;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int WPB = blockDim.x >> 6;
  const int lo = (int)((int64_t)nsets * blockIdx.x / gridDim.x);
  const int hi = (int)((int64_t)nsets * (blockIdx.x + 1) / gridDim.x);
  uint32_t acc = 0;
  uint4 buf[NBUF][NI];
  auto addr = [&](int q, int j) -> const uint8_t* {
    const int qc = min(q, nsets - 1);
    const int64_t sb = (int64_t)qc * 6000;
    if (PAT == kContig) return base + sb + 1024 * j + 16 * lane;
    if (PAT == kFrame32) {
      // instruction j: frames 2*(j/3) + (lane>>5), block j%3 of 3 (1536-B virtual stream, pad 36)
      const int f = 2 * (j / 3) + (lane >> 5), b = j % 3;
      return base + sb + 1500 * f - 36 + 512 * b + 16 * (lane & 31);
    }
    const int f = lane >> 4, col = lane & 15;
    const uint8_t* a = base + sb + 1500 * f - 36 + 256 * j + 16 * col;
    if (PAT == kFrame16a) return (const uint8_t*)((uintptr_t)a & ~(uintptr_t)15);
    if (PAT == kFrame16p && j == 0 && col < 2) return safe + 16 * col;
    return a;
  };
  auto load = [&](int q, uint4 (&x)[NI]) {
#pragma unroll
    for (int j = 0; j < NI; j++) {
      const g_u32x4* p = (const g_u32x4*)addr(q, j);
      const u32x4 v = NT ? __builtin_nontemporal_load(p) : *p;
      x[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  int q = lo + wid;
#pragma unroll
  for (int b = 0; b < NBUF - 1; b++) load(q + WPB * b, buf[b]);
  for (; q < hi; q += WPB * NBUF) {
#pragma unroll
    for (int b = 0; b < NBUF; b++) {
      load(q + WPB * (b + NBUF - 1), buf[(b + NBUF - 1) % NBUF]);
      if (q + WPB * b < hi) {
#pragma unroll
        for (int j = 0; j < NI; j++) acc ^= buf[b][j].x ^ buf[b][j].y ^ buf[b][j].z ^ buf[b][j].w;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// Claimed order (the lean kernel's schedule): wave i starts with lo + i, then takes the sets a
// per-workgroup atomic counter hands out; a claim is read one step after it is issued.
template <int NBUF>
__global__ __launch_bounds__(1024) void probe_claim(const uint8_t* __restrict__ base, int nsets, uint32_t* ctr,
                                                   uint32_t* out) {
  constexpr int NI = 6;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int WPB = blockDim.x >> 6;
  const int lo = (int)((int64_t)nsets * blockIdx.x / gridDim.x);
  const int hi = (int)((int64_t)nsets * (blockIdx.x + 1) / gridDim.x);
  uint32_t* c = ctr + blockIdx.x * 32;
  uint32_t acc = 0;
  uint4 buf[NBUF][NI];
  auto load = [&](int q, uint4 (&x)[NI]) {
    const int qc = min(q, nsets - 1);
    const int f = lane >> 4, col = lane & 15;
    const uint8_t* a = base + (int64_t)qc * 6000 + 1500 * f - 36 + 16 * col;
#pragma unroll
    for (int j = 0; j < NI; j++) {
      const u32x4 v = __builtin_nontemporal_load((const g_u32x4*)(a + 256 * j));
      x[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  auto claim = [&]() -> uint32_t {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  static_assert(NBUF == 2, "claim probe: depth 2");
  int q0 = lo + wid;
  uint32_t cl = claim();
  load(q0, buf[0]);
  int qc = q0;
  for (;;) {
    const int qn = lo + WPB + (int)__builtin_amdgcn_readfirstlane(cl);
    cl = claim();
    load(qn, buf[1]);
    if (qc >= hi) break;
#pragma unroll
    for (int j = 0; j < NI; j++) acc ^= buf[0][j].x ^ buf[0][j].y ^ buf[0][j].z ^ buf[0][j].w;
    const int qn2 = lo + WPB + (int)__builtin_amdgcn_readfirstlane(cl);
    cl = claim();
    load(qn2, buf[0]);
    if (qn >= hi) break;
#pragma unroll
    for (int j = 0; j < NI; j++) acc ^= buf[1][j].x ^ buf[1][j].y ^ buf[1][j].z ^ buf[1][j].w;
    qc = qn2;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int N = 1000000, NS = N / 4;
  const size_t BYTES = 1500ull * N + 4096;
  uint8_t* d;
  CK(hipMalloc(&d, BYTES + 4096));
  {  // random bytes (data-dependent power matters: a constant fill runs faster)
    std::vector<uint32_t> h((BYTES + 4096) / 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& v : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v = (uint32_t)x;
    }
    CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  uint8_t* base = d + 4096;  // room for the first frame's pad
  uint32_t* o;
  CK(hipMalloc(&o, 1 << 22));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 256;
  {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    ncu = pr.multiProcessorCount;
  }
  uint32_t* ctr;
  CK(hipMalloc(&ctr, 1 << 20));
  auto runc = [&](const char* nm, auto kern, int threads) {
    std::vector<float> ts;
    for (int r = 0; r < 26; r++) {
      CK(hipMemsetAsync(ctr, 0, ncu * 128));
      CK(hipEventRecord(e0));
      kern<<<ncu, threads>>>(base, NS, ctr, o);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-28s median %.4f ms  %.1f GB/s (1500 B/frame)\n", nm, ts[12], 1500.0 * N / ts[12] / 1e6);
    fflush(stdout);
  };
  auto run = [&](const char* nm, auto kern, int threads = 1024) {
    kern<<<ncu, threads>>>(base, NS, d, o);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 25; r++) {
      CK(hipEventRecord(e0));
      kern<<<ncu, threads>>>(base, NS, d, o);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%-28s median %.4f ms  %.1f GB/s (1500 B/frame)\n", nm, ts[12], 1500.0 * N / ts[12] / 1e6);
    fflush(stdout);
  };
  for (int rep = 0; rep < 2; rep++) {
    run("frame16 w8 nb2 NT", probe<kFrame16, 2, true>, 512);
    runc("claim w8 nb2 NT", probe_claim<2>, 512);
    run("frame16 w16 nb2 NT", probe<kFrame16, 2, true>);
    runc("claim w16 nb2 NT", probe_claim<2>, 1024);
  }
  printf("done\n");
  return 0;
}
