// Ceiling probe 3: permuting copies of 64-B row records (1e8 rows) -- the cost of keeping the
// row records physically sorted by the current dependency level's feature and moving them to
// the next level's order once per level, against the in-place random read-modify-write the
// column-gather level kernel pays.
//   gather : dst[i] = src[perm[i]]   (random 64-B reads, streaming writes)
//   scatter: dst[perm[i]] = src[i]   (streaming reads, random 64-B writes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// 4 lanes per record, 16 B each
template <int MODE, int NT>
__global__ __launch_bounds__(256) void k_perm(const uint32_t* __restrict__ perm, const Rec* __restrict__ src,
                                              Rec* __restrict__ dst, uint32_t n) {
  size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t i = (uint32_t)(t >> 2), c = (uint32_t)(t & 3);
  if (i >= n) return;
  uint32_t p = perm[i];
  const dv2* s = (const dv2*)(src + (MODE == 0 ? p : i)) + c;
  dv2* d = (dv2*)(dst + (MODE == 0 ? i : p)) + c;
  dv2 a = *s;
  a.x += 1.0;
  if (NT) __builtin_nontemporal_store(a, d); else *d = a;
}
// 32-B records, 2 lanes per record
template <int MODE>
__global__ __launch_bounds__(256) void k_perm32(const uint32_t* __restrict__ perm, const dv2* __restrict__ src,
                                                dv2* __restrict__ dst, uint32_t n) {
  size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t i = (uint32_t)(t >> 1), c = (uint32_t)(t & 1);
  if (i >= n) return;
  uint32_t p = perm[i];
  dv2 a = src[(size_t)(MODE == 0 ? p : i) * 2 + c];
  a.x += 1.0;
  dst[(size_t)(MODE == 0 ? i : p) * 2 + c] = a;
}
__global__ __launch_bounds__(256) void k_copy32(const dv2* __restrict__ src, dv2* __restrict__ dst, uint32_t n) {
  size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
  if (t >= (size_t)n * 2) return;
  dv2 a = src[t]; a.x += 1.0; dst[t] = a;
}
// in-place random RMW, 4 lanes per record
__global__ __launch_bounds__(256) void k_rmw4(const uint32_t* __restrict__ perm, Rec* recs, uint32_t n) {
  size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t i = (uint32_t)(t >> 2), c = (uint32_t)(t & 3);
  if (i >= n) return;
  dv2* p = (dv2*)(recs + perm[i]) + c;
  dv2 a = *p; a.x += 1.0; *p = a;
}
// streaming copy, 4 lanes per record
__global__ __launch_bounds__(256) void k_copy4(const Rec* __restrict__ src, Rec* __restrict__ dst, uint32_t n) {
  size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t i = (uint32_t)(t >> 2), c = (uint32_t)(t & 3);
  if (i >= n) return;
  dv2 a = ((const dv2*)(src + i))[c]; a.x += 1.0; ((dv2*)(dst + i))[c] = a;
}

int main(int argc, char** argv) {
  uint32_t n = argc > 1 ? atoi(argv[1]) : 100000000;
  std::vector<uint32_t> h(n); for (uint32_t i = 0; i < n; i++) h[i] = i;
  std::mt19937 g(1); std::shuffle(h.begin(), h.end(), g);
  uint32_t* perm; Rec *a, *b;
  CK(hipMalloc(&perm, (size_t)n * 4)); CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&b, (size_t)n * 64));
  CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(b, 0, (size_t)n * 64));
  CK(hipMemcpy(perm, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-36s n=%u %.3f ms  %.3g rows/s  %.0f GB/s (128 B/row)\n", name, n, ms, n / ms * 1e3, 128.0 * n / ms / 1e6);
  };
  unsigned g4 = (unsigned)(((size_t)n * 4 + 255) / 256);
  time("stream copy", [&] { k_copy4<<<g4, 256>>>(a, b, n); });
  time("random RMW in place", [&] { k_rmw4<<<g4, 256>>>(perm, a, n); });
  time("gather-permute", [&] { k_perm<0, 0><<<g4, 256>>>(perm, a, b, n); });
  time("gather-permute nt store", [&] { k_perm<0, 1><<<g4, 256>>>(perm, a, b, n); });
  time("scatter-permute", [&] { k_perm<1, 0><<<g4, 256>>>(perm, a, b, n); });
  time("scatter-permute nt store", [&] { k_perm<1, 1><<<g4, 256>>>(perm, a, b, n); });
  unsigned g2 = (unsigned)(((size_t)n * 2 + 255) / 256);
  time("32B stream copy (x0.5 B)", [&] { k_copy32<<<g2, 256>>>((const dv2*)a, (dv2*)b, n); });
  time("32B gather-permute (x0.5 B)", [&] { k_perm32<0><<<g2, 256>>>(perm, (const dv2*)a, (dv2*)b, n); });
  time("32B scatter-permute (x0.5 B)", [&] { k_perm32<1><<<g2, 256>>>(perm, (const dv2*)a, (dv2*)b, n); });
  // locality-bounded permutations: destinations random within windows of W rows
  for (uint32_t W : {1u << 16, 1u << 19, 1u << 21, 1u << 22}) {
    for (uint32_t i = 0; i < n; i++) h[i] = i;
    for (uint32_t c = 0; c < n; c += W) std::shuffle(h.begin() + c, h.begin() + std::min<size_t>(n, (size_t)c + W), g);
    CK(hipMemcpy(perm, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    char nm[64];
    snprintf(nm, 64, "scatter win %u", W); time(nm, [&] { k_perm<1, 0><<<g4, 256>>>(perm, a, b, n); });
    snprintf(nm, 64, "RMW win %u", W); time(nm, [&] { k_rmw4<<<g4, 256>>>(perm, a, n); });
  }
  return 0;
}
