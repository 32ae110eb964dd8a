// Ceiling probe for the level kernel's access pattern on MI355X: random 64-B record
// read-modify-write, with and without an index stream, at several occupancies.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int RW, int PER>
__global__ __launch_bounds__(256) void k_rand(const uint32_t* idx, Rec* recs, uint32_t n) {
  uint32_t base = (blockIdx.x * 256u + threadIdx.x) * PER;
  uint32_t r[PER]; double2 a[PER][4];
#pragma unroll
  for (int u = 0; u < PER; u++) r[u] = base + u < n ? idx[base + u] : 0;
#pragma unroll
  for (int u = 0; u < PER; u++) if (base + u < n) { const double2* p = (const double2*)(recs + r[u]); a[u][0]=p[0]; a[u][1]=p[1]; a[u][2]=p[2]; a[u][3]=p[3]; }
#pragma unroll
  for (int u = 0; u < PER; u++) if (base + u < n) {
    if (RW) { double2* p = (double2*)(recs + r[u]); a[u][0].x += 1.0; p[0]=a[u][0]; p[1]=a[u][1]; p[2]=a[u][2]; p[3]=a[u][3]; }
    else if (a[u][0].x == 12345.678) recs[0].v[0] = a[u][1].x + a[u][2].y + a[u][3].x;
  }
}
__global__ void k_stream(const Rec* a, Rec* b, uint32_t n) {
  uint32_t i = blockIdx.x * 256u + threadIdx.x; if (i >= n) return;
  const double2* p = (const double2*)(a + i); double2* q = (double2*)(b + i);
  q[0]=p[0]; q[1]=p[1]; q[2]=p[2]; q[3]=p[3];
}
int main(int argc, char** argv) {
  uint32_t n = argc > 1 ? atoi(argv[1]) : 10000000;
  std::vector<uint32_t> h(n); for (uint32_t i = 0; i < n; i++) h[i] = i;
  std::mt19937 g(1); std::shuffle(h.begin(), h.end(), g);
  uint32_t* idx; Rec* recs; Rec* r2;
  CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&recs, (size_t)n * 64)); CK(hipMalloc(&r2, (size_t)n * 64));
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice)); CK(hipMemset(recs, 0, (size_t)n * 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, double bytes, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int it = 0; it < 10; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
    printf("%-34s n=%u %.3f ms  %.0f GB/s\n", name, n, ms, bytes / ms / 1e6);
  };
  unsigned g1 = (n + 255) / 256;
  time("stream copy 64B/rec", 128.0 * n, [&] { k_stream<<<g1, 256>>>(recs, r2, n); });
  time("rand read 64B (+idx 4B) PER=1", 68.0 * n, [&] { k_rand<0, 1><<<g1, 256>>>(idx, recs, n); });
  time("rand RMW 64B (+idx) PER=1", 132.0 * n, [&] { k_rand<1, 1><<<g1, 256>>>(idx, recs, n); });
  time("rand RMW 64B (+idx) PER=2", 132.0 * n, [&] { k_rand<1, 2><<<(g1 + 1) / 2, 256>>>(idx, recs, n); });
  time("rand RMW 64B (+idx) PER=4", 132.0 * n, [&] { k_rand<1, 4><<<(g1 + 3) / 4, 256>>>(idx, recs, n); });
  // sorted-within-chunks index (like CSC columns: ascending rows)
  for (uint32_t c = 0; c + 400 <= n; c += 400) std::sort(h.begin() + c, h.begin() + c + 400);
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  time("rand RMW sorted-400 PER=1", 132.0 * n, [&] { k_rand<1, 1><<<g1, 256>>>(idx, recs, n); });
  return 0;
}
