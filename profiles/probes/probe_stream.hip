// Ceiling probe for a row-streaming level pass: sequential 64-B record RMW + two 8-B entry
// streams + two fp64 atomics per row into a per-feature table (random feature per row).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int ATOM>
__global__ __launch_bounds__(256) void k_pass(Rec* recs, const uint2* ent, const uint2* nxt, const double2* post, double* stats, uint32_t n) {
  for (uint32_t r = blockIdx.x * 256u + threadIdx.x; r < n; r += gridDim.x * 256u) {
    const double2* p = (const double2*)(recs + r);
    double2 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
    uint2 e = ent[r], nx = nxt[r];
    double2 po = post[e.x];
    double x = __uint_as_float(e.y), xn = __uint_as_float(nx.y);
    a0.x += x * po.x; a0.y += x * po.y; a1.x += a0.y * x; a2.x += a1.y * po.x;
    double h = a0.y - xn * 0.5;
    if (ATOM) { atomicAdd(&stats[2 * nx.x], xn * h * (a0.x + h)); atomicAdd(&stats[2 * nx.x + 1], xn * xn * h * h); }
    double2* q = (double2*)(recs + r);
    q[0] = a0; q[1] = a1; q[2] = a2; q[3] = a3;
  }
}
int main(int argc, char** argv) {
  uint32_t n = argc > 1 ? atoi(argv[1]) : 100000000, S = 125000;
  std::vector<uint2> h(n), h2(n); std::mt19937 g(1);
  for (uint32_t i = 0; i < n; i++) { h[i] = make_uint2(g() % S, 0x3f800000u); h2[i] = make_uint2(S + g() % S, 0x3f800000u); }
  Rec* recs; uint2 *ent, *nxt; double2* post; double* stats;
  CK(hipMalloc(&recs, (size_t)n * 64)); CK(hipMalloc(&ent, (size_t)n * 8)); CK(hipMalloc(&nxt, (size_t)n * 8));
  CK(hipMalloc(&post, 2 * S * 16)); CK(hipMalloc(&stats, 2 * S * 16));
  CK(hipMemcpy(ent, h.data(), (size_t)n * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(nxt, h2.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  CK(hipMemset(recs, 0, (size_t)n * 64)); CK(hipMemset(post, 0, 2 * S * 16)); CK(hipMemset(stats, 0, 2 * S * 16));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int it = 0; it < 10; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 10;
    printf("%-40s n=%u %.3f ms  %.0f GB/s (144 B/row)  %.3g rows/s\n", name, n, ms, 144.0 * n / ms / 1e6, n / ms * 1e3);
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64]; snprintf(nm, 64, "stream RMW + 2 f64 atomics grid=%d", grid);
    time(nm, [&] { k_pass<1><<<grid, 256>>>(recs, ent, nxt, post, stats, n); });
    snprintf(nm, 64, "stream RMW, no atomics grid=%d", grid);
    time(nm, [&] { k_pass<0><<<grid, 256>>>(recs, ent, nxt, post, stats, n); });
  }
  return 0;
}
