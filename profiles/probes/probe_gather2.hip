// Ceiling probe 2: random 64-B record RMW at 1e8 rows vs. the size of the sorted index
// groups (a column = one sorted group) and load/store cache policy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int NT>
__global__ __launch_bounds__(256) void k_rmw(const uint32_t* idx, Rec* recs, uint32_t n) {
  uint32_t i = blockIdx.x * 256u + threadIdx.x; if (i >= n) return;
  uint32_t r = idx[i];
  dv2* p = (dv2*)(recs + r);
  dv2 a0, a1, a2, a3;
  if (NT & 1) { a0 = __builtin_nontemporal_load(p); a1 = __builtin_nontemporal_load(p + 1); a2 = __builtin_nontemporal_load(p + 2); a3 = __builtin_nontemporal_load(p + 3); }
  else { a0 = p[0]; a1 = p[1]; a2 = p[2]; a3 = p[3]; }
  a0.x += 1.0;
  if (NT & 2) { __builtin_nontemporal_store(a0, p); __builtin_nontemporal_store(a1, p + 1); __builtin_nontemporal_store(a2, p + 2); __builtin_nontemporal_store(a3, p + 3); }
  else { p[0] = a0; p[1] = a1; p[2] = a2; p[3] = a3; }
}
// 4 lanes per record: lane l loads the 16-B chunk l%4 of record idx[i/4]
__global__ __launch_bounds__(256) void k_rmw4(const uint32_t* idx, Rec* recs, uint32_t n) {
  uint32_t t = blockIdx.x * 256u + threadIdx.x; uint32_t i = t >> 2, c = t & 3; if (i >= n) return;
  uint32_t r = idx[i];
  double2* p = (double2*)(recs + r) + c;
  double2 a = *p; a.x += 1.0; *p = a;
}
int main(int argc, char** argv) {
  uint32_t n = argc > 1 ? atoi(argv[1]) : 100000000;
  std::vector<uint32_t> h(n); for (uint32_t i = 0; i < n; i++) h[i] = i;
  std::mt19937 g(1); std::shuffle(h.begin(), h.end(), g);
  uint32_t* idx; Rec* recs;
  CK(hipMalloc(&idx, (size_t)n * 4)); CK(hipMalloc(&recs, (size_t)n * 64)); CK(hipMemset(recs, 0, (size_t)n * 64));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto time = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-44s %.3f ms  %.3g rows/s\n", name, ms, n / ms * 1e3);
  };
  unsigned g1 = (n + 255) / 256;
  uint32_t prev = 1;
  for (uint32_t grp : {1u, 400u, 800u, 3200u, 25600u, 204800u}) {
    for (uint32_t c = 0; c < n; c += grp) std::sort(h.begin() + c, h.begin() + std::min<size_t>(n, (size_t)c + grp));
    CK(hipMemcpy(idx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    char nm[96];
    snprintf(nm, 96, "sorted-%u plain", grp); time(nm, [&] { k_rmw<0><<<g1, 256>>>(idx, recs, n); });
    if (grp == 800) {
      time("sorted-800 nt load", [&] { k_rmw<1><<<g1, 256>>>(idx, recs, n); });
      time("sorted-800 nt store", [&] { k_rmw<2><<<g1, 256>>>(idx, recs, n); });
      time("sorted-800 nt both", [&] { k_rmw<3><<<g1, 256>>>(idx, recs, n); });
      time("sorted-800 4 lanes/rec", [&] { k_rmw4<<<(unsigned)(((size_t)n * 4 + 255) / 256), 256>>>(idx, recs, n); });
    }
    (void)prev;
  }
  return 0;
}
