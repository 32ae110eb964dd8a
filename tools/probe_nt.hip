// Ceiling probe 7: cache policy of the level kernel's scatter. 1e8 64-B records, runs of 800
// read contiguously, every record written whole (4 lanes x 16 B) to a random position:
// plain loads/stores vs non-temporal (nt) stores and/or loads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
constexpr int RUN = 800;

template <int BLOCK, bool NTL, bool NTS>
__global__ __launch_bounds__(BLOCK) void kB(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt)
{
	const size_t b = (size_t)blockIdx.x * RUN;
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		const dv2 *s = (const dv2 *)(src + b + i) + c;
		dv2 v = NTL ? __builtin_nontemporal_load(s) : *s;
		const uint32_t to = NTL ? __builtin_nontemporal_load(nxt + b + i) : nxt[b + i];
		dv2 *d = (dv2 *)(dst + to) + c;
		if (NTS) __builtin_nontemporal_store(v, d); else *d = v;
	}
}

int main()
{
	const uint32_t n = 100000000u, nrun = n / RUN;
	std::mt19937_64 g(3);
	std::vector<uint32_t> h(n);
	for (uint32_t i = 0; i < n; i++) h[i] = i;
	std::shuffle(h.begin(), h.end(), g);
	uint32_t *nx; Rec *a, *bb;
	CK(hipMalloc(&nx, (size_t)n * 4));
	CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(bb, 0, (size_t)n * 64));
	CK(hipMemcpy(nx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch();
		CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
		printf("%-40s %.3f ms\n", name, ms);
		fflush(stdout);
	};
	for (int rep = 0; rep < 2; rep++) {
		time("plain", [&] { kB<512, false, false><<<nrun, 512>>>(a, bb, nx); });
		time("nt store", [&] { kB<512, false, true><<<nrun, 512>>>(a, bb, nx); });
		time("nt load", [&] { kB<512, true, false><<<nrun, 512>>>(a, bb, nx); });
		time("nt load + nt store", [&] { kB<512, true, true><<<nrun, 512>>>(a, bb, nx); });
		time("nt load + nt store 1024", [&] { kB<1024, true, true><<<nrun, 1024>>>(a, bb, nx); });
	}
	return 0;
}
