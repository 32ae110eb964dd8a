// Ceiling probe 6: is the level kernel's random full-line scatter limited by address
// translation? The same scatter (1e8 64-B records, runs of 800 read contiguously, each record
// written to its permuted position) with the permutation confined to windows of W records
// (W*64 B of destination per window), and with buffers from hipDeviceMallocContiguous.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
constexpr int RUN = 800;

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void kB(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt)
{
	const size_t b = (size_t)blockIdx.x * RUN;
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		((dv2 *)(dst + nxt[b + i]))[c] = ((const dv2 *)(src + b + i))[c];
	}
}

int main()
{
	const uint32_t n = 100000000u, nrun = n / RUN;
	std::mt19937_64 g(3);
	std::vector<uint32_t> h(n);
	uint32_t *nx; Rec *a, *bb, *ca, *cb;
	CK(hipMalloc(&nx, (size_t)n * 4));
	CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(bb, 0, (size_t)n * 64));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, Rec *s, Rec *d) {
		kB<512><<<nrun, 512>>>(s, d, nx); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) kB<512><<<nrun, 512>>>(s, d, nx);
		CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
		printf("%-48s %.3f ms\n", name, ms);
		fflush(stdout);
	};
	const uint32_t wins[] = {100000000u, 25000000u, 6250000u, 1562500u, 400000u};
	for (uint32_t W : wins) {
		for (uint32_t i = 0; i < n; i++) h[i] = i;
		for (uint32_t b = 0; b < n; b += W) std::shuffle(h.begin() + b, h.begin() + std::min(n, b + W), g);
		CK(hipMemcpy(nx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
		char name[96];
		snprintf(name, sizeof name, "window %u records (%.0f MB)", W, W * 64.0 / 1e6);
		time(name, a, bb);
	}
	for (uint32_t i = 0; i < n; i++) h[i] = i;
	std::shuffle(h.begin(), h.end(), g);
	CK(hipMemcpy(nx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	time("full again (hipMalloc)", a, bb);
	hipError_t e = hipExtMallocWithFlags((void **)&ca, (size_t)n * 64, hipDeviceMallocContiguous);
	hipError_t e2 = hipExtMallocWithFlags((void **)&cb, (size_t)n * 64, hipDeviceMallocContiguous);
	printf("contiguous alloc: %s %s\n", hipGetErrorString(e), hipGetErrorString(e2));
	if (e == hipSuccess && e2 == hipSuccess) {
		CK(hipMemset(ca, 0, (size_t)n * 64)); CK(hipMemset(cb, 0, (size_t)n * 64));
		time("full (hipDeviceMallocContiguous)", ca, cb);
	}
	return 0;
}
