// Probe: is a level transition faster as a scatter (stream-read the run, write each 64-B record to
// its random slot: what k_level_lord does) or as a gather (read each record from its random slot,
// write the run contiguously)? Same bytes, the random side swapped. 4 lanes per record (16 B each),
// so every random access is one whole 64-B record.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_transition tools/probe_transition.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef double v2 __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ __launch_bounds__(512) void k_scatter(const v2 *__restrict__ src, v2 *__restrict__ dst,
                                                 const uint32_t *__restrict__ perm, uint64_t n)
{
	const uint64_t t = (uint64_t)blockIdx.x * 512 + threadIdx.x;   // piece index
	if (t >= n * 4) return;
	const v2 v = src[t];
	const uint32_t d = perm[t >> 2];
	if constexpr (NT) __builtin_nontemporal_store(v, dst + (uint64_t)d * 4 + (t & 3));
	else dst[(uint64_t)d * 4 + (t & 3)] = v;
}

template <bool NT>
__global__ __launch_bounds__(512) void k_gather(const v2 *__restrict__ src, v2 *__restrict__ dst,
                                                const uint32_t *__restrict__ perm, uint64_t n)
{
	const uint64_t t = (uint64_t)blockIdx.x * 512 + threadIdx.x;
	if (t >= n * 4) return;
	const uint32_t s = perm[t >> 2];
	const v2 v = src[(uint64_t)s * 4 + (t & 3)];
	if constexpr (NT) __builtin_nontemporal_store(v, dst + t);
	else dst[t] = v;
}

__global__ void k_fill(v2 *p, uint64_t n4)
{
	const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
	if (t < n4) p[t] = v2{(double)t, 1.0};
}

int main(int argc, char **argv)
{
	const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000000ull;
	const int reps = argc > 2 ? atoi(argv[2]) : 5;
	printf("records %llu (%.2f GB per buffer)\n", (unsigned long long)n, n * 64.0 / 1e9);
	std::vector<uint32_t> h(n);
	for (uint64_t i = 0; i < n; i++) h[i] = (uint32_t)i;
	std::mt19937_64 rng(12345);
	std::shuffle(h.begin(), h.end(), rng);
	v2 *a, *b;
	uint32_t *perm;
	CK(hipMalloc(&a, n * 64));
	CK(hipMalloc(&b, n * 64));
	CK(hipMalloc(&perm, n * 4));
	CK(hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice));
	k_fill<<<(unsigned)((n * 4 + 255) / 256), 256>>>(a, n * 4);
	k_fill<<<(unsigned)((n * 4 + 255) / 256), 256>>>(b, n * 4);
	CK(hipDeviceSynchronize());
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const unsigned grid = (unsigned)((n * 4 + 511) / 512);
	const double bytes = n * (64.0 + 64.0 + 4.0);
	auto run = [&](const char *name, auto launch) {
		launch();   // warm
		CK(hipDeviceSynchronize());
		float best = 1e30f, sum = 0.f;
		for (int r = 0; r < reps; r++) {
			CK(hipEventRecord(e0));
			launch();
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			best = std::min(best, ms);
			sum += ms;
		}
		printf("%-24s best %.3f ms  mean %.3f ms  %.1f ps/record  %.2f TB/s\n", name, best, sum / reps,
		       best * 1e9 / n, bytes / (best * 1e-3) / 1e12);
		fflush(stdout);
	};
	for (int round = 0; round < 2; round++) {
		run("scatter (plain stores)", [&] { k_scatter<false><<<grid, 512>>>(a, b, perm, n); });
		run("scatter (NT stores)", [&] { k_scatter<true><<<grid, 512>>>(a, b, perm, n); });
		run("gather (plain stores)", [&] { k_gather<false><<<grid, 512>>>(a, b, perm, n); });
		run("gather (NT stores)", [&] { k_gather<true><<<grid, 512>>>(a, b, perm, n); });
	}
	CK(hipFree(a));
	CK(hipFree(b));
	CK(hipFree(perm));
	return 0;
}
