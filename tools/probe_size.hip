// Probe 10 (round 4): does the level kernel's memory pattern itself run slower per record on a
// smaller store? For N = 2.5e6 .. 1e8 64-B records: a coalesced copy of the store, and the level
// kernel's pattern without its arithmetic (runs of 400 records, one 256-thread workgroup per
// run, every thread's loads in flight, the run staged through LDS, each record written whole to
// its slot of a uniformly random permutation -- the next level's order). Time per record per
// pass, 5 passes after one warm-up, one process, buffers allocated per size.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_size tools/probe_size.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t RUN = 400, BLOCK = 256, K = 8;   // 4 * 512 pieces / 256 threads

__global__ __launch_bounds__(256) void kcopy(const dv2 *__restrict__ src, dv2 *__restrict__ dst, size_t n)
{
	const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
	if (t < n) dst[t] = src[t];
}

__device__ inline uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

__global__ __launch_bounds__(BLOCK) void klds(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                              const uint32_t *__restrict__ nxt, uint32_t n)
{
	__shared__ dv2 recs[512 * 4];
	__shared__ uint32_t dsts[512];
	const uint32_t b = blockIdx.x * RUN;
	const uint32_t m = min(RUN, n - b);
	const uint32_t np = m * 4;
	dv2 v[K];
	uint32_t nr[2];
#pragma unroll
	for (uint32_t u = 0; u < 2; ++u) nr[u] = nxt[b + min(threadIdx.x + u * BLOCK, m - 1)];
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) v[k] = src[(size_t)b * 4 + min(threadIdx.x + k * BLOCK, np - 1)];
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) {
		const uint32_t t = threadIdx.x + k * BLOCK;
		recs[lslot(t >> 2, t & 3)] = v[k];
	}
#pragma unroll
	for (uint32_t u = 0; u < 2; ++u) dsts[threadIdx.x + u * BLOCK] = nr[u];
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < np; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		dst[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
	}
}

// argv[1] (optional): GB of device memory to allocate and touch first (the bench's data set holds
// 64+ GB of CSC / CSR beside the records at C4, 6.4 GB at C3); argv[2]: keep it (1) or free it (0)
int main(int argc, char **argv)
{
	const double pad_gb = argc > 1 ? atof(argv[1]) : 0.0;
	void *pad = nullptr;
	if (pad_gb > 0) {
		const size_t pb = (size_t)(pad_gb * 1e9);
		CK(hipMalloc(&pad, pb));
		CK(hipMemset(pad, 1, pb));
		CK(hipDeviceSynchronize());
		if (argc > 2 && atoi(argv[2]) == 0) { CK(hipFree(pad)); pad = nullptr; }
		printf("allocated %.0f GB first (%s)\n", pad_gb, pad ? "kept" : "freed");
	}
	const uint32_t sizes[] = {2500000u, 5000000u, 10000000u, 12500000u, 25000000u, 50000000u, 100000000u};
	std::mt19937_64 g(7);
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (uint32_t n : sizes) {
		std::vector<uint32_t> hp(n);
		for (uint32_t i = 0; i < n; i++) hp[i] = i;
		std::shuffle(hp.begin(), hp.end(), g);
		dv2 *a, *bb;
		uint32_t *np;
		CK(hipMalloc(&a, (size_t)n * 64));
		CK(hipMalloc(&bb, (size_t)n * 64));
		CK(hipMalloc(&np, (size_t)n * 4));
		CK(hipMemcpy(np, hp.data(), (size_t)n * 4, hipMemcpyHostToDevice));
		CK(hipMemset(a, 0, (size_t)n * 64));
		const uint32_t nrun = (n + RUN - 1) / RUN;
		float t[2] = {0.f, 0.f};
		for (int variant = 0; variant < 2; ++variant) {
			for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms up
				CK(hipEventRecord(e0));
				for (int it = 0; it < 5; ++it) {
					if (variant == 0) kcopy<<<(unsigned)(((size_t)n * 4 + 255) / 256), 256>>>(a, bb, (size_t)n * 4);
					else klds<<<nrun, BLOCK>>>(a, bb, np, n);
					std::swap(a, bb);
				}
				CK(hipEventRecord(e1));
				CK(hipEventSynchronize(e1));
				CK(hipEventElapsedTime(&t[variant], e0, e1));
			}
		}
		printf("N %10u  copy %8.4f ms (%5.2f ps/rec, %4.2f TB/s)  scatter %8.4f ms (%5.2f ps/rec)\n", n, t[0] / 5,
		       t[0] / 5 * 1e9 / n, 2.0 * 64 * n / (t[0] / 5 * 1e-3) / 1e12, t[1] / 5, t[1] / 5 * 1e9 / n);
		fflush(stdout);
		CK(hipFree(a));
		CK(hipFree(bb));
		CK(hipFree(np));
	}
	CK(hipGetLastError());
	return 0;
}
