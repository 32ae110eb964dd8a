// Ceiling probe 8: the level kernel's memory pattern with every load of a thread in flight
// (the pattern probes 1-7 used load/store loops, which the compiler serializes per piece).
// 1e8 64-B records in runs of ~800 (one workgroup per run, 512 threads), every record moved to
// a random slot of the next level (a random permutation), next position read per record.
//   copy      : coalesced read + coalesced write of all records (HBM streaming ceiling)
//   scatter   : coalesced read, 4 lanes per record, scattered whole-record writes; each thread
//               issues its 8 piece loads and 2 position loads before any store
//   lds       : as scatter, the run staged through LDS between a barrier (the level kernel's
//               structure minus the arithmetic)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_mlp tools/probe_mlp.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t RUN = 800, BLOCK = 512, K = 8;   // 4 * 1024 pieces / 512 threads

__global__ __launch_bounds__(256) void kcopy(const dv2 *__restrict__ src, dv2 *__restrict__ dst, size_t n)
{
	const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
	if (t < n) dst[t] = src[t];
}

__global__ __launch_bounds__(BLOCK) void kscatter(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                                  const uint32_t *__restrict__ nxt, uint32_t n)
{
	const uint32_t b = blockIdx.x * RUN;
	const uint32_t m = min(RUN, n - b);
	const uint32_t np = m * 4;
	dv2 v[K];
	uint32_t d[K];
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) {
		const uint32_t t = min(threadIdx.x + k * BLOCK, np - 1);
		v[k] = __builtin_nontemporal_load(src + (size_t)b * 4 + t);
		d[k] = nxt[b + (t >> 2)];
	}
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) {
		const uint32_t t = threadIdx.x + k * BLOCK;
		if (t < np) dst[(size_t)d[k] * 4 + (t & 3)] = v[k];
	}
}

__device__ inline uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

__global__ __launch_bounds__(BLOCK) void klds(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                              const uint32_t *__restrict__ nxt, uint32_t n)
{
	__shared__ dv2 recs[1024 * 4];
	__shared__ uint32_t dsts[1024];
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

int main()
{
	const uint32_t n = 100000000u;
	std::vector<uint32_t> hp(n);
	for (uint32_t i = 0; i < n; i++) hp[i] = i;
	std::mt19937_64 g(7);
	std::shuffle(hp.begin(), hp.end(), g);
	dv2 *a, *bb;
	uint32_t *np;
	CK(hipMalloc(&a, (size_t)n * 64));
	CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMalloc(&np, (size_t)n * 4));
	CK(hipMemcpy(np, hp.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemset(a, 0, (size_t)n * 64));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const uint32_t nrun = (n + RUN - 1) / RUN;
	for (int variant = 0; variant < 3; ++variant) {
		for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms up
			CK(hipEventRecord(e0));
			for (int it = 0; it < 5; ++it) {
				if (variant == 0) kcopy<<<(unsigned)(((size_t)n * 4 + 255) / 256), 256>>>(a, bb, (size_t)n * 4);
				else if (variant == 1) kscatter<<<nrun, BLOCK>>>(a, bb, np, n);
				else klds<<<nrun, BLOCK>>>(a, bb, np, n);
				std::swap(a, bb);
			}
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (rep) printf("%-8s %.3f ms per pass of 1e8 records (%.2f TB/s of 12.8 GB + 0.4 GB)\n",
			                variant == 0 ? "copy" : variant == 1 ? "scatter" : "lds", ms / 5,
			                (variant == 0 ? 12.8e9 : 13.2e9) / (ms / 5 * 1e-3) / 1e12);
		}
	}
	CK(hipGetLastError());
	return 0;
}
