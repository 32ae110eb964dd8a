// Ceiling probe 9: does the ORDER of records inside the next level's runs change the cost of
// the level kernel's scattered writes? 1e8 64-B records in runs of 800 (125k runs, one
// workgroup per run, 512 threads, LDS-staged as k_level_lord), every record moved to the next
// level; the next level's run of each record is a uniformly random run (balanced: every run
// receives 800 records). Within the destination run the record's slot is
//   rand   : a random slot (today's store: a run lists its rows in ascending row id, which
//            is random with respect to the source order)
//   arrival: the arrival rank in source order (a run lists its rows in the order of their
//            position in the previous level), so the workgroups in flight fill every
//            destination run front to back: writes of neighbouring source runs land next to
//            each other (full 128-B lines, open DRAM pages) instead of anywhere in the run.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_order tools/probe_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t RUN = 800, BLOCK = 512, K = 8;

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
	const uint32_t n = 100000000u, nrun = n / RUN;
	std::vector<uint32_t> lab(n), pr(n), pa(n), cnt(nrun, 0);
	for (uint32_t i = 0; i < n; i++) lab[i] = i / RUN;
	std::mt19937_64 g(7);
	std::shuffle(lab.begin(), lab.end(), g);          // destination run of source position i
	for (uint32_t i = 0; i < n; i++) pa[i] = lab[i] * RUN + cnt[lab[i]]++;
	// rand: the same destination runs, a random slot inside each run
	std::vector<uint32_t> slot(RUN);
	std::vector<std::vector<uint32_t>> members(nrun);
	for (uint32_t r = 0; r < nrun; r++) members[r].reserve(RUN);
	for (uint32_t i = 0; i < n; i++) members[lab[i]].push_back(i);
	for (uint32_t r = 0; r < nrun; r++) {
		for (uint32_t k = 0; k < RUN; k++) slot[k] = k;
		std::shuffle(slot.begin(), slot.end(), g);
		for (uint32_t k = 0; k < RUN; k++) pr[members[r][k]] = r * RUN + slot[k];
	}
	members.clear();
	dv2 *a, *bb;
	uint32_t *dr, *da;
	CK(hipMalloc(&a, (size_t)n * 64));
	CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMalloc(&dr, (size_t)n * 4));
	CK(hipMalloc(&da, (size_t)n * 4));
	CK(hipMemcpy(dr, pr.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(da, pa.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemset(a, 0, (size_t)n * 64));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (int round = 0; round < 3; ++round)
		for (int variant = 0; variant < 2; ++variant) {
			for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms up
				CK(hipEventRecord(e0));
				for (int it = 0; it < 5; ++it) {
					klds<<<nrun, BLOCK>>>(a, bb, variant ? da : dr, n);
					std::swap(a, bb);
				}
				CK(hipEventRecord(e1));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				if (rep) printf("round %d %-8s %.3f ms per pass of 1e8 records (%.2f TB/s of 12.8 GB + 0.4 GB)\n",
				                round, variant ? "arrival" : "rand", ms / 5, 13.2e9 / (ms / 5 * 1e-3) / 1e12);
			}
		}
	CK(hipGetLastError());
	return 0;
}
