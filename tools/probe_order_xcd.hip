// Probe 21 (round 6; probe 9, tools/probe_order.hip, found rand = arrival order): does the ORDER of rows inside a column change the level scatter's rate?
// The level kernel streams column j's run of records and scatters each 64-B record to its row's
// slot in the next level's order: slot = start of the row's next column + the row's rank in it.
// The columns are fixed by the data; the order of rows inside a column is free. Variants of that
// order, all with the same kernel over the same two buffers (one process, interleaved):
//   rand     ranks inside each destination column uniformly random (row-id order on uniform data)
//   src      ranks by the source column j: records written about the same time land next to each
//            other in every destination column (the launch walks the columns in blockIdx order)
//   src_xcd  as src, with workgroups mapped XCD-contiguously (blockIdx b runs column
//            (b % 8) * ceil(C / 8) + b / 8, so one XCD's L2 sees neighbouring columns)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_order_xcd tools/probe_order_xcd.hip
// Run:   tools/probe_order_xcd <records> <run length> <reps>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t BLOCK = 512, CAP = 1024;

__device__ inline uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

template <bool NT, bool XCD>
__global__ __launch_bounds__(BLOCK) void klevel(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                                const uint32_t *__restrict__ nxt, uint32_t n, uint32_t run,
                                                uint32_t ncol)
{
	__shared__ dv2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	uint32_t col = blockIdx.x;
	if constexpr (XCD) {
		const uint32_t per = (ncol + 7) / 8;
		col = (blockIdx.x % 8) * per + blockIdx.x / 8;
		if (col >= ncol) return;
	}
	const uint32_t b = col * run;
	if (b >= n) return;
	const uint32_t m = min(run, n - b);
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK)
		recs[lslot(t >> 2, t & 3)] = __builtin_nontemporal_load(src + (size_t)b * 4 + t);
	for (uint32_t i = threadIdx.x; i < m; i += BLOCK) dsts[i] = nxt[b + i];
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		if constexpr (NT) __builtin_nontemporal_store(recs[lslot(i, c)], dst + (size_t)dsts[i] * 4 + c);
		else dst[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
	}
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atof(argv[1]) : 100000000u;
	const uint32_t run = argc > 2 ? atoi(argv[2]) : 800;
	const int reps = argc > 3 ? atoi(argv[3]) : 6;
	if (run > CAP) { printf("run <= %u\n", CAP); return 1; }
	const uint32_t ncol = (n + run - 1) / run;
	// destination column of every record: a uniform permutation of the slots, cut into columns
	std::mt19937_64 g(12345);
	std::vector<uint32_t> perm(n);
	std::iota(perm.begin(), perm.end(), 0u);
	std::shuffle(perm.begin(), perm.end(), g);
	std::vector<uint32_t> rnd(perm), bysrc(n), byxcd(n);
	// src: inside each destination column, ranks follow the source position (column-major in time)
	{
		std::vector<uint32_t> fill(ncol, 0);
		for (uint32_t i = 0; i < n; ++i) {
			const uint32_t c = perm[i] / run;
			bysrc[i] = c * run + fill[c]++;
		}
	}
	// src_xcd: ranks follow the time a source column runs under the XCD-contiguous mapping
	{
		const uint32_t per = (ncol + 7) / 8;
		std::vector<uint32_t> order;   // source columns in launch order (blockIdx)
		for (uint32_t b = 0; b < 8 * per; ++b) {
			const uint32_t col = (b % 8) * per + b / 8;
			if (col < ncol) order.push_back(col);
		}
		std::vector<uint32_t> fill(ncol, 0);
		for (uint32_t col : order)
			for (uint32_t i = col * run; i < std::min(n, (col + 1) * run); ++i) {
				const uint32_t c = perm[i] / run;
				byxcd[i] = c * run + fill[c]++;
			}
	}
	dv2 *a, *d;
	uint32_t *ix[3];
	CK(hipMalloc(&a, (size_t)n * 64));
	CK(hipMalloc(&d, (size_t)n * 64));
	CK(hipMemset(a, 0, (size_t)n * 64));
	const std::vector<uint32_t> *hs[3] = {&rnd, &bysrc, &byxcd};
	for (int v = 0; v < 3; ++v) {
		CK(hipMalloc(&ix[v], (size_t)n * 4));
		CK(hipMemcpy(ix[v], hs[v]->data(), (size_t)n * 4, hipMemcpyHostToDevice));
	}
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const char *names[6] = {"rand", "src", "src_xcd", "rand_nt", "src_nt", "src_xcd_nt"};
	std::vector<float> best(6, 1e30f), sum(6, 0.f);
	const uint32_t grid_plain = ncol, grid_xcd = 8 * ((ncol + 7) / 8);
	for (int r = 0; r < reps; ++r)
		for (int k = 0; k < 6; ++k) {
			const int v = k % 3;
			const bool nt = k >= 3;
			CK(hipEventRecord(e0));
			if (v < 2) {
				if (nt) klevel<true, false><<<grid_plain, BLOCK>>>(a, d, ix[v], n, run, ncol);
				else klevel<false, false><<<grid_plain, BLOCK>>>(a, d, ix[v], n, run, ncol);
			} else {
				if (nt) klevel<true, true><<<grid_xcd, BLOCK>>>(a, d, ix[v], n, run, ncol);
				else klevel<false, true><<<grid_xcd, BLOCK>>>(a, d, ix[v], n, run, ncol);
			}
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (r) { best[k] = std::min(best[k], ms); sum[k] += ms; }
		}
	printf("records %u, run %u, columns %u, reps %d (first dropped); ms per launch best / mean, GB/s at 132 B per record\n",
	       n, run, ncol, reps);
	for (int k = 0; k < 6; ++k)
		printf("%-11s %8.4f %8.4f  %7.0f\n", names[k], best[k], sum[k] / (reps - 1), (double)n * 132 / best[k] / 1e6);
	return 0;
}
