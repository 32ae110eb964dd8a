// Probe 11 (round 4): the level kernel's memory pattern on the permutation a level transition of
// field-structured one-hot data really has, against a uniform random permutation of the same size.
// N rows, C columns per level: every row draws one column in level A and one in level B (uniform);
// the store holds the records in level A's order (columns ascending, rows ascending in a column),
// and each record moves to its row's slot in level B's order. One 512-thread workgroup per level-A
// column (up to 1024 records: all loads in flight, staged through LDS, whole-record scattered
// writes -- k_level_lord without its arithmetic); the uniform variant keeps the same runs but sends
// the records to a uniform random permutation. Time per record per pass, 5 passes after a warm-up.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_field tools/probe_field.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t BLOCK = 512, CAP = 1024, K = 4 * CAP / BLOCK;

__device__ inline uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

__global__ __launch_bounds__(BLOCK) void kmove(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                               const uint32_t *__restrict__ nxt, const uint32_t *__restrict__ cp)
{
	__shared__ dv2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	const uint32_t b = cp[blockIdx.x];
	const uint32_t m = min(cp[blockIdx.x + 1] - b, CAP);
	if (m == 0) return;
	const uint32_t np = m * 4;
	dv2 v[K];
	uint32_t nr[CAP / BLOCK];
#pragma unroll
	for (uint32_t u = 0; u < CAP / BLOCK; ++u) nr[u] = nxt[b + min(threadIdx.x + u * BLOCK, m - 1)];
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) v[k] = src[(size_t)b * 4 + min(threadIdx.x + k * BLOCK, np - 1)];
#pragma unroll
	for (uint32_t k = 0; k < K; ++k) {
		const uint32_t t = threadIdx.x + k * BLOCK;
		recs[lslot(t >> 2, t & 3)] = v[k];
	}
#pragma unroll
	for (uint32_t u = 0; u < CAP / BLOCK; ++u) dsts[threadIdx.x + u * BLOCK] = nr[u];
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < np; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		dst[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
	}
}

int main()
{
	struct Shape { uint32_t n, cols; };
	const Shape shapes[] = {{10000000u, 25000u}, {10000000u, 12500u}, {12500000u, 125000u},
	                        {50000000u, 62500u}, {100000000u, 125000u}, {100000000u, 250000u}};
	std::mt19937_64 g(11);
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (const Shape &s : shapes) {
		const uint32_t n = s.n, C = s.cols;
		std::vector<uint32_t> ca(n), cb(n), cntA(C + 1, 0), cntB(C + 1, 0);
		std::uniform_int_distribution<uint32_t> d(0, C - 1);
		for (uint32_t r = 0; r < n; r++) { ca[r] = d(g); cb[r] = d(g); cntA[ca[r] + 1]++; cntB[cb[r] + 1]++; }
		for (uint32_t c = 0; c < C; c++) { cntA[c + 1] += cntA[c]; cntB[c + 1] += cntB[c]; }
		std::vector<uint32_t> cp(cntA.begin(), cntA.end()), fa(cntA.begin(), cntA.end() - 1),
		    fb(cntB.begin(), cntB.end() - 1), posB(n), nxt(n);
		for (uint32_t r = 0; r < n; r++) posB[r] = fb[cb[r]]++;           // rows ascending in a column
		for (uint32_t r = 0; r < n; r++) nxt[fa[ca[r]]++] = posB[r];       // level-A order -> level-B slot
		std::vector<uint32_t> uni(n);
		for (uint32_t i = 0; i < n; i++) uni[i] = i;
		std::shuffle(uni.begin(), uni.end(), g);
		uint32_t maxc = 0;
		for (uint32_t c = 0; c < C; c++) maxc = std::max(maxc, cp[c + 1] - cp[c]);
		if (maxc > CAP) { printf("column of %u records > %u\n", maxc, CAP); return 1; }
		dv2 *a, *bb;
		uint32_t *dn, *du, *dcp;
		CK(hipMalloc(&a, (size_t)n * 64));
		CK(hipMalloc(&bb, (size_t)n * 64));
		CK(hipMalloc(&dn, (size_t)n * 4));
		CK(hipMalloc(&du, (size_t)n * 4));
		CK(hipMalloc(&dcp, (size_t)(C + 1) * 4));
		CK(hipMemcpy(dn, nxt.data(), (size_t)n * 4, hipMemcpyHostToDevice));
		CK(hipMemcpy(du, uni.data(), (size_t)n * 4, hipMemcpyHostToDevice));
		CK(hipMemcpy(dcp, cp.data(), (size_t)(C + 1) * 4, hipMemcpyHostToDevice));
		CK(hipMemset(a, 0, (size_t)n * 64));
		float t[2] = {0.f, 0.f};
		for (int variant = 0; variant < 2; ++variant) {
			for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms up
				CK(hipEventRecord(e0));
				for (int it = 0; it < 5; ++it) {
					kmove<<<C, BLOCK>>>(a, bb, variant == 0 ? dn : du, dcp);
					std::swap(a, bb);
				}
				CK(hipEventRecord(e1));
				CK(hipEventSynchronize(e1));
				CK(hipEventElapsedTime(&t[variant], e0, e1));
			}
		}
		printf("N %10u  %6u cols (%4u per col)  field %8.4f ms (%5.2f ps/rec)  uniform %8.4f ms (%5.2f ps/rec)\n", n,
		       C, n / C, t[0] / 5, t[0] / 5 * 1e9 / n, t[1] / 5, t[1] / 5 * 1e9 / n);
		fflush(stdout);
		CK(hipFree(a)); CK(hipFree(bb)); CK(hipFree(dn)); CK(hipFree(du)); CK(hipFree(dcp));
	}
	CK(hipGetLastError());
	return 0;
}
