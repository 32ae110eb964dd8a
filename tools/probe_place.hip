// Probe 12 (round 4): does the scattered-write rate of the level pattern depend on WHERE the two
// record buffers are placed? probe_size showed 26.9-35.6 ps per record for one size across
// processes (the streaming copy constant at 20.5 ps). Here, in one process, for N records: six
// buffer pairs allocated one after another (all kept), each timed twice (5 passes of the
// k_level_lord pattern: runs of 400, LDS-staged, whole-record scatter to a uniform random
// permutation), and once more after every pair was timed (persistence).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_place tools/probe_place.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t RUN = 400, BLOCK = 256, K = 8;

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

static float time_pair(dv2 *a, dv2 *b, const uint32_t *np, uint32_t n, hipEvent_t e0, hipEvent_t e1)
{
	const uint32_t nrun = (n + RUN - 1) / RUN;
	float ms = 0.f;
	for (int rep = 0; rep < 2; ++rep) {
		CK(hipEventRecord(e0));
		for (int it = 0; it < 6; ++it) klds<<<nrun, BLOCK>>>(it & 1 ? b : a, it & 1 ? a : b, np, n);
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		CK(hipEventElapsedTime(&ms, e0, e1));
	}
	return ms / 6 * 1e9f / n;   // ps per record
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
	const int pairs = argc > 2 ? atoi(argv[2]) : 6;
	std::vector<uint32_t> hp(n);
	for (uint32_t i = 0; i < n; i++) hp[i] = i;
	std::mt19937_64 g(7);
	std::shuffle(hp.begin(), hp.end(), g);
	uint32_t *np;
	CK(hipMalloc(&np, (size_t)n * 4));
	CK(hipMemcpy(np, hp.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	std::vector<dv2 *> A(pairs), B(pairs);
	std::vector<float> t1(pairs), t2(pairs), t3(pairs);
	for (int p = 0; p < pairs; ++p) {
		CK(hipMalloc(&A[p], (size_t)n * 64));
		CK(hipMalloc(&B[p], (size_t)n * 64));
		CK(hipMemset(A[p], 0, (size_t)n * 64));
		CK(hipMemset(B[p], 0, (size_t)n * 64));
		t1[p] = time_pair(A[p], B[p], np, n, e0, e1);
		t2[p] = time_pair(A[p], B[p], np, n, e0, e1);
	}
	for (int p = 0; p < pairs; ++p) t3[p] = time_pair(A[p], B[p], np, n, e0, e1);
	// cross pairs: the first pair's source with every other pair's destination
	printf("N %u records, %d buffer pairs (ps per record per pass)\n", n, pairs);
	for (int p = 0; p < pairs; ++p)
		printf("pair %d  a=%p b=%p  %.2f %.2f  later %.2f  (a0 -> b%d: %.2f)\n", p, (void *)A[p], (void *)B[p], t1[p],
		       t2[p], t3[p], p, time_pair(A[0], B[p], np, n, e0, e1));
	CK(hipGetLastError());
	return 0;
}
