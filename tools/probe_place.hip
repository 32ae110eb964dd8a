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

// mode 1 (argv[3] = 1): allocation strategies instead of plain pairs -- plain, one allocation of
// 2n records split in two, a 4x oversized allocation used from its middle, hipMallocAsync from the
// default pool, and plain after a 100 GB allocation was made and freed
static int strategies(uint32_t n, const uint32_t *np, hipEvent_t e0, hipEvent_t e1)
{
	const size_t B = (size_t)n * 64;
	const char *names[] = {"plain", "plain", "one 2n block", "4x block, middle", "hipMallocAsync", "plain after 100 GB"};
	for (int sidx = 0; sidx < 6; ++sidx) {
		void *pa = nullptr, *pb = nullptr;
		dv2 *a = nullptr, *b = nullptr;
		if (sidx <= 1) { CK(hipMalloc(&pa, B)); CK(hipMalloc(&pb, B)); a = (dv2 *)pa; b = (dv2 *)pb; }
		else if (sidx == 2) { CK(hipMalloc(&pa, 2 * B)); a = (dv2 *)pa; b = (dv2 *)((char *)pa + B); }
		else if (sidx == 3) { CK(hipMalloc(&pa, 4 * B)); a = (dv2 *)((char *)pa + B); b = (dv2 *)((char *)pa + 2 * B); }
		else if (sidx == 4) { CK(hipMallocAsync(&pa, B, 0)); CK(hipMallocAsync(&pb, B, 0)); CK(hipDeviceSynchronize()); a = (dv2 *)pa; b = (dv2 *)pb; }
		else {
			void *big = nullptr;
			CK(hipMalloc(&big, (size_t)100 << 30));
			CK(hipMemset(big, 0, (size_t)1 << 30));
			CK(hipFree(big));
			CK(hipMalloc(&pa, B)); CK(hipMalloc(&pb, B)); a = (dv2 *)pa; b = (dv2 *)pb;
		}
		CK(hipMemset(a, 0, B));
		CK(hipMemset(b, 0, B));
		const float t1 = time_pair(a, b, np, n, e0, e1), t2 = time_pair(a, b, np, n, e0, e1);
		printf("%-20s a=%p b=%p  %.2f %.2f ps/rec\n", names[sidx], (void *)a, (void *)b, t1, t2);
		fflush(stdout);
		if (sidx == 4) { CK(hipFreeAsync(pa, 0)); CK(hipFreeAsync(pb, 0)); CK(hipDeviceSynchronize()); }
		else { CK(hipFree(pa)); if (pb) CK(hipFree(pb)); }
	}
	return 0;
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
	const int pairs = argc > 2 ? atoi(argv[2]) : 6;
	const int mode = argc > 3 ? atoi(argv[3]) : 0;
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
	if (mode == 1) return strategies(n, np, e0, e1);
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
