// Probe 22 (round 6): can a record buffer be ASSEMBLED from fast physical memory? The level
// pattern's scatter rate follows the physical region behind the written buffer (probe 20,
// profiles/r06_placement/README.md), in runs several GB wide, and no allocation call selects the
// region. The virtual-memory API can: physical chunks (hipMemCreate) are scored one by one on the
// scatter pattern, and a buffer is then mapped from the fastest chunks into one virtual range.
//   1. a reference buffer and a uniform permutation (runs of 800 records, C4's level shape);
//   2. `scan` GB of physical chunks of `chunk` MB, each mapped and scored: runs streamed from the
//      reference, records scattered inside the chunk (ms per pass, best of 3);
//   3. buffers of n records assembled from the fastest chunks (F, F2), the slowest (S) and the
//      first ones in allocation order (M), plus a plain hipMalloc buffer (P);
//   4. the full level pattern (n records, runs of 800) from the reference into each, and the store's
//      ping-pong F <-> F2 against P <-> P2 (ms per pass).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_assemble tools/probe_assemble.hip
// Run:   tools/probe_assemble <records> <chunk MB> <scan GB>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t RUN = 800, BLOCK = 512;

__device__ inline uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

// one level's pattern: run b of RUN records streamed from src through LDS, each record written
// whole to dst[nxt[i]] (four 16-B pieces from four lanes); nxt < n
__global__ __launch_bounds__(BLOCK) void klevel(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                                const uint32_t *__restrict__ nxt, uint32_t n)
{
	__shared__ dv2 recs[1024 * 4];
	__shared__ uint32_t dsts[1024];
	const uint32_t b = blockIdx.x * RUN;
	if (b >= n) return;
	const uint32_t m = min(RUN, n - b);
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) recs[lslot(t >> 2, t & 3)] = src[(size_t)b * 4 + t];
	for (uint32_t i = threadIdx.x; i < m; i += BLOCK) dsts[i] = nxt[b + i];
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		dst[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
	}
}

static hipEvent_t e0, e1;

static float run_level(const dv2 *src, dv2 *dst, const uint32_t *nxt, uint32_t n, int reps)
{
	klevel<<<(n + RUN - 1) / RUN, BLOCK>>>(src, dst, nxt, n);   // warm-up
	float best = 1e30f;
	for (int r = 0; r < reps; ++r) {
		CK(hipEventRecord(e0));
		klevel<<<(n + RUN - 1) / RUN, BLOCK>>>(src, dst, nxt, n);
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		best = std::min(best, ms);
	}
	return best;
}

static std::vector<uint32_t> uniform_perm(uint32_t n, uint64_t seed)
{
	std::vector<uint32_t> p(n);
	std::iota(p.begin(), p.end(), 0u);
	std::mt19937_64 g(seed);
	std::shuffle(p.begin(), p.end(), g);
	return p;
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atof(argv[1]) : 100000000u;
	const size_t chunk = (argc > 2 ? (size_t)atoi(argv[2]) : 1024) << 20;
	const size_t scan = (argc > 3 ? (size_t)atoi(argv[3]) : 150) << 30;
	const size_t bytes = (size_t)n * 64;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	hipMemAllocationProp prop = {};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = 0;
	size_t gran = 0;
	CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
	if (chunk % gran) { printf("chunk must be a multiple of %zu\n", gran); return 1; }
	hipMemAccessDesc acc = {};
	acc.location = prop.location;
	acc.flags = hipMemAccessFlagsProtReadWrite;

	dv2 *ref;
	uint32_t *perm_n, *perm_c;
	CK(hipMalloc(&ref, bytes));
	CK(hipMemset(ref, 0, bytes));
	{
		auto p = uniform_perm(n, 7);
		CK(hipMalloc(&perm_n, (size_t)n * 4));
		CK(hipMemcpy(perm_n, p.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	}
	const uint32_t mc = (uint32_t)(chunk / 64);
	{
		auto p = uniform_perm(mc, 9);
		CK(hipMalloc(&perm_c, (size_t)mc * 4));
		CK(hipMemcpy(perm_c, p.data(), (size_t)mc * 4, hipMemcpyHostToDevice));
	}
	// plain buffers first (the store's own allocations come before any search)
	dv2 *P, *P2;
	CK(hipMalloc(&P, bytes));
	CK(hipMalloc(&P2, bytes));

	// 2. physical chunks, mapped one after another into one scratch range, scored one by one
	const size_t nch = scan / chunk;
	void *scratch = nullptr;
	CK(hipMemAddressReserve(&scratch, nch * chunk, 0, nullptr, 0));
	std::vector<hipMemGenericAllocationHandle_t> h(nch);
	std::vector<float> score(nch);
	size_t got = 0;
	for (; got < nch; ++got) {
		if (hipMemCreate(&h[got], chunk, &prop, 0) != hipSuccess) { (void)hipGetLastError(); break; }
		char *va = (char *)scratch + got * chunk;
		CK(hipMemMap(va, chunk, 0, h[got], 0));
		CK(hipMemSetAccess(va, chunk, &acc, 1));
		score[got] = run_level(ref, (dv2 *)va, perm_c, mc, 3);
	}
	printf("records %u (%.2f GB), chunks of %zu MB: %zu scored (%.0f GB)\n", n, bytes / 1e9, chunk >> 20, got,
	       got * (double)chunk / (1 << 30));
	printf("chunk scores (ms per pass of %u records), allocation order:\n", mc);
	for (size_t i = 0; i < got; ++i) printf("%.3f%s", score[i], (i + 1) % 16 ? " " : "\n");
	printf("\n");
	const size_t need = (bytes + chunk - 1) / chunk;
	if (got < 3 * need) { printf("not enough chunks for three buffers\n"); return 1; }
	std::vector<size_t> order(got);
	std::iota(order.begin(), order.end(), (size_t)0);
	std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return score[a] < score[b]; });

	// 3. assembled buffers: the same physical chunks mapped a second time into a buffer's own range
	auto assemble = [&](const std::vector<size_t> &ids) {
		void *va = nullptr;
		CK(hipMemAddressReserve(&va, need * chunk, 0, nullptr, 0));
		for (size_t k = 0; k < need; ++k) CK(hipMemMap((char *)va + k * chunk, chunk, 0, h[ids[k]], 0));
		CK(hipMemSetAccess(va, need * chunk, &acc, 1));
		return (dv2 *)va;
	};
	std::vector<size_t> fast(order.begin(), order.begin() + need), fast2(order.begin() + need, order.begin() + 2 * need),
		slow(order.end() - need, order.end()), first(need);
	std::iota(first.begin(), first.end(), (size_t)0);
	auto span = [&](const std::vector<size_t> &ids) {
		float lo = 1e30f, hi = 0;
		for (size_t i : ids) { lo = std::min(lo, score[i]); hi = std::max(hi, score[i]); }
		printf("[%.3f-%.3f]", lo, hi);
	};
	dv2 *F = assemble(fast), *F2 = assemble(fast2), *S = assemble(slow), *M = assemble(first);
	printf("F (fastest chunks) "); span(fast); printf(", F2 "); span(fast2); printf(", S (slowest) "); span(slow);
	printf(", M (first) "); span(first); printf("\n");

	// 4. the level pattern from the reference into each, then the ping-pong pairs
	const char *nm[6] = {"F", "F2", "S", "M", "P", "P2"};
	dv2 *bufs[6] = {F, F2, S, M, P, P2};
	for (int r = 0; r < 2; ++r) {
		printf("round %d, ref -> buffer (ms per pass):", r);
		for (int b = 0; b < 6; ++b) printf(" %s %.4f", nm[b], run_level(ref, bufs[b], perm_n, n, 4));
		printf("\n");
		const float ff = run_level(F, F2, perm_n, n, 4) + run_level(F2, F, perm_n, n, 4);
		const float pp = run_level(P, P2, perm_n, n, 4) + run_level(P2, P, perm_n, n, 4);
		printf("round %d, ping-pong (ms per pass, both directions averaged): F<->F2 %.4f, P<->P2 %.4f\n", r, ff / 2, pp / 2);
	}
	CK(hipDeviceSynchronize());
	return 0;
}
