// Probe 20 (round 6): what in a record buffer's placement sets the level
// pattern's scatter rate? For candidate buffers of n 64-B records -- plain hipMalloc ones allocated
// one after another, and buffers built with the virtual-memory API (hipMemCreate physical chunks of
// the recommended granularity, mapped into one reserved range) -- this times, per buffer:
//   w   the level pattern with the buffer as DESTINATION (runs of 400 streamed from a reference
//       buffer through LDS, whole records scattered into the candidate by a uniform permutation);
//   r   the same with the candidate as SOURCE (streamed) and the reference as destination;
//   t4k / t64k / t2m   dependent-free random 8-B reads, one per page of 4 KB / 64 KB / 2 MB
//       (2^22 touches): the address-translation cost for that fragment size -- a buffer backed by
//       small fragments misses the GPU's TLBs on the finer pages where one of large fragments hits;
//   c   a streaming copy reference -> candidate.
// If the scatter rate follows the translation probes, the fragment size of the backing is the
// cause (and an allocation that guarantees large fragments fixes it); if not, it is elsewhere.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_frag tools/probe_frag.hip
// Run:   tools/probe_frag <records> <plain buffers> <vmm buffers>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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

// the mirror pattern: run b of RUN consecutive destination records is gathered from random source
// positions (the same permutation, read as "where does my record come from"), staged through LDS,
// and written out contiguously
__global__ __launch_bounds__(BLOCK) void kgather(const dv2 *__restrict__ src, dv2 *__restrict__ dst,
                                                 const uint32_t *__restrict__ from, uint32_t n)
{
	__shared__ dv2 recs[512 * 4];
	const uint32_t b = blockIdx.x * RUN;
	const uint32_t m = min(RUN, n - b);
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		recs[lslot(i, c)] = src[(size_t)from[b + i] * 4 + c];
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK)
		dst[(size_t)b * 4 + t] = recs[lslot(t >> 2, t & 3)];
}

__global__ void kcopy(const dv2 *__restrict__ src, dv2 *__restrict__ dst, size_t n)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		dst[i] = src[i];
}

__device__ inline uint64_t mix(uint64_t z)
{
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

// one 8-B read per touch at a random page (of 2^pshift bytes) and a random line inside it; the
// sum goes to out so that nothing is optimised away
__global__ void ktouch(const double *__restrict__ buf, size_t bytes, uint32_t pshift, uint32_t touches, double *out)
{
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= touches) return;
	const uint64_t h = mix((uint64_t)i * 0x2545F4914F6CDD1Dull + pshift);
	const uint64_t pages = bytes >> pshift;
	const uint64_t page = h % pages;
	const uint64_t off = (page << pshift) + ((h >> 40) % ((1ull << pshift) / 64)) * 64;
	const double v = buf[off / 8];
	if (v == 1234.5) out[0] = v;
}

static hipEvent_t e0, e1;

static float timed(void (*f)(void *), void *arg, int reps)
{
	float best = 1e30f;
	for (int r = 0; r < reps; ++r) {
		CK(hipEventRecord(e0));
		f(arg);
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		best = std::min(best, ms);
	}
	return best;
}

struct Job {
	dv2 *a, *b;
	const uint32_t *perm;
	uint32_t n;
	double *out;
	uint32_t pshift;
};

static void run_scatter(void *p)
{
	Job *j = (Job *)p;
	const uint32_t nrun = (j->n + RUN - 1) / RUN;
	for (int it = 0; it < 4; ++it) klds<<<nrun, BLOCK>>>(j->a, j->b, j->perm, j->n);
}

static void run_gather(void *p)
{
	Job *j = (Job *)p;
	const uint32_t nrun = (j->n + RUN - 1) / RUN;
	for (int it = 0; it < 4; ++it) kgather<<<nrun, BLOCK>>>(j->a, j->b, j->perm, j->n);
}

static void run_copy(void *p)
{
	Job *j = (Job *)p;
	for (int it = 0; it < 4; ++it) kcopy<<<4096, 256>>>(j->a, j->b, (size_t)j->n * 4);
}

__global__ void kfill(dv2 *__restrict__ dst, size_t n, double v)
{
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		dst[i] = dv2{v, v};
}

static void run_fill(void *p)
{
	Job *j = (Job *)p;
	for (int it = 0; it < 8; ++it) kfill<<<4096, 256>>>(j->a, (size_t)j->n * 4, 1.0);
}

static void run_touch(void *p)
{
	Job *j = (Job *)p;
	const uint32_t touches = 1u << 22;
	ktouch<<<touches / 256, 256>>>((const double *)j->a, (size_t)j->n * 64, j->pshift, touches, j->out);
}

static float time_pair(dv2 *a, dv2 *b, const uint32_t *perm, uint32_t n)
{
	const uint32_t nrun = (n + RUN - 1) / RUN;
	float best = 1e30f;
	for (int rep = 0; rep < 3; ++rep) {
		CK(hipEventRecord(e0));
		for (int it = 0; it < 4; ++it) klds<<<nrun, BLOCK>>>(it & 1 ? b : a, it & 1 ? a : b, perm, n);
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		best = std::min(best, ms);
	}
	return best / 4 * 1e9f / n;
}

// mode "pads": both record buffers of the level pattern carved from ONE physical allocation
// (hipMemCreate) at a chosen distance: buffer B starts `pad` bytes after buffer A ends. If the
// rate is set by how the read and write streams' physical addresses alias in the memory system,
// it follows the pad systematically, the same way on every box
static int pads_mode(uint32_t n, const uint32_t *perm_d, int nalloc)
{
	const size_t bytes = (size_t)n * 64, MB = (size_t)1 << 20;
	const size_t pads[] = {0, 4096, 64 << 10, 256 << 10, 1 * MB, 2 * MB, 3 * MB, 4 * MB, 6 * MB, 8 * MB, 16 * MB, 32 * MB,
	                       64 * MB, 96 * MB, 128 * MB, 192 * MB, 256 * MB};
	const int np = sizeof(pads) / sizeof(pads[0]);
	hipMemAllocationProp prop = {};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = 0;
	const size_t total = 2 * bytes + 256 * MB + 2 * MB;
	for (int a = 0; a < nalloc; ++a) {
		void *va = nullptr;
		hipMemGenericAllocationHandle_t h;
		CK(hipMemAddressReserve(&va, total, 0, nullptr, 0));
		CK(hipMemCreate(&h, total, &prop, 0));
		CK(hipMemMap(va, total, 0, h, 0));
		hipMemAccessDesc acc = {};
		acc.location = prop.location;
		acc.flags = hipMemAccessFlagsProtReadWrite;
		CK(hipMemSetAccess(va, total, &acc, 1));
		CK(hipMemset(va, 0, total));
		printf("allocation %d at %p, pair pattern (ps per record) by pad:", a, va);
		for (int i = 0; i < np; ++i) {
			dv2 *A = (dv2 *)va, *B = (dv2 *)((char *)va + bytes + pads[i]);
			printf(" %zu:%.2f", pads[i] >> 10, time_pair(A, B, perm_d, n));
		}
		printf(" (pad in KB)\n");
		fflush(stdout);
		// the allocation stays: the next one comes from elsewhere in the pool
	}
	return 0;
}

// mode "bigwin": one large hipMalloc of `gb` GB; the level pattern (destination side, from a plain
// reference buffer) into windows of n records at every `step_mb` MB of it: does the rate vary inside
// one allocation, and with what period?
static int bigwin_mode(uint32_t n, const uint32_t *perm_d, int gb, int step_mb)
{
	const size_t bytes = (size_t)n * 64, total = (size_t)gb << 30, step = (size_t)step_mb << 20;
	dv2 *ref, *big;
	CK(hipMalloc(&ref, bytes));
	CK(hipMemset(ref, 0, bytes));
	CK(hipMalloc(&big, total));
	CK(hipMemset(big, 0, total));
	printf("one allocation of %d GB at %p; windows of %.2f GB every %d MB; w = ps per record (destination), "
	       "c = streaming copy into it\n", gb, (void *)big, bytes / 1e9, step_mb);
	for (size_t o = 0; o + bytes <= total; o += step) {
		dv2 *w = (dv2 *)((char *)big + o);
		Job jw = {ref, w, perm_d, n, nullptr, 0};
		const float ws = timed(run_scatter, &jw, 2) / 4 * 1e9f / n;
		const float c = timed(run_copy, &jw, 2) / 4 * 1e9f / n;
		printf("offset %6zu MB  w %6.2f  c %6.2f\n", o >> 20, ws, c);
		fflush(stdout);
	}
	return 0;
}

int main(int argc, char **argv)
{
	const uint32_t n = argc > 1 ? (uint32_t)atof(argv[1]) : 10000000u;
	const int nplain = argc > 2 ? atoi(argv[2]) : 12;
	const int nvmm = argc > 3 ? atoi(argv[3]) : 4;
	const size_t bytes = (size_t)n * 64;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	// uniform random permutation (host Fisher-Yates with a fixed seed)
	std::vector<uint32_t> perm(n);
	for (uint32_t i = 0; i < n; ++i) perm[i] = i;
	uint64_t s = 12345;
	for (uint32_t i = n - 1; i > 0; --i) {
		s = s * 6364136223846793005ull + 1442695040888963407ull;
		std::swap(perm[i], perm[(s >> 33) % (i + 1)]);
	}
	uint32_t *perm_d;
	double *out;
	dv2 *ref;
	CK(hipMalloc(&perm_d, (size_t)n * 4));
	CK(hipMemcpy(perm_d, perm.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMalloc(&out, 8));
	if (argc > 2 && std::string(argv[2]) == "pads") return pads_mode(n, perm_d, argc > 3 ? atoi(argv[3]) : 4);
	if (argc > 2 && std::string(argv[2]) == "bigwin")
		return bigwin_mode(n, perm_d, argc > 3 ? atoi(argv[3]) : 64, argc > 4 ? atoi(argv[4]) : 1024);
	CK(hipMalloc(&ref, bytes));
	CK(hipMemset(ref, 0, bytes));
	std::vector<dv2 *> bufs;
	std::vector<const char *> kind;
	for (int i = 0; i < nplain; ++i) {
		dv2 *p;
		CK(hipMalloc(&p, bytes));
		CK(hipMemset(p, 0, bytes));
		bufs.push_back(p);
		kind.push_back("plain");
	}
	// virtual-memory API: physical chunks of the recommended granularity mapped into one range
	hipMemAllocationProp prop = {};
	prop.type = hipMemAllocationTypePinned;
	prop.location.type = hipMemLocationTypeDevice;
	prop.location.id = 0;
	size_t gran = 0, gmin = 0;
	CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
	CK(hipMemGetAllocationGranularity(&gmin, &prop, hipMemAllocationGranularityMinimum));
	printf("vmm granularity: recommended %zu, minimum %zu\n", gran, gmin);
	const size_t vbytes = (bytes + gran - 1) / gran * gran;
	const size_t GB = (size_t)1 << 30;
	for (int i = 0; i < nvmm; ++i) {
		// kinds: one physical allocation of the whole buffer (default VA alignment); the same rounded
		// up to whole GB in a 1 GB-aligned range; 2 MB pieces; 64 MB pieces
		const int kd = i % 4;
		const size_t whole = kd == 1 ? (bytes + GB - 1) / GB * GB : vbytes;
		const size_t chunk = kd <= 1 ? whole : kd == 2 ? std::max(gran, (size_t)2 << 20) : std::max(gran, (size_t)64 << 20);
		const size_t total = (whole + chunk - 1) / chunk * chunk;
		void *va = nullptr;
		CK(hipMemAddressReserve(&va, total, kd == 1 ? GB : 0, nullptr, 0));
		for (size_t o = 0; o < total; o += chunk) {
			hipMemGenericAllocationHandle_t h;
			CK(hipMemCreate(&h, chunk, &prop, 0));
			CK(hipMemMap((char *)va + o, chunk, 0, h, 0));
		}
		hipMemAccessDesc acc = {};
		acc.location = prop.location;
		acc.flags = hipMemAccessFlagsProtReadWrite;
		CK(hipMemSetAccess(va, total, &acc, 1));
		CK(hipMemset(va, 0, bytes));
		bufs.push_back((dv2 *)va);
		kind.push_back(kd == 0 ? "vmm-1" : kd == 1 ? "vmm-1G" : kd == 2 ? "vmm-2M" : "vmm-64M");
		printf("buffer %zu: %s at %p (%zu bytes mapped)\n", bufs.size() - 1, kind.back(), va, total);
	}
	for (int i = 0; i < nplain; ++i) printf("buffer %d: plain at %p\n", i, (void *)bufs[i]);
	CK(hipDeviceSynchronize());
	printf("records %u (%.2f GB per buffer); ps per record for w / r / c, ns per touch for t4k / t64k / t2m\n", n,
	       bytes / 1e9);
	printf("%-3s %-8s %8s %8s %8s %8s %8s %8s %8s %8s\n", "#", "kind", "w", "r", "c", "t4k", "t64k", "t2m", "gsrc",
	       "gdst");
	for (int pass = 0; pass < 2; ++pass)
		for (size_t i = 0; i < bufs.size(); ++i) {
			Job jw = {ref, bufs[i], perm_d, n, out, 0}, jr = {bufs[i], ref, perm_d, n, out, 0};
			const float w = timed(run_scatter, &jw, 2) / 4 * 1e9f / n;
			const float r = timed(run_scatter, &jr, 2) / 4 * 1e9f / n;
			const float c = timed(run_copy, &jw, 2) / 4 * 1e9f / n;
			float t[3];
			const uint32_t sh[3] = {12, 16, 21};
			for (int q = 0; q < 3; ++q) {
				Job jt = {bufs[i], nullptr, nullptr, n, out, sh[q]};
				t[q] = timed(run_touch, &jt, 3) * 1e6f / (1u << 22);
			}
			// gather: the candidate as the randomly read source (gsrc), or as the contiguously written
			// destination of a gather from the reference (gdst)
			Job jg = {bufs[i], ref, perm_d, n, out, 0}, jg2 = {ref, bufs[i], perm_d, n, out, 0};
			const float gs = timed(run_gather, &jg, 2) / 4 * 1e9f / n;
			const float gd = timed(run_gather, &jg2, 2) / 4 * 1e9f / n;
			printf("%-3zu %-8s %8.2f %8.2f %8.2f %8.3f %8.3f %8.3f %8.2f %8.2f\n", i, kind[i], w, r, c, t[0], t[1], t[2],
			       gs, gd);
			fflush(stdout);
		}
	// streaming-write rate of each 256 MB window of every buffer (ps per 64 B): is a buffer slow as a
	// whole, or in patches?
	const size_t win = (size_t)256 << 20;
	if (bytes >= 2 * win) {
		printf("windows of 256 MB, streaming writes, ps per 64 B:\n");
		for (size_t i = 0; i < bufs.size(); ++i) {
			printf("%-3zu %-8s", i, kind[i]);
			for (size_t o = 0; o + win <= bytes; o += win) {
				Job jf = {(dv2 *)((char *)bufs[i] + o), nullptr, nullptr, (uint32_t)(win / 64), out, 0};
				printf(" %5.1f", timed(run_fill, &jf, 3) / 8 * 1e9f / (win / 64));
			}
			printf("\n");
			fflush(stdout);
		}
	}
	return 0;
}
