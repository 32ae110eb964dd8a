// Probe 9: the deferred split's posterior gather at ONE N = 8 RANK'S SHAPE (1.25e7 records in
// runs of 100, 125k columns per level, 256-thread workgroups, one record per thread: the shape
// k_lord_defer<256, 1> runs at; VERDICT r04 "next" item 1). Each variant streams a column's run
// into LDS, does a token amount of arithmetic and writes every record whole to a random slot
// (the level move); they differ only in the per-record posterior the deferred kernel gathers:
//   move        : no gather, 4-B next position per record (the fused kernel's pattern)
//   defer       : 8-B payload {next, prev feature}, 32-B gather tab[prev] (2 x 16-B loads) --
//                 the deferred kernel's pattern
//   indep       : the same gather, index hashed from the position (no wait on the payload):
//                 what the payload -> gather dependence costs
//   pair        : the gather split over two lanes per record (one 16-B load each, the pair on
//                 one line), the halves meeting in LDS
//   tab16       : a 16-B gather (one load): the floor of a smaller posterior
//   pipe        : persistent workgroups, the NEXT column's payload loaded while this column's
//                 records stream in (the gather of a column issues with its records)
// usage: probe_defer8 [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

struct __attribute__((aligned(64))) Rec { double v[8]; };
struct __attribute__((aligned(32))) Post { double mo, so, mu, sig; };
constexpr int RUN = 100, BLOCK = 256;
constexpr uint32_t NPREV = 125000;

__device__ __forceinline__ uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }
__device__ __forceinline__ uint32_t hash32(uint32_t x)
{
	x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
	return x;
}

enum { M_MOVE, M_DEFER, M_INDEP, M_PAIR, M_TAB16 };

typedef double ntv2 __attribute__((ext_vector_type(2)));

template <int MODE, bool NTL = false, bool NTS = false>
__global__ __launch_bounds__(BLOCK) void k_col(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                              const uint32_t *__restrict__ nxt, const uint2 *__restrict__ pay,
                                              const Post *__restrict__ tab, double *__restrict__ out)
{
	__shared__ double2 recs[BLOCK * 4];
	__shared__ uint32_t dsts[BLOCK];
	__shared__ double2 pst[BLOCK * 2];
	const uint32_t t = threadIdx.x;
	const size_t sb = (size_t)blockIdx.x * RUN;
	const uint32_t m = RUN;
	const uint32_t i = min(t, m - 1);
	uint2 q;
	if constexpr (MODE == M_MOVE) q = make_uint2(nxt[sb + i], 0u);
	else q = pay[sb + i];
	uint32_t pp = 0;   // pair: the previous feature of record t >> 1
	if constexpr (MODE == M_PAIR) pp = pay[sb + min(t >> 1, m - 1)].y;
	const double2 *s = reinterpret_cast<const double2 *>(src + sb);
	double2 v[4];
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t u = min(t + k * BLOCK, m * 4 - 1);
		if constexpr (NTL) {
			const ntv2 w = __builtin_nontemporal_load(reinterpret_cast<const ntv2 *>(s) + u);
			v[k] = make_double2(w.x, w.y);
		} else {
			v[k] = s[u];
		}
	}
	Post p = {0, 0, 0, 0};
	if constexpr (MODE == M_DEFER) p = tab[q.y];
	if constexpr (MODE == M_INDEP) p = tab[hash32((uint32_t)(sb + i)) % NPREV];
	if constexpr (MODE == M_TAB16) {
		const double2 h = reinterpret_cast<const double2 *>(tab)[q.y];
		p.mo = h.x; p.so = h.y;
	}
	if constexpr (MODE == M_PAIR) {
		if (t < 2 * m) pst[t] = reinterpret_cast<const double2 *>(tab)[2 * (size_t)pp + (t & 1)];
	}
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t u = t + k * BLOCK;
		recs[lslot(u >> 2, u & 3)] = v[k];
	}
	__syncthreads();
	double acc = 0.0;
	if (t < m) {
		if constexpr (MODE == M_PAIR) {
			const double2 a = pst[2 * t], b = pst[2 * t + 1];
			p.mo = a.x; p.so = a.y; p.mu = b.x; p.sig = b.y;
		}
		double2 r0 = recs[lslot(t, 0)], r1 = recs[lslot(t, 1)];
		r0.x += (p.mu - p.mo) * r0.y;
		r0.y += (p.sig - p.so) * r1.x;
		acc = r0.x * r0.y;
		recs[lslot(t, 0)] = r0;
		dsts[t] = q.x;
	}
	__syncthreads();
	double2 *d = reinterpret_cast<double2 *>(dst);
	for (uint32_t u = t; u < m * 4; u += BLOCK) {
		const double2 w = recs[lslot(u >> 2, u & 3)];
		const size_t o = (size_t)dsts[u >> 2] * 4 + (u & 3);
		if constexpr (NTS) {
			ntv2 z;
			z.x = w.x;
			z.y = w.y;
			__builtin_nontemporal_store(z, reinterpret_cast<ntv2 *>(d) + o);
		} else {
			d[o] = w;
		}
	}
	if (acc == 12345.0) out[blockIdx.x] = acc;   // keeps the arithmetic
}

// persistent: workgroup w sweeps columns w, w + G, ...; the next column's payload is loaded
// before this column's records are consumed
__global__ __launch_bounds__(BLOCK) void k_pipe(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                               const uint2 *__restrict__ pay, const Post *__restrict__ tab,
                                               double *__restrict__ out, uint32_t ncol)
{
	__shared__ double2 recs[BLOCK * 4];
	__shared__ uint32_t dsts[BLOCK];
	const uint32_t t = threadIdx.x;
	const uint32_t m = RUN;
	const uint32_t i = min(t, m - 1);
	uint32_t col = blockIdx.x;
	if (col >= ncol) return;
	uint2 q = pay[(size_t)col * RUN + i];
	double accs = 0.0;
	for (; col < ncol; col += gridDim.x) {
		const size_t sb = (size_t)col * RUN;
		const double2 *s = reinterpret_cast<const double2 *>(src + sb);
		double2 v[4];
#pragma unroll
		for (int k = 0; k < 4; ++k) v[k] = s[min(t + k * BLOCK, m * 4 - 1)];
		const Post p = tab[q.y];
		const uint32_t nc = col + gridDim.x;
		const uint2 qn = nc < ncol ? pay[(size_t)nc * RUN + i] : make_uint2(0u, 0u);
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			const uint32_t u = t + k * BLOCK;
			recs[lslot(u >> 2, u & 3)] = v[k];
		}
		__syncthreads();
		if (t < m) {
			double2 r0 = recs[lslot(t, 0)], r1 = recs[lslot(t, 1)];
			r0.x += (p.mu - p.mo) * r0.y;
			r0.y += (p.sig - p.so) * r1.x;
			accs += r0.x * r0.y;
			recs[lslot(t, 0)] = r0;
			dsts[t] = q.x;
		}
		__syncthreads();
		double2 *d = reinterpret_cast<double2 *>(dst);
		for (uint32_t u = t; u < m * 4; u += BLOCK) d[(size_t)dsts[u >> 2] * 4 + (u & 3)] = recs[lslot(u >> 2, u & 3)];
		__syncthreads();   // recs / dsts are rewritten by the next column
		q = qn;
	}
	if (accs == 12345.0) out[blockIdx.x] = accs;
}

// the previous level's posterior kernel: rewrites the table before each level (its lines then come
// from another XCD's L2 / the MALL, not from this XCD's L2)
__global__ void k_refresh(Post *tab, uint32_t n, double v)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) tab[i] = Post{v, v, v, v};
}

int main(int argc, char **argv)
{
	const int reps = argc > 1 ? atoi(argv[1]) : 3;
	const uint32_t ncol = 125000, n = ncol * RUN;
	std::mt19937_64 g(7);
	std::vector<uint32_t> perm(n);
	for (uint32_t i = 0; i < n; i++) perm[i] = i;
	std::shuffle(perm.begin(), perm.end(), g);
	std::vector<uint2> ph(n);
	for (uint32_t i = 0; i < n; i++) ph[i] = make_uint2(perm[i], (uint32_t)(g() % NPREV));
	Rec *a, *b;
	uint32_t *nx;
	uint2 *pay;
	Post *tab;
	double *out;
	CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&b, (size_t)n * 64));
	CK(hipMalloc(&nx, (size_t)n * 4)); CK(hipMalloc(&pay, (size_t)n * 8));
	CK(hipMalloc(&tab, (size_t)NPREV * sizeof(Post))); CK(hipMalloc(&out, (size_t)ncol * 8));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(b, 0, (size_t)n * 64));
	CK(hipMemset(tab, 0, (size_t)NPREV * sizeof(Post)));
	CK(hipMemcpy(nx, perm.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(pay, ph.data(), (size_t)n * 8, hipMemcpyHostToDevice));
	int cus = 0;
	CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0));
		for (int it = 0; it < 10; it++) launch();
		CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1));
		printf("%-44s %8.1f us\n", name, ms * 100.0f);   // ms / 10 launches -> us
		fflush(stdout);
	};
	printf("# 1.25e7 records, runs of %d, %u columns, 256-thread workgroups, %d CUs\n", RUN, ncol, cus);
	double rv = 0.0;
	auto refresh = [&] { k_refresh<<<(NPREV + 255) / 256, 256>>>(tab, NPREV, rv); rv += 1.0; };
	for (int r = 0; r < reps; r++) {
		time("refresh alone", [&] { refresh(); });
		time("move + refresh", [&] { refresh(); k_col<M_MOVE><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer + refresh", [&] { refresh(); k_col<M_DEFER><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer + refresh, NT loads", [&] { refresh(); k_col<M_DEFER, true, false><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer + refresh, NT stores", [&] { refresh(); k_col<M_DEFER, false, true><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer + refresh, NT loads + stores", [&] { refresh(); k_col<M_DEFER, true, true><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("move, NT loads + stores", [&] { k_col<M_MOVE, true, true><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer (static table), NT loads + stores", [&] { k_col<M_DEFER, true, true><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("move (fused pattern)", [&] { k_col<M_MOVE><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("defer (payload -> 32-B gather)", [&] { k_col<M_DEFER><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("indep (hashed index, 32-B gather)", [&] { k_col<M_INDEP><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("pair (2 lanes x 16 B per record)", [&] { k_col<M_PAIR><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		time("tab16 (one 16-B gather)", [&] { k_col<M_TAB16><<<ncol, BLOCK>>>(a, b, nx, pay, tab, out); std::swap(a, b); });
		for (int wpc : {4, 8, 16})
		{
			char nm[64];
			snprintf(nm, sizeof(nm), "pipe (%d workgroups per CU)", wpc);
			const unsigned grid = (unsigned)(cus * wpc);
			time(nm, [&] { k_pipe<<<grid, BLOCK>>>(a, b, pay, tab, out, ncol); std::swap(a, b); });
		}
	}
	return 0;
}
