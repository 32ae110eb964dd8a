// Ceiling probe 5: does the order of records inside the next level's columns matter for the
// level kernel's scatter? 1e8 records in runs of 800 (one workgroup per run), every record
// sent to a random column of the next level (125k columns).
//   rand : destination slots inside a column in random order (rows ascending = unrelated to
//          the source position: the level store as built today)
//   src  : destination slots inside a column in ascending SOURCE position (stable counting
//          sort of the source positions by destination column): workgroups running at the
//          same time write neighbouring slots of each destination column
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int RUN = 800;

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void kB(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt, const float *__restrict__ xs)
{
	const size_t b = (size_t)blockIdx.x * RUN;
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		dv2 a = ((const dv2 *)(src + b + i))[c];
		a.x += xs[b + i];
		((dv2 *)(dst + nxt[b + i]))[c] = a;
	}
}

__global__ void kcopy(const Rec *__restrict__ src, Rec *__restrict__ dst, uint32_t n)
{
	const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
	if (t < (size_t)n * 4) ((dv2 *)dst)[t] = ((const dv2 *)src)[t];
}

int main(int argc, char **argv)
{
	const uint32_t n = 100000000u, ncol = 125000;
	const uint32_t nrun = n / RUN;
	std::vector<uint32_t> col(n), cnt(ncol + 1, 0), hr(n), hs(n);
	std::mt19937_64 g(7);
	for (uint32_t p = 0; p < n; p++) { col[p] = (uint32_t)(g() % ncol); cnt[col[p] + 1]++; }
	for (uint32_t c = 0; c < ncol; c++) cnt[c + 1] += cnt[c];
	{
		std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
		for (uint32_t p = 0; p < n; p++) hs[p] = fill[col[p]]++;
	}
	// random order inside each column: shuffle each column's slot list
	{
		std::vector<uint32_t> inv(n);
		for (uint32_t p = 0; p < n; p++) inv[hs[p]] = p;
		for (uint32_t c = 0; c < ncol; c++) std::shuffle(inv.begin() + cnt[c], inv.begin() + cnt[c + 1], g);
		for (uint32_t q = 0; q < n; q++) hr[inv[q]] = q;
	}
	std::vector<uint32_t> hp(n);
	for (uint32_t i = 0; i < n; i++) hp[i] = i;
	std::shuffle(hp.begin(), hp.end(), g);
	uint32_t *nr, *ns, *np; Rec *a, *bb; float *xs;
	CK(hipMalloc(&nr, (size_t)n * 4)); CK(hipMalloc(&ns, (size_t)n * 4)); CK(hipMalloc(&np, (size_t)n * 4));
	CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMalloc(&xs, (size_t)n * 4));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(bb, 0, (size_t)n * 64)); CK(hipMemset(xs, 0, (size_t)n * 4));
	CK(hipMemcpy(nr, hr.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(ns, hs.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(np, hp.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
		printf("%-44s %.3f ms  %.3g rows/s\n", name, ms, n / ms * 1e3);
	};
	time("copy (streaming)", [&] { kcopy<<<(unsigned)(((size_t)n * 4 + 255) / 256), 256>>>(a, bb, n); });
	time("full random permutation 512", [&] { kB<512><<<nrun, 512>>>(a, bb, np, xs); });
	time("column slots random 512", [&] { kB<512><<<nrun, 512>>>(a, bb, nr, xs); });
	time("column slots by source 256", [&] { kB<256><<<nrun, 256>>>(a, bb, ns, xs); });
	time("column slots by source 512", [&] { kB<512><<<nrun, 512>>>(a, bb, ns, xs); });
	time("column slots by source 1024", [&] { kB<1024><<<nrun, 1024>>>(a, bb, ns, xs); });
	return 0;
}
