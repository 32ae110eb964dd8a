// Ceiling probe 8: the deferred split kernel's memory pattern. 1e8 64-B records in runs of 800
// read contiguously, each record written whole to a random position (the level move), plus
// per record one random gather from a posterior table (the previous level's correction):
//   none            : the move alone (= the fused level kernel's pattern)
//   tab 32B x 125k  : 4 MB table (C4: 125k features per level, 32-B posterior entries)
//   tab 16B x 125k  : 2 MB table
//   tab 32B x 16k   : 512 KB table
// and the same with the per-record index stream (lpidx + lpx, 8 B) the kernel reads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
constexpr int RUN = 800;

template <int BLOCK, int TB>
__global__ __launch_bounds__(BLOCK) void kD(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt, const uint32_t *__restrict__ pidx,
                                             const dv2 *__restrict__ tab)
{
	__shared__ dv2 lds[RUN * 4];
	const size_t b = (size_t)blockIdx.x * RUN;
	dv2 t0[2], t1[2];
	for (int u = 0; u < 2; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (TB > 0 && i < RUN) {
			const dv2 *tp = tab + (size_t)pidx[b + i] * (TB / 16);
			t0[u] = tp[0];
			t1[u] = TB == 32 ? tp[1] : t0[u];
		}
	}
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) lds[t] = ((const dv2 *)(src + b))[t];
	__syncthreads();
	for (int u = 0; u < 2; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (TB > 0 && i < RUN) {
			dv2 a = lds[i * 4];
			a.x += t0[u].x * t1[u].y;
			a.y += t0[u].y * t1[u].x;
			lds[i * 4] = a;
		}
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		((dv2 *)(dst + nxt[b + i]))[c] = lds[t];
	}
}


// the real kernel's per-record streams: lx, lnext, lpidx, lpx as four 4-B arrays (S4) or one
// packed 16-B record (PK)
template <int BLOCK, bool PK>
__global__ __launch_bounds__(BLOCK) void kE(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt, const uint32_t *__restrict__ pidx,
                                             const float *__restrict__ lx, const float *__restrict__ lpx,
                                             const uint4 *__restrict__ pay, const dv2 *__restrict__ tab)
{
	__shared__ dv2 lds[RUN * 4];
	__shared__ uint32_t dsts[RUN];
	const size_t b = (size_t)blockIdx.x * RUN;
	dv2 t0[2], t1[2];
	float xv[2], pxv[2];
	for (int u = 0; u < 2; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < RUN) {
			uint32_t pi;
			if (PK) {
				const uint4 q = pay[b + i];
				xv[u] = __uint_as_float(q.x); dsts[i] = q.y; pi = q.z; pxv[u] = __uint_as_float(q.w);
			} else {
				xv[u] = lx[b + i]; pi = pidx[b + i]; pxv[u] = lpx[b + i];
			}
			const dv2 *tp = tab + (size_t)pi * 2;
			t0[u] = tp[0];
			t1[u] = tp[1];
		}
	}
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) lds[t] = ((const dv2 *)(src + b))[t];
	__syncthreads();
	for (int u = 0; u < 2; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < RUN) {
			dv2 a = lds[i * 4];
			a.x += t0[u].x * t1[u].y * xv[u];
			a.y += t0[u].y * t1[u].x * pxv[u];
			lds[i * 4] = a;
			if (!PK) dsts[i] = nxt[b + i];
		}
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		((dv2 *)(dst + dsts[i]))[c] = lds[t];
	}
}

int main()
{
	const uint32_t n = 100000000u, nrun = n / RUN;
	std::mt19937_64 g(5);
	std::vector<uint32_t> h(n);
	for (uint32_t i = 0; i < n; i++) h[i] = i;
	std::shuffle(h.begin(), h.end(), g);
	uint32_t *nx, *p125, *p16; Rec *a, *bb; dv2 *tab;
	CK(hipMalloc(&nx, (size_t)n * 4)); CK(hipMalloc(&p125, (size_t)n * 4)); CK(hipMalloc(&p16, (size_t)n * 4));
	CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&bb, (size_t)n * 64)); CK(hipMalloc(&tab, 125000 * 32));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(bb, 0, (size_t)n * 64)); CK(hipMemset(tab, 0, 125000 * 32));
	CK(hipMemcpy(nx, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	for (uint32_t i = 0; i < n; i++) h[i] = (uint32_t)(g() % 125000);
	CK(hipMemcpy(p125, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	for (uint32_t i = 0; i < n; i++) h[i] = (uint32_t)(g() % 16000);
	CK(hipMemcpy(p16, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch();
		CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
		printf("%-40s %.3f ms\n", name, ms);
		fflush(stdout);
	};
	float *lx, *lpx; uint4 *pay;
	CK(hipMalloc(&lx, (size_t)n * 4)); CK(hipMalloc(&lpx, (size_t)n * 4)); CK(hipMalloc(&pay, (size_t)n * 16));
	CK(hipMemset(lx, 0, (size_t)n * 4)); CK(hipMemset(lpx, 0, (size_t)n * 4));
	{
		std::vector<uint32_t> nh(n), ph(n);
		CK(hipMemcpy(nh.data(), nx, (size_t)n * 4, hipMemcpyDeviceToHost));
		CK(hipMemcpy(ph.data(), p125, (size_t)n * 4, hipMemcpyDeviceToHost));
		std::vector<uint4> q(n);
		for (uint32_t i = 0; i < n; i++) q[i] = make_uint4(0u, nh[i], ph[i], 0u);
		CK(hipMemcpy(pay, q.data(), (size_t)n * 16, hipMemcpyHostToDevice));
	}
	for (int rep = 0; rep < 2; rep++) {
		time("4 streams + tab 32B + move", [&] { kE<512, false><<<nrun, 512>>>(a, bb, nx, p125, lx, lpx, pay, tab); });
		time("packed 16B + tab 32B + move", [&] { kE<512, true><<<nrun, 512>>>(a, bb, nx, p125, lx, lpx, pay, tab); });
		time("move only", [&] { kD<512, 0><<<nrun, 512>>>(a, bb, nx, p125, tab); });
		time("move + tab 32B x 125k (4 MB)", [&] { kD<512, 32><<<nrun, 512>>>(a, bb, nx, p125, tab); });
		time("move + tab 16B x 125k (2 MB)", [&] { kD<512, 16><<<nrun, 512>>>(a, bb, nx, p125, tab); });
		time("move + tab 32B x 16k (512 KB)", [&] { kD<512, 32><<<nrun, 512>>>(a, bb, nx, p16, tab); });
	}
	return 0;
}
