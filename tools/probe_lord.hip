// Ceiling probe 4: the memory pattern of the level-ordered sweep kernel without its
// arithmetic. 1e8 records in runs of 800 (one workgroup per run, like k_level_lord at C4),
// each run read contiguously and every record written to a random position (a permutation).
//   A: one lane per record, 4 x 16-B loads and 4 x 16-B stores per lane (k_level_lord today)
//   B: four lanes per record, one 16-B load / store each (fully coalesced instructions)
//   C: A's loads, records handed through LDS so that B's stores write them
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int RUN = 800;

template <int BLOCK, int R>
__global__ __launch_bounds__(BLOCK) void kA(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt, const float *__restrict__ xs)
{
	const size_t b = (size_t)blockIdx.x * RUN;
	dv2 v[R][4];
	uint32_t to[R];
	float x[R];
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < RUN) {
			const dv2 *p = (const dv2 *)(src + b + i);
			v[u][0] = p[0]; v[u][1] = p[1]; v[u][2] = p[2]; v[u][3] = p[3];
			to[u] = nxt[b + i]; x[u] = xs[b + i];
		}
	}
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < RUN) {
			v[u][0].x += x[u];
			dv2 *p = (dv2 *)(dst + to[u]);
			p[0] = v[u][0]; p[1] = v[u][1]; p[2] = v[u][2]; p[3] = v[u][3];
		}
	}
}

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

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void kC(const Rec *__restrict__ src, Rec *__restrict__ dst,
                                             const uint32_t *__restrict__ nxt, const float *__restrict__ xs)
{
	__shared__ dv2 lds[RUN * 4];
	const size_t b = (size_t)blockIdx.x * RUN;
	// coalesced load into LDS, per-record compute from LDS, coalesced random-line store
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) lds[t] = ((const dv2 *)(src + b))[t];
	__syncthreads();
	for (uint32_t i = threadIdx.x; i < RUN; i += BLOCK) {
		dv2 a = lds[i * 4];
		a.x += xs[b + i];
		lds[i * 4] = a;
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < RUN * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		((dv2 *)(dst + nxt[b + i]))[c] = lds[t];
	}
}

int main(int argc, char **argv)
{
	const uint32_t n = 100000000u;
	const uint32_t nrun = n / RUN;
	std::vector<uint32_t> h(n);
	for (uint32_t i = 0; i < n; i++) h[i] = i;
	std::mt19937 g(1);
	std::shuffle(h.begin(), h.end(), g);
	uint32_t *nxt; Rec *a, *bb; float *xs;
	CK(hipMalloc(&nxt, (size_t)n * 4)); CK(hipMalloc(&a, (size_t)n * 64)); CK(hipMalloc(&bb, (size_t)n * 64));
	CK(hipMalloc(&xs, (size_t)n * 4));
	CK(hipMemset(a, 0, (size_t)n * 64)); CK(hipMemset(bb, 0, (size_t)n * 64)); CK(hipMemset(xs, 0, (size_t)n * 4));
	CK(hipMemcpy(nxt, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 5; it++) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
		printf("%-40s %.3f ms  %.3g rows/s\n", name, ms, n / ms * 1e3);
	};
	time("A 512x2 1 lane/rec", [&] { kA<512, 2><<<nrun, 512>>>(a, bb, nxt, xs); });
	time("A 256x4 1 lane/rec", [&] { kA<256, 4><<<nrun, 256>>>(a, bb, nxt, xs); });
	time("A 1024x1 1 lane/rec", [&] { kA<1024, 1><<<nrun, 1024>>>(a, bb, nxt, xs); });
	time("B 256 4 lanes/rec", [&] { kB<256><<<nrun, 256>>>(a, bb, nxt, xs); });
	time("B 512 4 lanes/rec", [&] { kB<512><<<nrun, 512>>>(a, bb, nxt, xs); });
	time("B 1024 4 lanes/rec", [&] { kB<1024><<<nrun, 1024>>>(a, bb, nxt, xs); });
	time("C 256 LDS", [&] { kC<256><<<nrun, 256>>>(a, bb, nxt, xs); });
	time("C 512 LDS", [&] { kC<512><<<nrun, 512>>>(a, bb, nxt, xs); });
	return 0;
}
