// Ceiling probe 9: the online learner's short level sweeps. A mini-batch of 200k 64-B row
// records (12.8 MB, MALL-resident), 25k columns of 8 rows per level, 40 levels as 40
// dependent launches, G = 8 lanes per column (k_ov_v_level's shape):
//   empty   : 40 launches of an empty kernel of the same grid
//   gather  : rows in row order: gather the column's records, butterfly-reduce, write them
//             back in place (the column layout k_ov_v_level uses)
//   lorder  : rows in the level's column order: read the column's run (consecutive records),
//             reduce, write each record to its position in the next level (one lane per
//             record, four 16-B stores), i.e. a per-batch level-ordered store
//   lorder4 : the same with the scattered writes staged through LDS, four lanes per record
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
struct __attribute__((aligned(64))) Rec { double v[8]; };
typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint32_t NROW = 200000, NCOL = 25000, CLEN = 8, LEVELS = 40;

__global__ __launch_bounds__(256) void k_empty() {}

__global__ __launch_bounds__(256) void k_gather(Rec *rows, const uint32_t *ent)
{
	const uint32_t col = blockIdx.x * 32 + threadIdx.x / 8, lane = threadIdx.x % 8;
	if (col >= NCOL) return;
	const uint32_t r = ent[(size_t)col * CLEN + lane];
	dv2 *p = (dv2 *)(rows + r);
	dv2 a = p[0], b = p[1], c = p[2], d = p[3];
	double s = a.x * b.y + c.x;
	for (int o = 4; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
	a.y += s * 1e-9; d.x += a.x * 1e-9;
	p[0] = a; p[1] = b; p[2] = c; p[3] = d;
}

__global__ __launch_bounds__(256) void k_lorder(const Rec *src, Rec *dst, const uint32_t *nxt)
{
	const uint32_t i = blockIdx.x * 256 + threadIdx.x;
	if (i >= NROW) return;
	const dv2 *p = (const dv2 *)(src + i);
	dv2 a = p[0], b = p[1], c = p[2], d = p[3];
	double s = a.x * b.y + c.x;
	for (int o = 4; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
	a.y += s * 1e-9; d.x += a.x * 1e-9;
	dv2 *q = (dv2 *)(dst + nxt[i]);
	q[0] = a; q[1] = b; q[2] = c; q[3] = d;
}

__global__ __launch_bounds__(256) void k_lorder4(const Rec *src, Rec *dst, const uint32_t *nxt)
{
	__shared__ dv2 lds[256 * 4];
	__shared__ uint32_t to[256];
	const uint32_t base = blockIdx.x * 256;
	const uint32_t m = min(256u, NROW - base);
	for (uint32_t t = threadIdx.x; t < m * 4; t += 256) lds[t] = ((const dv2 *)(src + base))[t];
	__syncthreads();
	if (threadIdx.x < m) {
		dv2 a = lds[threadIdx.x * 4], b = lds[threadIdx.x * 4 + 1], c = lds[threadIdx.x * 4 + 2];
		double s = a.x * b.y + c.x;
		for (int o = 4; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
		a.y += s * 1e-9;
		lds[threadIdx.x * 4] = a;
		to[threadIdx.x] = nxt[base + threadIdx.x];
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += 256) ((dv2 *)(dst + to[t >> 2]))[t & 3] = lds[t];
}

int main()
{
	std::mt19937 gen(3);
	std::vector<uint32_t> h((size_t)LEVELS * NCOL * CLEN), hn((size_t)LEVELS * NROW);
	for (uint32_t l = 0; l < LEVELS; ++l) {
		std::vector<uint32_t> perm(NROW);
		for (uint32_t i = 0; i < NROW; ++i) perm[i] = i;
		std::shuffle(perm.begin(), perm.end(), gen);
		for (uint32_t i = 0; i < NCOL * CLEN; ++i) h[(size_t)l * NCOL * CLEN + i] = perm[i];
		std::shuffle(perm.begin(), perm.end(), gen);
		for (uint32_t i = 0; i < NROW; ++i) hn[(size_t)l * NROW + i] = perm[i];
	}
	Rec *rows, *alt; uint32_t *ents, *nxt;
	CK(hipMalloc(&rows, (size_t)NROW * 64)); CK(hipMalloc(&alt, (size_t)NROW * 64));
	CK(hipMalloc(&ents, h.size() * 4)); CK(hipMalloc(&nxt, hn.size() * 4));
	CK(hipMemset(rows, 0, (size_t)NROW * 64)); CK(hipMemset(alt, 0, (size_t)NROW * 64));
	CK(hipMemcpy(ents, h.data(), h.size() * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(nxt, hn.data(), hn.size() * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
	auto time = [&](const char *name, auto launch) {
		launch(); CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0)); for (int it = 0; it < 20; it++) launch(); CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms; CK(hipEventElapsedTime(&ms, e0, e1));
		printf("%-28s %.2f us per level\n", name, ms * 1000.0 / 20 / LEVELS);
		fflush(stdout);
	};
	for (int rep = 0; rep < 2; rep++) {
		time("empty", [&] { for (uint32_t l = 0; l < LEVELS; ++l) k_empty<<<(NCOL + 31) / 32, 256>>>(); });
		time("gather (column layout)", [&] {
			for (uint32_t l = 0; l < LEVELS; ++l) k_gather<<<(NCOL + 31) / 32, 256>>>(rows, ents + (size_t)l * NCOL * CLEN);
		});
		time("lorder 1 lane/rec", [&] {
			for (uint32_t l = 0; l < LEVELS; ++l)
				k_lorder<<<(NROW + 255) / 256, 256>>>(l & 1 ? alt : rows, l & 1 ? rows : alt, nxt + (size_t)l * NROW);
		});
		time("lorder 4 lanes/rec (LDS)", [&] {
			for (uint32_t l = 0; l < LEVELS; ++l)
				k_lorder4<<<(NROW + 255) / 256, 256>>>(l & 1 ? alt : rows, l & 1 ? rows : alt, nxt + (size_t)l * NROW);
		});
	}
	return 0;
}
