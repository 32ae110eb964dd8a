// Ceiling probe 10: what a per-level launch costs when the work is tiny (the online learner's
// mini-batch levels: ~780 workgroups of 256 threads, ~12 us each), against keeping one
// cooperative kernel resident and separating the levels with a grid-wide barrier.
//   launch : 2000 back-to-back launches of an empty 780 x 256 kernel (stream order)
//   touch  : the same, each workgroup reading and writing 16 KB (12.8 MB per launch, MALL-resident)
//   gsync  : one cooperative 780 x 256 kernel, 2000 grid barriers (cooperative_groups grid.sync)
//   gtouch : the same with the 16 KB read + write per workgroup between barriers
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_sync tools/probe_sync.hip
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <cstdlib>
namespace cg = cooperative_groups;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int WG = 780, TPB = 256, ITERS = 2000;
constexpr size_t PER_WG = 16384 / 16;   // double2 per workgroup

__global__ __launch_bounds__(TPB) void kempty(double2 *) {}

__global__ __launch_bounds__(TPB) void ktouch(double2 *buf, int it)
{
	double2 *b = buf + (size_t)blockIdx.x * PER_WG;
	for (size_t i = threadIdx.x; i < PER_WG; i += TPB) {
		double2 v = b[i];
		v.x += it;
		b[(i + 64 * (it & 7)) % PER_WG] = v;
	}
}

__global__ __launch_bounds__(TPB) void kgsync(double2 *buf, int touch)
{
	cg::grid_group g = cg::this_grid();
	double2 *b = buf + (size_t)blockIdx.x * PER_WG;
	for (int it = 0; it < ITERS; ++it) {
		if (touch) {
			for (size_t i = threadIdx.x; i < PER_WG; i += TPB) {
				double2 v = b[i];
				v.x += it;
				b[(i + 64 * (it & 7)) % PER_WG] = v;
			}
		}
		g.sync();
	}
}

int main()
{
	double2 *buf;
	CK(hipMalloc(&buf, (size_t)WG * PER_WG * 16));
	CK(hipMemset(buf, 0, (size_t)WG * PER_WG * 16));
	int dev = 0, coop = 0, nb = 0;
	CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
	CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kgsync, TPB, 0));
	hipDeviceProp_t p;
	CK(hipGetDeviceProperties(&p, dev));
	printf("cooperative launch %d, %d CUs, %d resident workgroups per CU for kgsync\n", coop,
	       p.multiProcessorCount, nb);
	if (!coop || nb * p.multiProcessorCount < WG) {
		printf("grid of %d workgroups cannot be co-resident: no cooperative probe\n", WG);
		return 0;
	}
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (int round = 0; round < 2; ++round) {
		for (int variant = 0; variant < 4; ++variant) {
			CK(hipDeviceSynchronize());
			CK(hipEventRecord(e0));
			if (variant == 0) {
				for (int i = 0; i < ITERS; ++i) kempty<<<WG, TPB>>>(buf);
			} else if (variant == 1) {
				for (int i = 0; i < ITERS; ++i) ktouch<<<WG, TPB>>>(buf, i);
			} else {
				int touch = variant == 3;
				void *args[] = {&buf, &touch};
				CK(hipLaunchCooperativeKernel((void *)kgsync, dim3(WG), dim3(TPB), args, 0, 0));
			}
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			CK(hipGetLastError());
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			const char *nm[] = {"launch", "touch", "gsync", "gtouch"};
			printf("round %d %-7s %.2f us per level\n", round, nm[variant], ms * 1000.0f / ITERS);
		}
	}
	return 0;
}
