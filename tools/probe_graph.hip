// Ceiling probe 11: does a hipGraph of the level launches cost less per level than launching
// them one by one? The same kernels as probe_sync (an empty 780 x 256 kernel; one whose
// workgroups read and write 16 KB each), 2000 dependent launches on a created stream, either
// launched from the host or captured once into a graph and replayed.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_graph tools/probe_graph.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
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

static void enqueue(int touch, double2 *buf, hipStream_t s)
{
	for (int i = 0; i < ITERS; ++i) {
		if (touch) ktouch<<<WG, TPB, 0, s>>>(buf, i);
		else kempty<<<WG, TPB, 0, s>>>(buf);
	}
}

int main()
{
	double2 *buf;
	CK(hipMalloc(&buf, (size_t)WG * PER_WG * 16));
	CK(hipMemset(buf, 0, (size_t)WG * PER_WG * 16));
	hipStream_t s;
	CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	hipGraphExec_t ge[2];
	for (int touch = 0; touch < 2; ++touch) {
		hipGraph_t g;
		CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
		enqueue(touch, buf, s);
		CK(hipStreamEndCapture(s, &g));
		CK(hipGraphInstantiate(&ge[touch], g, nullptr, nullptr, 0));
		CK(hipGraphDestroy(g));
	}
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (int round = 0; round < 3; ++round) {
		for (int variant = 0; variant < 4; ++variant) {
			const int touch = variant & 1, graph = variant >> 1;
			CK(hipStreamSynchronize(s));
			CK(hipEventRecord(e0, s));
			if (graph) CK(hipGraphLaunch(ge[touch], s));
			else enqueue(touch, buf, s);
			CK(hipEventRecord(e1, s));
			CK(hipEventSynchronize(e1));
			CK(hipGetLastError());
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			printf("round %d %-6s %-5s %.2f us per level\n", round, graph ? "graph" : "stream", touch ? "touch" : "empty",
			       ms * 1000.0f / ITERS);
		}
	}
	CK(hipGraphExecDestroy(ge[0]));
	CK(hipGraphExecDestroy(ge[1]));
	return 0;
}
