// vbfm_replay.hip -- the reference's initial draws generated on the device.
//
// After srand(seed) the reference draws, in this order, fm.v (k*D normals with stdev
// init_stdev, fm_model.h:97), fm.w (D, libfm.cpp:307), mu_w_dash (D, 0.1*N(0,1)) and mu_v_dash
// (k*D, f-major) (fm_learn_vb.h:709-711), every normal by Leva's ratio-of-uniforms method
// (src/util/random.h:150-164) on glibc's rand() (random.h:174-176). vbfm_init_params_host
// replays that sequentially (~5e7 normals/s: ~21 s at C4); here the same stream is produced in
// parallel, bit for bit:
//   1. glibc's TYPE_3 generator is the linear recurrence y_n = y_{n-31} + y_{n-3} (mod 2^32),
//      output y_n >> 1. The host computes the 31-word state at the start of every chunk of
//      C outputs by jump-ahead (the 31x31 transition matrix raised to C, mod 2^32); each
//      device thread then generates its chunk.
//   2. A Leva attempt takes two consecutive uniforms (u, v) and either accepts (v/u) or
//      rejects; attempts start at every second position, except that a zero u is redrawn
//      (`while (u == 0.0)`), which shifts the later attempts by one. Zeros (1 in 2^31 outputs)
//      are located on the device and the host splits the stream into segments of aligned
//      attempts.
//   3. Accept flags -> exclusive scan -> the i-th accepted attempt is the i-th normal, routed to
//      fm.v / fm.w / mu_w_dash / mu_v_dash in the device's feature-major {mu, sigma} layout.
//   The one transcendental in the acceptance test (log u) may differ from glibc's by an ulp;
//   attempts whose test is that close to its boundary are re-decided on the host with
//   std::log (in practice none).
#include "vbfm_ctx.h"
#include "vbfm_rng.h"

#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#define DEVI __device__ __forceinline__

using namespace vbi;

namespace {

constexpr uint32_t CHUNK = 31 * 2048;   // outputs per generator thread (a multiple of 31)
constexpr uint32_t MAX_ZEROS = 4096, MAX_UNSURE = 4096;

// outputs [t*CHUNK, (t+1)*CHUNK) of the stream from the state y_{n-31..n-1} of its start
__global__ __launch_bounds__(256) void k_glibc_chunks(const uint32_t *__restrict__ states, uint32_t nchunks,
                                                      int32_t *__restrict__ out)
{
	const uint32_t t = blockIdx.x * 256u + threadIdx.x;
	if (t >= nchunks) return;
	uint32_t s[31];
#pragma unroll
	for (int i = 0; i < 31; ++i) s[i] = states[(size_t)t * 31 + i];
	int32_t *o = out + (size_t)t * CHUNK;
	for (uint32_t b = 0; b < CHUNK / 31; ++b) {
#pragma unroll
		for (int i = 0; i < 31; ++i) {
			s[i] = s[i] + (i < 3 ? s[i + 28] : s[i - 3]);   // y_{n+i} = y_{n+i-31} + y_{n+i-3}
			o[(size_t)b * 31 + i] = (int32_t)(s[i] >> 1);
		}
	}
}

__global__ void k_find_zeros(const int32_t *out, uint64_t n, uint64_t *pos, uint32_t *cnt)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n && out[i] == 0) {
		const uint32_t k = atomicAdd(cnt, 1u);
		if (k < MAX_ZEROS) pos[k] = i;
	}
}

struct Seg { uint64_t pos, first; };   // attempts first.. start at pos, pos+2, ...

DEVI uint64_t attempt_pos(const Seg *seg, uint32_t nseg, uint64_t i)
{
	uint32_t k = nseg - 1;
	while (k > 0 && seg[k].first > i) --k;
	return seg[k].pos + 2 * (i - seg[k].first);
}

DEVI double uniform_of(int32_t r) { return r / ((double)2147483647 + 1); }   // random.h:174-176

// Leva's test (random.h:150-164) for attempt i: 1 accept, 0 reject
__global__ void k_leva_flags(const int32_t *out, const Seg *seg, uint32_t nseg, uint64_t nattempt, uint32_t *flag,
                             uint64_t *unsure, uint32_t *nunsure)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= nattempt) return;
	const uint64_t s = attempt_pos(seg, nseg, i);
	const double u = uniform_of(out[s]);
	const double v = 1.7156 * (uniform_of(out[s + 1]) - 0.5);
	const double x = u - 0.449871;
	const double y = fabs(v) + 0.386595;
	const double Q = x * x + y * (0.19600 * y - 0.25472 * x);
	uint32_t acc;
	if (Q < 0.27597) acc = 1;
	else if (Q > 0.27846) acc = 0;
	else {
		const double lhs = v * v, rhs = -4.0 * u * u * log(u);
		acc = (lhs > rhs) ? 0 : 1;
		if (fabs(lhs - rhs) <= 1e-12 * fabs(rhs)) {
			const uint32_t k = atomicAdd(nunsure, 1u);
			if (k < MAX_UNSURE) unsure[k] = i;
		}
	}
	flag[i] = acc;
}

struct Route {
	uint64_t n_fmv, n_fmw, D, k;   // normals of fm.v, fm.w; then D of mu_w, k*D of mu_v
	double init_stdev;
	uint64_t total;                // normals drawn in all
	uint64_t *end;                 // stream position after the last one (the next rand() call)
};

// the idx-th normal to its destination (fm_model.h:97, libfm.cpp:307, fm_learn_vb.h:709-711)
__global__ void k_leva_route(const int32_t *out, const Seg *seg, uint32_t nseg, uint64_t nattempt,
                             const uint32_t *flag, const uint32_t *offs, Route r, double *fm_v, double *fm_w,
                             double2 *ms_w, double2 *ms_v)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= nattempt || !flag[i]) return;
	uint64_t idx = offs[i];
	const uint64_t s = attempt_pos(seg, nseg, i);
	if (idx + 1 == r.total) *r.end = s + 2;
	const double u = uniform_of(out[s]);
	const double v = 1.7156 * (uniform_of(out[s + 1]) - 0.5);
	const double g = v / u;
	if (idx < r.n_fmv) { if (fm_v) fm_v[idx] = 0 + r.init_stdev * g; return; }   // gaussian(0, init_stdev)
	idx -= r.n_fmv;
	if (idx < r.n_fmw) { if (fm_w) fm_w[idx] = 0 + r.init_stdev * g; return; }
	idx -= r.n_fmw;
	const double mu = 0.1 * (0 + 1 * g);                                           // 0.1 * gaussian(0, 1)
	if (idx < r.D) { ms_w[idx] = make_double2(mu, .02); return; }
	idx -= r.D;
	if (idx < r.k * r.D) {
		const uint64_t f = idx / r.D, j = idx % r.D;                                   // mu_v_dash[f][j]
		ms_v[j * r.k + f] = make_double2(mu, .02);
	}
}

inline unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

// ---- host: the stream's state and its jump-ahead ------------------------------------------
typedef std::vector<uint32_t> Mat;   // 31 x 31, row-major, arithmetic mod 2^32

Mat mat_mul(const Mat &a, const Mat &b)
{
	Mat c(31 * 31, 0);
	for (int i = 0; i < 31; i++)
		for (int k = 0; k < 31; k++) {
			const uint32_t x = a[i * 31 + k];
			if (!x) continue;
			for (int j = 0; j < 31; j++) c[i * 31 + j] += x * b[k * 31 + j];
		}
	return c;
}

// transition of (y_{n-31}, ..., y_{n-1}) by one output, raised to the power p
Mat jump_matrix(uint64_t p)
{
	Mat m(31 * 31, 0), r(31 * 31, 0);
	for (int i = 0; i < 30; i++) m[i * 31 + i + 1] = 1;   // shift
	m[30 * 31 + 0] = 1;                                    // y_n = y_{n-31} + y_{n-3}
	m[30 * 31 + 28] += 1;
	for (int i = 0; i < 31; i++) r[i * 31 + i] = 1;
	while (p) {
		if (p & 1) r = mat_mul(r, m);
		m = mat_mul(m, m);
		p >>= 1;
	}
	return r;
}

}  // namespace

namespace vbi {
// the glibc window (y_{n-31..n-1}) after srand(seed), the warm-up and `pos` more outputs
void glibc_state_at(uint32_t seed, uint64_t pos, uint32_t st[31])
{
	uint32_t st0[31];
	vbrng::glibc_warm_state(seed, st0);
	const Mat J = jump_matrix(pos);
	for (int i = 0; i < 31; i++) {
		uint32_t a = 0;
		for (int j = 0; j < 31; j++) a += J[i * 31 + j] * st0[j];
		st[i] = a;
	}
}
}  // namespace vbi

extern "C" int vbfm_init_params_replay(vbfm_ctx *c, uint32_t seed, double init_stdev, double *fm_v_out,
                                       double *fm_w_out)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		const uint64_t kD = (uint64_t)c->k * c->D, D = c->D;
		Route r;
		r.init_stdev = init_stdev;
		const bool model_draws = !(init_stdev == 0.0 || std::isnan(init_stdev));   // random.h:166-172
		r.n_fmv = model_draws ? kD : 0;
		r.n_fmw = model_draws ? D : 0;
		r.D = D;
		r.k = (uint64_t)c->k;
		const uint64_t nnorm = r.n_fmv + r.n_fmw + D + kD;
		r.total = nnorm;
		uint64_t end_h = 0;
		r.end = dalloc<uint64_t>(1);
		HIPCHK(hipMemsetAsync(r.end, 0, 8, c->s));
		uint32_t st0[31];
		vbrng::glibc_warm_state(seed, st0);
		double *fmv_d = fm_v_out && r.n_fmv ? dalloc<double>(r.n_fmv) : nullptr;
		double *fmw_d = fm_w_out && r.n_fmw ? dalloc<double>(r.n_fmw) : nullptr;
		// ~2.74 uniforms per Leva normal; grow the stream if it falls short
		uint64_t nuni = (uint64_t)(2.8 * (double)nnorm) + 4 * CHUNK;
		for (int attempt = 0;; attempt++) {
			const uint32_t nchunks = (uint32_t)((nuni + CHUNK - 1) / CHUNK);
			nuni = (uint64_t)nchunks * CHUNK;
			// chunk start states
			const Mat J = jump_matrix(CHUNK);
			std::vector<uint32_t> states((size_t)nchunks * 31);
			std::copy(st0, st0 + 31, states.begin());
			for (uint32_t t = 1; t < nchunks; t++) {
				const uint32_t *p = &states[(size_t)(t - 1) * 31];
				uint32_t *q = &states[(size_t)t * 31];
				for (int i = 0; i < 31; i++) {
					uint32_t a = 0;
					for (int j = 0; j < 31; j++) a += J[i * 31 + j] * p[j];
					q[i] = a;
				}
			}
			uint32_t *states_d = dalloc<uint32_t>(states.size());
			int32_t *out = dalloc<int32_t>(nuni);
			uint64_t *zpos = dalloc<uint64_t>(MAX_ZEROS);
			uint32_t *cnt = dalloc<uint32_t>(2);
			HIPCHK(hipMemcpyAsync(states_d, states.data(), states.size() * 4, hipMemcpyHostToDevice, c->s));
			HIPCHK(hipMemsetAsync(cnt, 0, 8, c->s));
			k_glibc_chunks<<<grid_of(nchunks), 256, 0, c->s>>>(states_d, nchunks, out);
			HIPCHK(hipGetLastError());
			k_find_zeros<<<grid_of(nuni), 256, 0, c->s>>>(out, nuni, zpos, cnt);
			HIPCHK(hipGetLastError());
			uint32_t nz = 0;
			HIPCHK(d2h(c, &nz, cnt, 4));
			sync(c);
			if (nz > MAX_ZEROS) throw std::string("init replay: too many zero outputs");
			std::vector<uint64_t> z(nz);
			if (nz) HIPCHK(hipMemcpy(z.data(), zpos, nz * 8, hipMemcpyDeviceToHost));
			std::sort(z.begin(), z.end());
			// segments of aligned attempts: a zero where an attempt would start shifts the rest
			std::vector<Seg> seg{Seg{0, 0}};
			for (uint64_t zp : z) {
				Seg &cur = seg.back();
				if (zp < cur.pos || ((zp - cur.pos) & 1)) continue;   // a v position, or before
				const uint64_t first = cur.first + (zp - cur.pos) / 2;
				seg.push_back(Seg{zp + 1, first});
			}
			const Seg &last = seg.back();
			const uint64_t nattempt = nuni >= last.pos + 2 ? last.first + (nuni - last.pos) / 2 : last.first;
			Seg *seg_d = dalloc<Seg>(seg.size());
			HIPCHK(hipMemcpy(seg_d, seg.data(), seg.size() * sizeof(Seg), hipMemcpyHostToDevice));
			uint32_t *flag = dalloc<uint32_t>(nattempt), *offs = dalloc<uint32_t>(nattempt);
			uint64_t *unsure = dalloc<uint64_t>(MAX_UNSURE);
			k_leva_flags<<<grid_of(nattempt), 256, 0, c->s>>>(out, seg_d, (uint32_t)seg.size(), nattempt, flag, unsure,
			                                                  cnt + 1);
			HIPCHK(hipGetLastError());
			uint32_t nu = 0;
			HIPCHK(d2h(c, &nu, cnt + 1, 4));
			sync(c);
			if (nu > MAX_UNSURE) throw std::string("init replay: too many borderline attempts");
			if (nu) {   // re-decide with the host's log (the reference's libm)
				std::vector<uint64_t> ui(nu);
				HIPCHK(hipMemcpy(ui.data(), unsure, nu * 8, hipMemcpyDeviceToHost));
				for (uint64_t i : ui) {
					uint64_t k = seg.size() - 1;
					while (k > 0 && seg[k].first > i) --k;
					const uint64_t s = seg[k].pos + 2 * (i - seg[k].first);
					int32_t w[2];
					HIPCHK(hipMemcpy(w, out + s, 8, hipMemcpyDeviceToHost));
					const double u = w[0] / ((double)2147483647 + 1);
					const double v = 1.7156 * (w[1] / ((double)2147483647 + 1) - 0.5);
					const uint32_t acc = ((v * v) > (-4.0 * u * u * std::log(u))) ? 0u : 1u;
					HIPCHK(hipMemcpy(flag + i, &acc, 4, hipMemcpyHostToDevice));
				}
			}
			size_t tb = 0;
			HIPCHK(rocprim::exclusive_scan(nullptr, tb, flag, offs, 0u, (size_t)nattempt, rocprim::plus<uint32_t>(), c->s));
			void *tmp = dalloc<uint8_t>(tb);
			HIPCHK(rocprim::exclusive_scan(tmp, tb, flag, offs, 0u, (size_t)nattempt, rocprim::plus<uint32_t>(), c->s));
			uint32_t tail[2] = {0, 0};
			if (nattempt) {
				HIPCHK(d2h(c, &tail[0], offs + nattempt - 1, 4));
				HIPCHK(d2h(c, &tail[1], flag + nattempt - 1, 4));
			}
			sync(c);
			const uint64_t accepted = (uint64_t)tail[0] + tail[1];
			if (accepted >= nnorm)
				k_leva_route<<<grid_of(nattempt), 256, 0, c->s>>>(out, seg_d, (uint32_t)seg.size(), nattempt, flag, offs,
				                                                  r, fmv_d, fmw_d, c->ms_w, c->ms_v);
			HIPCHK(hipGetLastError());
			sync(c);
			dfree(tmp); dfree(flag); dfree(offs); dfree(unsure); dfree(seg_d);
			dfree(states_d); dfree(out); dfree(zpos); dfree(cnt);
			if (accepted >= nnorm) break;
			if (attempt > 8) throw std::string("init replay: stream too short");
			nuni = nuni + nuni / 4;
		}
		// attributes past the drawn ones keep their values; fm_learn_vb::init scalars (:693-712)
		HIPCHK(hipMemcpy(&end_h, r.end, 8, hipMemcpyDeviceToHost));
		dfree(r.end);
		c->init_stream_seed = seed;
		c->init_stream_end = end_h;   // outputs after the warm-up that the draws consumed
		if (fmv_d) HIPCHK(hipMemcpy(fm_v_out, fmv_d, r.n_fmv * 8, hipMemcpyDeviceToHost));
		if (fmw_d) HIPCHK(hipMemcpy(fm_w_out, fmw_d, r.n_fmw * 8, hipMemcpyDeviceToHost));
		dfree(fmv_d); dfree(fmw_d);
		std::fill(c->hyp_w.begin(), c->hyp_w.end(), 1.0);
		std::fill(c->hyp_v.begin(), c->hyp_v.end(), 1.0);
		upload_hyp(c);
		c->alpha = 1.0; c->sigma_0 = 1.0; c->mu0 = 0.0; c->s0d = 0.02;
		c->q_ready[0] = c->q_ready[1] = -1;
		sync(c);
	});
}
