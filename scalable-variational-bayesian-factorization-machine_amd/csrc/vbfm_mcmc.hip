// vbfm_mcmc.hip -- CDNA4 kernels of the MCMC / ALS learner (fm_learn_mcmc, -method mcmc|als).
//
// Same structure as the VB sweep (vbfm_kernels.hip): dependency levels, one workgroup per
// feature column, deterministic block reductions, the q-cache of factor f+1 accumulated
// while factor f is swept (slot f%2 / (f+1)%2 of the row record), bit-exact per-row sums.
// Row cache convention of the MCMC learner: e = yhat - y (fm_learn_mcmc_simultaneous.h:76-80),
// kept in RowRec::e; the q-cache is RowRec::q (slot 0) / RowRec::q1 (slot 1).
// Random numbers: z[j] holds the standard normal the reference's stream supplies for
// feature j (host replay of glibc rand(), see vbfm_rng.h), or -- in device-RNG mode -- a
// counter-based normal keyed by (seed, iteration, factor, feature), the same on every shard.
#include "vbfm_device.h"

#define DEVI __device__ __forceinline__
#include "vbfm_mc_math.h"

namespace {

DEVI double wave_sum(double v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	return v;
}

template <int BLOCK>
DEVI void block_sum2(double &a, double &b, double *lds)
{
	a = wave_sum(a);
	b = wave_sum(b);
	if constexpr (BLOCK > 64) {
		const int w = threadIdx.x >> 6;
		if ((threadIdx.x & 63) == 0) { lds[2 * w] = a; lds[2 * w + 1] = b; }
		__syncthreads();
		a = lds[0]; b = lds[1];
#pragma unroll
		for (int i = 1; i < BLOCK / 64; ++i) { a += lds[2 * i]; b += lds[2 * i + 1]; }
	}
}

template <int BLOCK>
DEVI double block_sum1(double a, double *lds)
{
	a = wave_sum(a);
	if constexpr (BLOCK > 64) {
		const int w = threadIdx.x >> 6;
		__syncthreads();
		if ((threadIdx.x & 63) == 0) lds[w] = a;
		__syncthreads();
		a = lds[0];
#pragma unroll
		for (int i = 1; i < BLOCK / 64; ++i) a += lds[i];
	}
	return a;
}

DEVI float ent_x(uint2 ent) { return __uint_as_float(ent.y); }
// q-cache term of the next factor: cache[i].q += v_if * x_li (fm_learn_mcmc.h:404)
template <int S> DEVI void mc_qacc(RowRec &r, float x, bool first, double vn)
{
	const double a = vn * x;
	double &q = S == 0 ? r.q : r.q1;
	q = first ? 0.0 + a : q + a;
}

template <int S> DEVI double mc_q(const RowRec &r) { return S == 0 ? r.q : r.q1; }
template <int S> DEVI double &mc_qref(RowRec &r) { return S == 0 ? r.q : r.q1; }

// ---- draw_v over one level -------------------------------------------------------------
// MODE 0: fused; 1: per-feature statistics of this shard's rows into a.stats; 2: draw and
// correction from the all-reduced a.stats (row-sharded multi-GPU form)
template <int BLOCK, int P, bool NEXT, int MODE>
__global__ __launch_bounds__(BLOCK) void k_mc_v_level(McArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	if constexpr (MODE == 2) debug_skew(a.skew);
	const double vo = a.par[(size_t)j * a.stride].x;
	double sm = 0.0, ss = 0.0;
	if constexpr (MODE != 2) {
		for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {    // :785-792
			const uint2 ent = col[i];
			const RowRec &r = a.rows[ent.x & ROW_MASK];
			const float x = ent_x(ent);
			const double h = x * (mc_q<P>(r) - x * vo);
			sm += h * r.e;
			ss += h * h;
		}
		block_sum2<BLOCK>(sm, ss, lds);
		if constexpr (MODE == 1) {
			if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(sm, ss);
			return;
		}
	} else {
		const double2 st = a.stats[blockIdx.x];
		sm = st.x;
		ss = st.y;
	}
	const double vn = NEXT ? a.par_next[(size_t)j * a.next_stride].x : 0.0;
	const double vp = a.pk ? a.par_prev[(size_t)j * a.next_stride].x : 0.0;   // fused re-prediction
	const uint32_t g = mc_group(a, j);
	double v;
	const bool go = mc_draw(sm, ss, vo, mc_lambda(a, g), mc_mu(a, g), a.alpha,
	                        mc_z(a, j), a.z != nullptr, a.sample, true, v, a.counters, threadIdx.x == 0);
	// MODE 2: every wave has used the old value (the draw) before it is overwritten
	if constexpr (MODE == 2) __syncthreads();   // [raw-barrier]
	if (threadIdx.x == 0) a.par[(size_t)j * a.stride].x = v;
	if (!go && !NEXT && !a.pk) return;
	auto entry = [&](uint2 ent) {
		RowRec &r = a.rows[ent.x & ROW_MASK];
		const float x = ent_x(ent);
		const bool first = (ent.x & ROW_FIRST) != 0;
		if (go) {
			const double h = x * (mc_q<P>(r) - x * vo);
			mc_qref<P>(r) -= x * (vo - v);
			r.e -= h * (vo - v);
		}
		if constexpr (NEXT) mc_qacc<1 - P>(r, x, first, vn);
		if (a.pk) mc_pred_acc(r.tq, r.tz, r.t, x, first, vp, a.pk);   // MCMC leaves tq, tz, t free
	};
	if (a.dup[j]) {   // a column listing a row twice: sequential, as the reference
		__syncthreads();
		if (threadIdx.x == 0)
			for (uint32_t i = 0; i < n; ++i) entry(col[i]);
		return;
	}
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) entry(col[i]);   // :826-834
}

// ---- draw_w over one level (+ q-cache of factor 0 into slot 0) ---------------------------
template <int BLOCK, bool NEXT, int MODE>
__global__ __launch_bounds__(BLOCK) void k_mc_w_level(McArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	if constexpr (MODE == 2) debug_skew(a.skew);
	const double wo = a.par[(size_t)j * a.stride].x;
	double sm = 0.0, ss = 0.0;
	if constexpr (MODE != 2) {
		for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {    // :674-679
			const uint2 ent = col[i];
			const float x = ent_x(ent);
			sm += x * (a.rows[ent.x & ROW_MASK].e - wo * x);
			ss += x * x;                                       // fp32 product
		}
		block_sum2<BLOCK>(sm, ss, lds);
		if constexpr (MODE == 1) {
			if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(sm, ss);
			return;
		}
	} else {
		const double2 st = a.stats[blockIdx.x];
		sm = st.x;
		ss = st.y;
	}
	const double vn = NEXT ? a.par_next[(size_t)j * a.next_stride].x : 0.0;
	const uint32_t g = mc_group(a, j);
	double w;
	const bool go = mc_draw(sm, ss, wo, mc_lambda(a, g), mc_mu(a, g), a.alpha,
	                        mc_z(a, j), a.z != nullptr, a.sample, false, w, a.counters, threadIdx.x == 0);
	// MODE 2: every wave has used the old value (the draw) before it is overwritten
	if constexpr (MODE == 2) __syncthreads();   // [raw-barrier]
	if (threadIdx.x == 0) a.par[(size_t)j * a.stride].x = w;
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		__syncthreads();
		if (threadIdx.x == 0)
			for (uint32_t i = 0; i < n; ++i) {
				const uint2 ent = col[i];
				RowRec &r = a.rows[ent.x & ROW_MASK];
				const float x = ent_x(ent);
				if (go) { const double h = x; r.e -= h * (wo - w); }
				if constexpr (NEXT) mc_qacc<0>(r, x, (ent.x & ROW_FIRST) != 0, vn);
			}
		return;
	}
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {        // :712-717
		const uint2 ent = col[i];
		RowRec &r = a.rows[ent.x & ROW_MASK];
		const float x = ent_x(ent);
		if (go) { const double h = x; r.e -= h * (wo - w); }
		if constexpr (NEXT) mc_qacc<0>(r, x, (ent.x & ROW_FIRST) != 0, vn);
	}
}

// parameters of attributes without train rows (j in [nf_train, D)): drawn from the prior,
// fm_learn_mcmc.h:449-457 / :569-577
__global__ void k_mc_prior(McArgs a, uint32_t j0, uint32_t j1, int is_v)
{
	const uint32_t j = j0 + blockIdx.x * 256u + threadIdx.x;
	if (j >= j1) return;
	const uint32_t g = mc_group(a, j);
	const double cur = a.par[(size_t)j * a.stride].x;
	double out;
	mc_draw(0.0, 0.0, cur, mc_lambda(a, g), mc_mu(a, g), a.alpha, mc_z(a, j),
	        a.z != nullptr, a.sample, is_v != 0, out, a.counters, true);
	a.par[(size_t)j * a.stride].x = out;
}

// q-cache of one factor from scratch (add_main_q, fm_learn_mcmc.h:384-409), row-parallel
__global__ void k_mc_qcache(const uint64_t *row_ptr, const uint2 *csr, const double2 *par_f, uint32_t stride,
                            RowRec *rows, uint32_t n, int slot, const uint32_t *pos)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	double q = 0.0;
	for (uint64_t p = row_ptr[r]; p < row_ptr[r + 1]; ++p) {
		const uint2 ent = csr[p];
		q += par_f[(size_t)ent.x * stride].x * ent_x(ent);
	}
	RowRec &rec = rows[pos ? pos[r] : r];   // record index of row r (level-ordered store: level-0 position)
	if (slot == 0) rec.q = q; else rec.q1 = q;
}

// per block: mode 0 sum e^2 (draw_alpha :908-910), mode 1 sum (e - w0) (draw_w0 :635-637)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_mc_row_sums(const RowRec *rows, uint32_t n, int mode, double w0, double *out)
{
	__shared__ double lds[BLOCK / 64];
	double s = 0.0;
	for (uint32_t r = blockIdx.x * BLOCK + threadIdx.x; r < n; r += gridDim.x * BLOCK) {
		const double e = rows[r].e;
		s += mode == 0 ? e * e : e - w0;
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ void k_mc_e_shift(RowRec *rows, uint32_t n, double d)
{
	// cache[i].e -= (w0_old - w0)  (fm_learn_mcmc.h:665-667)
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r < n) rows[r].e -= d;
}

DEVI double clip(double p, double mn, double mx)
{
	p = (p < mx) ? p : mx;
	p = (mn < p) ? p : mn;
	return p;
}

// after the full re-predict of train (fm_learn_mcmc_simultaneous.h:153-162): per block
// sum (clip(yhat) - y)^2, and e = yhat - y
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_mc_train_update(RowRec *rows, const double *yhat, const float *target,
                                                           uint32_t n, double mn, double mx, double *out,
                                                           const uint32_t *pos)
{
	__shared__ double lds[BLOCK / 64];
	double s = 0.0;
	for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < n; c += gridDim.x * BLOCK) {
		const double yh = yhat[c];
		const double err = clip(yh, mn, mx) - target[c];
		s += err * err;
		rows[pos ? pos[c] : c].e = yh - target[c];
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// the end of the fused train re-prediction (fm_learn_mcmc.h:117-348; the v sweeps of factors
// 1..k-1 accumulated factors 0..k-2 into each record's tq / tz / t, mc_pred_acc): the last
// factor's q and its squared terms, then the w terms, from the row's entries in ascending
// feature order, yhat = e + q (+ w0) into yhat[row] (k_mc_train_update follows). The last
// factor's v and the w are read from compact copies (vlast[j],
// wc[j]: 8 B per attribute, MALL-resident at the bench scale). The q of step 1 and the squared
// terms of step 2 go to separate accumulators, each in the reference's order, so one pass over
// the entries serves both; the w terms follow every squared term (step 3). A row without
// entries predicts w0.
__global__ __launch_bounds__(256) void k_mc_pred_final(const uint64_t *row_ptr, const uint2 *csr, const double *vlast,
                                                       const double *wc, int k, int k1, int k0, double w0, int pk_done,
                                                       const RowRec *rows, const uint32_t *pos, uint32_t n, double *yhat)
{
	const uint32_t c = blockIdx.x * 256u + threadIdx.x;   // one row per thread: every gather chain in flight
	if (c >= n) return;
	const uint64_t b = row_ptr[c], e = row_ptr[c + 1];
	double ev = 0.0, q2 = 0.0;
	if (pk_done && e > b) {
		const RowRec &rec = rows[pos ? pos[c] : c];
		ev = rec.tz + 0.5 * rec.tq * rec.tq;   // fold factor k-2
		q2 = rec.t;
	}
	if (k > 0) {
		double q = 0.0;
		for (uint64_t p = b; p < e; ++p) {
			const uint2 ent = csr[p];
			const double v = vlast[ent.x];
			const float x = ent_x(ent);
			q += v * x;
			q2 -= 0.5 * v * v * x * x;
		}
		ev += 0.5 * q * q;
	}
	if (k1)
		for (uint64_t p = b; p < e; ++p) {
			const uint2 ent = csr[p];
			q2 += wc[ent.x] * ent_x(ent);
		}
	double yh = ev + q2;
	if (k0) yh += w0;
	yhat[c] = yh;
}

// out[j] = p[j * stride].x: one factor's (or w's) values as a compact array
__global__ void k_mc_extract(const double2 *p, uint32_t stride, uint32_t D, double *out)
{
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	if (j < D) out[j] = p[(size_t)j * stride].x;
}

// test side (:143-151 and _evaluate :261-279): pred_this = yhat, pred_sum_all += clip(yhat);
// per block (sum err_this^2, sum |err_this|, sum err_all^2, sum |err_all|)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_mc_test_update(const double *e_test, const float *target, uint32_t n,
                                                          double mn, double mx, double inv_iters, double *pred_this,
                                                          double *pred_sum, double *out)
{
	__shared__ double lds[BLOCK / 64];
	double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
	for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < n; c += gridDim.x * BLOCK) {
		const double p = e_test[c];
		pred_this[c] = p;
		const double sum = pred_sum[c] + clip(p, mn, mx);
		pred_sum[c] = sum;
		const double et = clip(p * 1.0, mn, mx) - target[c];
		const double ea = clip(sum * inv_iters, mn, mx) - target[c];
		s0 += et * et;
		s1 += fabs(et);
		s2 += ea * ea;
		s3 += fabs(ea);
	}
	s0 = block_sum1<BLOCK>(s0, lds);
	s1 = block_sum1<BLOCK>(s1, lds);
	s2 = block_sum1<BLOCK>(s2, lds);
	s3 = block_sum1<BLOCK>(s3, lds);
	if (threadIdx.x == 0) {
		double *o = out + 4 * (size_t)blockIdx.x;
		o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3;
	}
}

// hyper-prior sums over one chunk of a (w or factor f, group g) segment: mode 0 sum p,
// mode 1 sum (p - c)^2 with c = the segment's prior mean (draw_w_mu / draw_w_lambda,
// draw_v_mu / draw_v_lambda: fm_learn_mcmc.h:931-1089)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_mc_param_sums(const double2 *pw, const double2 *pv, const uint32_t *perm,
                                                         const vbk::Chunk *chunks, int mode, const double *cw,
                                                         const double *cv, int k, double *out)
{
	__shared__ double lds[BLOCK / 64];
	const vbk::Chunk c = chunks[blockIdx.x];
	const double2 *p = c.f < 0 ? pw : pv + c.f;
	const size_t stride = c.f < 0 ? 1 : (size_t)k;
	const double ctr = mode == 0 ? 0.0 : (c.f < 0 ? cw[c.g] : cv[(size_t)c.g * k + c.f]);
	double s = 0.0;
	for (uint32_t i = c.begin + threadIdx.x; i < c.end; i += BLOCK) {
		const double v = p[(size_t)perm[i] * stride].x;
		s += mode == 0 ? v : (v - ctr) * (v - ctr);
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

namespace vbk {

template <int BLOCK, int MODE>
static void launch_v(const McArgs &a, hipStream_t s)
{
	const bool nx = a.par_next != nullptr;
	if (a.slot == 0) {
		if (nx) k_mc_v_level<BLOCK, 0, true, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
		else k_mc_v_level<BLOCK, 0, false, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
	} else {
		if (nx) k_mc_v_level<BLOCK, 1, true, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
		else k_mc_v_level<BLOCK, 1, false, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
	}
}

template <int BLOCK, int MODE>
static void launch_w(const McArgs &a, hipStream_t s)
{
	if (a.par_next) k_mc_w_level<BLOCK, true, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
	else k_mc_w_level<BLOCK, false, MODE><<<a.nfeat, BLOCK, 0, s>>>(a);
}

// threads per column from the level's mean column length (the VB kernels' shapes; the
// level-ordered MCMC kernel uses the same BLOCK, so both reduce a column in one order)
template <int MODE>
static void launch_level(const McArgs &a, bool is_w, hipStream_t s)
{
	dispatch_shape(a.avg_len, [&](auto B, auto) {
		if (is_w) launch_w<B(), MODE>(a, s);
		else launch_v<B(), MODE>(a, s);
	});
}

static hipError_t mc_level(const McArgs &a, int mode, bool is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (mode == 0) launch_level<0>(a, is_w, s);
	else if (mode == 1) launch_level<1>(a, is_w, s);
	else launch_level<2>(a, is_w, s);
	return hipGetLastError();
}

hipError_t mc_v_level(const McArgs &a, int mode, hipStream_t s) { return mc_level(a, mode, false, s); }
hipError_t mc_w_level(const McArgs &a, int mode, hipStream_t s) { return mc_level(a, mode, true, s); }

hipError_t mc_prior(const McArgs &a, uint32_t j0, uint32_t j1, int is_v, hipStream_t s)
{
	if (j1 <= j0) return hipSuccess;
	k_mc_prior<<<grid_for(j1 - j0), 256, 0, s>>>(a, j0, j1, is_v);
	return hipGetLastError();
}

hipError_t mc_qcache(const uint64_t *row_ptr, const uint2 *csr, const double2 *par_f, uint32_t stride, RowRec *rows,
                     uint32_t n, int slot, const uint32_t *pos, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_mc_qcache<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, par_f, stride, rows, n, slot, pos);
	return hipGetLastError();
}

hipError_t mc_row_sums(const RowRec *rows, uint32_t n, int mode, double w0, double *out, uint32_t nblocks, hipStream_t s)
{
	k_mc_row_sums<256><<<nblocks, 256, 0, s>>>(rows, n, mode, w0, out);
	return hipGetLastError();
}

hipError_t mc_e_shift(RowRec *rows, uint32_t n, double d, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_mc_e_shift<<<grid_for(n), 256, 0, s>>>(rows, n, d);
	return hipGetLastError();
}

hipError_t mc_train_update(RowRec *rows, const double *yhat, const float *target, uint32_t n, double mn, double mx,
                           double *out, uint32_t nblocks, const uint32_t *pos, hipStream_t s)
{
	k_mc_train_update<256><<<nblocks, 256, 0, s>>>(rows, yhat, target, n, mn, mx, out, pos);
	return hipGetLastError();
}

hipError_t mc_pred_final(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k,
                         int k1, int k0, double w0, int pk_done, const RowRec *rows, const uint32_t *pos, uint32_t n,
                         uint32_t D, double *scratch, double *yhat, hipStream_t s)
{
	double *vlast = scratch, *wc = scratch + D;
	if (D && k > 0) k_mc_extract<<<grid_for(D), 256, 0, s>>>(ms_v + (k - 1), (uint32_t)k, D, vlast);
	if (D && k1) k_mc_extract<<<grid_for(D), 256, 0, s>>>(ms_w, 1, D, wc);
	if (n) k_mc_pred_final<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, vlast, wc, k, k1, k0, w0, pk_done, rows, pos, n, yhat);
	return hipGetLastError();
}

hipError_t mc_test_update(const double *e_test, const float *target, uint32_t n, double mn, double mx,
                          double inv_iters, double *pred_this, double *pred_sum, double *out, uint32_t nblocks,
                          hipStream_t s)
{
	k_mc_test_update<256><<<nblocks, 256, 0, s>>>(e_test, target, n, mn, mx, inv_iters, pred_this, pred_sum, out);
	return hipGetLastError();
}

hipError_t mc_param_sums(const double2 *pw, const double2 *pv, const uint32_t *perm, const Chunk *chunks,
                         uint32_t nchunks, int mode, const double *cw, const double *cv, int k, double *out,
                         hipStream_t s)
{
	if (nchunks == 0) return hipSuccess;
	k_mc_param_sums<256><<<nchunks, 256, 0, s>>>(pw, pv, perm, chunks, mode, cw, cv, k, out);
	return hipGetLastError();
}

}  // namespace vbk
