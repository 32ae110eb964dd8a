// vbfm_math.h -- device arithmetic shared by the sweep kernels of both row layouts
// (vbfm_kernels.hip: column-gather; vbfm_lorder.hip: level-ordered row store): deterministic
// wave / block reductions, the 64-B row record accessors, and the per-entry statistics,
// posterior + guards and correction of update_v / update_w restated expression by
// expression from the reference (citations relative to /root/reference).
#pragma once
#include "vbfm_device.h"

#define DEVI __device__ __forceinline__

namespace {


DEVI double wave_sum(double v)
{
	// xor butterfly: lanes i and i^o add the same two values (a+b == b+a), so every lane
	// ends with the identical, order-fixed sum
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	return v;
}

template <int BLOCK>
DEVI void block_sum2(double &a, double &b, double *lds /* [2*BLOCK/64] */)
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

DEVI bool dnan(double v) { return __builtin_isnan(v); }
DEVI bool dinf(double v) { return __builtin_isinf(v); }

// ------------------------------------------------------------------------------------
// row record access. v[0] = (e, q0), v[1] = (tq0, tz0), v[2] = (t, q1), v[3] = (tq1, tz1)
typedef double2 Rec[4];

// 16-B vector loads / stores, element-wise into the record: a piece a kernel leaves untouched
// then stays in registers (a whole-struct copy can leave it as a memcpy through scratch / LDS)
typedef double rec_v2 __attribute__((ext_vector_type(2)));
DEVI void load_rec(const RowRec *rows, uint32_t r, Rec &v)
{
	const rec_v2 *p = reinterpret_cast<const rec_v2 *>(rows + r);
#pragma unroll
	for (int c = 0; c < 4; ++c) {
		const rec_v2 t = p[c];
		v[c].x = t.x;
		v[c].y = t.y;
	}
}

DEVI void store_rec(RowRec *rows, uint32_t r, const Rec &v)
{
	rec_v2 *p = reinterpret_cast<rec_v2 *>(rows + r);
#pragma unroll
	for (int c = 0; c < 4; ++c) {
		rec_v2 t;
		t.x = v[c].x;
		t.y = v[c].y;
		p[c] = t;
	}
}

template <int S> DEVI double &Q(Rec &v) { return S == 0 ? v[0].y : v[2].y; }
template <int S> DEVI double &TQ(Rec &v) { return S == 0 ? v[1].x : v[3].x; }
template <int S> DEVI double &TZ(Rec &v) { return S == 0 ? v[1].y : v[3].y; }
DEVI double &E(Rec &v) { return v[0].x; }
DEVI double &T(Rec &v) { return v[2].x; }

// add_main_q term of one entry into slot S (fm_learn_vb.h:374-376); `first` marks the
// row's smallest feature, where the reference's zeroed cache (:411-415) starts the sum
template <int S>
DEVI void qacc(Rec &v, float x, bool first, double2 nx)
{
	const double a = nx.x * x;
	const double b = nx.y * x * x;
	const double c = nx.x * nx.x * x * x;
	double &q = Q<S>(v), &tq = TQ<S>(v), &tz = TZ<S>(v);
	if (first) { q = 0.0 + a; tq = 0.0 + b; tz = 0.0 + c; }
	else { q += a; tq += b; tz += c; }
}

// ------------------------------------------------------------------------------------
// v sweep: update_v (src/libfm/src/fm_learn_vb.h:577-644)

// stats term of one entry (fm_learn_vb.h:592-595)
DEVI void v_stat(float x, double e, double q, double tq, double mo, double so, double &vm, double &vs)
{
	const float xx = x * x;
	const double h = q - x * mo;
	const double h1 = tq - xx * so;
	vm += x * h * (e + x * mo * h);
	vs += xx * h * h + xx * h1;
}

// posterior + guards (fm_learn_vb.h:597-619); returns false when the correction is skipped
DEVI bool v_post(double vm, double vs, double sv_g, double alpha, double mo, double so,
                 double &mu, double &sig, uint32_t *counters, bool leader)
{
	sig = (double)1.0 / (sv_g + alpha * vs);
	mu = sig * alpha * vm;
	if (dnan(sig) || dinf(sig)) {
		sig = so;
		if (leader) atomicAdd(&counters[CNT_NAN_SIGMA_V], 1u);
	}
	if (dnan(mu)) {
		mu = mo;
		if (leader) atomicAdd(&counters[CNT_NAN_MU_V], 1u);
		return false;
	}
	if (dinf(mu)) {
		mu = mo;
		if (leader) atomicAdd(&counters[CNT_INF_MU_V], 1u);
		return false;
	}
	return true;
}

// correction of one row (fm_learn_vb.h:623-643)
DEVI void v_corr(float x, double mo, double so, double mu, double sig, double &e, double &q, double &tq,
                 double &tz, double &t)
{
	const float xx = x * x;
	const double h = x * (q - x * mo);
	const double h1 = xx * (tq - xx * so);
	const double h2 = xx * (tz - xx * mo * mo);
	q += x * (mu - mo);
	tq += xx * (sig - so);
	tz += xx * (mu * mu - mo * mo);
	e += h * (mo - mu);
	t += (h1 + h2) * (sig - so);
	t += h1 * (mu * mu - mo * mo);
}

// everything that happens to one row record of the column after the posterior: the
// correction (when the guards let it run) and the fused q-cache term of factor f+1
template <int P, bool NEXT>
DEVI void v_apply(Rec &v, float x, bool first, bool go, double mo, double so, double mu, double sig, double2 nx)
{
	if (go) v_corr(x, mo, so, mu, sig, E(v), Q<P>(v), TQ<P>(v), TZ<P>(v), T(v));
	if constexpr (NEXT) qacc<1 - P>(v, x, first, nx);
}

DEVI void w_stat(float x, double e, double mo, double &wm, double &ws)
{
	wm += x * (e + x * mo);
	ws += x * x;   // fp32 product
}

DEVI bool w_post(double wm, double ws, double sw_g, double alpha, double mo, double so, double &mu,
                 double &sig, uint32_t *counters, bool leader)
{
	sig = (double)1.0 / (sw_g + alpha * ws);
	mu = sig * alpha * wm;
	if (dnan(sig) || dinf(sig)) {
		if (leader) atomicAdd(&counters[CNT_NAN_SIGMA_W], 1u);
		sig = so;
	}
	if (dnan(mu)) {
		if (leader) atomicAdd(&counters[CNT_NAN_MU_W], 1u);
		mu = mo;
		return false;
	}
	if (dinf(mu)) {
		if (leader) atomicAdd(&counters[CNT_INF_MU_W], 1u);
		mu = mo;
		return false;
	}
	return true;
}

template <bool NEXT>
DEVI void w_apply(Rec &v, float x, bool first, bool go, double mo, double so, double mu, double sig, double2 nx)
{
	if (go) {
		const double h = x;
		E(v) += h * (mo - mu);
		T(v) += h * h * (sig - so);
	}
	if constexpr (NEXT) qacc<0>(v, x, first, nx);
}

}  // namespace
