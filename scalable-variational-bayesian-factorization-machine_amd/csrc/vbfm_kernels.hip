// vbfm_kernels.hip -- CDNA4 (gfx950) kernels of the VB factorization-machine sweep.
//
// Every kernel restates one loop of the reference (citations relative to /root/reference)
// with the reference's arithmetic, expression by expression: x is fp32 and a product of
// two fp32 values is rounded to fp32 before it meets a double (FM_FLOAT,
// src/fm_core/fm_data.h:25). Built with -ffp-contract=off so no FMA is formed. Where a
// sum runs over many independent terms (a column's sufficient statistics, a data set's
// residual energy) the device sums in a fixed tree order: deterministic run to run, equal
// to the reference up to summation order (~1e-16 relative). Per-row sums (q-cache,
// predictions) keep the reference's sequential ascending-feature order and are bit-exact.
//
// Parallel schedule: the reference updates features one at a time in ascending id order
// (Gauss-Seidel). Two features interact only through rows they share, so the features are
// grouped into dependency levels (level(j) = 1 + max level of an earlier feature sharing a
// row); all features of one level are updated concurrently, one workgroup per feature
// column, which reproduces the sequential result exactly (each row is touched by at most
// one feature per level, in the same relative order as the reference).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "vbfm_math.h"

namespace {

template <int P, bool NEXT>
DEVI void v_apply_serial(const uint2 *col, uint32_t n, RowRec *rows, bool go, double mo, double so, double mu,
                         double sig, double2 nx, uint32_t fm)
{
	// a column listing some row twice: the reference corrects entry after entry, a repeated
	// row seeing its own earlier update
	for (uint32_t i = 0; i < n; ++i) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(rows, ent.x & ROW_MASK, v);
		v_apply<P, NEXT>(v, ent_x(ent), (ent.x & fm) != 0, go, mo, so, mu, sig, nx);
		store_rec(rows, ent.x & ROW_MASK, v);
	}
}

// One workgroup per feature column of the level. Entries i = tid + u*BLOCK for u < R are
// gathered once (one 64-B record each) and kept in registers from the stats pass to the
// write-back; longer columns re-gather the overflow entries.
template <int BLOCK, int R, int P, bool NEXT>
__global__ __launch_bounds__(BLOCK) void k_v_level_fused(LevelArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	if (a.long_min && n > a.long_min && !a.dup[j]) return;   // segment kernels (col_long)
	const uint2 *col = a.csc + cb;
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double mo = msj.x, so = msj.y;
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];

	uint32_t row[R];
	float xv[R];
	Rec rec[R];
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		// unconditional, index clamped (entries and records past the column are never used;
		// an empty column reads row 0): a guarded load is sunk into its branch and waited on
		// there, so the entries and then the records would arrive one after the other
		const uint2 ent = n ? col[min(i, n - 1)] : make_uint2(0u, 0u);
		row[u] = ent.x;
		xv[u] = ent_x(ent);
	}
#pragma unroll
	for (int u = 0; u < R; ++u) load_rec(a.rows, row[u] & ROW_MASK, rec[u]);
	double vm = 0.0, vs = 0.0;
#pragma unroll
	for (int u = 0; u < R; ++u)
		if (threadIdx.x + u * BLOCK < n) v_stat(xv[u], E(rec[u]), Q<P>(rec[u]), TQ<P>(rec[u]), mo, so, vm, vs);
	for (uint32_t i = threadIdx.x + R * BLOCK; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		v_stat(ent_x(ent), E(v), Q<P>(v), TQ<P>(v), mo, so, vm, vs);
	}
	block_sum2<BLOCK>(vm, vs, lds);

	double mu, sig;
	const double sv_g = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool go = v_post(vm, vs, sv_g, a.alpha, mo, so, mu, sig, a.counters, threadIdx.x == 0);
	if (threadIdx.x == 0) a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		__syncthreads();
		if (threadIdx.x == 0) v_apply_serial<P, NEXT>(col, n, a.rows, go, mo, so, mu, sig, nx, a.first_mask);
		return;
	}
#pragma unroll
	for (int u = 0; u < R; ++u)
		if (threadIdx.x + u * BLOCK < n) {
			v_apply<P, NEXT>(rec[u], xv[u], (row[u] & a.first_mask) != 0, go, mo, so, mu, sig, nx);
			store_rec(a.rows, row[u] & ROW_MASK, rec[u]);
		}
	for (uint32_t i = threadIdx.x + R * BLOCK; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		v_apply<P, NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

// Long columns on the column-gather layout (as lord_long on the level store): the fused
// kernels skip columns longer than a.long_min (except columns listing a row twice, which stay
// sequential); one workgroup per segment writes the segment's statistics and the column's
// parameters before the level, then one workgroup per segment sums the column's partials in
// segment order, computes the (identical) posterior and corrects its rows.
template <bool IS_W, int P>
__global__ __launch_bounds__(256) void k_col_long_stats(LevelArgs a)
{
	__shared__ double lds[2 * (256 / 64)];
	const LongSeg g = a.segs[blockIdx.x];
	const uint32_t j = level_feat(a, g.col);
	const uint2 *col = a.csc + a.col_ptr[j] + g.start;
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	double s1 = 0.0, s2 = 0.0;
	for (uint32_t i = threadIdx.x; i < g.len; i += 256) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		if constexpr (IS_W) w_stat(ent_x(ent), E(v), msj.x, s1, s2);
		else v_stat(ent_x(ent), E(v), Q<P>(v), TQ<P>(v), msj.x, msj.y, s1, s2);
	}
	block_sum2<256>(s1, s2, lds);
	if (threadIdx.x == 0) {
		a.seg_part[2 * blockIdx.x] = make_double2(s1, s2);
		a.seg_part[2 * blockIdx.x + 1] = msj;
	}
}

template <bool IS_W, int P, bool NEXT>
__global__ __launch_bounds__(256) void k_col_long_correct(LevelArgs a)
{
	const LongSeg g = a.segs[blockIdx.x];
	const uint32_t j = level_feat(a, g.col);
	const uint2 *col = a.csc + a.col_ptr[j] + g.start;
	double s1 = 0.0, s2 = 0.0;
	for (uint32_t q = 0; q < g.nseg; ++q) {
		const double2 p = a.seg_part[2 * (g.seg0 + q)];
		s1 += p.x;
		s2 += p.y;
	}
	const double2 msj = a.seg_part[2 * g.seg0 + 1];
	const double mo = msj.x, so = msj.y;
	const double2 nx = NEXT ? a.ms_next[(size_t)j * a.ms_stride_next] : make_double2(0.0, 0.0);
	const double hyp = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool lead = threadIdx.x == 0 && blockIdx.x == g.seg0;
	double mu, sig;
	const bool go = IS_W ? w_post(s1, s2, hyp, a.alpha, mo, so, mu, sig, a.counters, lead)
	                     : v_post(s1, s2, hyp, a.alpha, mo, so, mu, sig, a.counters, lead);
	if (lead) a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	if (!go && !NEXT) return;
	for (uint32_t i = threadIdx.x; i < g.len; i += 256) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		if constexpr (IS_W) w_apply<NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		else v_apply<P, NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

// split form for the row-sharded multi-GPU mode: stats -> (all-reduce) -> correction
template <int BLOCK, int P>
__global__ __launch_bounds__(BLOCK) void k_v_level_stats(LevelArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	double vm = 0.0, vs = 0.0;
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		v_stat(ent_x(ent), E(v), Q<P>(v), TQ<P>(v), msj.x, msj.y, vm, vs);
	}
	block_sum2<BLOCK>(vm, vs, lds);
	if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(vm, vs);
}

template <int BLOCK, int P, bool NEXT>
__global__ __launch_bounds__(BLOCK) void k_v_level_correct(LevelArgs a)
{
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	debug_skew(a.skew);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double2 st = a.stats[blockIdx.x];
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];
	double mu, sig;
	const double sv_g = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool go = v_post(st.x, st.y, sv_g, a.alpha, msj.x, msj.y, mu, sig, a.counters, threadIdx.x == 0);
	// every wave has used the old value (v_post above) before it is overwritten: without the
	// barrier a wave of this workgroup could still read the new one as its "old"
	__syncthreads();   // [raw-barrier]
	if (threadIdx.x == 0) a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		if (threadIdx.x == 0) v_apply_serial<P, NEXT>(col, n, a.rows, go, msj.x, msj.y, mu, sig, nx, a.first_mask);
		return;
	}
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		v_apply<P, NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, msj.x, msj.y, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

// ------------------------------------------------------------------------------------
// w sweep: update_w (fm_learn_vb.h:527-574). With NEXT the sweep also accumulates the
// q-cache of factor 0 into slot 0 (add_main_q(train, 0), fm_learn_vb.h:354-381).
template <bool NEXT>
DEVI void w_apply_serial(const uint2 *col, uint32_t n, RowRec *rows, bool go, double mo, double so, double mu,
                         double sig, double2 nx, uint32_t fm)
{
	for (uint32_t i = 0; i < n; ++i) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(rows, ent.x & ROW_MASK, v);
		w_apply<NEXT>(v, ent_x(ent), (ent.x & fm) != 0, go, mo, so, mu, sig, nx);
		store_rec(rows, ent.x & ROW_MASK, v);
	}
}

template <int BLOCK, int R, bool NEXT>
__global__ __launch_bounds__(BLOCK) void k_w_level_fused(LevelArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	if (a.long_min && n > a.long_min && !a.dup[j]) return;   // segment kernels (col_long)
	const uint2 *col = a.csc + cb;
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double mo = msj.x, so = msj.y;
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];
	uint32_t row[R];
	float xv[R];
	Rec rec[R];
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		// unconditional, index clamped (entries and records past the column are never used;
		// an empty column reads row 0): a guarded load is sunk into its branch and waited on
		// there, so the entries and then the records would arrive one after the other
		const uint2 ent = n ? col[min(i, n - 1)] : make_uint2(0u, 0u);
		row[u] = ent.x;
		xv[u] = ent_x(ent);
	}
#pragma unroll
	for (int u = 0; u < R; ++u) load_rec(a.rows, row[u] & ROW_MASK, rec[u]);
	double wm = 0.0, ws = 0.0;
#pragma unroll
	for (int u = 0; u < R; ++u)
		if (threadIdx.x + u * BLOCK < n) w_stat(xv[u], E(rec[u]), mo, wm, ws);
	for (uint32_t i = threadIdx.x + R * BLOCK; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		w_stat(ent_x(ent), a.rows[ent.x & ROW_MASK].e, mo, wm, ws);
	}
	block_sum2<BLOCK>(wm, ws, lds);
	double mu, sig;
	const double sw_g = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool go = w_post(wm, ws, sw_g, a.alpha, mo, so, mu, sig, a.counters, threadIdx.x == 0);
	if (threadIdx.x == 0) a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		__syncthreads();
		if (threadIdx.x == 0) w_apply_serial<NEXT>(col, n, a.rows, go, mo, so, mu, sig, nx, a.first_mask);
		return;
	}
#pragma unroll
	for (int u = 0; u < R; ++u)
		if (threadIdx.x + u * BLOCK < n) {
			w_apply<NEXT>(rec[u], xv[u], (row[u] & a.first_mask) != 0, go, mo, so, mu, sig, nx);
			store_rec(a.rows, row[u] & ROW_MASK, rec[u]);
		}
	for (uint32_t i = threadIdx.x + R * BLOCK; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		w_apply<NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_w_level_stats(LevelArgs a)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	const double mo = a.ms[(size_t)j * a.ms_stride].x;
	double wm = 0.0, ws = 0.0;
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		w_stat(ent_x(ent), a.rows[ent.x & ROW_MASK].e, mo, wm, ws);
	}
	block_sum2<BLOCK>(wm, ws, lds);
	if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(wm, ws);
}

template <int BLOCK, bool NEXT>
__global__ __launch_bounds__(BLOCK) void k_w_level_correct(LevelArgs a)
{
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t cb = a.col_ptr[j];
	const uint32_t n = (uint32_t)(a.col_ptr[j + 1] - cb);
	const uint2 *col = a.csc + cb;
	debug_skew(a.skew);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double2 st = a.stats[blockIdx.x];
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];
	double mu, sig;
	const double sw_g = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool go = w_post(st.x, st.y, sw_g, a.alpha, msj.x, msj.y, mu, sig, a.counters, threadIdx.x == 0);
	// every wave has used the old value (w_post above) before it is overwritten: without the
	// barrier a wave of this workgroup could still read the new one as its "old"
	__syncthreads();   // [raw-barrier]
	if (threadIdx.x == 0) a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		if (threadIdx.x == 0) w_apply_serial<NEXT>(col, n, a.rows, go, msj.x, msj.y, mu, sig, nx, a.first_mask);
		return;
	}
	for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		w_apply<NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, msj.x, msj.y, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

// ------------------------------------------------------------------------------------
// q-cache of factor f: add_main_q (fm_learn_vb.h:354-381) after zeroing (:411-415).
// Row-parallel over the feature-sorted CSR: each row sums its entries in ascending
// feature order, exactly the order the reference's column loop adds them in.
__global__ __launch_bounds__(256) void k_qcache(const uint64_t *__restrict__ row_ptr, const uint2 *__restrict__ csr,
                                                 const double2 *__restrict__ ms_f, uint32_t stride,
                                                 RowRec *__restrict__ rows, uint32_t n, int slot,
                                                 const uint32_t *__restrict__ pos)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	double q = 0.0, tq = 0.0, tz = 0.0;
	for (uint64_t p = b; p < e; ++p) {
		const uint2 ent = csr[p];
		const float x = ent_x(ent);
		const double2 m = ms_f[(size_t)ent.x * stride];
		q += m.x * x;
		tq += m.y * x * x;
		tz += m.x * m.x * x * x;
	}
	RowRec *rec = rows + (pos ? pos[r] : r);   // record index of row r
	if (slot == 0) {
		rec->q = q;
		reinterpret_cast<double2 *>(rec)[1] = make_double2(tq, tz);
	} else {
		rec->q1 = q;
		reinterpret_cast<double2 *>(rec)[3] = make_double2(tq, tz);
	}
}

// flag the CSC entry of each row's first (smallest-feature) CSR entry: binary search for the
// row in that column (rows ascend within a column; the first of repeated rows is taken)
__global__ void k_mark_first(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, uint2 *csc, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r];
	if (row_ptr[r + 1] == b) return;
	const uint32_t j = csr[b].x;
	uint64_t lo = col_ptr[j], hi = col_ptr[j + 1];
	while (lo < hi) {
		const uint64_t mid = (lo + hi) >> 1;
		if ((csc[mid].x & ROW_MASK) < r) lo = mid + 1; else hi = mid;
	}
	csc[lo].x |= ROW_FIRST;
}

// predict_data_and_write_to_eterms for one data set (fm_learn_vb.h:70-203), row-parallel.
// Exact form: the reference's order (factor-major sums, each over the row's ascending ids).
__global__ __launch_bounds__(256) void k_predict_e(const uint64_t *__restrict__ row_ptr, const uint2 *__restrict__ csr,
                                                    const double2 *__restrict__ ms_v, const double2 *__restrict__ ms_w,
                                                    int k, int k1, int k0, double mu0, double *__restrict__ out, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
	double e = 0.0;
	for (int f = 0; f < k; ++f) {                          // (1) :93-133
		double q = 0.0;
		for (uint64_t p = b; p < en; ++p) { const uint2 ent = csr[p]; q += ms_v[(size_t)ent.x * k + f].x * ent_x(ent); }
		e += 0.5 * q * q;
	}
	double q = 0.0;
	for (int f = 0; f < k; ++f) {                          // (2) :136-163
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const double v = ms_v[(size_t)ent.x * k + f].x;
			const float x = ent_x(ent);
			q -= 0.5 * v * v * x * x;
		}
	}
	if (k1)                                                // (3) :166-188
		for (uint64_t p = b; p < en; ++p) { const uint2 ent = csr[p]; q += ms_w[ent.x].x * ent_x(ent); }
	e = e + q;                                             // merge :190-202
	if (k0) e += mu0;
	out[r] = e;
}

// Blocked form for large data sets: one pass over the row per block of C factors reading
// C contiguous {mu, sigma} pairs per entry; every per-factor sum keeps the reference's
// order, the -1/2 sum v^2 x^2 term is summed block-major.
template <int C>
__global__ __launch_bounds__(256) void k_predict_e_blocked(const uint64_t *__restrict__ row_ptr,
                                                            const uint2 *__restrict__ csr,
                                                            const double2 *__restrict__ ms_v,
                                                            const double2 *__restrict__ ms_w, int k, int k1, int k0,
                                                            double mu0, double *__restrict__ out, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
	double e = 0.0, qq = 0.0;
	for (int f0 = 0; f0 < k; f0 += C) {
		double q[C];
#pragma unroll
		for (int c = 0; c < C; ++c) q[c] = 0.0;
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const float x = ent_x(ent);
			const double2 *m = ms_v + (size_t)ent.x * k + f0;
#pragma unroll
			for (int c = 0; c < C; ++c)
				if (f0 + c < k) {
					const double v = m[c].x;
					q[c] += v * x;
					qq -= 0.5 * v * v * x * x;
				}
		}
#pragma unroll
		for (int c = 0; c < C; ++c)
			if (f0 + c < k) e += 0.5 * q[c] * q[c];
	}
	if (k1)
		for (uint64_t p = b; p < en; ++p) { const uint2 ent = csr[p]; qq += ms_w[ent.x].x * ent_x(ent); }
	e = e + qq;
	if (k0) e += mu0;
	out[r] = e;
}

// predict_t_and_write_to_qterms (fm_learn_vb.h:207-312), row-parallel; writes rows[].t
__global__ __launch_bounds__(256) void k_predict_t(const uint64_t *__restrict__ row_ptr, const uint2 *__restrict__ csr,
                                                    const double2 *__restrict__ ms_v, const double2 *__restrict__ ms_w,
                                                    int k, int k1, int k0, double s0d, RowRec *__restrict__ rows,
                                                    uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
	double t = 0.0;
	for (int f = 0; f < k; ++f) {                          // (1) :222-254
		double q = 0.0, z = 0.0;
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const double2 vm = ms_v[(size_t)ent.x * k + f];
			const float x = ent_x(ent);
			q += vm.x * x * vm.x * x;
			z += vm.y * x * x;
		}
		t += (0.5 * z * z + z * q);
	}
	double q = 0.0;
	for (int f = 0; f < k; ++f) {                          // (2) :257-281
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const double2 vm = ms_v[(size_t)ent.x * k + f];
			const float x = ent_x(ent);
			q -= (vm.x * vm.x * x * x * x * x * vm.y + 0.5 * x * x * x * x * vm.y * vm.y);
		}
	}
	if (k1)                                                // (3) :284-301
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const float x = ent_x(ent);
			q += ms_w[ent.x].y * x * x;
		}
	t = t + q;                                             // :304-311
	if (k0) t += s0d;
	rows[r].t = t;
}

template <int C>
__global__ __launch_bounds__(256) void k_predict_t_blocked(const uint64_t *__restrict__ row_ptr,
                                                            const uint2 *__restrict__ csr,
                                                            const double2 *__restrict__ ms_v,
                                                            const double2 *__restrict__ ms_w, int k, int k1, int k0,
                                                            double s0d, RowRec *__restrict__ rows, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
	double t = 0.0, qq = 0.0;
	for (int f0 = 0; f0 < k; f0 += C) {
		double q[C], z[C];
#pragma unroll
		for (int c = 0; c < C; ++c) { q[c] = 0.0; z[c] = 0.0; }
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const float x = ent_x(ent);
			const double2 *m = ms_v + (size_t)ent.x * k + f0;
#pragma unroll
			for (int c = 0; c < C; ++c)
				if (f0 + c < k) {
					const double2 vm = m[c];
					q[c] += vm.x * x * vm.x * x;
					z[c] += vm.y * x * x;
					qq -= (vm.x * vm.x * x * x * x * x * vm.y + 0.5 * x * x * x * x * vm.y * vm.y);
				}
		}
#pragma unroll
		for (int c = 0; c < C; ++c)
			if (f0 + c < k) t += (0.5 * z[c] * z[c] + z[c] * q[c]);
	}
	if (k1)
		for (uint64_t p = b; p < en; ++p) {
			const uint2 ent = csr[p];
			const float x = ent_x(ent);
			qq += ms_w[ent.x].y * x * x;
		}
	t = t + qq;
	if (k0) t += s0d;
	rows[r].t = t;
}

// entries whose factor runs a wave-form prediction kernel loads before accumulating them (in
// entry order): several independent gathers in flight per wave instead of one
constexpr int wave_pu(int KP) { return KP >= 4 ? 2 : (KP == 2 ? 4 : 8); }

template <int KP, int PU>
DEVI void wave_gather(uint2 mine, uint32_t cnt, uint32_t i0, uint32_t lane, const double2 *__restrict__ ms_v, int k,
                      double2 (&mv)[PU][KP], float (&xs)[PU])
{
#pragma unroll
	for (int u = 0; u < PU; ++u) {
		const int i = (int)min(i0 + u, cnt - 1);
		const uint32_t j = __shfl(mine.x, i, 64);
		xs[u] = __uint_as_float(__shfl(mine.y, i, 64));
#pragma unroll
		for (int c = 0; c < KP; ++c) {
			const int f = (int)lane + 64 * c;
			mv[u][c] = make_double2(0.0, 0.0);
			if (f < k && i0 + u < cnt) mv[u][c] = ms_v[(size_t)j * k + f];
		}
	}
}

// Wave form (large data sets): one 64-lane wave per row, factor f on lane f % 64 (pass
// f / 64, KP passes). Each entry's k {mu, sigma} pairs are one contiguous run, read by the
// wave as whole 1 KiB pieces instead of one strided pair per thread; the row's entries are
// loaded once (one lane each) and broadcast. Every lane keeps the reference's order over the
// row's entries for its factors; the per-factor terms are summed across lanes in a fixed
// butterfly (~1 ulp from the reference's sequential factor order, like the blocked form),
// the linear term is added after them in the reference's entry order.
// COMPACT: the factors come from a plain [j*k + f] array of mu (vc) instead of the {mu, sigma}
// pairs: half the bytes per entry (the MCMC learner's per-iteration re-prediction, where the
// pairs hold {v, 0})
template <int KP, bool COMPACT = false>
__global__ __launch_bounds__(256) void k_predict_e_wave(const uint64_t *__restrict__ row_ptr,
                                                         const uint2 *__restrict__ csr,
                                                         const double2 *__restrict__ ms_v,
                                                         const double2 *__restrict__ ms_w, int k, int k1, int k0,
                                                         double mu0, double *__restrict__ out, uint32_t n,
                                                         const double *__restrict__ vc = nullptr)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t nwaves = gridDim.x * 4;
	for (uint32_t r = (blockIdx.x * 256 + threadIdx.x) >> 6; r < n; r += nwaves) {
		const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
		double q[KP];
#pragma unroll
		for (int c = 0; c < KP; ++c) q[c] = 0.0;
		double qq = 0.0;
		constexpr int PU = wave_pu(KP);
		for (uint64_t p0 = b; p0 < en; p0 += 64) {
			const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
			const uint2 mine = lane < cnt ? csr[p0 + lane] : make_uint2(0u, 0u);
			for (uint32_t i0 = 0; i0 < cnt; i0 += PU) {
				// PU entries' factors in flight at once, then accumulated in entry order
				double v[PU][KP];
				float xs[PU];
#pragma unroll
				for (int u = 0; u < PU; ++u) {
					const int i = (int)min(i0 + u, cnt - 1);
					const uint32_t j = __shfl(mine.x, i, 64);
					xs[u] = __uint_as_float(__shfl(mine.y, i, 64));
#pragma unroll
					for (int c = 0; c < KP; ++c) {
						const int f = (int)lane + 64 * c;
						v[u][c] = 0.0;
						if (f < k && i0 + u < cnt) v[u][c] = COMPACT ? vc[(size_t)j * k + f] : ms_v[(size_t)j * k + f].x;
					}
				}
#pragma unroll
				for (int u = 0; u < PU; ++u) {
					if (i0 + u >= cnt) break;
					const float x = xs[u];
#pragma unroll
					for (int c = 0; c < KP; ++c)
						if ((int)lane + 64 * c < k) {
							q[c] += v[u][c] * x;                       // :93-133
							qq -= 0.5 * v[u][c] * v[u][c] * x * x;     // :136-163
						}
				}
			}
		}
		double e = 0.0;
#pragma unroll
		for (int c = 0; c < KP; ++c)
			if ((int)lane + 64 * c < k) e += 0.5 * q[c] * q[c];
		e = wave_sum(e);
		qq = wave_sum(qq);
		if (k1) {                                              // (3) :166-188
			// every lane gathers one entry's w, the wave adds them in entry order
			for (uint64_t p0 = b; p0 < en; p0 += 64) {
				const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
				double pe = 0.0;
				if (lane < cnt) { const uint2 ent = csr[p0 + lane]; pe = ms_w[ent.x].x * ent_x(ent); }
				for (uint32_t i = 0; i < cnt; ++i) qq += __shfl(pe, (int)i, 64);
			}
		}
		e = e + qq;
		if (k0) e += mu0;
		if (lane == 0) out[r] = e;
	}
}

template <int KP>
__global__ __launch_bounds__(256) void k_predict_t_wave(const uint64_t *__restrict__ row_ptr,
                                                         const uint2 *__restrict__ csr,
                                                         const double2 *__restrict__ ms_v,
                                                         const double2 *__restrict__ ms_w, int k, int k1, int k0,
                                                         double s0d, RowRec *__restrict__ rows, uint32_t n)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t nwaves = gridDim.x * 4;
	for (uint32_t r = (blockIdx.x * 256 + threadIdx.x) >> 6; r < n; r += nwaves) {
		const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
		double q[KP], z[KP];
#pragma unroll
		for (int c = 0; c < KP; ++c) { q[c] = 0.0; z[c] = 0.0; }
		double qq = 0.0;
		constexpr int PU = wave_pu(KP);
		for (uint64_t p0 = b; p0 < en; p0 += 64) {
			const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
			const uint2 mine = lane < cnt ? csr[p0 + lane] : make_uint2(0u, 0u);
			for (uint32_t i0 = 0; i0 < cnt; i0 += PU) {
				double2 mv[PU][KP];
				float xs[PU];
				wave_gather<KP, PU>(mine, cnt, i0, lane, ms_v, k, mv, xs);
#pragma unroll
				for (int u = 0; u < PU; ++u) {
					if (i0 + u >= cnt) break;
					const float x = xs[u];
#pragma unroll
					for (int c = 0; c < KP; ++c)
						if ((int)lane + 64 * c < k) {
							const double2 vm = mv[u][c];
							q[c] += vm.x * x * vm.x * x;               // :222-254
							z[c] += vm.y * x * x;
							qq -= (vm.x * vm.x * x * x * x * x * vm.y + 0.5 * x * x * x * x * vm.y * vm.y);   // :257-281
						}
				}
			}
		}
		double t = 0.0;
#pragma unroll
		for (int c = 0; c < KP; ++c)
			if ((int)lane + 64 * c < k) t += (0.5 * z[c] * z[c] + z[c] * q[c]);
		t = wave_sum(t);
		qq = wave_sum(qq);
		if (k1) {                                              // (3) :284-301
			for (uint64_t p0 = b; p0 < en; p0 += 64) {
				const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
				double pt = 0.0;
				if (lane < cnt) {
					const uint2 ent = csr[p0 + lane];
					const float x = ent_x(ent);
					pt = ms_w[ent.x].y * x * x;
				}
				for (uint32_t i = 0; i < cnt; ++i) qq += __shfl(pt, (int)i, 64);
			}
		}
		t = t + qq;                                            // :304-311
		if (k0) t += s0d;
		if (lane == 0) rows[r].t = t;
	}
}

// Both predictions of a data set's rows in one pass over the parameters (the caches a fresh
// train set or mini-batch starts from, fm_learn_vb_simultaneous.h:37-44 /
// fm_learn_vb_online_simultaneous.h:111-139): k_predict_e_wave's and k_predict_t_wave's
// arithmetic, accumulator by accumulator in the same order (bit-identical to the two kernels),
// from one read of each entry's {mu, sigma} run; e = y - yhat written with T.
template <int KP>
__global__ __launch_bounds__(256) void k_predict_et_wave(const uint64_t *__restrict__ row_ptr,
                                                          const uint2 *__restrict__ csr,
                                                          const double2 *__restrict__ ms_v,
                                                          const double2 *__restrict__ ms_w, int k, int k1, int k0,
                                                          double mu0, double s0d, const float *__restrict__ target,
                                                          RowRec *__restrict__ rows, uint32_t n)
{
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t nwaves = gridDim.x * 4;
	for (uint32_t r = (blockIdx.x * 256 + threadIdx.x) >> 6; r < n; r += nwaves) {
		const uint64_t b = row_ptr[r], en = row_ptr[r + 1];
		double qe[KP], q[KP], z[KP];
#pragma unroll
		for (int c = 0; c < KP; ++c) { qe[c] = 0.0; q[c] = 0.0; z[c] = 0.0; }
		double qqe = 0.0, qq = 0.0;
		constexpr int PU = wave_pu(KP);
		for (uint64_t p0 = b; p0 < en; p0 += 64) {
			const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
			const uint2 mine = lane < cnt ? csr[p0 + lane] : make_uint2(0u, 0u);
			for (uint32_t i0 = 0; i0 < cnt; i0 += PU) {
				double2 mv[PU][KP];
				float xs[PU];
				wave_gather<KP, PU>(mine, cnt, i0, lane, ms_v, k, mv, xs);
#pragma unroll
				for (int u = 0; u < PU; ++u) {
					if (i0 + u >= cnt) break;
					const float x = xs[u];
#pragma unroll
					for (int c = 0; c < KP; ++c)
						if ((int)lane + 64 * c < k) {
							const double2 vm = mv[u][c];
							qe[c] += vm.x * x;                          // fm_learn_vb.h:93-133
							qqe -= 0.5 * vm.x * vm.x * x * x;           // :136-163
							q[c] += vm.x * x * vm.x * x;                // :222-254
							z[c] += vm.y * x * x;
							qq -= (vm.x * vm.x * x * x * x * x * vm.y + 0.5 * x * x * x * x * vm.y * vm.y);   // :257-281
						}
				}
			}
		}
		double e = 0.0, t = 0.0;
#pragma unroll
		for (int c = 0; c < KP; ++c)
			if ((int)lane + 64 * c < k) {
				e += 0.5 * qe[c] * qe[c];
				t += (0.5 * z[c] * z[c] + z[c] * q[c]);
			}
		e = wave_sum(e);
		qqe = wave_sum(qqe);
		t = wave_sum(t);
		qq = wave_sum(qq);
		if (k1) {                                               // :166-188 / :284-301
			for (uint64_t p0 = b; p0 < en; p0 += 64) {
				const uint32_t cnt = (uint32_t)min<uint64_t>(64, en - p0);
				double pe = 0.0, pt = 0.0;
				if (lane < cnt) {
					const uint2 ent = csr[p0 + lane];
					const float x = ent_x(ent);
					const double2 w = ms_w[ent.x];
					pe = w.x * x;
					pt = w.y * x * x;
				}
				for (uint32_t i = 0; i < cnt; ++i) {
					qqe += __shfl(pe, (int)i, 64);
					qq += __shfl(pt, (int)i, 64);
				}
			}
		}
		e = e + qqe;
		if (k0) e += mu0;
		t = t + qq;                                             // :304-311
		if (k0) t += s0d;
		if (lane == 0) {
			rows[r].e = target[r] - e;
			rows[r].t = t;
		}
	}
}

// e = y - yhat (fm_learn_vb_simultaneous.h:42-44)
__global__ void k_residual_init(RowRec *rows, const double *yhat, const float *target, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r < n) rows[r].e = target[r] - yhat[r];
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_row_sums(const RowRec *rows, uint32_t n, int mode, double mu0, double *out)
{
	__shared__ double lds[BLOCK / 64];
	double s = 0.0;
	for (uint32_t r = blockIdx.x * BLOCK + threadIdx.x; r < n; r += gridDim.x * BLOCK) {
		const double e = rows[r].e;
		if (mode == 0) s += e + mu0;                       // update_w0 (fm_learn_vb.h:512-514)
		else s += e * e + rows[r].t;                       // alpha / free energy (:450-452, :659-661)
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ void k_w0_apply(RowRec *rows, uint32_t n, double de, double dt)
{
	// fm_learn_vb.h:517-520
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r < n) { rows[r].e = rows[r].e + de; rows[r].t = rows[r].t + dt; }
}

// std::min(max_target, p) then std::max(min_target, p)
DEVI double clip(double p, double mn, double mx)
{
	p = (p < mx) ? p : mx;
	p = (mn < p) ? p : mn;
	return p;
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_test_metrics(const double *e_test, const float *target, uint32_t n, double mn,
                                                        double mx, double *pred, double *out)
{
	__shared__ double lds[2 * (BLOCK / 64)];
	double s2 = 0.0, s1 = 0.0;
	for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < n; c += gridDim.x * BLOCK) {
		double p = clip(e_test[c], mn, mx);                // fm_learn_vb_simultaneous.h:143-150
		pred[c] = p;
		p = clip(p * 1.0, mn, mx);                         // _evaluate (:266-274)
		const double err = p - target[c];
		s2 += err * err;
		s1 += fabs(err);
	}
	block_sum2<BLOCK>(s2, s1, lds);
	if (threadIdx.x == 0) { out[2 * blockIdx.x] = s2; out[2 * blockIdx.x + 1] = s1; }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_train_quirk(const RowRec *rows, uint32_t n, double mn, double mx, double *out)
{
	__shared__ double lds[BLOCK / 64];
	double s = 0.0;
	for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < n; c += gridDim.x * BLOCK) {
		const double p = clip(rows[c].e, mn, mx);          // :153-161
		s += p * p;
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// hyper-parameter sums (mode 0, fm_learn_vb.h:477-497: mu^2 + sigma) and free-energy terms
// (mode 1, :665-676) over one chunk of attributes of one (factor, group) segment.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_param_sums(const double2 *ms_w, const double2 *ms_v, const uint32_t *perm,
                                                      uint32_t D, const vbk::Chunk *chunks, int mode,
                                                      const double *hyp_w, const double *hyp_v, int k, double *out)
{
	__shared__ double lds[BLOCK / 64];
	const vbk::Chunk c = chunks[blockIdx.x];
	const double2 *ms = c.f < 0 ? ms_w : ms_v + c.f;       // ms_v is feature-major: [j*k + f]
	const size_t stride = c.f < 0 ? 1 : (size_t)k;
	const double hs = mode == 0 ? 0.0 : (c.f < 0 ? hyp_w[c.g] : hyp_v[(size_t)c.g * k + c.f]);
	double s = 0.0;
	for (uint32_t i = c.begin + threadIdx.x; i < c.end; i += BLOCK) {
		const double2 m = ms[(size_t)perm[i] * stride];
		if (mode == 0) s += m.x * m.x + m.y;
		else s += -0.5 * hs * (m.x * m.x + m.y) + 0.5 * log(m.y * hs) + .5;
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// The same sums over the factors, every factor of a chunk of one group's attributes in one
// workgroup: ms_v is feature-major, so attribute j's {mu, sigma} of all k factors are one
// contiguous run of 16k bytes, and P = 256 / k attributes are read side by side, one factor per
// thread (coalesced, each byte of ms_v read once; the per-(f, g) chunk walk above reads every
// 16-B pair on its own line, k times over the array). Per-factor partials of the chunk in a
// fixed order: part[chunk * k + f].
//   MODEL 0 (VB):   mode 0  mu^2 + sigma                               (fm_learn_vb.h:477-497)
//                   mode 1  the free-energy term with h = hyp_v[g][f]   (:665-676)
//   MODEL 1 (MCMC): mode 0  v ; mode 1 (v - h)^2 with h = v_mu[g][f]   (fm_learn_mcmc.h:1010-1089)
template <int MODEL>
__global__ __launch_bounds__(256) void k_vsums(const double2 *ms_v, const uint32_t *perm, const vbk::Chunk *chunks,
                                               int mode, const double *hv, int k, double *part)
{
	__shared__ double lds[256];
	const vbk::Chunk c = chunks[blockIdx.x];
	for (int fb = 0; fb < k; fb += 256) {
		const int kk = min(k - fb, 256);
		const int P = 256 / kk;
		const int sub = (int)threadIdx.x / kk;
		const int f = fb + (int)threadIdx.x % kk;
		double s = 0.0;
		if (sub < P) {
			const double h = mode == 0 ? 0.0 : hv[(size_t)c.g * k + f];
#pragma unroll 4
			for (uint32_t i = c.begin + sub; i < c.end; i += P) {
				const double2 m = ms_v[(size_t)perm[i] * k + f];
				if constexpr (MODEL == 0) {
					if (mode == 0) s += m.x * m.x + m.y;
					else s += -0.5 * h * (m.x * m.x + m.y) + 0.5 * log(m.y * h) + .5;
				} else {
					s += mode == 0 ? m.x : (m.x - h) * (m.x - h);
				}
			}
		}
		lds[threadIdx.x] = s;
		__syncthreads();
		if ((int)threadIdx.x < kk) {
			double t = lds[threadIdx.x];
			for (int p = 1; p < P; ++p) t += lds[p * kk + threadIdx.x];
			part[(size_t)blockIdx.x * k + f] = t;
		}
		__syncthreads();
	}
}

// seg[f * G + g] = group g's chunk partials of factor f summed in a fixed order (16 strided
// runs of chunks, then the 16 run sums in order); 64 factors per 1024-thread workgroup
__global__ __launch_bounds__(1024) void k_vsums_finish(const double *part, const uint32_t *gchunk, int k, uint32_t G,
                                                       double *seg)
{
	__shared__ double lds[1024];
	const uint32_t g = blockIdx.y;
	const int fl = (int)threadIdx.x % 64, sub = (int)threadIdx.x / 64;
	const int f = (int)blockIdx.x * 64 + fl;
	double s = 0.0;
	if (f < k) {
#pragma unroll 4
		for (uint32_t ch = gchunk[g] + sub; ch < gchunk[g + 1]; ch += 16) s += part[(size_t)ch * k + f];
	}
	lds[threadIdx.x] = s;
	__syncthreads();
	if (sub == 0 && f < k) {
		double t = lds[fl];
		for (int p = 1; p < 16; ++p) t += lds[p * 64 + fl];
		seg[(size_t)f * G + g] = t;
	}
}

// ------------------------------------------------------------------------------------
// dependency levels: relax level[b] >= level[a] + 1 over consecutive distinct features
// a < b of every row until nothing changes (least fixed point = longest-path levels).
__global__ void k_level_init(uint32_t *level, uint32_t nf)
{
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	if (j < nf) level[j] = 1;
}

__global__ void k_level_relax(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t *level, uint32_t *changed)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	if (e - b < 2) return;
	uint32_t prev = csr[b].x;
	uint32_t lp = __hip_atomic_load(&level[prev], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	bool ch = false;
	for (uint64_t p = b + 1; p < e; ++p) {
		const uint32_t cur = csr[p].x;
		if (cur == prev) continue;
		const uint32_t old = atomicMax(&level[cur], lp + 1);
		if (old < lp + 1) { ch = true; lp = lp + 1; } else lp = old;
		prev = cur;
	}
	if (ch) atomicOr(changed, 1u);
}

// The same levels in one pass over the edges (Kahn's order, level-synchronous): the relaxation
// needs one round per row switch on the longest path (365 rounds of the whole CSR for the
// multi-hot bench's 785 levels); here a feature's level is fixed in the round its last
// predecessor is processed. Edges are counted per entry: every entry (r, j) has the edge to the
// next distinct feature of row r, counted once per entry by k_kahn_indeg and consumed once per
// entry by k_kahn_round, whatever the order of a column's rows or repeated ids.
__global__ void k_kahn_indeg(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t *indeg)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	if (e - b < 2) return;
	uint32_t nx = csr[e - 1].x, cnt = 0;   // next distinct feature after the current run
	for (uint64_t q = e - 1; q > b; --q) {
		const uint32_t cur = csr[q - 1].x;
		if (cur != csr[q].x) {
			if (cnt) atomicAdd(&indeg[nx], cnt);
			nx = csr[q].x;
			cnt = 0;
		}
		if (cur != nx) cnt++;
	}
	if (cnt) atomicAdd(&indeg[nx], cnt);
}

// lanes with want append val to order[] (one atomic per wave); every lane of the wave calls
DEVI void wave_append(bool want, uint32_t val, uint32_t *tail, uint32_t *order)
{
	const uint64_t m = __ballot(want);
	if (!m) return;
	const int lane = threadIdx.x & 63;
	const int leader = __ffsll((unsigned long long)m) - 1;
	uint32_t base = 0;
	if (lane == leader) base = atomicAdd(tail, (uint32_t)__popcll(m));
	base = __shfl(base, leader);
	if (want) order[base + __popcll(m & ((1ull << lane) - 1ull))] = val;
}

__global__ __launch_bounds__(256) void k_kahn_seed(const uint32_t *indeg, uint32_t nf, uint32_t *level,
                                                   uint32_t *order, uint32_t *tail)
{
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	const bool src = j < nf && indeg[j] == 0;
	if (src) level[j] = 1;
	wave_append(src, j, tail, order);
}

// frontier bounds: the features of level t+1 are order[bounds[t] .. bounds[t+1])
__global__ void k_kahn_close(const uint32_t *tail, uint32_t *bounds, int slot)
{
	if (threadIdx.x == 0) bounds[slot] = *tail;
}

// round t: every entry of a frontier column consumes its edge; a feature whose last edge
// goes gets level t+2 and joins the next frontier. One wave per column (lanes over entries).
__global__ __launch_bounds__(256) void k_kahn_round(const uint64_t *col_ptr, const uint2 *csc, const uint64_t *row_ptr,
                                                    const uint2 *csr, const uint32_t *bounds, int t, uint32_t *indeg,
                                                    uint32_t *level, uint32_t *order, uint32_t *tail)
{
	const uint32_t s = bounds[t], e = bounds[t + 1];
	const uint32_t lane = threadIdx.x & 63u;
	const uint32_t nw = gridDim.x * 4u;
	for (uint32_t i = s + ((blockIdx.x * 256u + threadIdx.x) >> 6); i < e; i += nw) {
		const uint32_t j = order[i];
		const uint64_t cb = col_ptr[j], ce = col_ptr[j + 1];
		for (uint64_t p0 = cb; p0 < ce; p0 += 64) {
			const uint64_t p = p0 + lane;
			bool ready = false;
			uint32_t nxt = 0;
			if (p < ce) {
				const uint32_t r = csc[p].x & ROW_MASK;
				uint64_t lo = row_ptr[r], hi = row_ptr[r + 1];
				const uint64_t end = hi;
				while (lo < hi) {   // first entry of the row past feature j
					const uint64_t mid = (lo + hi) >> 1;
					if (csr[mid].x <= j) lo = mid + 1;
					else hi = mid;
				}
				if (lo < end) {
					nxt = csr[lo].x;
					ready = atomicSub(&indeg[nxt], 1u) == 1u;
				}
			}
			if (ready) level[nxt] = (uint32_t)t + 2u;
			wave_append(ready, nxt, tail, order);
		}
	}
}

__global__ void k_mark_dups(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint8_t *dup)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	for (uint64_t p = b + 1; p < e; ++p)
		if (csr[p].x == csr[p - 1].x) dup[csr[p].x] = 1;
}

// ------------------------------------------------------------------------------------
// field-structured synthetic generator (tests/synth.py is the specification)
DEVI uint64_t splitmix64(uint64_t z)
{
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}
DEVI uint64_t hstream(uint64_t seed, uint64_t stream, uint64_t i)
{
	return splitmix64(seed * 0x9E3779B97F4A7C15ull + stream * 0xD1B54A32D192ED03ull + i);
}

// order-independent 64-bit fingerprint of n words: the wrapping sum of splitmix64(word ^ f(index))
// (integer, so the atomic sum is exact in any order)
template <class W>
__global__ __launch_bounds__(256) void k_fingerprint(const W *a, uint64_t n, uint64_t salt, unsigned long long *out)
{
	unsigned long long s = 0;
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u)
		s += splitmix64((uint64_t)a[i] ^ (i * 0xD1B54A32D192ED03ull + salt));
	for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
	if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

__global__ void k_synth_entries(uint32_t n, uint32_t F, uint32_t S, uint64_t seed, int xmode, uint64_t row0, uint2 *csr)
{
	const uint64_t idx = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (idx >= (uint64_t)n * F) return;
	const uint32_t fld = (uint32_t)(idx % F);
	const uint64_t g = idx + row0 * F;      // entry index in the global (one-rank) data set
	const uint32_t feat = fld * S + (uint32_t)(hstream(seed, 1, g) % S);
	float x = 1.0f;
	if (xmode) x = 0.5f + (float)(hstream(seed, 2, g) >> 40) * 0x1p-24f;
	csr[idx] = make_uint2(feat, __float_as_uint(x));
}

DEVI double synth_unit(uint64_t seed, uint64_t stream, uint64_t i)
{
	return (double)(hstream(seed, stream, i) >> 11) * 0x1p-53;
}

// planted model: bias b(j) and rank-2 factors p(j, .) from the model seed, summed in field
// order with separate multiply and add (the file is built with -ffp-contract=off)
__global__ void k_synth_rows(uint32_t n, uint32_t F, uint64_t seed, uint64_t model_seed, uint64_t row0, double bgain,
                             double igain, const uint2 *csr, uint64_t *row_ptr, float *target)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r > n) return;
	row_ptr[r] = (uint64_t)r * F;
	if (r == n) return;
	double s = 0.0, s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
	for (uint32_t f = 0; f < F; ++f) {
		const uint64_t j = csr[(uint64_t)r * F + f].x;
		s = s + (synth_unit(model_seed, 3, j) - 0.5) * bgain;
		const double a0 = synth_unit(model_seed, 5, 2 * j) - 0.5;
		const double a1 = synth_unit(model_seed, 5, 2 * j + 1) - 0.5;
		s0 = s0 + a0;
		s1 = s1 + a1;
		q0 = q0 + a0 * a0;
		q1 = q1 + a1 * a1;
	}
	const double t = 0.5 * (s0 * s0 - q0) + 0.5 * (s1 * s1 - q1);
	const double noise = synth_unit(seed, 4, row0 + r) - 0.5;
	double y = rint(((3.0 + s) + igain * t) + 1.5 * noise);
	y = y < 1.0 ? 1.0 : (y > 5.0 ? 5.0 : y);
	target[r] = (float)y;
}

__global__ void k_synth_field_keys(const uint2 *csr, uint32_t n, uint32_t F, uint32_t S, uint32_t field, uint32_t *keys,
                                   uint32_t *vals)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	keys[r] = csr[(uint64_t)r * F + field].x - field * S;
	vals[r] = r;
}

__global__ void k_synth_field_scatter(const uint32_t *sorted_rows, const uint2 *csr, uint32_t n, uint32_t F, uint32_t field,
                                      uint2 *out)
{
	const uint32_t p = blockIdx.x * 256u + threadIdx.x;
	if (p >= n) return;
	const uint32_t r = sorted_rows[p];
	out[p] = make_uint2(r, csr[(uint64_t)r * F + field].y);
}

// multi-hot rows without field structure (tests/synth.py generate_multihot is the
// specification): row R holds L = lo + h(6, R) % (hi - lo + 1) distinct ids, id i drawn in
// stratum [i D / L, (i + 1) D / L) (ascending by construction); gains per L from the host table
__global__ void k_mh_len(uint32_t n, uint32_t lo, uint32_t hi, uint64_t seed, uint64_t row0, uint64_t *len)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r > n) return;
	len[r] = r < n ? lo + hstream(seed, 6, row0 + r) % (uint64_t)(hi - lo + 1) : 0;
}

__global__ void k_mh_fill(uint32_t n, uint32_t D, uint64_t seed, int xmode, uint64_t model_seed, uint64_t row0,
                          const double *gains, uint32_t lo, const uint64_t *row_ptr, uint2 *csr, uint32_t *row_of,
                          float *target)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t R = row0 + r, b = row_ptr[r];
	const uint32_t L = (uint32_t)(row_ptr[r + 1] - b);
	double s = 0.0, s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
	for (uint32_t i = 0; i < L; ++i) {
		const uint64_t a = (uint64_t)i * D / L, e = (uint64_t)(i + 1) * D / L;
		const uint64_t j = a + hstream(seed, 7, R * 64 + i) % (e - a);
		float x = 1.0f;
		if (xmode) x = 0.5f + (float)(hstream(seed, 2, R * 64 + i) >> 40) * 0x1p-24f;
		csr[b + i] = make_uint2((uint32_t)j, __float_as_uint(x));
		row_of[b + i] = r;
		s = s + (synth_unit(model_seed, 3, j) - 0.5);
		const double a0 = synth_unit(model_seed, 5, 2 * j) - 0.5;
		const double a1 = synth_unit(model_seed, 5, 2 * j + 1) - 0.5;
		s0 = s0 + a0;
		s1 = s1 + a1;
		q0 = q0 + a0 * a0;
		q1 = q1 + a1 * a1;
	}
	const double t = 0.5 * (s0 * s0 - q0) + 0.5 * (s1 * s1 - q1);
	const double noise = synth_unit(seed, 4, R) - 0.5;
	double y = rint(((3.0 + gains[2 * (L - lo)] * s) + gains[2 * (L - lo) + 1] * t) + 1.5 * noise);
	y = y < 1.0 ? 1.0 : (y > 5.0 ? 5.0 : y);
	target[r] = (float)y;
}

__global__ void k_mh_keys(const uint2 *csr, uint64_t nnz, uint32_t *keys, uint32_t *vals)
{
	const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (p >= nnz) return;
	keys[p] = csr[p].x;
	vals[p] = (uint32_t)p;
}

// CSC entries from the entries sorted (stably) by feature: {row, x} of entry p
__global__ void k_mh_scatter(const uint32_t *sorted_p, const uint2 *csr, const uint32_t *row_of, uint64_t nnz, uint2 *csc)
{
	const uint64_t q = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (q >= nnz) return;
	const uint32_t p = sorted_p[q];
	csc[q] = make_uint2(row_of[p], csr[p].y);
}

__global__ void k_count_features(const uint2 *csr, uint64_t nnz, unsigned long long *counts)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i < nnz) atomicAdd(&counts[csr[i].x], 1ull);
}

// {scale * N(0,1), second}: Box-Muller on two splitmix64 uniforms in (0, 1]
__global__ void k_init_normal_pairs(double2 *ms, size_t n, uint64_t seed, uint64_t stream, double scale, double second)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	const double u1 = ((double)(hstream(seed, stream, 2 * i) >> 11) + 1.0) * 0x1p-53;
	const double u2 = (double)(hstream(seed, stream, 2 * i + 1) >> 11) * 0x1p-53;
	const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
	ms[i] = make_double2(scale * z, second);
}

// out[j*rows + f] = {a[f*D + j], b[f*D + j]}
__global__ void k_pack(const double *a, const double *b, double2 *out, uint32_t rows, size_t D)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= (size_t)rows * D) return;
	const size_t j = i / rows, f = i % rows;
	out[i] = make_double2(a[f * D + j], b[f * D + j]);
}

__global__ void k_unpack(const double2 *in, double *a, double *b, uint32_t rows, size_t D)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= (size_t)rows * D) return;
	const size_t j = i / rows, f = i % rows;
	a[f * D + j] = in[i].x;
	b[f * D + j] = in[i].y;
}

// ------------------------------------------------------------------------------------
// feature-sharded passes (the north star's feature-column partition; Jacobi across shards):
// every shard holds all rows and starts a pass from the same row caches; afterwards the
// shards' changes of e and t and their partial q-caches of the next factor are summed.
// base[r] = e, base[n + r] = t at the start of a pass; the next factor's q-cache slot zeroed
__global__ void k_fs_begin(RowRec *rows, uint32_t n, double *base, int next_slot)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	RowRec &x = rows[r];
	base[r] = x.e;
	base[(size_t)n + r] = x.t;
	if (next_slot == 0) { x.q = 0.0; x.tq = 0.0; x.tz = 0.0; }
	else if (next_slot == 1) { x.q1 = 0.0; x.tq1 = 0.0; x.tz1 = 0.0; }
}

// buf = [e - e0 | t - t0 | q | tq | tz of the next slot], written (acc = 0) or added to
__global__ void k_fs_pack(const RowRec *rows, uint32_t n, const double *base, double *buf, int next_slot, int acc)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const RowRec &x = rows[r];
	double v[5] = {x.e - base[r], x.t - base[(size_t)n + r], 0.0, 0.0, 0.0};
	if (next_slot == 0) { v[2] = x.q; v[3] = x.tq; v[4] = x.tz; }
	else if (next_slot == 1) { v[2] = x.q1; v[3] = x.tq1; v[4] = x.tz1; }
	const int m = next_slot < 0 ? 2 : 5;
	for (int i = 0; i < m; ++i) {
		double *d = buf + (size_t)i * n + r;
		*d = acc ? *d + v[i] : v[i];
	}
}

__global__ void k_fs_unpack(RowRec *rows, uint32_t n, const double *base, const double *buf, int next_slot)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	RowRec &x = rows[r];
	x.e = base[r] + buf[r];
	x.t = base[(size_t)n + r] + buf[(size_t)n + r];
	const double q = buf[2 * (size_t)n + r], tq = buf[3 * (size_t)n + r], tz = buf[4 * (size_t)n + r];
	if (next_slot == 0) { x.q = q; x.tq = tq; x.tz = tz; }
	else if (next_slot == 1) { x.q1 = q; x.tq1 = tq; x.tz1 = tz; }
}

// to_buf: pbuf[j] = ms[j*stride] for the listed features; else ms[j*stride] = pbuf[j]
__global__ void k_fs_params(double2 *ms, uint32_t stride, const uint32_t *feats, uint32_t nfeat, double2 *pbuf,
                            int to_buf)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= nfeat) return;
	const uint32_t j = feats[i];
	if (to_buf) pbuf[j] = ms[(size_t)j * stride];
	else ms[(size_t)j * stride] = pbuf[j];
}

// ------------------------------------------------------------------------------------
// CSR of an uploaded data set from its CSC (Data.h keeps both; the device builds the row copy):
// each entry's (row; feature, x), then a stable radix sort by row keeps every row's entries in
// ascending feature order -- the order the reference's column loops visit a row in.
__global__ __launch_bounds__(256) void k_csc_expand(const uint64_t *col_ptr, const uint2 *csc, uint32_t *rows,
                                                    uint2 *fx)
{
	const uint32_t j = blockIdx.x;
	const uint64_t b = col_ptr[j], e = col_ptr[j + 1];
	for (uint64_t p = b + threadIdx.x; p < e; p += 256) {
		const uint2 ent = csc[p];
		rows[p] = ent.x & ROW_MASK;
		fx[p] = make_uint2(j, ent.y);
	}
}

__global__ void k_count_u32(const uint32_t *keys, uint64_t n, unsigned long long *counts)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n) atomicAdd(&counts[keys[i]], 1ull);
}

// ------------------------------------------------------------------------------------
// schedule check (VBFM_CHECK=1): within one level every row may be touched by one column at
// most (a column listing a row twice is corrected sequentially and counted once), or two
// workgroups of the level would update the same row concurrently
__global__ __launch_bounds__(256) void k_check_level(const uint32_t *feats, const uint64_t *col_ptr, const uint2 *csc,
                                                     const uint8_t *dup, uint32_t *owner, uint32_t *bad)
{
	const uint32_t j = feats[blockIdx.x];
	const uint64_t b = col_ptr[j], e = col_ptr[j + 1];
	for (uint64_t p = b + threadIdx.x; p < e; p += 256) {
		const uint32_t r = csc[p].x & ROW_MASK;
		const uint32_t prev = atomicCAS(&owner[r], 0xFFFFFFFFu, j);
		if (prev != 0xFFFFFFFFu && !(prev == j && dup[j])) atomicAdd(bad, 1u);
	}
}

inline unsigned grid_for(uint64_t n, unsigned block = 256) { return (unsigned)((n + block - 1) / block); }

}  // namespace

// ------------------------------------------------------------------------------------
// a collective that never completes, for the deadline test (VBFM_FAULT=comm_stall): the wave
// polls a flag in coherent host memory with loads only and leaves when the host sets it, or after
// 60 s of the 100 MHz constant clock whatever happens: every wave reaches the exit
__global__ __launch_bounds__(64) void k_stall(const volatile uint32_t *flag)
{
	const uint64_t t0 = wall_clock64();
	while (*flag == 0u && wall_clock64() - t0 < 6000000000ull) __builtin_amdgcn_s_sleep(127);
}

namespace vbk {

// Column-length-adaptive launch shape: threads per column and entries held per thread
// from the level's mean column length (dispatch_shape, vbfm_device.h).
template <int P, bool NEXT>
hipError_t launch_v_fused(const LevelArgs &a, hipStream_t s)
{
	dispatch_shape(a.avg_len, [&](auto B, auto R) { k_v_level_fused<B(), R(), P, NEXT><<<a.nfeat, B(), 0, s>>>(a); });
	return hipGetLastError();
}

template <bool NEXT>
hipError_t launch_w_fused(const LevelArgs &a, hipStream_t s)
{
	dispatch_shape(a.avg_len, [&](auto B, auto R) { k_w_level_fused<B(), R(), NEXT><<<a.nfeat, B(), 0, s>>>(a); });
	return hipGetLastError();
}

hipError_t stall(const uint32_t *flag, hipStream_t s)
{
	hipLaunchKernelGGL(k_stall, dim3(1), dim3(64), 0, s, flag);
	return hipGetLastError();
}

hipError_t v_level_fused(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (a.slot == 0) return nx ? launch_v_fused<0, true>(a, s) : launch_v_fused<0, false>(a, s);
	return nx ? launch_v_fused<1, true>(a, s) : launch_v_fused<1, false>(a, s);
}
hipError_t w_level_fused(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	return a.ms_next ? launch_w_fused<true>(a, s) : launch_w_fused<false>(a, s);
}
hipError_t col_long(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nsegs == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (is_w) {
		k_col_long_stats<true, 0><<<a.nsegs, 256, 0, s>>>(a);
		if (nx) k_col_long_correct<true, 0, true><<<a.nsegs, 256, 0, s>>>(a);
		else k_col_long_correct<true, 0, false><<<a.nsegs, 256, 0, s>>>(a);
	} else if (a.slot == 0) {
		k_col_long_stats<false, 0><<<a.nsegs, 256, 0, s>>>(a);
		if (nx) k_col_long_correct<false, 0, true><<<a.nsegs, 256, 0, s>>>(a);
		else k_col_long_correct<false, 0, false><<<a.nsegs, 256, 0, s>>>(a);
	} else {
		k_col_long_stats<false, 1><<<a.nsegs, 256, 0, s>>>(a);
		if (nx) k_col_long_correct<false, 1, true><<<a.nsegs, 256, 0, s>>>(a);
		else k_col_long_correct<false, 1, false><<<a.nsegs, 256, 0, s>>>(a);
	}
	return hipGetLastError();
}
hipError_t v_level_stats(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	// the fused kernel's BLOCK: the same reduction tree, so the split form equals the fused one
	dispatch_shape(a.avg_len, [&](auto B, auto) {
		if (a.slot == 0) k_v_level_stats<B(), 0><<<a.nfeat, B(), 0, s>>>(a);
		else k_v_level_stats<B(), 1><<<a.nfeat, B(), 0, s>>>(a);
	});
	return hipGetLastError();
}
hipError_t v_level_correct(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (a.slot == 0) {
		if (nx) k_v_level_correct<256, 0, true><<<a.nfeat, 256, 0, s>>>(a);
		else k_v_level_correct<256, 0, false><<<a.nfeat, 256, 0, s>>>(a);
	} else {
		if (nx) k_v_level_correct<256, 1, true><<<a.nfeat, 256, 0, s>>>(a);
		else k_v_level_correct<256, 1, false><<<a.nfeat, 256, 0, s>>>(a);
	}
	return hipGetLastError();
}
hipError_t w_level_stats(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	dispatch_shape(a.avg_len, [&](auto B, auto) { k_w_level_stats<B()><<<a.nfeat, B(), 0, s>>>(a); });
	return hipGetLastError();
}
hipError_t w_level_correct(const LevelArgs &a, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (a.ms_next) k_w_level_correct<256, true><<<a.nfeat, 256, 0, s>>>(a);
	else k_w_level_correct<256, false><<<a.nfeat, 256, 0, s>>>(a);
	return hipGetLastError();
}

hipError_t qcache(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_f, uint32_t stride, RowRec *rows,
                  uint32_t n, int slot, const uint32_t *pos, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_qcache<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, ms_f, stride, rows, n, slot, pos);
	return hipGetLastError();
}

hipError_t mark_first(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, uint2 *csc, uint32_t n,
                      hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_mark_first<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, col_ptr, csc, n);
	return hipGetLastError();
}

hipError_t predict_e(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k, int k1,
                     int k0, double mu0, double *out, uint32_t n, int blocked, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const unsigned wg = (unsigned)std::min<uint64_t>(((uint64_t)n + 3) / 4, 8192);   // 4 waves (rows) per workgroup
	if (blocked == 2 && k <= 64) k_predict_e_wave<1><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n);
	else if (blocked == 2 && k <= 128) k_predict_e_wave<2><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n);
	else if (blocked == 2 && k <= 256) k_predict_e_wave<4><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n);
	else if (blocked) k_predict_e_blocked<8><<<grid_for(n), 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n);
	else k_predict_e<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n);
	return hipGetLastError();
}

hipError_t predict_t(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k, int k1,
                     int k0, double s0d, RowRec *rows, uint32_t n, int blocked, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const unsigned wg = (unsigned)std::min<uint64_t>(((uint64_t)n + 3) / 4, 8192);
	if (blocked == 2 && k <= 64) k_predict_t_wave<1><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n);
	else if (blocked == 2 && k <= 128) k_predict_t_wave<2><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n);
	else if (blocked == 2 && k <= 256) k_predict_t_wave<4><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n);
	else if (blocked) k_predict_t_blocked<8><<<grid_for(n), 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n);
	else k_predict_t<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n);
	return hipGetLastError();
}

__global__ void k_compact_mu(const double2 *__restrict__ ms, double *__restrict__ out, size_t n)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n) out[i] = ms[i].x;
}

// predict_e with the factors' mu compacted into vc ([j*k + f], refreshed here from ms_v) where
// the wave form applies; otherwise predict_e itself. Same arithmetic and order: bit-identical.
hipError_t predict_e_compact(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k,
                             int k1, int k0, double mu0, double *out, uint32_t n, int blocked, double *vc, size_t kd,
                             bool refresh, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	if (blocked != 2 || k > 256 || !vc) return predict_e(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n, blocked, s);
	if (refresh && kd) k_compact_mu<<<(unsigned)((kd + 255) / 256), 256, 0, s>>>(ms_v, vc, kd);
	const unsigned wg = (unsigned)std::min<uint64_t>(((uint64_t)n + 3) / 4, 8192);
	if (k <= 64) k_predict_e_wave<1, true><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n, vc);
	else if (k <= 128) k_predict_e_wave<2, true><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n, vc);
	else k_predict_e_wave<4, true><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, out, n, vc);
	return hipGetLastError();
}

// e = y - yhat and T of a train set's rows; the one-pass kernel where the wave form applies
hipError_t predict_et(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k, int k1,
                      int k0, double mu0, double s0d, const float *target, double *scratch, RowRec *rows, uint32_t n,
                      int blocked, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const unsigned wg = (unsigned)std::min<uint64_t>(((uint64_t)n + 3) / 4, 8192);
	if (blocked == 2 && k <= 256) {
		if (k <= 64) k_predict_et_wave<1><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, s0d, target, rows, n);
		else if (k <= 128) k_predict_et_wave<2><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, s0d, target, rows, n);
		else k_predict_et_wave<4><<<wg, 256, 0, s>>>(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, s0d, target, rows, n);
		return hipGetLastError();
	}
	hipError_t e = predict_e(row_ptr, csr, ms_v, ms_w, k, k1, k0, mu0, scratch, n, blocked, s);
	if (e == hipSuccess) e = predict_t(row_ptr, csr, ms_v, ms_w, k, k1, k0, s0d, rows, n, blocked, s);
	if (e == hipSuccess) e = residual_init(rows, scratch, target, n, s);
	return e;
}

hipError_t residual_init(RowRec *rows, const double *yhat, const float *target, uint32_t n, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_residual_init<<<grid_for(n), 256, 0, s>>>(rows, yhat, target, n);
	return hipGetLastError();
}

hipError_t row_sums(const RowRec *rows, uint32_t n, int mode, double mu0, double *out, uint32_t nblocks, hipStream_t s)
{
	k_row_sums<256><<<nblocks, 256, 0, s>>>(rows, n, mode, mu0, out);
	return hipGetLastError();
}

hipError_t w0_apply(RowRec *rows, uint32_t n, double de, double dt, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_w0_apply<<<grid_for(n), 256, 0, s>>>(rows, n, de, dt);
	return hipGetLastError();
}

hipError_t test_metrics(const double *e_test, const float *target, uint32_t n, double mn, double mx, double *pred,
                        double *out, uint32_t nblocks, hipStream_t s)
{
	k_test_metrics<256><<<nblocks, 256, 0, s>>>(e_test, target, n, mn, mx, pred, out);
	return hipGetLastError();
}

hipError_t train_quirk(const RowRec *rows, uint32_t n, double mn, double mx, double *out, uint32_t nblocks, hipStream_t s)
{
	k_train_quirk<256><<<nblocks, 256, 0, s>>>(rows, n, mn, mx, out);
	return hipGetLastError();
}

hipError_t param_sums(const double2 *ms_w, const double2 *ms_v, const uint32_t *perm, uint32_t D, const Chunk *chunks,
                      uint32_t nchunks, int mode, const double *hyp_w, const double *hyp_v, int k, double *out,
                      hipStream_t s)
{
	if (nchunks == 0) return hipSuccess;
	k_param_sums<256><<<nchunks, 256, 0, s>>>(ms_w, ms_v, perm, D, chunks, mode, hyp_w, hyp_v, k, out);
	return hipGetLastError();
}

hipError_t fingerprint(const void *a, uint64_t n, int word_bytes, uint64_t salt, unsigned long long *out,
                       hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const unsigned grid = (unsigned)std::min<uint64_t>(4096, (n + 255) / 256);
	if (word_bytes == 8) k_fingerprint<uint64_t><<<grid, 256, 0, s>>>((const uint64_t *)a, n, salt, out);
	else k_fingerprint<uint32_t><<<grid, 256, 0, s>>>((const uint32_t *)a, n, salt, out);
	return hipGetLastError();
}

hipError_t vsums(const double2 *ms_v, const uint32_t *perm, const Chunk *chunks, uint32_t nchunks,
                 const uint32_t *gchunk, uint32_t G, int model, int mode, const double *hv, int k, double *part,
                 double *seg, hipStream_t s)
{
	if (nchunks == 0 || k <= 0 || G == 0) return hipSuccess;
	if (model == 0) k_vsums<0><<<nchunks, 256, 0, s>>>(ms_v, perm, chunks, mode, hv, k, part);
	else k_vsums<1><<<nchunks, 256, 0, s>>>(ms_v, perm, chunks, mode, hv, k, part);
	k_vsums_finish<<<dim3((unsigned)(k + 63) / 64, G), 1024, 0, s>>>(part, gchunk, k, G, seg);
	return hipGetLastError();
}

hipError_t level_init(uint32_t *level, uint32_t nf, hipStream_t s)
{
	if (nf == 0) return hipSuccess;
	k_level_init<<<grid_for(nf), 256, 0, s>>>(level, nf);
	return hipGetLastError();
}

hipError_t level_relax(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t nf, uint32_t *level,
                       uint32_t *changed, hipStream_t s)
{
	(void)nf;
	if (n == 0) return hipSuccess;
	k_level_relax<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, n, level, changed);
	return hipGetLastError();
}

hipError_t kahn_init(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t nf, uint32_t *indeg,
                     uint32_t *level, uint32_t *order, uint32_t *tail, uint32_t *bounds, hipStream_t s)
{
	if (nf == 0) return hipSuccess;
	hipError_t err = hipMemsetAsync(indeg, 0, (size_t)nf * 4, s);
	if (err == hipSuccess) err = hipMemsetAsync(tail, 0, 4, s);
	if (err == hipSuccess) err = hipMemsetAsync(bounds, 0, 4, s);
	if (err != hipSuccess) return err;
	if (n) k_kahn_indeg<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, n, indeg);
	k_kahn_seed<<<grid_for(nf), 256, 0, s>>>(indeg, nf, level, order, tail);
	k_kahn_close<<<1, 64, 0, s>>>(tail, bounds, 1);
	return hipGetLastError();
}

hipError_t kahn_round(const uint64_t *col_ptr, const uint2 *csc, const uint64_t *row_ptr, const uint2 *csr,
                      uint32_t *bounds, int t, uint32_t *indeg, uint32_t *level, uint32_t *order, uint32_t *tail,
                      hipStream_t s)
{
	k_kahn_round<<<1024, 256, 0, s>>>(col_ptr, csc, row_ptr, csr, bounds, t, indeg, level, order, tail);
	k_kahn_close<<<1, 64, 0, s>>>(tail, bounds, t + 2);
	return hipGetLastError();
}

hipError_t mark_dups(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint8_t *dup, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_mark_dups<<<grid_for(n), 256, 0, s>>>(row_ptr, csr, n, dup);
	return hipGetLastError();
}

hipError_t fs_begin(RowRec *rows, uint32_t n, double *base, int next_slot, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_fs_begin<<<grid_for(n), 256, 0, s>>>(rows, n, base, next_slot);
	return hipGetLastError();
}

hipError_t fs_pack(const RowRec *rows, uint32_t n, const double *base, double *buf, int next_slot, int acc,
                   hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_fs_pack<<<grid_for(n), 256, 0, s>>>(rows, n, base, buf, next_slot, acc);
	return hipGetLastError();
}

hipError_t fs_unpack(RowRec *rows, uint32_t n, const double *base, const double *buf, int next_slot, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_fs_unpack<<<grid_for(n), 256, 0, s>>>(rows, n, base, buf, next_slot);
	return hipGetLastError();
}

hipError_t fs_params(double2 *ms, uint32_t stride, const uint32_t *feats, uint32_t nfeat, double2 *pbuf, int to_buf,
                     hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_fs_params<<<grid_for(nfeat), 256, 0, s>>>(ms, stride, feats, nfeat, pbuf, to_buf);
	return hipGetLastError();
}

hipError_t synth_csr(uint32_t n, uint32_t F, uint32_t S, uint64_t seed, int xmode, uint64_t model_seed, uint64_t row0,
                     uint64_t *row_ptr, uint2 *csr, float *target, hipStream_t s)
{
	const uint64_t nnz = (uint64_t)n * F;
	const double bgain = sqrt(12.0 / (double)F);
	const double igain = F >= 2 ? sqrt(72.0 / ((double)F * (double)(F - 1) / 2.0)) : 0.0;
	if (nnz) k_synth_entries<<<grid_for(nnz), 256, 0, s>>>(n, F, S, seed, xmode, row0, csr);
	k_synth_rows<<<grid_for((uint64_t)n + 1), 256, 0, s>>>(n, F, seed, model_seed, row0, bgain, igain, csr, row_ptr,
	                                                      target);
	return hipGetLastError();
}

hipError_t synth_field_keys(const uint2 *csr, uint32_t n, uint32_t F, uint32_t S, uint32_t field, uint32_t *keys,
                            uint32_t *vals, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_synth_field_keys<<<grid_for(n), 256, 0, s>>>(csr, n, F, S, field, keys, vals);
	return hipGetLastError();
}

hipError_t synth_field_scatter(const uint32_t *sorted_rows, const uint2 *csr, uint32_t n, uint32_t F, uint32_t field,
                               uint2 *out, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_synth_field_scatter<<<grid_for(n), 256, 0, s>>>(sorted_rows, csr, n, F, field, out);
	return hipGetLastError();
}

hipError_t synth_mh_len(uint32_t n, uint32_t lo, uint32_t hi, uint64_t seed, uint64_t row0, uint64_t *len, hipStream_t s)
{
	k_mh_len<<<grid_for((uint64_t)n + 1), 256, 0, s>>>(n, lo, hi, seed, row0, len);
	return hipGetLastError();
}

hipError_t synth_mh_fill(uint32_t n, uint32_t D, uint64_t seed, int xmode, uint64_t model_seed, uint64_t row0,
                         const double *gains, uint32_t lo, const uint64_t *row_ptr, uint2 *csr, uint32_t *row_of,
                         float *target, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_mh_fill<<<grid_for(n), 256, 0, s>>>(n, D, seed, xmode, model_seed, row0, gains, lo, row_ptr, csr, row_of, target);
	return hipGetLastError();
}

hipError_t mh_keys(const uint2 *csr, uint64_t nnz, uint32_t *keys, uint32_t *vals, hipStream_t s)
{
	if (nnz == 0) return hipSuccess;
	k_mh_keys<<<grid_for(nnz), 256, 0, s>>>(csr, nnz, keys, vals);
	return hipGetLastError();
}

hipError_t synth_mh_scatter(const uint32_t *sorted_p, const uint2 *csr, const uint32_t *row_of, uint64_t nnz, uint2 *csc,
                            hipStream_t s)
{
	if (nnz == 0) return hipSuccess;
	k_mh_scatter<<<grid_for(nnz), 256, 0, s>>>(sorted_p, csr, row_of, nnz, csc);
	return hipGetLastError();
}

hipError_t count_features(const uint2 *csr, uint64_t nnz, uint64_t *counts, hipStream_t s)
{
	if (nnz == 0) return hipSuccess;
	k_count_features<<<grid_for(nnz), 256, 0, s>>>(csr, nnz, reinterpret_cast<unsigned long long *>(counts));
	return hipGetLastError();
}

hipError_t build_csr(const uint64_t *col_ptr, const uint2 *csc, uint32_t nf, uint32_t n, uint64_t nnz,
                     uint64_t *row_ptr, uint2 *csr, hipStream_t s)
{
	hipError_t err = hipSuccess;
	uint32_t *ki = nullptr, *ko = nullptr;
	uint2 *vi = nullptr;
	unsigned long long *counts = nullptr;
	void *tmp = nullptr;
	size_t tb = 0, tb2 = 0;
	int bits = 1;
	while (bits < 32 && (1ull << bits) < n) bits++;
#define BC(x) do { err = (x); if (err != hipSuccess) goto done; } while (0)
	BC(hipMalloc(&counts, ((size_t)n + 1) * 8));
	BC(hipMemsetAsync(counts, 0, ((size_t)n + 1) * 8, s));
	if (nnz) {
		BC(hipMalloc(&ki, nnz * 4));
		BC(hipMalloc(&ko, nnz * 4));
		BC(hipMalloc(&vi, nnz * 8));
		if (nf) k_csc_expand<<<nf, 256, 0, s>>>(col_ptr, csc, ki, vi);
		BC(hipGetLastError());
		BC(rocprim::radix_sort_pairs(nullptr, tb, ki, ko, vi, csr, (size_t)nnz, 0, bits, s));
		BC(hipMalloc(&tmp, tb));
		BC(rocprim::radix_sort_pairs(tmp, tb, ki, ko, vi, csr, (size_t)nnz, 0, bits, s));
		k_count_u32<<<grid_for(nnz), 256, 0, s>>>(ko, nnz, counts);
		BC(hipGetLastError());
		BC(hipStreamSynchronize(s));
		BC(hipFree(tmp));
		tmp = nullptr;
	}
	BC(exclusive_scan_u64(nullptr, &tb2, reinterpret_cast<uint64_t *>(counts), row_ptr, (size_t)n + 1, s));
	BC(hipMalloc(&tmp, tb2));
	BC(exclusive_scan_u64(tmp, &tb2, reinterpret_cast<uint64_t *>(counts), row_ptr, (size_t)n + 1, s));
	BC(hipStreamSynchronize(s));
#undef BC
done:
	if (ki) (void)hipFree(ki);
	if (ko) (void)hipFree(ko);
	if (vi) (void)hipFree(vi);
	if (counts) (void)hipFree(counts);
	if (tmp) (void)hipFree(tmp);
	return err;
}

hipError_t check_level(const uint32_t *feats, uint32_t nfeat, const uint64_t *col_ptr, const uint2 *csc,
                       const uint8_t *dup, uint32_t *owner, uint32_t *bad, hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_check_level<<<nfeat, 256, 0, s>>>(feats, col_ptr, csc, dup, owner, bad);
	return hipGetLastError();
}

hipError_t sort_pairs_u32(void *tmp, size_t *tmp_bytes, const uint32_t *ki, uint32_t *ko, const uint32_t *vi,
                          uint32_t *vo, size_t n, int bits, hipStream_t s)
{
	return rocprim::radix_sort_pairs(tmp, *tmp_bytes, ki, ko, vi, vo, n, 0, bits, s);
}

hipError_t exclusive_scan_u64(void *tmp, size_t *tmp_bytes, const uint64_t *in, uint64_t *out, size_t n, hipStream_t s)
{
	return rocprim::exclusive_scan(tmp, *tmp_bytes, in, out, (uint64_t)0, n, rocprim::plus<uint64_t>(), s);
}

hipError_t init_normal_pairs(double2 *ms, size_t n, uint64_t seed, uint64_t stream, double scale, double second,
                             hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_init_normal_pairs<<<grid_for(n), 256, 0, s>>>(ms, n, seed, stream, scale, second);
	return hipGetLastError();
}

hipError_t pack_pairs(const double *a, const double *b, double2 *out, uint32_t rows, size_t D, hipStream_t s)
{
	const size_t n = (size_t)rows * D;
	if (n == 0) return hipSuccess;
	k_pack<<<grid_for(n), 256, 0, s>>>(a, b, out, rows, D);
	return hipGetLastError();
}

hipError_t unpack_pairs(const double2 *in, double *a, double *b, uint32_t rows, size_t D, hipStream_t s)
{
	const size_t n = (size_t)rows * D;
	if (n == 0) return hipSuccess;
	k_unpack<<<grid_for(n), 256, 0, s>>>(in, a, b, rows, D);
	return hipGetLastError();
}

}  // namespace vbk
