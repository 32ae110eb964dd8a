// vbfm_lorder.hip -- the level-ordered row store: sweep kernels that stream the row caches
// instead of gathering them.
//
// The column-gather kernels (vbfm_kernels.hip) keep the row records in row order; a level
// reads and writes back one 64-B record at a random address per entry, twice per row per
// level (read, later write), and run at the random read-modify-write ceiling of HBM
// (~2e10 rows/s). When every dependency level holds each row exactly once
// (field-structured one-hot data: one level per field, every row one entry per field) the
// records can instead be kept physically in the order of the current level's CSC entries:
// position p of level l is the p-th entry of the level's columns taken in ascending
// feature order (ascending rows within a column), so a column's records are one contiguous
// run. A level then
//   * streams its records (coalesced, one pass),
//   * reduces each column's statistics, computes the posterior and applies the correction
//     exactly as update_v / update_w do (fm_learn_vb.h:577-644, :527-574), and
//   * writes every record once to its row's position in the NEXT level's order
//     (lnext[p]; the last level maps back to level 0, where every sweep starts):
// one streaming read + one random full-line write per row per level instead of a random
// read + a random write of the same line. The i-th entry of a column is the same (row, x)
// in both layouts and is reduced in the same tree order, so both layouts compute
// bit-identical column statistics, posteriors and corrections.
//
// Build (once per train set): level-ordered segment starts lcp (host), then per level the
// row -> position map (k_lord_pos) and the entry payload x / lnext (k_lord_fill), walking
// the levels backwards so that one row-sized scratch array holds the next level's map.
#include "vbfm_math.h"
#include "vbfm_mc_math.h"

namespace {

// What one level does to one record, as a policy of the staging loops below.
// VB (update_v :587-596/:623-643, update_w :534-539/:567-573): statistics, then the
// correction with the new posterior; NEXT adds the q-cache term of the next factor.
template <bool IS_W, int P, bool NEXT>
struct VbOp {
	double mo, so, mu, sig;
	double2 nx;
	bool go;
	DEVI void stat(Rec &v, float x, double &s1, double &s2) const
	{
		if constexpr (IS_W) w_stat(x, E(v), mo, s1, s2);
		else v_stat(x, E(v), Q<P>(v), TQ<P>(v), mo, so, s1, s2);
	}
	DEVI void apply(Rec &v, float x, bool first) const
	{
		if constexpr (IS_W) w_apply<NEXT>(v, x, first, go, mo, so, mu, sig, nx);
		else v_apply<P, NEXT>(v, x, first, go, mo, so, mu, sig, nx);
	}
};

template <bool IS_W>
DEVI bool vb_post(double s1, double s2, double hyp, double alpha, double mo, double so, double &mu, double &sig,
                  uint32_t *counters, bool leader)
{
	if constexpr (IS_W) return w_post(s1, s2, hyp, alpha, mo, so, mu, sig, counters, leader);
	else return v_post(s1, s2, hyp, alpha, mo, so, mu, sig, counters, leader);
}

// MCMC / ALS (draw_v :785-792/:826-834, draw_w :674-679/:712-717); row caches e (= yhat - y)
// and the q-cache of factor f in slot P, of factor f+1 (or 0 after draw_w) in the other
template <bool IS_W, int P, bool NEXT>
struct McOp {
	double vo, v, vn;
	bool go;
	double vp = 0.0;   // v_{f-1}[j] for the fused train re-prediction (McArgs::pk), pk 0: off
	int pk = 0;
	DEVI void stat(Rec &r, float x, double &s1, double &s2) const
	{
		if constexpr (IS_W) {
			s1 += x * (E(r) - vo * x);
			s2 += x * x;                                       // fp32 product
		} else {
			const double h = x * (Q<P>(r) - x * vo);
			s1 += h * E(r);
			s2 += h * h;
		}
	}
	DEVI void apply(Rec &r, float x, bool first) const
	{
		if (go) {
			if constexpr (IS_W) {
				const double h = x;
				E(r) -= h * (vo - v);
			} else {
				const double h = x * (Q<P>(r) - x * vo);
				Q<P>(r) -= x * (vo - v);
				E(r) -= h * (vo - v);
			}
		}
		if constexpr (NEXT) {
			const double a = vn * x;
			double &q = IS_W ? Q<0>(r) : Q<1 - P>(r);
			q = first ? 0.0 + a : q + a;
		}
		if constexpr (!IS_W) {
			if (pk) mc_pred_acc(TQ<0>(r), TZ<0>(r), T(r), x, first, vp, pk);   // MCMC leaves tq, tz, t free
		}
	}
};

// ---- LDS staging -------------------------------------------------------------------------
// A run of records moves between HBM and LDS four lanes per 64-B record (one 16-B piece
// each), so that every wave instruction reads or writes whole records: the scattered writes
// to the next level's order are then full-line writes. (One lane per record with four 16-B
// stores runs ~35 % slower: tools/probe_lord.hip.) In LDS piece c of record i sits at
// i*4 + (c ^ ((i >> 2) & 3)): the per-record ds_read_b128 / ds_write_b128 of 16 consecutive
// lanes then touch 16 distinct 16-B bank groups.
DEVI uint32_t lslot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

typedef double ntv2 __attribute__((ext_vector_type(2)));

// m <= BLOCK*R records = at most 4R pieces per thread; recs holds BLOCK*R records. Every
// piece is loaded into registers (straight-line, index clamped to the run) before the first
// LDS write, so a thread keeps 4R reads in flight; a load/write loop waits on each read before
// issuing the next (s_waitcnt vmcnt(0) per piece). stage_load / stage_store split the two
// halves so that a kernel can issue dependent loads (the deferred posterior gathers) between
// them. NT: non-temporal loads (records read once: keep L2 for gathered tables).
template <int BLOCK, int R, bool NT>
DEVI void stage_load(double2 (&v)[4 * R], const double2 *src, uint32_t m)
{
	const uint32_t np = max(m * 4, 1u);
#pragma unroll
	for (int k = 0; k < 4 * R; ++k) {
		const uint32_t t = min(threadIdx.x + k * BLOCK, np - 1);
		if constexpr (NT) {
			const ntv2 w = __builtin_nontemporal_load(reinterpret_cast<const ntv2 *>(src) + t);
			v[k] = make_double2(w.x, w.y);
		} else {
			v[k] = src[t];
		}
	}
}

// unconditional: slots past the run (copies of its last piece) are never read, and a
// conditional write lets the compiler sink each load next to it
template <int BLOCK, int R>
DEVI void stage_store(double2 *recs, const double2 (&v)[4 * R])
{
#pragma unroll
	for (int k = 0; k < 4 * R; ++k) {
		const uint32_t t = threadIdx.x + k * BLOCK;
		recs[lslot(t >> 2, t & 3)] = v[k];
	}
}

template <int BLOCK, int R, bool NT = false>
DEVI void stage_in(double2 *recs, const double2 *src, uint32_t m)
{
	if (m == 0) return;
	double2 v[4 * R];
	stage_load<BLOCK, R, NT>(v, src, m);
	stage_store<BLOCK, R>(recs, v);
}

template <int BLOCK, int R>
DEVI void stage_in_nt(double2 *recs, const double2 *src, uint32_t m)
{
	stage_in<BLOCK, R, true>(recs, src, m);
}

DEVI void lds_get(const double2 *recs, uint32_t i, Rec &v)
{
#pragma unroll
	for (uint32_t c = 0; c < 4; ++c) v[c] = recs[lslot(i, c)];
}

DEVI void lds_put(double2 *recs, uint32_t i, const Rec &v)
{
#pragma unroll
	for (uint32_t c = 0; c < 4; ++c) recs[lslot(i, c)] = v[c];
}

// statistics of a run of n records in chunks of CAP (the last chunk stays in LDS)
template <int BLOCK, uint32_t CAP, class Op>
DEVI void lord_stats(double2 *recs, const RowRec *src, const float *lx, uint32_t n, const Op &op, double &s1,
                     double &s2)
{
	const double2 *s = reinterpret_cast<const double2 *>(src);
	for (uint32_t base = 0; base < n; base += CAP) {
		const uint32_t m = min(CAP, n - base);
		if (base) __syncthreads();
		// this chunk's x in registers before its records stream in (a per-record load after
		// the barrier would wait once per record)
		constexpr int R = CAP / BLOCK;
		float xr[R];
#pragma unroll
		for (int u = 0; u < R; ++u) xr[u] = lx ? lx[base + min(threadIdx.x + u * BLOCK, m - 1)] : 1.0f;
		stage_in<BLOCK, R>(recs, s + (size_t)base * 4, m);
		__syncthreads();
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			if (i < m) {
				Rec v;
				lds_get(recs, i, v);
				op.stat(v, xr[u], s1, s2);
			}
		}
	}
}

// correction of every record of the run and its move to the next level's order. resident:
// the run (n <= CAP) is still in LDS from lord_stats. Every record is written even when the
// guards skip the correction: the write IS the move.
// ENT (the entry store, build_estore): bit 31 of a next position marks the row's first entry
// (the q-cache restart), which the level-uniform `first` gives in the field store
constexpr uint32_t ENT_FIRST = 0x80000000u;

// one 16-B piece of a moved record. NT (the entry store): a non-temporal store -- a slot is read
// by a later level of the row, rarely the next one, so the moved records are not kept in L2 and
// the launch boundary has no dirty lines to write back (multi-hot bench: v sweep 799 -> 706 ms,
// profiles/probes/ab_entry_nt_store.txt; the field store, whose next level reads every record,
// gains nothing from it)
template <bool NT>
DEVI void put_piece(double2 *d, size_t idx, const double2 &v)
{
	if constexpr (NT) {
		ntv2 w;
		w.x = v.x;
		w.y = v.y;
		__builtin_nontemporal_store(w, reinterpret_cast<ntv2 *>(d) + idx);
	} else {
		d[idx] = v;
	}
}

template <int BLOCK, uint32_t CAP, class Op, bool ENT = false>
DEVI void lord_move(double2 *recs, uint32_t *dsts, const RowRec *src, const float *lx, const uint32_t *nxt, uint32_t n,
                    bool resident, RowRec *dst, bool first, const Op &op)
{
	const double2 *s = reinterpret_cast<const double2 *>(src);
	double2 *d = reinterpret_cast<double2 *>(dst);
	for (uint32_t base = 0; base < n; base += CAP) {
		const uint32_t m = min(CAP, n - base);
		// x and next positions of the chunk in registers before its records stream in
		constexpr int R = CAP / BLOCK;
		float xr[R];
		uint32_t nr[R];
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t ic = base + min(threadIdx.x + u * BLOCK, m - 1);
			nr[u] = nxt[ic];
			xr[u] = lx ? lx[ic] : 1.0f;
		}
		if (!resident) {
			__syncthreads();
			stage_in<BLOCK, R>(recs, s + (size_t)base * 4, m);
			__syncthreads();
		}
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			if (i < m) {
				Rec v;
				lds_get(recs, i, v);
				op.apply(v, xr[u], ENT ? (nr[u] & ENT_FIRST) != 0 : first);
				lds_put(recs, i, v);
				dsts[i] = ENT ? nr[u] & ~ENT_FIRST : nr[u];
			}
		}
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
			const uint32_t i = t >> 2, c = t & 3;
			put_piece<ENT>(d, (size_t)dsts[i] * 4 + c, recs[lslot(i, c)]);
		}
	}
}

// A run that fits LDS (n <= CAP = BLOCK*R), thread-owned entries i = threadIdx.x + u*BLOCK
// (the order lord_stats / lord_move visit them): each entry's x and next position are loaded
// into registers BEFORE the records stream in, so their latency hides under the run's load
// instead of following it (the stats loop then touches no global memory; 15 % per launch at C4
// measured with the x array present, gpurun_out/r24).
template <int BLOCK, int R>
DEVI void res_prefetch(const float *lx, const uint32_t *nxt, uint32_t n, float (&xr)[R], uint32_t (&nr)[R])
{
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		xr[u] = 1.0f;
		nr[u] = 0;
		if (i < n) {
			nr[u] = nxt[i];
			if (lx) xr[u] = lx[i];
		}
	}
}

template <int BLOCK, int R, class Op>
DEVI void res_stats(const double2 *recs, uint32_t n, const float (&xr)[R], const Op &op, double &s1, double &s2)
{
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < n) {
			Rec v;
			lds_get(recs, i, v);
			op.stat(v, xr[u], s1, s2);
		}
	}
}

template <int BLOCK, int R, class Op, bool ENT = false>
DEVI void res_move(double2 *recs, uint32_t *dsts, uint32_t n, const float (&xr)[R], const uint32_t (&nr)[R],
                   RowRec *dst, bool first, const Op &op)
{
#pragma unroll
	for (int u = 0; u < R; ++u) {
		const uint32_t i = threadIdx.x + u * BLOCK;
		if (i < n) {
			Rec v;
			lds_get(recs, i, v);
			op.apply(v, xr[u], ENT ? (nr[u] & ENT_FIRST) != 0 : first);
			lds_put(recs, i, v);
			dsts[i] = ENT ? nr[u] & ~ENT_FIRST : nr[u];
		}
	}
	__syncthreads();
	double2 *d = reinterpret_cast<double2 *>(dst);
	for (uint32_t t = threadIdx.x; t < n * 4; t += BLOCK) {
		const uint32_t i = t >> 2, c = t & 3;
		put_piece<ENT>(d, (size_t)dsts[i] * 4 + c, recs[lslot(i, c)]);
	}
}

// One workgroup per column of the level: stream the column's run of records into LDS,
// reduce its statistics (update_v :587-596 / update_w :534-539), posterior + guards, then
// correct and move every record. Runs longer than CAP = BLOCK*R records are streamed twice
// (contiguous, L2-warm).
template <int BLOCK, int R, bool IS_W, int P, bool NEXT, bool ENT>
__global__ __launch_bounds__(BLOCK) void k_level_lord(const uint64_t *lcp, const uint32_t *feats, const RowRec *src_l,
                                                      const uint32_t *lnext_l, const float *lx_l, double2 *ms,
                                                      uint32_t ms_stride, LevelArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	__shared__ double lds[2 * (BLOCK / 64)];
	// the column's run bounds and its parameters first, from preloaded arguments only (LordLead):
	// the feature's index into ms (relative to the level's first feature on field data) ...
	// (no branch around a load: a branch puts a wait behind it; the feature-list load reads lcp's
	// word instead when there is no list)
	const uint64_t sb = lcp[blockIdx.x];
	const uint64_t se = lcp[blockIdx.x + 1];
	const uint32_t fj = *(feats ? feats + blockIdx.x : reinterpret_cast<const uint32_t *>(lcp + blockIdx.x));
	const uint32_t jr = feats ? fj : blockIdx.x;
	const uint32_t n = (uint32_t)(se - sb);
	const double2 msj = ms[(size_t)jr * ms_stride];
	// ... and every LevelArgs field the workgroup reads, fetched in one batch with them (left to
	// itself the compiler fetches them in several batches, each after a wait); the empty asm only
	// pins them to this point
	asm volatile("; k_level_lord: LevelArgs fields" ::"s"(a.long_min), "s"(a.lbase), "s"(a.hyp_uniform), "s"(a.hyp0),
	             "s"(a.alpha), "s"(a.counters), "s"(a.dst), "s"(a.first_level), "s"(a.feat_base),
	             "s"(a.ms_next), "s"(a.ms_stride_next), "s"(a.pf_lcp), "s"(a.pf_feats), "s"(a.pf_n));
	const uint32_t j = feats ? jr : a.feat_base + jr;   // the feature id
	if (a.long_min && n > a.long_min) return;      // a long column: the segment kernels' (lord_long)
	const RowRec *src = src_l + (sb - a.lbase);
	const float *lx = lx_l ? lx_l + sb : nullptr;   // null: every x is 1 (lx not stored)
	VbOp<IS_W, P, NEXT> op;
	op.mo = msj.x; op.so = msj.y;
	op.nx = NEXT ? a.ms_next[(size_t)j * a.ms_stride_next] : make_double2(0.0, 0.0);

	double s1 = 0.0, s2 = 0.0;
	// one attribute group: the prior by value (no attr_group -> hyp load chain)
	const double hyp = a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride];
	if (n <= CAP) {   // the run stays in LDS from the statistics to the move
		float xr[R];
		uint32_t nr[R];
		res_prefetch<BLOCK, R>(lx, lnext_l + sb, n, xr, nr);
		stage_in<BLOCK, R>(recs, reinterpret_cast<const double2 *>(src), n);
		__syncthreads();
		// the next level's column bounds (and feature id) of this workgroup index into this XCD's
		// L2 (the next launch puts workgroup blockIdx.x on the same XCD): its first load then hits
		// L2 instead of HBM. Issued after the run is staged, so the run's stream does not evict
		// it (the moves below are non-temporal on the entry store); the value is kept by a test
		// that never holds, at the end
		uint64_t pf = 0;
		if (blockIdx.x < a.pf_n) {   // uniform: scalar loads, whose counter the stores do not share
			pf = a.pf_lcp[blockIdx.x];
			if (a.pf_feats) pf += a.pf_feats[blockIdx.x];
		}
		res_stats<BLOCK, R>(recs, n, xr, op, s1, s2);
		block_sum2<BLOCK>(s1, s2, lds);
		op.go = vb_post<IS_W>(s1, s2, hyp, a.alpha, op.mo, op.so, op.mu, op.sig, a.counters, threadIdx.x == 0);
		if (threadIdx.x == 0) ms[(size_t)jr * ms_stride] = make_double2(op.mu, op.sig);
		res_move<BLOCK, R, VbOp<IS_W, P, NEXT>, ENT>(recs, dsts, n, xr, nr, a.dst, a.first_level != 0, op);
		if (pf == ~0ull) a.counters[CNT_N - 1] = 0u;   // never: positions and ids are < 2^63
		return;
	}
	lord_stats<BLOCK, CAP>(recs, src, lx, n, op, s1, s2);
	block_sum2<BLOCK>(s1, s2, lds);
	op.go = vb_post<IS_W>(s1, s2, hyp, a.alpha, op.mo, op.so, op.mu, op.sig, a.counters, threadIdx.x == 0);
	if (threadIdx.x == 0) ms[(size_t)jr * ms_stride] = make_double2(op.mu, op.sig);
	lord_move<BLOCK, CAP, VbOp<IS_W, P, NEXT>, ENT>(recs, dsts, src, lx, lnext_l + sb, n, false, a.dst,
	                                                a.first_level != 0, op);
}

// Long columns (skewed data: a popular item): one workgroup would stream the whole run while
// the rest of the level is long done. Their runs are cut into segments, one workgroup each:
// k_lord_long_stats writes each segment's statistics (and the column's parameters before the
// level), k_lord_long_move sums the column's segment partials in segment order (every
// workgroup of the column the same sum, so the same posterior), the column's first segment
// writes the new parameters, and every segment corrects and moves its records. The column's
// sum is taken in another order than one workgroup's (segments, then the tree): ~1e-16.
constexpr uint32_t LONG_BLOCK = 512, LONG_CAP = 1024;

template <bool IS_W, int P>
__global__ __launch_bounds__(LONG_BLOCK) void k_lord_long_stats(LevelArgs a)
{
	__shared__ double2 recs[LONG_CAP * 4];
	__shared__ double lds[2 * (LONG_BLOCK / 64)];
	const LongSeg g = a.segs[blockIdx.x];
	const uint32_t j = level_feat(a, g.col);
	const uint64_t sb = a.lcp[g.col] + g.start;
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	VbOp<IS_W, P, false> op;
	op.mo = msj.x; op.so = msj.y;
	double s1 = 0.0, s2 = 0.0;
	lord_stats<LONG_BLOCK, LONG_CAP>(recs, a.src + (sb - a.lbase), a.lx ? a.lx + sb : nullptr, g.len, op, s1, s2);
	block_sum2<LONG_BLOCK>(s1, s2, lds);
	if (threadIdx.x == 0) {
		a.seg_part[2 * blockIdx.x] = make_double2(s1, s2);
		a.seg_part[2 * blockIdx.x + 1] = msj;
	}
}

template <bool IS_W, int P, bool NEXT>
__global__ __launch_bounds__(LONG_BLOCK) void k_lord_long_move(LevelArgs a)
{
	__shared__ double2 recs[LONG_CAP * 4];
	__shared__ uint32_t dsts[LONG_CAP];
	const LongSeg g = a.segs[blockIdx.x];
	const uint32_t j = level_feat(a, g.col);
	const uint64_t sb = a.lcp[g.col] + g.start;
	double s1 = 0.0, s2 = 0.0;
	for (uint32_t q = 0; q < g.nseg; ++q) {
		const double2 p = a.seg_part[2 * (g.seg0 + q)];
		s1 += p.x;
		s2 += p.y;
	}
	const double2 msj = a.seg_part[2 * g.seg0 + 1];   // before this level (the first segment rewrites ms)
	VbOp<IS_W, P, NEXT> op;
	op.mo = msj.x; op.so = msj.y;
	op.nx = NEXT ? a.ms_next[(size_t)j * a.ms_stride_next] : make_double2(0.0, 0.0);
	const double hyp = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	const bool lead = threadIdx.x == 0 && blockIdx.x == g.seg0;
	op.go = vb_post<IS_W>(s1, s2, hyp, a.alpha, op.mo, op.so, op.mu, op.sig, a.counters, lead);
	if (lead) a.ms[(size_t)j * a.ms_stride] = make_double2(op.mu, op.sig);
	lord_move<LONG_BLOCK, LONG_CAP>(recs, dsts, a.src + (sb - a.lbase), a.lx ? a.lx + sb : nullptr, a.lnext + sb, g.len,
	                                false, a.dst, a.first_level != 0, op);
}

// split form (row-sharded multi-GPU): statistics of the local rows -> all-reduce -> move. The
// launch shape is the fused kernel's (launch_lord): the same BLOCK gives the same reduction tree,
// and a column's run takes no more LDS than it needs (with a fixed 256 x 2 shape the 100-entry
// columns of one N = 8 rank held 33-35 KB per workgroup: 13-15 resident waves per CU, 336 + 472 us
// per level against 341 us fused, profiles/r05_split/)
template <int BLOCK, int R, bool IS_W, int P>
__global__ __launch_bounds__(BLOCK) void k_level_lord_stats(LevelArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t sb = a.lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(a.lcp[blockIdx.x + 1] - sb);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	VbOp<IS_W, P, false> op;
	op.mo = msj.x; op.so = msj.y;
	double s1 = 0.0, s2 = 0.0;
	lord_stats<BLOCK, CAP>(recs, a.src + (sb - a.lbase), a.lx ? a.lx + sb : nullptr, n, op, s1, s2);
	block_sum2<BLOCK>(s1, s2, lds);
	if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(s1, s2);
}

template <int BLOCK, int R, bool IS_W, int P, bool NEXT, bool ENT = false>
__global__ __launch_bounds__(BLOCK) void k_level_lord_move(LevelArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t sb = a.lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(a.lcp[blockIdx.x + 1] - sb);
	debug_skew(a.skew);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double2 st = a.stats[blockIdx.x];
	VbOp<IS_W, P, NEXT> op;
	op.mo = msj.x; op.so = msj.y;
	op.nx = NEXT ? a.ms_next[(size_t)j * a.ms_stride_next] : make_double2(0.0, 0.0);
	const double hyp = (a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride]);
	op.go = vb_post<IS_W>(st.x, st.y, hyp, a.alpha, op.mo, op.so, op.mu, op.sig, a.counters, threadIdx.x == 0);
	// every wave has used the old value (vb_post above) before it is overwritten: without the
	// barrier a wave of this workgroup could still read the new one as its "old"
	__syncthreads();   // [raw-barrier]
	if (threadIdx.x == 0) a.ms[(size_t)j * a.ms_stride] = make_double2(op.mu, op.sig);
	lord_move<BLOCK, CAP, VbOp<IS_W, P, NEXT>, ENT>(recs, dsts, a.src + (sb - a.lbase), a.lx ? a.lx + sb : nullptr,
	                                                a.lnext + sb, n, false, a.dst, a.first_level != 0, op);
}

// ---- MCMC / ALS on the level-ordered store -----------------------------------------------
// MODE 0: fused; 1: statistics of this shard's rows into a.stats; 2: draw from the
// all-reduced a.stats, correct and move. Launch shape (BLOCK) as the column-gather MCMC
// kernel so that both reduce a column in the same order.
template <int BLOCK, int R, bool IS_W, int P, bool NEXT, int MODE, bool ENT = false>
__global__ __launch_bounds__(BLOCK) void k_mc_level_lord(McArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[MODE == 1 ? 1 : CAP];
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t sb = a.lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(a.lcp[blockIdx.x + 1] - sb);
	const RowRec *src = a.src + (sb - a.lbase);
	const float *lx = a.lx ? a.lx + sb : nullptr;
	McOp<IS_W, P, NEXT> op;
	if constexpr (MODE == 2) debug_skew(a.skew);
	op.vo = a.par[(size_t)j * a.stride].x;
	op.vn = NEXT ? a.par_next[(size_t)j * a.next_stride].x : 0.0;
	op.pk = IS_W ? 0 : a.pk;
	op.vp = op.pk ? a.par_prev[(size_t)j * a.next_stride].x : 0.0;
	double sm = 0.0, ss = 0.0;
	if constexpr (MODE == 0) {
		if (n <= CAP) {   // resident run, x / next positions prefetched (as k_level_lord)
			float xr[R];
			uint32_t nr[R];
			res_prefetch<BLOCK, R>(lx, a.lnext + sb, n, xr, nr);
			stage_in<BLOCK, R>(recs, reinterpret_cast<const double2 *>(src), n);
			__syncthreads();
			res_stats<BLOCK, R>(recs, n, xr, op, sm, ss);
			block_sum2<BLOCK>(sm, ss, lds);
			const uint32_t g = mc_group(a, j);
			op.go = mc_draw(sm, ss, op.vo, mc_lambda(a, g), mc_mu(a, g), a.alpha,
			                mc_z(a, j), a.z != nullptr, a.sample, !IS_W, op.v, a.counters, threadIdx.x == 0);
			if (threadIdx.x == 0) a.par[(size_t)j * a.stride].x = op.v;
			res_move<BLOCK, R, McOp<IS_W, P, NEXT>, ENT>(recs, dsts, n, xr, nr, a.dst, a.first_level != 0, op);
			return;
		}
	}
	if constexpr (MODE != 2) {
		lord_stats<BLOCK, CAP>(recs, src, lx, n, op, sm, ss);
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
	if constexpr (MODE != 1) {
		const uint32_t g = mc_group(a, j);
		op.go = mc_draw(sm, ss, op.vo, mc_lambda(a, g), mc_mu(a, g), a.alpha,
		                mc_z(a, j), a.z != nullptr, a.sample, !IS_W, op.v, a.counters, threadIdx.x == 0);
		// MODE 2: every wave has used the old value (the draw) before it is overwritten (no
		// barrier since the kernel began; without one a wave could read the new value as "old")
		if constexpr (MODE == 2) __syncthreads();   // [raw-barrier]
		if (threadIdx.x == 0) a.par[(size_t)j * a.stride].x = op.v;
		lord_move<BLOCK, CAP, McOp<IS_W, P, NEXT>, ENT>(recs, dsts, src, lx, a.lnext + sb, n, false, a.dst,
		                                                a.first_level != 0, op);
	}
}

// ---- placement probe ---------------------------------------------------------------------
// The level kernel's memory pattern without its arithmetic: level 0's runs (one workgroup per
// column, LDS-staged in chunks of 512 records) moved whole to their slots of level 1 (lnext).
// Used to time a pair of record buffers before the store adopts it: the scattered-write rate of
// the pattern depends on where the buffers were placed by up to ~20 %, persistently per
// allocation (tools/probe_place.hip); the copy rate does not.
__global__ __launch_bounds__(256) void k_place_move(const RowRec *src, RowRec *dst, const uint64_t *lcp,
                                                    const uint32_t *lnext)
{
	constexpr uint32_t CAP = 512;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	const uint64_t sb = lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(lcp[blockIdx.x + 1] - sb);
	const double2 *s = reinterpret_cast<const double2 *>(src + sb);
	double2 *d = reinterpret_cast<double2 *>(dst);
	for (uint32_t base = 0; base < n; base += CAP) {
		const uint32_t m = min(CAP, n - base);
		if (base) __syncthreads();
		double2 v[8];
		uint32_t nr[2];
#pragma unroll
		for (int u = 0; u < 2; ++u) nr[u] = lnext[sb + base + min(threadIdx.x + u * 256, m - 1)];
		stage_load<256, 2, false>(v, s + (size_t)base * 4, m);
		stage_store<256, 2>(recs, v);
#pragma unroll
		for (int u = 0; u < 2; ++u) dsts[threadIdx.x + u * 256] = nr[u];
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < m * 4; t += 256) {
			const uint32_t i = t >> 2, c = t & 3;
			d[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
		}
	}
}

// ---- build -------------------------------------------------------------------------------
__global__ void k_lord_pack(const float *lx, const uint32_t *lnext, const uint32_t *lpidx, const float *lpx, uint4 *lpay,
                            uint64_t nnz)
{
	const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (p < nnz)
		lpay[p] = make_uint4(__float_as_uint(lx ? lx[p] : 1.0f), lnext[p], lpidx[p], __float_as_uint(lpx[p]));
}

__global__ void k_lord_pack2(const uint32_t *lnext, const uint32_t *lpidx, uint2 *lpay2, uint64_t nnz)
{
	const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (p < nnz) lpay2[p] = make_uint2(lnext[p], lpidx[p]);
}

// pos[row] = level-relative position of the row's entry in this level
__global__ __launch_bounds__(256) void k_lord_pos(const uint32_t *feats, const uint64_t *lcp, uint64_t lbase,
                                                  const uint64_t *col_ptr, const uint2 *csc, uint32_t *pos)
{
	const uint32_t j = feats[blockIdx.x];
	const uint64_t cb = col_ptr[j];
	const uint32_t n = (uint32_t)(col_ptr[j + 1] - cb);
	const uint32_t p0 = (uint32_t)(lcp[blockIdx.x] - lbase);
	for (uint32_t i = threadIdx.x; i < n; i += 256) pos[csc[cb + i].x & ROW_MASK] = p0 + i;
}

// payload of the level's entries: x, the row's position in the next level, and (level 0)
// the row id of every position
__global__ __launch_bounds__(256) void k_lord_fill(const uint32_t *feats, const uint64_t *lcp, uint64_t lbase,
                                                   const uint64_t *col_ptr, const uint2 *csc, const uint32_t *pos_next,
                                                   float *lx, uint32_t *lnext, uint32_t *row0)
{
	const uint32_t j = feats[blockIdx.x];
	const uint64_t cb = col_ptr[j];
	const uint32_t n = (uint32_t)(col_ptr[j + 1] - cb);
	const uint64_t g0 = lcp[blockIdx.x];
	for (uint32_t i = threadIdx.x; i < n; i += 256) {
		const uint2 ent = csc[cb + i];
		const uint32_t r = ent.x & ROW_MASK;
		if (lx) lx[g0 + i] = ent_x(ent);
		lnext[g0 + i] = pos_next[r];
		if (row0) row0[g0 + i - lbase] = r;
	}
}

// the entry store's deferred payload (row shards): for every slot, the global level-feature
// index and the x of the row's previous entry (the first entry's previous is the row's last:
// the correction a sweep leaves pending at its end, carried into the next sweep or flushed)
__global__ __launch_bounds__(256) void k_estore_prev(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr,
                                                     const uint2 *csc, const uint32_t *lvpos, const uint64_t *lcp,
                                                     uint32_t n, uint32_t *lpidx, float *lpx)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	for (uint64_t p = b; p < e; ++p) {
		const uint32_t j = csr[p].x;
		uint64_t lo = col_ptr[j], hi = col_ptr[j + 1];   // rows ascending: the row's entry of column j
		const uint64_t c0 = lo;
		while (lo < hi) {
			const uint64_t mid = (lo + hi) >> 1;
			if ((csc[mid].x & ROW_MASK) < r) lo = mid + 1;
			else hi = mid;
		}
		const uint32_t slot = (uint32_t)(lcp[lvpos[j]] + (lo - c0));
		const uint2 prev = csr[p == b ? e - 1 : p - 1];
		lpidx[slot] = lvpos[prev.x];
		lpx[slot] = ent_x(prev);
	}
}

// number of entries whose x is not 1.0f (the level store then keeps x per entry)
__global__ __launch_bounds__(256) void k_count_x_ne1(const uint2 *csc, uint64_t nnz, uint32_t *cnt)
{
	uint32_t m = 0;
	for (uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x; p < nnz; p += (uint64_t)gridDim.x * 256u)
		m |= ent_x(csc[p]) != 1.0f;
	m = __any(m);
	if (m && (threadIdx.x & 63) == 0) atomicAdd(cnt, 1u);
}

// record permutations between row order and level-0 order; 4 lanes per 64-B record
__global__ __launch_bounds__(256) void k_rows_gather(RowRec *__restrict__ dst, const RowRec *__restrict__ src,
                                                     const uint32_t *__restrict__ idx, uint32_t n)
{
	const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	const uint32_t p = (uint32_t)(t >> 2), c = (uint32_t)(t & 3);
	if (p >= n) return;
	reinterpret_cast<double2 *>(dst + p)[c] = reinterpret_cast<const double2 *>(src + idx[p])[c];
}

__global__ __launch_bounds__(256) void k_rows_scatter(RowRec *__restrict__ dst, const RowRec *__restrict__ src,
                                                      const uint32_t *__restrict__ idx, uint32_t n)
{
	const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	const uint32_t p = (uint32_t)(t >> 2), c = (uint32_t)(t & 3);
	if (p >= n) return;
	reinterpret_cast<double2 *>(dst + idx[p])[c] = reinterpret_cast<const double2 *>(src + p)[c];
}

// The entry store (data whose levels miss rows: multi-hot rows without fields): slot s of the
// store is the s-th entry of the train set taken level by level (the level's columns in
// ascending feature order, rows ascending in a column: the field store's order), and a row's
// record waits in the slot of the entry its next level will sweep. A row's features ascend
// with their levels (the schedule's definition), so its CSR entries come in level order: per
// row, each entry's slot (its rank in its column by binary search), then for every slot the
// slot of the row's next entry (the last entry -> the first: the next sweep), bit 31 on the
// row's first entry (the q-cache restart), the entry's x, and the row's first slot. A row
// without entries is never swept: its record waits in a parking slot past the entries, nnz + r.
__global__ __launch_bounds__(256) void k_estore_build(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr,
                                                      const uint2 *csc, const uint32_t *lvpos, const uint64_t *lcp,
                                                      uint32_t n, uint64_t nnz, uint32_t *lnext, float *lx,
                                                      uint32_t *lfirst)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint64_t b = row_ptr[r], e = row_ptr[r + 1];
	if (e == b) {
		lfirst[r] = (uint32_t)(nnz + r);
		return;
	}
	auto slot_of = [&](uint2 ent) -> uint32_t {
		const uint32_t j = ent.x;
		uint64_t lo = col_ptr[j], hi = col_ptr[j + 1];   // rows ascending: first entry with row >= r
		const uint64_t c0 = lo;
		while (lo < hi) {
			const uint64_t mid = (lo + hi) >> 1;
			if ((csc[mid].x & ROW_MASK) < r) lo = mid + 1;
			else hi = mid;
		}
		return (uint32_t)(lcp[lvpos[j]] + (lo - c0));
	};
	const uint32_t s0 = slot_of(csr[b]);
	uint32_t s = s0;
	for (uint64_t p = b; p < e; ++p) {
		const uint32_t sn = p + 1 < e ? slot_of(csr[p + 1]) : s0;
		lnext[s] = sn | (p == b ? ENT_FIRST : 0u);
		if (lx) lx[s] = ent_x(csr[p]);
		s = sn;
	}
	lfirst[r] = s0;
}

// The leading (preloaded, -amdgpu-kernarg-preload-count) arguments of k_level_lord: everything the
// loads of a column's bounds and parameters need, so they issue at wave start. On field data ms
// arrives offset to the level's first feature (feats null: the column's index is blockIdx.x)
struct LordLead {
	const uint64_t *lcp;
	const uint32_t *feats;
	const RowRec *src;
	const uint32_t *lnext;
	const float *lx;
	double2 *ms;
	uint32_t ms_stride;
};
#define LORD_LEAD_ARGS(L) L.lcp, L.feats, L.src, L.lnext, L.lx, L.ms, L.ms_stride

inline LordLead lord_lead(const LevelArgs &a)
{
	LordLead L;
	L.lcp = a.lcp;
	L.feats = a.feat_contig ? nullptr : a.feats;
	L.src = a.src;
	L.lnext = a.lnext;
	L.lx = a.lx;
	L.ms = a.feat_contig ? a.ms + (size_t)a.feat_base * a.ms_stride : a.ms;
	L.ms_stride = a.ms_stride;
	return L;
}

template <bool IS_W, int P, bool NEXT>
void launch_lord(const LevelArgs &a, hipStream_t s)
{
	const LordLead L = lord_lead(a);
	dispatch_shape(a.avg_len, [&](auto B, auto R) {
		if (a.ent) k_level_lord<B(), R(), IS_W, P, NEXT, true><<<a.nfeat, B(), 0, s>>>(LORD_LEAD_ARGS(L), a);
		else k_level_lord<B(), R(), IS_W, P, NEXT, false><<<a.nfeat, B(), 0, s>>>(LORD_LEAD_ARGS(L), a);
	});
}

template <bool IS_W, int P, bool NEXT, bool ENT>
void launch_lord_move_shape(const LevelArgs &a, hipStream_t s)
{
	dispatch_shape(a.avg_len, [&](auto B, auto R) { k_level_lord_move<B(), R(), IS_W, P, NEXT, ENT><<<a.nfeat, B(), 0, s>>>(a); });
}

template <bool IS_W, int P>
void launch_lord_move(const LevelArgs &a, hipStream_t s)
{
	if (a.ent) {
		if (a.ms_next) launch_lord_move_shape<IS_W, P, true, true>(a, s);
		else launch_lord_move_shape<IS_W, P, false, true>(a, s);
		return;
	}
	if (a.ms_next) launch_lord_move_shape<IS_W, P, true, false>(a, s);
	else launch_lord_move_shape<IS_W, P, false, false>(a, s);
}

template <bool IS_W, int P>
void launch_lord_stats(const LevelArgs &a, hipStream_t s)
{
	dispatch_shape(a.avg_len, [&](auto B, auto R) { k_level_lord_stats<B(), R(), IS_W, P><<<a.nfeat, B(), 0, s>>>(a); });
}


// ---- deferred correction (row-sharded split) ---------------------------------------------
// The split form above streams every level's records twice (statistics, then after the
// all-reduce the move). Deferred: level l's kernel applies level l-1's correction to each
// record (its posterior from the table the previous post kernel wrote, gathered by the row's
// level-(l-1) feature; the row's level-(l-1) x rides along in lpx), reduces level l's
// statistics from the corrected records and moves them, still without level l's own
// correction, to level l+1's order. After the all-reduce a small kernel turns the statistics
// into posteriors (parameters + table); the next level applies them, a flush kernel after the
// last level of a sweep. Same arithmetic per row as the fused kernel: bit-identical results.
// the previous level's correction (without its q-cache term: each level adds its own term
// of the next factor's q-cache in its kernel, in the same per-row order as the fused kernel)
// an entry's deferred payload {x, next position, previous-level feature, its x}: the 16-B
// record, or the 8-B {next, previous} one when every x is 1
template <bool PAY8, class A> DEVI uint4 pay_load(const A &a, uint64_t p)
{
	if constexpr (PAY8) {
		const uint2 w = a.lpay2[p];
		return make_uint4(0x3f800000u, w.x, w.y, 0x3f800000u);
	} else {
		return a.lpay[p];
	}
}

template <class A> DEVI uint4 pay_at(const A &a, uint64_t p)
{
	if (a.lpay2) {
		const uint2 w = a.lpay2[p];
		return make_uint4(0x3f800000u, w.x, w.y, 0x3f800000u);
	}
	return a.lpay[p];
}

template <bool IS_W, int P>
DEVI void apply_pending(Rec &v, const PostT &t, float x)
{
	VbOp<IS_W, P, false> op;
	op.mo = t.mo; op.so = t.so; op.sig = t.sig; op.nx = make_double2(0.0, 0.0);
	op.go = !__builtin_isnan(t.mu);
	op.mu = op.go ? t.mu : t.mo;
	op.apply(v, x, false);
}

// this level's term of the next factor's q-cache (slot 0 after the w sweep, 1-P after v)
template <bool IS_W, int P>
DEVI void add_next_q(Rec &v, float x, bool first, double2 nx)
{
	if constexpr (IS_W) qacc<0>(v, x, first, nx);
	else qacc<1 - P>(v, x, first, nx);
}

// PK: which level's correction is pending -- 0: the previous level of this sweep; at level 0 of
// a v sweep the previous sweep's last level, left unflushed: 1 = v with the other q-cache slot
// (the previous factor), 2 = w (the w sweep before factor 0)
// ENT (the entry store under row shards): a row's previous entry sits in any earlier level, so
// the posteriors live in one table over all level features (tab[global index], written by each
// level's post kernel at tab_base) and the pending correction is decided per entry: the row's
// first entry (ENT_FIRST) carries the previous sweep's last correction (PK, or nothing when
// that sweep was flushed), every other entry the correction of the row's previous entry in
// this sweep; records move to their rows' next slots in the same store (non-temporal stores)
template <int BLOCK, int R, bool IS_W, int P, bool NEXT, int PK, bool PAY8, bool ENT = false>
__global__ __launch_bounds__(BLOCK) void k_lord_defer(LevelArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t sb = a.lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(a.lcp[blockIdx.x + 1] - sb);
	const RowRec *src = a.src + (sb - a.lbase);
	const double2 *s = reinterpret_cast<const double2 *>(src);
	double2 *d = reinterpret_cast<double2 *>(a.dst);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	VbOp<IS_W, P, NEXT> op;
	op.mo = msj.x; op.so = msj.y;
	const double2 nx = NEXT ? a.ms_next[(size_t)j * a.ms_stride_next] : make_double2(0.0, 0.0);
	const bool first = a.first_level != 0;
	const bool pending = (a.pending & 1) != 0;
	double s1 = 0.0, s2 = 0.0;
	for (uint32_t base = 0; base < n; base += CAP) {
		const uint32_t m = min(CAP, n - base);
		if (base) __syncthreads();
		// each entry's {x, next position, previous-level feature, its x} in one 16-B load; the
		// posteriors of the records' previous-level features are gathered (L2 / MALL: one line
		// each) while the run streams into LDS
		// payloads, then the run's records, then the posteriors the payloads point at (the
		// gathers wait for the payloads only), then the LDS writes: three round trips overlap
		PostT t[R];
		uint4 q[R];
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			q[u] = pay_load<PAY8>(a, sb + base + min(i, m - 1));
		}
		double2 sv[4 * R];
		// records read once: non-temporal loads on large shards (pending bit 1); on a shard the
		// size of C4's on 8 GPUs (1.25e7 rows) plain loads are 1.5 % faster
		// (profiles/probes/ab_defer_loads.txt)
		if (a.pending & 2) stage_load<BLOCK, R, true>(sv, s + (size_t)base * 4, m);
		else stage_load<BLOCK, R, false>(sv, s + (size_t)base * 4, m);
		// unconditional (a.tab always holds a previous level's width; unused unless pending):
		// a branch here lets the compiler sink half of each payload load after the records'
#pragma unroll
		for (int u = 0; u < R; ++u) t[u] = a.tab[q[u].z];
		stage_store<BLOCK, R>(recs, sv);
		__syncthreads();
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			if (i >= m) continue;
			Rec v;
			lds_get(recs, i, v);
			const float x = __uint_as_float(q[u].x);
			const float px = __uint_as_float(q[u].w);
			bool fe = first;
			if constexpr (ENT) {
				fe = (q[u].y & ENT_FIRST) != 0;
				if (!fe) apply_pending<IS_W, P>(v, t[u], px);
				else if constexpr (PK == 1) apply_pending<false, 1 - P>(v, t[u], px);
				else if constexpr (PK == 2) apply_pending<true, 0>(v, t[u], px);
			} else if (pending) {
				if constexpr (PK == 0) apply_pending<IS_W, P>(v, t[u], px);
				else if constexpr (PK == 1) apply_pending<false, 1 - P>(v, t[u], px);
				else apply_pending<true, 0>(v, t[u], px);
			}
			if constexpr (NEXT) add_next_q<IS_W, P>(v, x, fe, nx);
			if (ENT || pending || NEXT) lds_put(recs, i, v);
			op.stat(v, x, s1, s2);
			dsts[i] = ENT ? q[u].y & ~ENT_FIRST : q[u].y;
		}
		__syncthreads();
		// non-temporal record stores (pending bit 2; always on the entry store): with non-temporal
		// loads too the moved records no longer push the posterior table out of L2
		// (tools/probe_defer8.hip: the gather's cost 43 -> 23 us per level at one N = 8 rank's shape)
		if (ENT || (a.pending & 4)) {
			for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
				const uint32_t i = t >> 2, c = t & 3;
				put_piece<true>(d, (size_t)dsts[i] * 4 + c, recs[lslot(i, c)]);
			}
		} else {
			for (uint32_t t = threadIdx.x; t < m * 4; t += BLOCK) {
				const uint32_t i = t >> 2, c = t & 3;
				put_piece<false>(d, (size_t)dsts[i] * 4 + c, recs[lslot(i, c)]);
			}
		}
	}
	block_sum2<BLOCK>(s1, s2, lds);
	if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(s1, s2);
}

// posteriors of the level's features from the all-reduced statistics (update_v :597-619 /
// update_w :540-565): parameters, and the table the next level's kernel reads
template <bool IS_W, bool NEXT>
__global__ __launch_bounds__(256) void k_lord_defer_post(LevelArgs a)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= a.nfeat) return;
	const uint32_t j = level_feat(a, i);
	const double2 msj = a.ms[(size_t)j * a.ms_stride];
	const double2 st = a.stats[i];
	const double hyp = a.hyp_uniform ? a.hyp0 : a.hyp[(size_t)a.attr_group[j] * a.hyp_stride];
	double mu, sig;
	const bool go = vb_post<IS_W>(st.x, st.y, hyp, a.alpha, msj.x, msj.y, mu, sig, a.counters, true);
	a.ms[(size_t)j * a.ms_stride] = make_double2(mu, sig);
	PostT t;
	t.mo = msj.x; t.so = msj.y; t.sig = sig;
	t.mu = go ? mu : __builtin_nan("");
	a.tab[a.tab_base + i] = t;
}

// the last level's correction, in place on the records (level-0 order after the last move)
template <bool IS_W, int P, bool NEXT>
__global__ __launch_bounds__(256) void k_lord_defer_flush(LevelArgs a, uint32_t n)
{
	__shared__ double2 recs[256 * 4];
	const uint32_t b = blockIdx.x * 256u;
	const uint32_t m = min(256u, n - b);
	double2 *r = reinterpret_cast<double2 *>(a.dst) + (size_t)b * 4;
	stage_in_nt<256, 1>(recs, r, m);
	__syncthreads();
	if (threadIdx.x < m) {
		Rec v;
		lds_get(recs, threadIdx.x, v);
		const uint4 q = pay_at(a, b + threadIdx.x);
		apply_pending<IS_W, P>(v, a.tab[q.z], __uint_as_float(q.w));
		lds_put(recs, threadIdx.x, v);
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += 256) r[t] = recs[lslot(t >> 2, t & 3)];
}

// the entry store's flush: after a sweep every row's record waits in its first slot with the
// correction of its last entry pending (the first slot's payload names that entry: the cycle)
template <bool IS_W, int P>
__global__ __launch_bounds__(256) void k_lord_defer_flush_ent(LevelArgs a, uint32_t n)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	const uint32_t s = a.lfirst[r];
	if (s >= a.ent_nnz) return;   // a row without entries: never swept
	double2 *p = reinterpret_cast<double2 *>(a.dst + s);
	Rec v;
#pragma unroll
	for (int c = 0; c < 4; ++c) v[c] = p[c];
	const uint4 q = pay_at(a, s);
	apply_pending<IS_W, P>(v, a.tab[q.z], __uint_as_float(q.w));
#pragma unroll
	for (int c = 0; c < 4; ++c) p[c] = v[c];
}

// build: prev_i[row] / prev_x[row] = (index within its level, x) of the row's entry in a level
__global__ __launch_bounds__(256) void k_lord_prev_map(const uint32_t *feats, const uint64_t *col_ptr, const uint2 *csc,
                                                       uint32_t *prev_i, float *prev_x)
{
	const uint32_t j = feats[blockIdx.x];
	for (uint64_t p = col_ptr[j] + threadIdx.x; p < col_ptr[j + 1]; p += 256) {
		const uint2 ent = csc[p];
		prev_i[ent.x & ROW_MASK] = blockIdx.x;
		prev_x[ent.x & ROW_MASK] = __uint_as_float(ent.y);
	}
}

// lpidx / lpx of a level's entries (global positions lcp[i] + k) from the previous level's map
__global__ __launch_bounds__(256) void k_lord_prev_fill(const uint32_t *feats, const uint64_t *lcp,
                                                        const uint64_t *col_ptr, const uint2 *csc, const uint32_t *prev_i,
                                                        const float *prev_x, uint32_t *lpidx, float *lpx)
{
	const uint32_t j = feats[blockIdx.x];
	const uint64_t cb = col_ptr[j], g0 = lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(col_ptr[j + 1] - cb);
	for (uint32_t k = threadIdx.x; k < n; k += 256) {
		const uint32_t r = csc[cb + k].x & ROW_MASK;
		lpidx[g0 + k] = prev_i[r];
		lpx[g0 + k] = prev_x[r];
	}
}


template <bool IS_W, int P, bool NEXT, int PK, bool ENT>
void launch_defer_shape(const LevelArgs &a, hipStream_t s)
{
	if (a.lpay2) {   // every x 1: 8-B payloads
		dispatch_shape(a.avg_len, [&](auto B, auto R) {
			k_lord_defer<B(), R(), IS_W, P, NEXT, PK, true, ENT><<<a.nfeat, B(), 0, s>>>(a);
		});
		return;
	}
	dispatch_shape(a.avg_len, [&](auto B, auto R) {
		k_lord_defer<B(), R(), IS_W, P, NEXT, PK, false, ENT><<<a.nfeat, B(), 0, s>>>(a);
	});
}

template <bool IS_W, int P, bool NEXT, int PK>
void launch_defer_pk(const LevelArgs &a, hipStream_t s)
{
	if (a.ent) launch_defer_shape<IS_W, P, NEXT, PK, true>(a, s);
	else launch_defer_shape<IS_W, P, NEXT, PK, false>(a, s);
}

template <bool IS_W, int P, bool NEXT>
void launch_defer(const LevelArgs &a, hipStream_t s)
{
	if constexpr (!IS_W) {
		if (a.pend_kind == 1) return launch_defer_pk<IS_W, P, NEXT, 1>(a, s);
		if (a.pend_kind == 2) return launch_defer_pk<IS_W, P, NEXT, 2>(a, s);
	}
	launch_defer_pk<IS_W, P, NEXT, 0>(a, s);
}

template <bool IS_W, int P, bool NEXT>
void launch_flush(const LevelArgs &a, uint32_t n, hipStream_t s)
{
	if (a.ent) k_lord_defer_flush_ent<IS_W, P><<<(n + 255) / 256, 256, 0, s>>>(a, n);
	else k_lord_defer_flush<IS_W, P, NEXT><<<(n + 255) / 256, 256, 0, s>>>(a, n);
}

// ---- MCMC / ALS deferred split (row shards) ------------------------------------------------
// As k_lord_defer for VB: level l's kernel applies level l-1's correction (fm_learn_mcmc.h
// draw_v :826-834 / draw_w :712-717) from the table the previous post kernel wrote after its
// all-reduce, adds level l's term of the next q-cache, reduces level l's statistics from the
// corrected records and moves them; k_mc_lord_defer_post draws the level's parameters from the
// all-reduced statistics (mc_draw, the same random input per attribute as the fused kernel).
// The same arithmetic per row as the fused kernel: bit-identical results.
template <bool IS_W, int P>
DEVI void mc_apply_pending(Rec &r, const PostT &t, float x)
{
	if (__builtin_isnan(t.mu)) return;   // the draw was refused: no correction
	McOp<IS_W, P, false> op;
	op.vo = t.mo; op.v = t.mu; op.vn = 0.0; op.go = true;
	op.apply(r, x, false);
}

template <bool IS_W, int P>
DEVI void mc_add_next_q(Rec &r, float x, bool first, double vn)
{
	const double aq = vn * x;
	double &q = IS_W ? Q<0>(r) : Q<1 - P>(r);
	q = first ? 0.0 + aq : q + aq;
}

template <int BLOCK, int R, bool IS_W, int P, bool NEXT, bool PAY8>
__global__ __launch_bounds__(BLOCK) void k_mc_lord_defer(McArgs a)
{
	constexpr uint32_t CAP = BLOCK * R;
	__shared__ double2 recs[CAP * 4];
	__shared__ uint32_t dsts[CAP];
	__shared__ double lds[2 * (BLOCK / 64)];
	const uint32_t j = level_feat(a, blockIdx.x);
	const uint64_t sb = a.lcp[blockIdx.x];
	const uint32_t n = (uint32_t)(a.lcp[blockIdx.x + 1] - sb);
	const double2 *s = reinterpret_cast<const double2 *>(a.src + (sb - a.lbase));
	double2 *d = reinterpret_cast<double2 *>(a.dst);
	McOp<IS_W, P, false> op;
	op.vo = a.par[(size_t)j * a.stride].x;
	const double vn = NEXT ? a.par_next[(size_t)j * a.next_stride].x : 0.0;
	const int pk = IS_W ? 0 : a.pk;
	const double vp = pk ? a.par_prev[(size_t)j * a.next_stride].x : 0.0;
	const bool first = a.first_level != 0;
	const bool pending = (a.pending & 1) != 0;
	double sm = 0.0, ss = 0.0;
	for (uint32_t base = 0; base < n; base += CAP) {
		const uint32_t m = min(CAP, n - base);
		if (base) __syncthreads();
		// payloads, then the run's records, then the posteriors the payloads point at (the
		// gathers wait for the payloads only), then the LDS writes: three round trips overlap
		PostT t[R];
		uint4 q[R];
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			q[u] = pay_load<PAY8>(a, sb + base + min(i, m - 1));
		}
		double2 sv[4 * R];
		stage_load<BLOCK, R, true>(sv, s + (size_t)base * 4, m);   // records read once: non-temporal
		// unconditional (a.tab always holds a previous level's width; unused unless pending):
		// a branch here lets the compiler sink half of each payload load after the records'
#pragma unroll
		for (int u = 0; u < R; ++u) t[u] = a.tab[q[u].z];
		stage_store<BLOCK, R>(recs, sv);
		__syncthreads();
#pragma unroll
		for (int u = 0; u < R; ++u) {
			const uint32_t i = threadIdx.x + u * BLOCK;
			if (i >= m) continue;
			Rec v;
			lds_get(recs, i, v);
			const float x = __uint_as_float(q[u].x);
			if (pending) mc_apply_pending<IS_W, P>(v, t[u], __uint_as_float(q[u].w));
			if constexpr (NEXT) mc_add_next_q<IS_W, P>(v, x, first, vn);
			if (pk) mc_pred_acc(TQ<0>(v), TZ<0>(v), T(v), x, first, vp, pk);
			if (pending || NEXT || pk) lds_put(recs, i, v);
			op.stat(v, x, sm, ss);
			dsts[i] = q[u].y;
		}
		__syncthreads();
		if (a.pending & 4) {   // non-temporal record stores (as k_lord_defer)
			for (uint32_t tt = threadIdx.x; tt < m * 4; tt += BLOCK) {
				const uint32_t i = tt >> 2, c = tt & 3;
				put_piece<true>(d, (size_t)dsts[i] * 4 + c, recs[lslot(i, c)]);
			}
		} else {
			for (uint32_t tt = threadIdx.x; tt < m * 4; tt += BLOCK) {
				const uint32_t i = tt >> 2, c = tt & 3;
				d[(size_t)dsts[i] * 4 + c] = recs[lslot(i, c)];
			}
		}
	}
	block_sum2<BLOCK>(sm, ss, lds);
	if (threadIdx.x == 0) a.stats[blockIdx.x] = make_double2(sm, ss);
}

template <bool IS_W>
__global__ __launch_bounds__(256) void k_mc_lord_defer_post(McArgs a)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= a.nfeat) return;
	const uint32_t j = level_feat(a, i);
	const double vo = a.par[(size_t)j * a.stride].x;
	const double2 st = a.stats[i];
	const uint32_t g = mc_group(a, j);
	double v = vo;
	const bool go = mc_draw(st.x, st.y, vo, mc_lambda(a, g), mc_mu(a, g), a.alpha,
	                        mc_z(a, j), a.z != nullptr, a.sample, !IS_W, v, a.counters, true);
	a.par[(size_t)j * a.stride].x = v;
	PostT t;
	t.mo = vo; t.so = 0.0; t.sig = 0.0;
	t.mu = go ? v : __builtin_nan("");
	a.tab[i] = t;
}

template <bool IS_W, int P>
__global__ __launch_bounds__(256) void k_mc_lord_defer_flush(McArgs a, uint32_t n)
{
	__shared__ double2 recs[256 * 4];
	const uint32_t b = blockIdx.x * 256u;
	const uint32_t m = min(256u, n - b);
	double2 *r = reinterpret_cast<double2 *>(a.dst) + (size_t)b * 4;
	stage_in_nt<256, 1>(recs, r, m);
	__syncthreads();
	if (threadIdx.x < m) {
		Rec v;
		lds_get(recs, threadIdx.x, v);
		const uint4 q = pay_at(a, b + threadIdx.x);
		mc_apply_pending<IS_W, P>(v, a.tab[q.z], __uint_as_float(q.w));
		lds_put(recs, threadIdx.x, v);
	}
	__syncthreads();
	for (uint32_t t = threadIdx.x; t < m * 4; t += 256) r[t] = recs[lslot(t >> 2, t & 3)];
}

template <bool IS_W, int P, bool NEXT>
void launch_mc_defer(const McArgs &a, hipStream_t s)
{
	if (a.lpay2) {   // every x 1: 8-B payloads
		dispatch_shape(a.avg_len, [&](auto B, auto R) {
			k_mc_lord_defer<B(), R(), IS_W, P, NEXT, true><<<a.nfeat, B(), 0, s>>>(a);
		});
		return;
	}
	dispatch_shape(a.avg_len, [&](auto B, auto R) {
		k_mc_lord_defer<B(), R(), IS_W, P, NEXT, false><<<a.nfeat, B(), 0, s>>>(a);
	});
}

template <int BLOCK, int R, int MODE, bool ENT>
void launch_mc_lord_ent(const McArgs &a, int is_w, hipStream_t s)
{
	const bool nx = a.par_next != nullptr;
	if (is_w) {
		if (nx) k_mc_level_lord<BLOCK, R, true, 0, true, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
		else k_mc_level_lord<BLOCK, R, true, 0, false, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
	} else if (a.slot == 0) {
		if (nx) k_mc_level_lord<BLOCK, R, false, 0, true, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
		else k_mc_level_lord<BLOCK, R, false, 0, false, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
	} else {
		if (nx) k_mc_level_lord<BLOCK, R, false, 1, true, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
		else k_mc_level_lord<BLOCK, R, false, 1, false, MODE, ENT><<<a.nfeat, BLOCK, 0, s>>>(a);
	}
}

// every mode on both stores: the entry store's next slots carry the row's-first-entry flag in
// bit 31 (ENT_FIRST), which only the ENT kernels strip before the move
template <int BLOCK, int R, int MODE>
void launch_mc_lord(const McArgs &a, int is_w, hipStream_t s)
{
	if (a.ent) return launch_mc_lord_ent<BLOCK, R, MODE, true>(a, is_w, s);
	launch_mc_lord_ent<BLOCK, R, MODE, false>(a, is_w, s);
}

template <int MODE>
void launch_mc_lord_shape(const McArgs &a, int is_w, hipStream_t s)
{
	// the column-gather MCMC kernel's BLOCK (vbfm_mcmc.hip launch_level), records per thread
	// as the VB level kernel
	dispatch_shape(a.avg_len, [&](auto B, auto R) { launch_mc_lord<B(), R(), MODE>(a, is_w, s); });
}

}  // namespace

namespace vbk {

hipError_t mc_lord_level(const McArgs &a, int mode, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (mode == 0) launch_mc_lord_shape<0>(a, is_w, s);
	else if (mode == 1) launch_mc_lord_shape<1>(a, is_w, s);
	else launch_mc_lord_shape<2>(a, is_w, s);
	return hipGetLastError();
}

hipError_t mc_lord_defer_level(const McArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const bool nx = a.par_next != nullptr;
	if (is_w) nx ? launch_mc_defer<true, 0, true>(a, s) : launch_mc_defer<true, 0, false>(a, s);
	else if (a.slot == 0) nx ? launch_mc_defer<false, 0, true>(a, s) : launch_mc_defer<false, 0, false>(a, s);
	else nx ? launch_mc_defer<false, 1, true>(a, s) : launch_mc_defer<false, 1, false>(a, s);
	return hipGetLastError();
}

hipError_t mc_lord_defer_post(const McArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const unsigned g = (a.nfeat + 255) / 256;
	if (is_w) k_mc_lord_defer_post<true><<<g, 256, 0, s>>>(a);
	else k_mc_lord_defer_post<false><<<g, 256, 0, s>>>(a);
	return hipGetLastError();
}

hipError_t mc_lord_defer_flush(const McArgs &a, int is_w, uint32_t n, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const unsigned g = (n + 255) / 256;
	if (is_w) k_mc_lord_defer_flush<true, 0><<<g, 256, 0, s>>>(a, n);
	else if (a.slot == 0) k_mc_lord_defer_flush<false, 0><<<g, 256, 0, s>>>(a, n);
	else k_mc_lord_defer_flush<false, 1><<<g, 256, 0, s>>>(a, n);
	return hipGetLastError();
}

hipError_t lord_level(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (is_w) nx ? launch_lord<true, 0, true>(a, s) : launch_lord<true, 0, false>(a, s);
	else if (a.slot == 0) nx ? launch_lord<false, 0, true>(a, s) : launch_lord<false, 0, false>(a, s);
	else nx ? launch_lord<false, 1, true>(a, s) : launch_lord<false, 1, false>(a, s);
	return hipGetLastError();
}

hipError_t lord_long(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nsegs == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (is_w) k_lord_long_stats<true, 0><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	else if (a.slot == 0) k_lord_long_stats<false, 0><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	else k_lord_long_stats<false, 1><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	if (is_w) {
		if (nx) k_lord_long_move<true, 0, true><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
		else k_lord_long_move<true, 0, false><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	} else if (a.slot == 0) {
		if (nx) k_lord_long_move<false, 0, true><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
		else k_lord_long_move<false, 0, false><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	} else {
		if (nx) k_lord_long_move<false, 1, true><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
		else k_lord_long_move<false, 1, false><<<a.nsegs, LONG_BLOCK, 0, s>>>(a);
	}
	return hipGetLastError();
}

hipError_t lord_level_stats(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (is_w) launch_lord_stats<true, 0>(a, s);
	else if (a.slot == 0) launch_lord_stats<false, 0>(a, s);
	else launch_lord_stats<false, 1>(a, s);
	return hipGetLastError();
}

hipError_t lord_level_move(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (is_w) launch_lord_move<true, 0>(a, s);
	else if (a.slot == 0) launch_lord_move<false, 0>(a, s);
	else launch_lord_move<false, 1>(a, s);
	return hipGetLastError();
}

hipError_t lord_defer_level(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (is_w) nx ? launch_defer<true, 0, true>(a, s) : launch_defer<true, 0, false>(a, s);
	else if (a.slot == 0) nx ? launch_defer<false, 0, true>(a, s) : launch_defer<false, 0, false>(a, s);
	else nx ? launch_defer<false, 1, true>(a, s) : launch_defer<false, 1, false>(a, s);
	return hipGetLastError();
}

hipError_t lord_defer_post(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const unsigned g = (a.nfeat + 255) / 256;
	if (is_w) { if (a.ms_next) k_lord_defer_post<true, true><<<g, 256, 0, s>>>(a); else k_lord_defer_post<true, false><<<g, 256, 0, s>>>(a); }
	else { if (a.ms_next) k_lord_defer_post<false, true><<<g, 256, 0, s>>>(a); else k_lord_defer_post<false, false><<<g, 256, 0, s>>>(a); }
	return hipGetLastError();
}

hipError_t lord_defer_flush(const LevelArgs &a, int is_w, uint32_t n, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	const bool nx = a.ms_next != nullptr;
	if (is_w) nx ? launch_flush<true, 0, true>(a, n, s) : launch_flush<true, 0, false>(a, n, s);
	else if (a.slot == 0) nx ? launch_flush<false, 0, true>(a, n, s) : launch_flush<false, 0, false>(a, n, s);
	else nx ? launch_flush<false, 1, true>(a, n, s) : launch_flush<false, 1, false>(a, n, s);
	return hipGetLastError();
}

hipError_t lord_prev_map(const uint32_t *feats, uint32_t nfeat, const uint64_t *col_ptr, const uint2 *csc,
                         const float *, uint32_t *prev_i, float *prev_x, hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_lord_prev_map<<<nfeat, 256, 0, s>>>(feats, col_ptr, csc, prev_i, prev_x);
	return hipGetLastError();
}

hipError_t lord_prev_fill(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, const uint64_t *col_ptr,
                          const uint2 *csc, const uint32_t *prev_i, const float *prev_x, uint32_t *lpidx, float *lpx,
                          hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_lord_prev_fill<<<nfeat, 256, 0, s>>>(feats, lcp, col_ptr, csc, prev_i, prev_x, lpidx, lpx);
	return hipGetLastError();
}

hipError_t lord_pos(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, uint64_t lbase, const uint64_t *col_ptr,
                    const uint2 *csc, uint32_t *pos, hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_lord_pos<<<nfeat, 256, 0, s>>>(feats, lcp, lbase, col_ptr, csc, pos);
	return hipGetLastError();
}

hipError_t lord_fill(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, uint64_t lbase, const uint64_t *col_ptr,
                     const uint2 *csc, const uint32_t *pos_next, float *lx, uint32_t *lnext, uint32_t *row0,
                     hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_lord_fill<<<nfeat, 256, 0, s>>>(feats, lcp, lbase, col_ptr, csc, pos_next, lx, lnext, row0);
	return hipGetLastError();
}

hipError_t count_x_ne1(const uint2 *csc, uint64_t nnz, uint32_t *cnt, hipStream_t s)
{
	const hipError_t e = hipMemsetAsync(cnt, 0, 4, s);
	if (e != hipSuccess || nnz == 0) return e;
	const uint64_t g = std::min<uint64_t>((nnz + 255) / 256, 8192);
	k_count_x_ne1<<<(unsigned)g, 256, 0, s>>>(csc, nnz, cnt);
	return hipGetLastError();
}

hipError_t lord_pack2(const uint32_t *lnext, const uint32_t *lpidx, uint2 *lpay2, uint64_t nnz, hipStream_t s)
{
	if (nnz == 0) return hipSuccess;
	k_lord_pack2<<<(unsigned)((nnz + 255) / 256), 256, 0, s>>>(lnext, lpidx, lpay2, nnz);
	return hipGetLastError();
}

hipError_t lord_pack(const float *lx, const uint32_t *lnext, const uint32_t *lpidx, const float *lpx, uint4 *lpay,
                     uint64_t nnz, hipStream_t s)
{
	if (nnz == 0) return hipSuccess;
	k_lord_pack<<<(unsigned)((nnz + 255) / 256), 256, 0, s>>>(lx, lnext, lpidx, lpx, lpay, nnz);
	return hipGetLastError();
}

hipError_t rows_gather(RowRec *dst, const RowRec *src, const uint32_t *idx, uint32_t n, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_rows_gather<<<(unsigned)(((uint64_t)n * 4 + 255) / 256), 256, 0, s>>>(dst, src, idx, n);
	return hipGetLastError();
}

hipError_t estore_build(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, const uint2 *csc,
                        const uint32_t *lvpos, const uint64_t *lcp, uint32_t n, uint64_t nnz, uint32_t *lnext,
                        float *lx, uint32_t *lfirst, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_estore_build<<<(n + 255) / 256, 256, 0, s>>>(row_ptr, csr, col_ptr, csc, lvpos, lcp, n, nnz, lnext, lx, lfirst);
	return hipGetLastError();
}

hipError_t estore_prev(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, const uint2 *csc,
                       const uint32_t *lvpos, const uint64_t *lcp, uint32_t n, uint32_t *lpidx, float *lpx, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_estore_prev<<<(n + 255) / 256, 256, 0, s>>>(row_ptr, csr, col_ptr, csc, lvpos, lcp, n, lpidx, lpx);
	return hipGetLastError();
}

hipError_t place_move(const RowRec *src, RowRec *dst, const uint64_t *lcp, const uint32_t *lnext, uint32_t nfeat,
                      hipStream_t s)
{
	if (nfeat == 0) return hipSuccess;
	k_place_move<<<nfeat, 256, 0, s>>>(src, dst, lcp, lnext);
	return hipGetLastError();
}

hipError_t rows_scatter(RowRec *dst, const RowRec *src, const uint32_t *idx, uint32_t n, hipStream_t s)
{
	if (n == 0) return hipSuccess;
	k_rows_scatter<<<(unsigned)(((uint64_t)n * 4 + 255) / 256), 256, 0, s>>>(dst, src, idx, n);
	return hipGetLastError();
}

}  // namespace vbk
