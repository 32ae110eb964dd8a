// vbfm_online.hip -- the online VB learner (OVBFM, `-method vb_online`): fm_learn_vb_online
// (src/libfm/src/fm_learn_vb_online.h) driven by fm_learn_vb_online_simultaneous::_learn
// (src/libfm/src/fm_learn_vb_online_simultaneous.h:20-290), citations relative to
// /root/reference.
//
// The reference writes every epoch's mini-batches to text files and re-parses them; here the
// train set stays resident in HBM and each epoch regroups it on the device:
//   1. the epoch's permutation: std::random_shuffle on the reference's rand() stream (host,
//      the swaps are sequential), uploaded once;
//   2. batch of row r = ceil(shuffle[r] / size) (:87-95), rows grouped by batch in file order
//      (stable radix sort) and numbered within their batch;
//   3. the CSC entries re-keyed to (batch, local row) and stably sorted by batch: inside a batch
//      the entries stay column-major with ascending rows -- the transposed copy
//      Data::create_data_t(num_attribute) builds for the batch file (Data.h:511-560);
//      per-(batch, column) counts give every batch's col_ptr as a slice of one prefix sum;
//   4. per batch: its rows' CSR gathered for the predictions, then fm_learn_vb_online::
//      update_all on the batch -- the VB learner's level sweeps with the natural-gradient
//      posterior (k_ov_*_level below), update_w0 and the hyper-parameter steps on the host.
// Parallel reductions sum a column's per-entry natural-parameter terms in a tree: equal to the
// reference's sequential sums up to summation order (every term rounded as the reference
// rounds it). One GPU: the learner refuses a communicator or feature shards.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "vbfm_ctx.h"
#include "vbfm_math.h"
#include "vbfm_rng.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace vbi;

namespace {

// fm_learn_vb_online::init (fm_learn_vb_online.h:686-700): fixed learning-rate schedule
constexpr double LAMDA = 0.5;
constexpr uint32_t T0 = 1;   // t0_w0 = t0_wj = t0_vj

// ---- mini-batch grouping ------------------------------------------------------------------
// batch of every row: ceil((double)shuffle[r] / size_except_last) - 1 (:91-94)
__global__ void k_ov_batch(const uint32_t *sh, uint32_t n, uint32_t size, uint32_t *bat, uint32_t *iota)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r >= n) return;
	bat[r] = (uint32_t)ceil((double)sh[r] / size) - 1u;
	iota[r] = r;
}

// position of each row inside its batch
__global__ void k_ov_local(const uint32_t *rows_sorted, const uint32_t *bat, const uint64_t *rstart, uint32_t n,
                           uint32_t *loc)
{
	const uint32_t p = blockIdx.x * 256u + threadIdx.x;
	if (p >= n) return;
	const uint32_t r = rows_sorted[p];
	loc[r] = p - (uint32_t)rstart[bat[r]];
}

// every CSC entry keyed by its row's batch, its row renumbered within the batch (the
// first-entry flag kept: a row's smallest feature is the same in the batch), and the
// (batch, level position) histogram. The columns are taken in level order (column i of the
// level-ordered feature list at lvcp[i]), so that after the stable sort by batch a batch's
// columns are in level order too and its col_ptr is indexed by level position.
__global__ __launch_bounds__(256) void k_ov_entries(const uint64_t *col_ptr, const uint2 *csc, const uint32_t *feats,
                                                    const uint64_t *lvcp, const uint32_t *bat, const uint32_t *loc,
                                                    uint32_t nf, uint16_t *key, uint2 *val, uint32_t *cnt)
{
	const uint32_t i = blockIdx.x, j = feats[i];
	const uint64_t b = col_ptr[j], e = col_ptr[j + 1], o = lvcp[i] - b;
	for (uint64_t p = b + threadIdx.x; p < e; p += 256) {
		const uint2 ent = csc[p];
		const uint32_t r = ent.x & ROW_MASK;
		const uint32_t bb = bat[r];
		key[o + p] = (uint16_t)bb;
		val[o + p] = make_uint2(loc[r] | (ent.x & ROW_FIRST), ent.y);
		atomicAdd(&cnt[(size_t)bb * nf + i], 1u);
	}
}

// the batch's rows (global ids, ascending) -> lengths of their CSR rows
__global__ void k_ov_rowlen(const uint32_t *rows, uint32_t n, const uint64_t *row_ptr, uint64_t *len)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) len[i] = row_ptr[rows[i] + 1] - row_ptr[rows[i]];
}

// one wave per batch row: copy its feature-sorted entries and its target
__global__ __launch_bounds__(256) void k_ov_gather(const uint32_t *rows, uint32_t n, const uint64_t *row_ptr,
                                                   const uint2 *csr, const float *target, const uint64_t *rp_b,
                                                   uint2 *csr_b, float *t_b)
{
	const uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6);
	const uint32_t lane = threadIdx.x & 63;
	if (i >= n) return;
	const uint32_t r = rows[i];
	const uint64_t b = row_ptr[r], len = row_ptr[r + 1] - b, o = rp_b[i];
	for (uint64_t p = lane; p < len; p += 64) csr_b[o + p] = csr[b + p];
	if (lane == 0) t_b[i] = target[r];
}

// first entry of every level of every batch: lvl[b * (L+1) + l] = gptr[b * nf + level_ptr[l]]
__global__ void k_ov_level_bases(const uint64_t *gptr, const uint32_t *level_ptr, uint32_t L, uint32_t nf, uint32_t nb,
                                 uint64_t *lvl)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i >= nb * (L + 1)) return;
	const uint32_t b = i / (L + 1), l = i % (L + 1);
	lvl[i] = gptr[(size_t)b * nf + level_ptr[l]];
}

// ---- update_w0 (fm_learn_vb_online.h:471-497): sum of the per-row natural-mean terms
// (1 - new_w0) * mu_old + new_w0 * _size * alpha * (e + mu_0_dash)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_ov_w0_sum(const RowRec *rows, uint32_t n, double keep, double scale,
                                                     double mu0, double *out)
{
	__shared__ double lds[BLOCK / 64];
	double s = 0.0;
	for (uint32_t r = blockIdx.x * BLOCK + threadIdx.x; r < n; r += gridDim.x * BLOCK) {
		const double w0_temp = rows[r].e + mu0;
		s += keep + scale * w0_temp;
	}
	s = block_sum1<BLOCK>(s, lds);
	if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// fm_learn_vb_online::init (:706-758): col_count from the train set, natural parameters
// natural_mu = mu / 0.02, natural_sigma = 1 / sigma
__global__ void k_ov_ccount(const uint64_t *col_ptr, uint32_t nf, uint32_t D, uint32_t *cc)
{
	const uint32_t j = blockIdx.x * 256u + threadIdx.x;
	if (j < D) cc[j] = j < nf ? (uint32_t)(col_ptr[j + 1] - col_ptr[j]) : 0u;
}

__global__ void k_ov_nat_init(const double2 *ms, size_t n, double2 *nat)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n) nat[i] = make_double2(ms[i].x / 0.02, 1 / ms[i].y);
}

// the same for v: ms_v feature-major [j][f] -> nat_v factor-major [f][j]
__global__ void k_ov_nat_init_v(const double2 *ms, uint32_t k, uint32_t D, double2 *nat)
{
	const size_t i = (size_t)blockIdx.x * 256u + threadIdx.x;   // index in nat: f * D + j
	if (i >= (size_t)k * D) return;
	const size_t f = i / D, j = i % D;
	const double2 m = ms[j * k + f];
	nat[i] = make_double2(m.x / 0.02, 1 / m.y);
}

__global__ void k_ov_fill(double *p, uint32_t n, double v)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < n) p[i] = v;
}

// new_vj(i) = pow(t0_vj + t_vj(i), -lamda) for every attribute (:401-403)
__global__ void k_ov_steps(const uint32_t *t, double *rho, uint32_t D)
{
	const uint32_t i = blockIdx.x * 256u + threadIdx.x;
	if (i < D) rho[i] = pow((double)(T0 + t[i]), -LAMDA);
}

// ---- the level sweeps ------------------------------------------------------------------------
// A mini-batch holds ~1/num_batch of every column, so its columns are short: G threads serve one
// column (G = 4 .. 64 lanes of a wave, several columns per 256-thread workgroup, sums by xor
// butterflies inside the lane group; or G = 256, one column per workgroup).
template <int G>
DEVI void group_sum2(double &a, double &b, double *lds)
{
	if constexpr (G <= 64) {
#pragma unroll
		for (int o = G / 2; o > 0; o >>= 1) {
			a += __shfl_xor(a, o, 64);
			b += __shfl_xor(b, o, 64);
		}
	} else {
		block_sum2<G>(a, b, lds);
	}
}

// update_v (fm_learn_vb_online.h:558-627) for the batch's entries of one column per lane group.
// The per-entry statistics are VB's (v_stat); each becomes the natural-parameter terms
//   (1 - new_vj) * sigma_old + new_vj * (sigma_v_g + alpha * col_count * v_sigma_sqr)
//   (1 - new_vj) * mu_old    + new_vj * col_count * alpha * v_mean
// whose mean over the entries is the new natural parameter; the correction is VB's (v_apply).
template <int G, int P, bool NEXT>
__global__ __launch_bounds__(256) void k_ov_v_level(LevelArgs a)
{
	__shared__ double lds[2 * (256 / 64)];
	const uint32_t col_i = G <= 64 ? blockIdx.x * (256 / G) + threadIdx.x / G : blockIdx.x;
	const uint32_t lane = G <= 64 ? threadIdx.x % G : threadIdx.x;
	if (col_i >= a.nfeat) return;   // whole lane groups (G <= 64) or the whole workgroup
	// the batch's col_ptr is indexed by level position (ov_regroup): coalesced, and the
	// column's entries can be fetched in parallel with its parameters (the feature id is
	// loaded with the bounds, before the branch on the column length)
	const uint32_t j = level_feat(a, col_i);
	const uint64_t cb = a.col_ptr[col_i];
	const uint32_t n = (uint32_t)(a.col_ptr[col_i + 1] - cb);
	if (n == 0) return;   // columns without entries in the batch are skipped (:389-394)
	const uint2 *col = a.csc + cb;
	// the lane's first two entries stay in registers from the statistics to the correction
	// (named, not an array: an array of records gets demoted to LDS / scratch)
	const bool h0 = lane < n, h1 = lane + G < n;
	uint2 ent0 = make_uint2(0u, 0u), ent1 = make_uint2(0u, 0u);
	Rec v0, v1;
	if (h0) {
		ent0 = col[lane];
		load_rec(a.rows, ent0.x & ROW_MASK, v0);
	}
	if (h1) {
		ent1 = col[lane + G];
		load_rec(a.rows, ent1.x & ROW_MASK, v1);
	}
	const size_t pi = (size_t)j * a.ms_stride;
	const double2 msj = a.ms[pi], natj = a.nat[(size_t)j * a.nat_stride];
	const double mo = msj.x, so = msj.y;
	const double rho = a.rho[j];
	const uint32_t cc = a.ccount[j];
	const double sv_g = a.hyp[(size_t)a.attr_group[j] * a.hyp_stride];
	const double keep_m = (1 - rho) * natj.x, keep_s = (1 - rho) * natj.y;
	const double acc = a.alpha * cc;          // alpha * col_count(col)
	const double rca = rho * cc * a.alpha;    // new_vj(col) * col_count(col) * alpha
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];
	double eta1 = 0.0, eta2 = 0.0;
	auto stat = [&](uint2 e, Rec &r) {
		double vm = 0.0, vs = 0.0;
		v_stat(ent_x(e), E(r), Q<P>(r), TQ<P>(r), mo, so, vm, vs);
		eta2 += keep_s + rho * (sv_g + acc * vs);
		eta1 += keep_m + rca * vm;
	};
	if (h0) stat(ent0, v0);
	if (h1) stat(ent1, v1);
	for (uint32_t i = lane + 2 * G; i < n; i += G) {
		const uint2 e = col[i];
		Rec r;
		load_rec(a.rows, e.x & ROW_MASK, r);
		stat(e, r);
	}
	group_sum2<G>(eta1, eta2, lds);
	const double nmu = eta1 / n, nsig = eta2 / n;
	double mu = nmu / nsig, sig = 1 / nsig;
	bool go = true;
	const bool leader = lane == 0;
	if (dnan(sig) || dinf(sig)) {
		sig = so;
		if (leader) atomicAdd(&a.counters[CNT_NAN_SIGMA_V], 1u);
	}
	if (dnan(mu)) {
		if (leader) atomicAdd(&a.counters[CNT_NAN_MU_V], 1u);
		mu = mo;
		go = false;
	} else if (dinf(mu)) {
		if (leader) atomicAdd(&a.counters[CNT_INF_MU_V], 1u);
		mu = mo;
		go = false;
	}
	if (leader) {
		a.nat[(size_t)j * a.nat_stride] = make_double2(nmu, nsig);
		a.ms[pi] = make_double2(mu, sig);
		if (a.tcount) a.tcount[j] += n;   // t_vj(i) += size at factor 0 (:396-399)
	}
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		// a row listed twice: the reference corrects entry after entry
		if constexpr (G > 64) __syncthreads();
		if (leader)
			for (uint32_t i = 0; i < n; ++i) {
				const uint2 ent = col[i];
				Rec v;
				load_rec(a.rows, ent.x & ROW_MASK, v);
				v_apply<P, NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
				store_rec(a.rows, ent.x & ROW_MASK, v);
			}
		return;
	}
	if (h0) {
		v_apply<P, NEXT>(v0, ent_x(ent0), (ent0.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent0.x & ROW_MASK, v0);
	}
	if (h1) {
		v_apply<P, NEXT>(v1, ent_x(ent1), (ent1.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent1.x & ROW_MASK, v1);
	}
	for (uint32_t i = lane + 2 * G; i < n; i += G) {
		const uint2 e = col[i];
		Rec r;
		load_rec(a.rows, e.x & ROW_MASK, r);
		v_apply<P, NEXT>(r, ent_x(e), (e.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, e.x & ROW_MASK, r);
	}
}

// update_w (fm_learn_vb_online.h:499-556): as above with VB's w statistics; t_wj / new_wj are
// advanced by the column itself (:519-520)
template <int G, bool NEXT>
__global__ __launch_bounds__(256) void k_ov_w_level(LevelArgs a)
{
	__shared__ double lds[2 * (256 / 64)];
	const uint32_t col_i = G <= 64 ? blockIdx.x * (256 / G) + threadIdx.x / G : blockIdx.x;
	const uint32_t lane = G <= 64 ? threadIdx.x % G : threadIdx.x;
	if (col_i >= a.nfeat) return;
	const uint64_t cb = a.col_ptr[col_i];
	const uint32_t n = (uint32_t)(a.col_ptr[col_i + 1] - cb);
	if (n == 0) return;   // (:364-368)
	const uint32_t j = level_feat(a, col_i);
	const uint2 *col = a.csc + cb;
	const size_t pi = (size_t)j * a.ms_stride;
	const double2 msj = a.ms[pi], natj = a.nat[(size_t)j * a.nat_stride];
	const double mo = msj.x, so = msj.y;
	const double rho = a.rho[j];
	const uint32_t cc = a.ccount[j];
	const double sw_g = a.hyp[(size_t)a.attr_group[j] * a.hyp_stride];
	const double keep_m = (1 - rho) * natj.x, keep_s = (1 - rho) * natj.y;
	const double acc = a.alpha * cc;
	const double rca = rho * cc * a.alpha;
	double2 nx = make_double2(0.0, 0.0);
	if constexpr (NEXT) nx = a.ms_next[(size_t)j * a.ms_stride_next];
	double eta1 = 0.0, eta2 = 0.0;
	for (uint32_t i = lane; i < n; i += G) {
		const uint2 ent = col[i];
		const float x = ent_x(ent);
		const double w_mean = x * (a.rows[ent.x & ROW_MASK].e + x * mo);
		const double w_sigma_sqr = x * x;   // fp32 product
		eta2 += keep_s + rho * (sw_g + acc * w_sigma_sqr);
		eta1 += keep_m + rca * w_mean;
	}
	group_sum2<G>(eta1, eta2, lds);
	const double nmu = eta1 / n, nsig = eta2 / n;
	double mu = nmu / nsig, sig = 1 / nsig;
	bool go = true;
	const bool leader = lane == 0;
	if (dnan(sig) || dinf(sig)) {
		if (leader) atomicAdd(&a.counters[CNT_NAN_SIGMA_W], 1u);
		sig = so;
	}
	if (dnan(mu)) {
		if (leader) atomicAdd(&a.counters[CNT_NAN_MU_W], 1u);
		mu = mo;
		go = false;
	} else if (dinf(mu)) {
		if (leader) atomicAdd(&a.counters[CNT_INF_MU_W], 1u);
		mu = mo;
		go = false;
	}
	if (leader) {
		a.nat[(size_t)j * a.nat_stride] = make_double2(nmu, nsig);
		a.ms[pi] = make_double2(mu, sig);
		const uint32_t t = a.tcount[j] + n;
		a.tcount[j] = t;
		a.rho[j] = pow((double)(T0 + t), -LAMDA);
	}
	if (!go && !NEXT) return;
	if (a.dup[j]) {
		if constexpr (G > 64) __syncthreads();
		if (leader)
			for (uint32_t i = 0; i < n; ++i) {
				const uint2 ent = col[i];
				Rec v;
				load_rec(a.rows, ent.x & ROW_MASK, v);
				w_apply<NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
				store_rec(a.rows, ent.x & ROW_MASK, v);
			}
		return;
	}
	for (uint32_t i = lane; i < n; i += G) {
		const uint2 ent = col[i];
		Rec v;
		load_rec(a.rows, ent.x & ROW_MASK, v);
		w_apply<NEXT>(v, ent_x(ent), (ent.x & a.first_mask) != 0, go, mo, so, mu, sig, nx);
		store_rec(a.rows, ent.x & ROW_MASK, v);
	}
}

// ---- the per-batch level-ordered store --------------------------------------------------------
// When every level holds each row of the batch exactly once (field-structured data) the
// batch's records are kept in the current level's order: position p of level l is the p-th
// entry of the level's batch columns, which are contiguous in ent_sorted (level order, rows
// ascending in a column). A level then reads each column's records as one run and writes every
// record, corrected, to its row's position in the next level (lnx): one random line per record
// instead of a random read and a random write of the same line (tools/probe_ovlevel.hip: 7.7 vs
// 12.6 us per level at C3's batch shape). Column statistics, posteriors and corrections are the
// column kernels' (same entries, same lanes, same butterfly): bit-identical; only data-set sums
// (w0, alpha, free energy) add the rows in another order.
//
// level of a batch entry (by its index g in ent_sorted) and its position in that level
DEVI uint32_t ov_level_of(const uint64_t *base, uint32_t L, uint64_t g)
{
	uint32_t lo = 0, hi = L;   // base[lo] <= g < base[hi]
	while (hi - lo > 1) {
		const uint32_t mid = (lo + hi) >> 1;
		if (base[mid] <= g) lo = mid;
		else hi = mid;
	}
	return lo;
}

// The padded layout (levels >= 1 of a batch whose every workgroup run fits PAD_CAP records): the
// run of workgroup w (level columns [w cpw, (w+1) cpw), cpw = 256 / G of the level's kernel) starts
// at record w * PAD_CAP of the level's buffer, so a level kernel issues its run's loads at once
// instead of after a load of the run's column bound. Level 0 stays packed (the data-set sums of
// the batch read its records in level-0 order, n of them).
struct OvPad {
	const uint64_t *gp;        // the batch's col_ptr by level position (o.gptr + b * nf)
	const uint32_t *lptr;      // level_ptr [L+1]
	const uint32_t *cpw;       // columns per workgroup of each level
	uint32_t cap;              // PAD_CAP, or 0: every level packed
	const uint64_t *off;       // [L] start of each level's lnx region (packed: base[l] - base[0])
};

// pos[l * n + row] = position of the row in level l; base[L+1] = first entry of every level
// (packed layout: one thread per entry)
__global__ void k_ov_lord_pos(const uint2 *ent, const uint64_t *base, uint32_t L, uint32_t n, uint32_t *pos)
{
	const uint64_t g = base[0] + (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (g >= base[L]) return;
	const uint32_t l = ov_level_of(base, L, g);
	pos[(size_t)l * n + (ent[g].x & ROW_MASK)] = (uint32_t)(g - base[l]);
}

// lnx[g - base[0]] = the entry's row position in the next level (the last level -> level 0)
__global__ void k_ov_lord_next(const uint2 *ent, const uint64_t *base, uint32_t L, uint32_t n, const uint32_t *pos,
                               uint32_t *lnx)
{
	const uint64_t g = base[0] + (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (g >= base[L]) return;
	const uint32_t l = ov_level_of(base, L, g), ln = l + 1 == L ? 0 : l + 1;
	lnx[g - base[0]] = pos[(size_t)ln * n + (ent[g].x & ROW_MASK)];
}

// the padded layout: one workgroup per workgroup run (level l, group w; gbase[l] = the groups of
// the levels before l), its entries [gs, ge) coalesced; level 0 packed (position g - gp[0]),
// levels >= 1 at w * cap + (g - gs). NEXT: lnx[off[l] + position] = the row's position in the next
// level (the last level -> level 0); else pos[l * n + row] = position.
template <bool NEXT>
__global__ __launch_bounds__(256) void k_ov_pad_pos(const uint2 *ent, OvPad pd, const uint32_t *gbase, uint32_t L,
                                                    uint32_t n, uint32_t *pos, uint32_t *lnx)
{
	uint32_t lo = 0, hi = L;   // the level of this group: gbase[lo] <= blockIdx.x < gbase[lo + 1]
	while (hi - lo > 1) {
		const uint32_t mid = (lo + hi) >> 1;
		if (gbase[mid] <= blockIdx.x) lo = mid;
		else hi = mid;
	}
	const uint32_t l = lo, w = blockIdx.x - gbase[l];
	const uint32_t p0 = pd.lptr[l] + w * pd.cpw[l], p1 = min(p0 + pd.cpw[l], pd.lptr[l + 1]);
	const uint64_t gs = pd.gp[p0], ge = pd.gp[p1];
	const uint64_t first = l == 0 ? pd.gp[0] : gs - (uint64_t)w * pd.cap;
	const uint32_t ln = l + 1 == L ? 0 : l + 1;
	for (uint64_t g = gs + threadIdx.x; g < ge; g += 256) {
		const uint32_t row = ent[g].x & ROW_MASK, at = (uint32_t)(g - first);
		if constexpr (NEXT) lnx[pd.off[l] + at] = pos[(size_t)ln * n + row];
		else pos[(size_t)l * n + row] = at;
	}
}

// per batch: does some workgroup run of a level >= 1 exceed PAD_CAP records? (thread per
// (batch, level position): the positions that start a workgroup's columns)
__global__ void k_ov_pad_check(const uint64_t *gptr, const uint32_t *lptr, const uint32_t *cpw, uint32_t L,
                               uint32_t nf, uint32_t nb, uint32_t cap, uint32_t *bad)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= (uint64_t)nb * nf) return;
	const uint32_t b = (uint32_t)(i / nf), p = (uint32_t)(i % nf);
	uint32_t lo = 0, hi = L;   // the level of position p: lptr[lo] <= p < lptr[lo + 1]
	while (hi - lo > 1) {
		const uint32_t mid = (lo + hi) >> 1;
		if (lptr[mid] <= p) lo = mid;
		else hi = mid;
	}
	if (lo == 0 || (p - lptr[lo]) % cpw[lo] != 0) return;
	const uint32_t e = min(p + cpw[lo], lptr[lo + 1]);
	const uint64_t *g = gptr + (size_t)b * nf;
	if (g[e] - g[p] > cap) bad[b] = 1u;
}

// One level of the w (IS_W) or v sweep of a mini-batch on the level-ordered store. A workgroup
// serves 256/G consecutive columns, i.e. one contiguous run of the level's records: the run
// (up to CAP records) and its next-level positions are staged in LDS with coalesced loads, four
// lanes per record; G lanes per column reduce the statistics as k_ov_{w,v}_level do (same
// entries per lane, same butterfly), the corrected records go back to their LDS slots, and the
// run is written out four lanes per record to a.dst[lnext] (every record: the write is the
// move, also when the guards skip the correction). Records past CAP (a run longer than CAP)
// are read and written directly.
constexpr uint32_t OV_CAP = 512;

// Diagnostic build only (tools/ov_stamps.sh, -DVBFM_OV_STAMPS; never in lib/libvbfm.so): every wave
// reads the 100-MHz real-time counter at five points (entry, staged, posterior, corrected, stores
// issued) into registers; at the end thread 0 of every workgroup of one chosen level launch writes
// them to a buffer of its own (only then is the buffer's address needed, so the stamps do not hold
// the entry up on a kernarg load)
#ifdef VBFM_OV_STAMPS
#define OV_STAMP_DECL unsigned long long ov_st_[5] = {0, 0, 0, 0, 0}
#define OV_STAMP(i) (ov_st_[i] = __builtin_amdgcn_s_memrealtime())
#define OV_STAMP_FLUSH                                                                                 \
	do {                                                                                               \
		if (a.stamp && threadIdx.x == 0)                                                               \
			for (int i_ = 0; i_ < 5; ++i_) a.stamp[(size_t)blockIdx.x * 5 + i_] = ov_st_[i_];           \
	} while (0)
#else
#define OV_STAMP_DECL do {} while (0)
#define OV_STAMP(i) do {} while (0)
#define OV_STAMP_FLUSH do {} while (0)
#endif

DEVI uint32_t ov_slot(uint32_t i, uint32_t c) { return i * 4 + (c ^ ((i >> 2) & 3)); }

// The pointers a workgroup's first loads need come as leading scalar arguments: with
// -amdgpu-kernarg-preload-count (Makefile) the dispatcher preloads them into SGPRs, so the run's
// record loads and the columns' parameter loads issue at wave start instead of after a scalar load
// of the (freshly written, cold) kernarg segment; LevelArgs follows by value for the rest.
//
// FAST (v sweeps on the padded layout of field data, ov_lord_fast): only 14 argument dwords are
// preloaded, so the two values those loads still need travel in the unused top 16 bits of the
// 48-bit pointers -- the level's column count (col_ptr: low half, src: high half) and the stride
// of ms (lnext) -- and ms / nat / rho / ccount arrive offset to the level's first feature. Every
// load of the staging phase then issues at wave start: one memory round trip to the barrier
// instead of three (kernarg -> column bounds -> records and parameters).
constexpr uint64_t OV_PTR_MASK = (1ull << 48) - 1;
// (through a global-address-space pointer: the loads stay global_load, not flat)
template <class T> DEVI T *ov_untag(T *p)
{
	typedef __attribute__((address_space(1))) T gT;
	return (T *)reinterpret_cast<gT *>(reinterpret_cast<uintptr_t>(p) & OV_PTR_MASK);
}
template <class T> DEVI uint32_t ov_tag(T *p) { return (uint32_t)(reinterpret_cast<uintptr_t>(p) >> 48); }

template <int G, bool IS_W, int P, bool NEXT, bool PAD, bool FAST>
__global__ __launch_bounds__(256) void k_ov_lord(const uint64_t *__restrict__ col_ptr_t, const RowRec *src_t,
                                                 const uint32_t *lnext_t, double2 *ms, double2 *nat, double *rho_p,
                                                 const uint32_t *ccount, uint32_t nfeat_arg, LevelArgs a)
{
	static_assert(G <= 64, "lane groups inside one wave");
	static_assert(!FAST || (PAD && !IS_W), "the tagged arguments serve the v sweep's padded levels");
	__shared__ double2 stage[OV_CAP * 4];
	__shared__ uint32_t dsts[OV_CAP];
	OV_STAMP_DECL;
	OV_STAMP(0);
	const uint64_t *col_ptr = FAST ? ov_untag(col_ptr_t) : col_ptr_t;
	const RowRec *src = FAST ? ov_untag(src_t) : src_t;
	const uint32_t *lnext = FAST ? ov_untag(lnext_t) : lnext_t;
	const uint32_t nfeat = FAST ? ov_tag(col_ptr_t) | ov_tag(src_t) << 16 : nfeat_arg;
	const uint32_t ms_stride = FAST ? ov_tag(lnext_t) : a.ms_stride;
	const uint32_t nat_stride = FAST ? 1u : a.nat_stride;   // FAST: factor-major nat (ov_lord_fast checks)
	// the run's pieces into registers first, only as many rounds as the run needs (uniform
	// bound), the per-column loads below overlap them, the LDS writes come last (a load/write
	// loop waits on every read before issuing the next)
	constexpr int KS = OV_CAP * 4 / 256, KD = OV_CAP / 256;
	// the slot's first KP rounds (256 records: the run is 256 +- 16 at C3's batch shape) and every
	// next position are loaded at once (PAD: before anything else); the rest only if the run is
	// that long, once the column bounds are in -- inside the staging's bandwidth-bound wait, so
	// the half of the workgroups that need a 5th round lose nothing by it, and every workgroup
	// reads 64 fewer records (C3 epoch -0.7 % against KP = 5; 3: no gain; 4 plus half a round at
	// once for 128 lanes: +1.7 %, profiles/r05_online/kp_ab/)
	constexpr int KP = 4, KDP = 1;
	double2 sv[KS];
	uint32_t dv[KD];
	if constexpr (PAD) {
		const double2 *s2 = reinterpret_cast<const double2 *>(src + blockIdx.x * OV_CAP);
		const uint32_t *nx2 = lnext + blockIdx.x * OV_CAP;
#pragma unroll
		for (int k = 0; k < KS; ++k) {
			sv[k] = make_double2(0.0, 0.0);
			if (k < KP) sv[k] = s2[threadIdx.x + k * 256];
		}
#pragma unroll
		// the first 256 next positions at once, the rest with the records' later rounds (C3 epoch
		// -0.7 % against both at once, profiles/r05_online/kp_ab/)
		for (int k = 0; k < KD; ++k) {
			dv[k] = 0;
			if (k < KDP) dv[k] = nx2[threadIdx.x + k * 256];
		}
	}
	const uint32_t c0 = blockIdx.x * (256 / G);
	const uint32_t c1 = min(c0 + 256 / G, nfeat);
	const uint64_t wb = col_ptr[c0], we = col_ptr[c1];
	// the column's id and bounds (a dead lane of the level's last workgroup loads its first
	// column's: no branch around the loads)
	const uint32_t col_i = c0 + threadIdx.x / G;
	const uint32_t lane = threadIdx.x % G;
	const bool live = col_i < nfeat;
	const uint32_t ci = live ? col_i : c0;
	const uint32_t j = FAST ? a.feat_base + ci : level_feat(a, ci);   // the feature id
	const uint32_t pj = FAST ? ci : j;                                   // its index into ms / nat / rho / ccount
	const uint64_t cb = col_ptr[ci];
	const uint64_t ce = col_ptr[ci + 1];
	double2 msj, natj, nx = make_double2(0.0, 0.0);
	double rho;
	uint32_t cc;
	const size_t pi = (size_t)pj * ms_stride;
	// every per-column load issued at once: on field data the feature id is arithmetic
	// (feat_contig), so these wait for nothing -- not for the column bounds (a column empty in
	// this batch loads its parameters for nothing)
	msj = ms[pi];
	natj = nat[(size_t)pj * nat_stride];
	rho = rho_p[pj];
	cc = ccount[pj];
	if constexpr (NEXT) nx = FAST ? ms[pi + 1] : a.ms_next[(size_t)j * a.ms_stride_next];
	if constexpr (FAST) {
		// the LevelArgs fields the rest of the workgroup reads, fetched here in one batch while the
		// loads above are in flight (left to itself the compiler fetches them in two more batches,
		// each a round trip after the previous wait); the empty asm only pins them to this point
		asm volatile("; k_ov_lord: LevelArgs fields" ::"s"(a.x_one), "s"(a.first_level), "s"(a.first_mask), "s"(a.csc),
		             "s"(a.hyp_uniform), "s"(a.hyp0), "s"(a.alpha), "s"(a.tcount), "s"(a.counters), "s"(a.dst),
		             "s"(a.feat_base));
	}
	const uint32_t n = live ? (uint32_t)(ce - cb) : 0u;
	const uint32_t m = (uint32_t)min<uint64_t>(we - wb, OV_CAP);
	// the run's first record in the level's buffer: from the column bound, or (PAD) the slot
	const uint32_t rb = PAD ? blockIdx.x * OV_CAP : (uint32_t)(wb - a.lbase);
	const uint32_t np = m * 4;
	const uint32_t ks = (np + 255) / 256, kd = (m + 255) / 256;
	const double2 *s2 = reinterpret_cast<const double2 *>(src + rb);
	const uint32_t *nx2 = lnext + rb;
	if constexpr (PAD) {
#pragma unroll
		for (int k = KP; k < KS; ++k)
			if (k < (int)ks) sv[k] = s2[threadIdx.x + k * 256];
#pragma unroll
		for (int k = KDP; k < KD; ++k)
			if (k < (int)kd) dv[k] = nx2[threadIdx.x + k * 256];
	} else {
#pragma unroll
		for (int k = 0; k < KS; ++k) {
			sv[k] = make_double2(0.0, 0.0);
			if (k < (int)ks) sv[k] = s2[min(threadIdx.x + k * 256, np - 1)];
		}
#pragma unroll
		for (int k = 0; k < KD; ++k) {
			dv[k] = 0;
			if (k < (int)kd) dv[k] = nx2[min(threadIdx.x + k * 256, m - 1)];
		}
	}
	const uint32_t o0 = (uint32_t)(cb - wb);   // the column's first record in the run
	const uint2 *col = a.csc + cb;
	// x of the lane's first two entries in registers before the barrier (the stats loop then
	// waits on no CSC load); none at all when every x is 1. `first` is level-uniform on the store.
	float xr0 = 1.0f, xr1 = 1.0f;
	if (!a.x_one) {
		if (lane < n) xr0 = ent_x(col[lane]);
		if (lane + G < n) xr1 = ent_x(col[lane + G]);
	}
	const bool fe_uniform = a.first_level >= 0, fe = a.first_level > 0;   // -1: the per-entry bit (A/B)
	auto xof = [&](uint32_t i, uint32_t it) -> float {
		if (a.x_one) return 1.0f;
		return it == 0 ? xr0 : it == 1 ? xr1 : ent_x(col[i]);
	};
	auto fof = [&](uint32_t i) -> bool { return fe_uniform ? fe : (col[i].x & a.first_mask) != 0; };
	// these two follow a pointer from the kernarg segment (used after the statistics loop / only
	// with several attribute groups)
	double hg = a.hyp0;
	uint32_t tc = 0;
	if (!a.hyp_uniform) hg = a.hyp[(size_t)a.attr_group[j] * a.hyp_stride];
	if (a.tcount) tc = a.tcount[j];
	// unconditional: slots past the run are never read, and a guarded write lets the compiler
	// merge it with its load and wait there
#pragma unroll
	for (int k = 0; k < KS; ++k) {
		const uint32_t t = threadIdx.x + k * 256;
		stage[ov_slot(t >> 2, t & 3)] = sv[k];
	}
#pragma unroll
	for (int k = 0; k < KD; ++k) dsts[threadIdx.x + k * 256] = dv[k];
	__syncthreads();
	OV_STAMP(1);
	auto get = [&](uint32_t i, Rec &r) {
		const uint32_t o = o0 + i;
		if (o < m) {
#pragma unroll
			for (uint32_t c = 0; c < 4; ++c) r[c] = stage[ov_slot(o, c)];
		} else {
			load_rec(src, rb + o, r);
		}
	};
	const double mo = msj.x, so = msj.y;
	const double keep_m = (1 - rho) * natj.x, keep_s = (1 - rho) * natj.y;
	const double acc = a.alpha * cc;
	const double rca = rho * cc * a.alpha;
	double eta1 = 0.0, eta2 = 0.0;
	for (uint32_t i = lane, it = 0; i < n; i += G, ++it) {
		Rec r;
		get(i, r);
		const float x = xof(i, it);
		if constexpr (IS_W) {
			const double w_mean = x * (E(r) + x * mo);
			const double w_sigma_sqr = x * x;   // fp32 product
			eta2 += keep_s + rho * (hg + acc * w_sigma_sqr);
			eta1 += keep_m + rca * w_mean;
		} else {
			double vm = 0.0, vs = 0.0;
			v_stat(x, E(r), Q<P>(r), TQ<P>(r), mo, so, vm, vs);
			eta2 += keep_s + rho * (hg + acc * vs);
			eta1 += keep_m + rca * vm;
		}
	}
	group_sum2<G>(eta1, eta2, nullptr);
	double mu = mo, sig = so;
	bool go = false;
	if (n) {
		const double nmu = eta1 / n, nsig = eta2 / n;
		mu = nmu / nsig;
		sig = 1 / nsig;
		go = true;
		const bool leader = lane == 0;
		const int c_sig = IS_W ? CNT_NAN_SIGMA_W : CNT_NAN_SIGMA_V, c_nan = IS_W ? CNT_NAN_MU_W : CNT_NAN_MU_V,
		          c_inf = IS_W ? CNT_INF_MU_W : CNT_INF_MU_V;
		if (dnan(sig) || dinf(sig)) {
			sig = so;
			if (leader) atomicAdd(&a.counters[c_sig], 1u);
		}
		if (dnan(mu)) {
			if (leader) atomicAdd(&a.counters[c_nan], 1u);
			mu = mo;
			go = false;
		} else if (dinf(mu)) {
			if (leader) atomicAdd(&a.counters[c_inf], 1u);
			mu = mo;
			go = false;
		}
		if (leader) {
			nat[(size_t)pj * nat_stride] = make_double2(nmu, nsig);
			ms[pi] = make_double2(mu, sig);
			if constexpr (IS_W) {
				const uint32_t t = tc + n;
				a.tcount[j] = t;
				rho_p[pj] = pow((double)(T0 + t), -LAMDA);
			} else {
				if (a.tcount) a.tcount[j] = tc + n;
			}
		}
	}
	OV_STAMP(2);
	for (uint32_t i = lane, it = 0; i < n; i += G, ++it) {
		Rec r;
		get(i, r);
		const float x = xof(i, it);
		if constexpr (IS_W) w_apply<NEXT>(r, x, fof(i), go, mo, so, mu, sig, nx);
		else v_apply<P, NEXT>(r, x, fof(i), go, mo, so, mu, sig, nx);
		const uint32_t o = o0 + i;
		if (o < m) {
#pragma unroll
			for (uint32_t c = 0; c < 4; ++c) stage[ov_slot(o, c)] = r[c];
		} else {
			store_rec(a.dst, lnext[rb + o], r);
		}
	}
	__syncthreads();
	OV_STAMP(3);
	// non-temporal stores: v sweep 1129 -> 1086 ms per C3 epoch (profiles/probes/ab_online_nt_store.txt;
	// write-through stores were 8 % slower, ab_write_through.txt)
	typedef double ntv2 __attribute__((ext_vector_type(2)));
	ntv2 *d = reinterpret_cast<ntv2 *>(a.dst);
	for (uint32_t t = threadIdx.x; t < m * 4; t += 256) {
		const double2 v = stage[ov_slot(t >> 2, t & 3)];
		ntv2 w;
		w.x = v.x;
		w.y = v.y;
		__builtin_nontemporal_store(w, d + (size_t)dsts[t >> 2] * 4 + (t & 3));
	}
	OV_STAMP(4);
	OV_STAMP_FLUSH;
}

inline unsigned grid_of(uint64_t n, unsigned block = 256) { return (unsigned)((n + block - 1) / block); }

}  // namespace

// ------------------------------------------------------------------------------------------
namespace vbk {
template <int G>
hipError_t launch_ov(const LevelArgs &a, int is_w, hipStream_t s)
{
	const unsigned grid = G <= 64 ? (a.nfeat + 256 / G - 1) / (256 / G) : a.nfeat;
	const bool nx = a.ms_next != nullptr;
	if (is_w) {
		if (nx) k_ov_w_level<G, true><<<grid, 256, 0, s>>>(a);
		else k_ov_w_level<G, false><<<grid, 256, 0, s>>>(a);
	} else if (a.slot == 0) {
		if (nx) k_ov_v_level<G, 0, true><<<grid, 256, 0, s>>>(a);
		else k_ov_v_level<G, 0, false><<<grid, 256, 0, s>>>(a);
	} else {
		if (nx) k_ov_v_level<G, 1, true><<<grid, 256, 0, s>>>(a);
		else k_ov_v_level<G, 1, false><<<grid, 256, 0, s>>>(a);
	}
	return hipGetLastError();
}

template <int G, bool PAD>
void launch_ov_lord_pad(const LevelArgs &a, int is_w, hipStream_t s)
{
	const unsigned grid = (a.nfeat + 256 / G - 1) / (256 / G);
	const bool nx = a.ms_next != nullptr;
#define OV_LORD_ARGS a.col_ptr, a.src, a.lnext, a.ms, a.nat, a.rho, a.ccount, a.nfeat, a
	if (is_w) {
		if (nx) k_ov_lord<G, true, 0, true, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
		else k_ov_lord<G, true, 0, false, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
	} else if (a.slot == 0) {
		if (nx) k_ov_lord<G, false, 0, true, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
		else k_ov_lord<G, false, 0, false, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
	} else {
		if (nx) k_ov_lord<G, false, 1, true, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
		else k_ov_lord<G, false, 1, false, PAD, false><<<grid, 256, 0, s>>>(OV_LORD_ARGS);
	}
#undef OV_LORD_ARGS
}

// the tagged-argument form of a v sweep's padded level (k_ov_lord FAST): field data (the level's
// features are consecutive ids), factor-major nat, the next factor's {mu, sigma} adjacent in ms (or
// none), and pointers / values that fit the tags; false: the caller takes the plain form
template <int G>
bool launch_ov_lord_fast(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (is_w || !a.pad_cap || !a.ov_fast || !a.feat_contig || a.nat_stride != 1) return false;
	// the kernel reads factor f+1 as ms[pi + 1] with factor f's stride
	if (a.ms_next && (a.ms_next != a.ms + 1 || a.ms_stride_next != a.ms_stride)) return false;
	auto fits = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) >> 48) == 0; };
	if (!fits(a.col_ptr) || !fits(a.src) || !fits(a.lnext) || a.ms_stride > 0xffffu) return false;
	auto tag = [](const void *p, uint64_t v) {
		return reinterpret_cast<uintptr_t>(p) | (uintptr_t)(v << 48);
	};
	const uint64_t *cp = reinterpret_cast<const uint64_t *>(tag(a.col_ptr, a.nfeat & 0xffffu));
	const RowRec *sr = reinterpret_cast<const RowRec *>(tag(a.src, a.nfeat >> 16));
	const uint32_t *ln = reinterpret_cast<const uint32_t *>(tag(a.lnext, a.ms_stride));
	double2 *ms = a.ms + (size_t)a.feat_base * a.ms_stride;
	double2 *nat = a.nat + a.feat_base;
	double *rho = a.rho + a.feat_base;
	const uint32_t *cc = a.ccount + a.feat_base;
	const unsigned grid = (a.nfeat + 256 / G - 1) / (256 / G);
#define OV_FAST_ARGS cp, sr, ln, ms, nat, rho, cc, a.nfeat, a
	if (a.slot == 0) {
		if (a.ms_next) k_ov_lord<G, false, 0, true, true, true><<<grid, 256, 0, s>>>(OV_FAST_ARGS);
		else k_ov_lord<G, false, 0, false, true, true><<<grid, 256, 0, s>>>(OV_FAST_ARGS);
	} else {
		if (a.ms_next) k_ov_lord<G, false, 1, true, true, true><<<grid, 256, 0, s>>>(OV_FAST_ARGS);
		else k_ov_lord<G, false, 1, false, true, true><<<grid, 256, 0, s>>>(OV_FAST_ARGS);
	}
#undef OV_FAST_ARGS
	return true;
}

template <int G>
hipError_t launch_ov_lord(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.pad_cap) {
		if (!launch_ov_lord_fast<G>(a, is_w, s)) launch_ov_lord_pad<G, true>(a, is_w, s);
	} else {
		launch_ov_lord_pad<G, false>(a, is_w, s);
	}
	return hipGetLastError();
}

// one level on the batch's level-ordered store (a.src / a.dst / a.lnext / a.lbase set)
hipError_t ov_lord_level(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	if (a.pad_cap && a.pad_cap != OV_CAP) return hipErrorInvalidValue;
	switch (ov_lord_g(a.avg_len)) {
	case 4: return launch_ov_lord<4>(a, is_w, s);
	case 8: return launch_ov_lord<8>(a, is_w, s);
	case 16: return launch_ov_lord<16>(a, is_w, s);
	case 32: return launch_ov_lord<32>(a, is_w, s);
	default: return launch_ov_lord<64>(a, is_w, s);
	}
}

uint32_t ov_lord_g(uint32_t m)
{
	return m <= 6 ? 4 : m <= 12 ? 8 : m <= 24 ? 16 : m <= 48 ? 32 : 64;
}

uint32_t ov_pad_cap() { return OV_CAP; }

// lanes per column from the batch's mean column length (LevelArgs::avg_len, set by
// ov_level_args): about one entry per lane
hipError_t ov_level(const LevelArgs &a, int is_w, hipStream_t s)
{
	if (a.nfeat == 0) return hipSuccess;
	const uint32_t m = a.avg_len;
	if (m <= 6) return launch_ov<4>(a, is_w, s);
	if (m <= 12) return launch_ov<8>(a, is_w, s);
	if (m <= 24) return launch_ov<16>(a, is_w, s);
	if (m <= 48) return launch_ov<32>(a, is_w, s);
	if (m <= 160) return launch_ov<64>(a, is_w, s);
	return launch_ov<256>(a, is_w, s);
}
}  // namespace vbk

// ------------------------------------------------------------------------------------------
struct OvState {
	uint32_t num_batch = 50;
	uint32_t n_total = 0;          // total_cases
	uint32_t size = 0;             // size_except_last = ceil(N / num_batch)
	vbrng::Glibc stream;           // the reference's rand() after the initial draws
	std::vector<uint32_t> shuffle; // kept across epochs (:58-62)
	// the next epoch's shuffle, drawn on a host thread while the GPU sweeps this epoch's batches
	// (the permutation depends on the rand() stream and the last permutation only)
	std::vector<uint32_t> sh_next;
	vbrng::Glibc stream_next;
	std::thread pre;
	void pre_join()
	{
		if (pre.joinable()) pre.join();
	}
	~OvState() { pre_join(); }
	double2 *nat_w = nullptr, *nat_v = nullptr;   // natural_{mu,sigma}_{w,v}_dash; nat_v factor-major [f][j]
	                                              // (the reference's layout): a level's columns are
	                                              // consecutive ids, so their natural parameters are one
	                                              // coalesced run instead of one line per column
	double *new_wj = nullptr, *new_vj = nullptr;
	uint32_t *t_wj = nullptr, *t_vj = nullptr, *ccount = nullptr;
	double nat_mu0 = 0.0, nat_sig0 = 0.0, new_w0 = 1.0;
	uint32_t t_w0 = 0;
	// epoch regrouping
	uint32_t *sh_d = nullptr, *bat_d = nullptr, *iota_d = nullptr, *rows_sorted = nullptr, *bat_sorted = nullptr,
	         *loc_d = nullptr;
	uint16_t *key_in = nullptr, *key_out = nullptr;
	uint2 *ent_sorted = nullptr;   // all entries, batch-major, column-major inside a batch
	uint2 *ent_tmp = nullptr;
	uint32_t *cnt = nullptr;       // [num_batch * nf] (batch, column) entry counts
	uint64_t *gptr = nullptr;      // [num_batch * nf + 1] their prefix sums: col_ptr of every batch,
	                               // indexed by level position (level_feats order)
	uint64_t *lvcp = nullptr;      // [nf + 1] start of each level-ordered column in the whole train set
	std::vector<uint64_t> rstart;  // [num_batch + 1] first sorted row of each batch
	uint64_t *rstart_d = nullptr;
	void *tmp = nullptr;
	size_t tmp_bytes = 0;
	// the batch being processed
	uint32_t cap_rows = 0;
	uint64_t cap_nnz = 0;
	uint64_t *rp_b = nullptr, *len_b = nullptr;
	uint2 *csr_b = nullptr;
	float *t_b = nullptr;
	RowRec *rows_b = nullptr;
	hipEvent_t ev[4] = {};
	std::vector<hipEvent_t> bev;   // [num_batch * 6] phase marks of every batch
	uint32_t launches_v = 0;
	// the per-batch level-ordered store (k_ov_lord)
	uint32_t *level_ptr_d = nullptr;   // [L+1] level bounds in level positions
	bool x_one = false;                // every train x is 1.0f (one-hot): k_ov_lord loads no x
	// the padded layout of levels >= 1 (OvPad): columns per workgroup of every level, each level's
	// slot count, the padded levels' lnx prefix (batch-independent), the batches it applies to
	uint32_t *cpw_d = nullptr, *pad_bad_d = nullptr;
	uint64_t *lnx_off_d = nullptr;     // [L] lnx region of each level for the current batch
	std::vector<uint32_t> cpw_h, ngroups_h, gbase_h;   // gbase: groups of the levels before l [L + 1]
	uint32_t *gbase_d = nullptr;
	std::vector<uint64_t> pad_prefix;  // [L + 1] sum over levels 1..l-1 of ngroups * cap
	std::vector<uint8_t> batch_pad;    // [num_batch]
	uint64_t pad_rows = 0;             // records a padded level's buffer needs (max over levels)
	bool pad_on = false;               // the batch being processed uses the padded layout
	bool fast = true;                  // v levels on it take k_ov_lord's tagged arguments (VBFM_OV_FAST)
	bool legacy = false;               // A/B: the round-3 kernel's per-entry x and flag (VBFM_OV_LEGACY)
	uint32_t cur_n = 0;                // its rows
	uint64_t *lvl_d = nullptr;         // [num_batch * (L+1)] first entry of every level of every batch
	std::vector<uint64_t> lvl_h;
	std::vector<uint8_t> batch_lord;   // [num_batch] the batch's levels are complete
	uint32_t *lpos = nullptr, *lnx = nullptr;
	RowRec *rows_b2 = nullptr;
	uint32_t lord_cap_rows = 0;
	uint64_t lord_cap_nnz = 0;
	bool lord_on = false;              // the batch being processed uses the store
	const uint64_t *lvl_cur = nullptr; // its level bases (host)
	RowRec *rows_other = nullptr;      // the second record buffer of the ping-pong
};

namespace vbi {

void ov_free(vbfm_ctx *c)
{
	if (!c->ov) return;
	OvState &o = *c->ov;
	dfree(o.nat_w); dfree(o.nat_v); dfree(o.new_wj); dfree(o.new_vj); dfree(o.t_wj); dfree(o.t_vj);
	dfree(o.ccount); dfree(o.sh_d); dfree(o.bat_d); dfree(o.iota_d); dfree(o.rows_sorted); dfree(o.bat_sorted);
	dfree(o.loc_d); dfree(o.key_in); dfree(o.key_out); dfree(o.ent_sorted); dfree(o.ent_tmp); dfree(o.cnt);
	dfree(o.gptr); dfree(o.lvcp); dfree(o.rstart_d); dfree(o.tmp); dfree(o.rp_b); dfree(o.len_b); dfree(o.csr_b); dfree(o.t_b);
	dfree(o.rows_b);
	dfree(o.level_ptr_d); dfree(o.lvl_d); dfree(o.lpos); dfree(o.lnx); dfree(o.rows_b2);
	dfree(o.cpw_d); dfree(o.pad_bad_d); dfree(o.lnx_off_d); dfree(o.gbase_d);
	for (hipEvent_t e : o.ev)
		if (e) (void)hipEventDestroy(e);
	for (hipEvent_t e : o.bev) (void)hipEventDestroy(e);
	delete c->ov;
	c->ov = nullptr;
}

void ov_level_args(vbfm_ctx *c, LevelArgs &a, bool is_w, int f)
{
	OvState &o = *c->ov;
	a.nat = is_w ? o.nat_w : o.nat_v + (size_t)f * c->D;   // factor-major: the level's columns are one run
	a.nat_stride = 1;
	a.rho = is_w ? o.new_wj : o.new_vj;
	a.ccount = o.ccount;
	a.tcount = is_w ? o.t_wj : (f == 0 ? o.t_vj : nullptr);
	if (!is_w) o.launches_v++;
	a.avg_len = a.avg_len / std::max(o.num_batch, 1u);   // the batch's share of the mean column
	a.hyp_uniform = c->G == 1;
	a.hyp0 = c->G == 1 ? (is_w ? c->hyp_w[0] : c->hyp_v[f]) : 0.0;
	a.col_ptr += a.feats - c->level_feats;               // the batch's col_ptr by level position
}

// one level of the batch's sweep: on the batch's level-ordered store when it is in use (the
// records move to the next level's order), else the column kernels
void ov_launch_level(vbfm_ctx *c, LevelArgs &a, uint32_t l, bool is_w)
{
	OvState &o = *c->ov;
	if (!o.lord_on) {
		HIPCHK(vbk::ov_level(a, is_w, c->s));
		return;
	}
	a.src = c->rows;
	a.dst = o.rows_other;
	a.lbase = o.lvl_cur[l];
	a.lnext = o.lnx + (o.lvl_cur[l] - o.lvl_cur[0]);
	if (o.pad_on && l > 0) {   // the padded layout: slot w of the level's buffer, lnx likewise
		a.pad_cap = vbk::ov_pad_cap();
		a.lnext = o.lnx + o.cur_n + o.pad_prefix[l];
		a.ov_fast = o.fast;
	}
	// every level of the store holds each batch row once and a row's features ascend with the
	// levels: level 0 holds every row's first entry (the ROW_FIRST bit of its CSC entries)
	a.first_level = l == 0 && a.first_mask != 0;
	a.x_one = o.x_one;
	if (o.legacy) {   // A/B (VBFM_OV_LEGACY=1): x and the first-entry bit from the CSC per entry
		a.first_level = -1;
		a.x_one = 0;
	}
#ifdef VBFM_OV_STAMPS
	// VBFM_OV_STAMP=<n>: the n-th v-level launch of the process (and every 1000th after it) stamps
	// its workgroups; the stamps go to stderr as one line per workgroup after the launch
	static long launch_no = 0;
	static const long want = [] { const char *e = getenv("VBFM_OV_STAMP"); return e ? atol(e) : -1L; }();
	unsigned long long *st = nullptr;
	const unsigned nwg = (a.nfeat + 31) / 32 + 4096;
	if (!is_w && want >= 0 && launch_no >= want && (launch_no - want) % 1000 == 0) {
		HIPCHK(hipMalloc(&st, (size_t)nwg * 5 * 8 * 8));
		HIPCHK(hipMemsetAsync(st, 0, (size_t)nwg * 5 * 8 * 8, c->s));
	}
	a.stamp = st;
	if (!is_w) launch_no++;
	HIPCHK(vbk::ov_lord_level(a, is_w, c->s));
	if (st) {
		std::vector<unsigned long long> h((size_t)nwg * 5 * 8);
		HIPCHK(d2h(c, h.data(), st, h.size() * 8));
		sync(c);
		(void)hipFree(st);
		fprintf(stderr, "OVSTAMP launch %ld nfeat %u avg %u\n", launch_no - 1, a.nfeat, a.avg_len);
		for (size_t w = 0; w * 5 < h.size() && h[w * 5] != 0; w++)
			fprintf(stderr, "OVSTAMP %zu %llu %llu %llu %llu %llu\n", w, h[w * 5], h[w * 5 + 1], h[w * 5 + 2],
			        h[w * 5 + 3], h[w * 5 + 4]);
	}
	a.stamp = nullptr;
#else
	HIPCHK(vbk::ov_lord_level(a, is_w, c->s));
#endif
	std::swap(c->rows, o.rows_other);
}

}  // namespace vbi

namespace {

// temp storage of rocprim calls: grow on demand
void *ov_tmp(OvState &o, size_t bytes)
{
	if (bytes > o.tmp_bytes) {
		dfree(o.tmp);
		o.tmp = dalloc<uint8_t>(bytes);
		o.tmp_bytes = bytes;
	}
	return o.tmp;
}

// std::random_shuffle(sh, sh + N) (libstdc++: i from 1, j = rand() % (i + 1))
void ov_shuffle(std::vector<uint32_t> &sh, vbrng::Glibc &stream)
{
	const uint32_t N = (uint32_t)sh.size();
	for (uint32_t i = 1; i < N; i++) {
		const uint32_t j = (uint32_t)(stream.next() % (int32_t)(i + 1));
		if (j != i) std::swap(sh[i], sh[j]);
	}
}

// the next epoch's permutation on a host thread; called once this epoch's has reached the device
void ov_prefetch_shuffle(OvState &o)
{
	o.pre_join();
	o.pre = std::thread([&o] {
		o.sh_next = o.shuffle;
		o.stream_next = o.stream;
		ov_shuffle(o.sh_next, o.stream_next);
	});
}

// steps 1-3 of the file header: the epoch's batches
void ov_regroup(vbfm_ctx *c)
{
	OvState &o = *c->ov;
	const uint32_t N = o.n_total, nf = c->tr.nf, nb = o.num_batch;
	const uint64_t nnz = c->tr.nnz;
	if (o.pre.joinable()) {   // drawn during the last epoch
		o.pre_join();
		std::swap(o.shuffle, o.sh_next);
		o.stream = o.stream_next;
	} else {
		ov_shuffle(o.shuffle, o.stream);
	}
	HIPCHK(hipMemcpyAsync(o.sh_d, o.shuffle.data(), (size_t)N * 4, hipMemcpyHostToDevice, c->s));
	k_ov_batch<<<grid_of(N), 256, 0, c->s>>>(o.sh_d, N, o.size, o.bat_d, o.iota_d);
	HIPCHK(hipGetLastError());
	int bits = 1;
	while ((1u << bits) < nb) bits++;
	size_t tb = 0;
	HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, o.bat_d, o.bat_sorted, o.iota_d, o.rows_sorted, (size_t)N, 0, bits,
	                                 c->s));
	HIPCHK(rocprim::radix_sort_pairs(ov_tmp(o, tb), tb, o.bat_d, o.bat_sorted, o.iota_d, o.rows_sorted, (size_t)N, 0,
	                                 bits, c->s));
	// batch row counts: the shuffle is a permutation of 1..N, so batch b holds the rows with
	// shuffle values in (b*size, (b+1)*size]
	o.rstart.assign((size_t)nb + 1, 0);
	for (uint32_t b = 0; b <= nb; b++) o.rstart[b] = std::min<uint64_t>((uint64_t)b * o.size, N);
	HIPCHK(hipMemcpyAsync(o.rstart_d, o.rstart.data(), ((size_t)nb + 1) * 8, hipMemcpyHostToDevice, c->s));
	k_ov_local<<<grid_of(N), 256, 0, c->s>>>(o.rows_sorted, o.bat_d, o.rstart_d, N, o.loc_d);
	HIPCHK(hipGetLastError());
	// entries
	HIPCHK(hipMemsetAsync(o.cnt, 0, (size_t)nb * nf * 4, c->s));
	if (nf)
		k_ov_entries<<<nf, 256, 0, c->s>>>(c->tr.col_ptr, c->tr.csc, c->level_feats, o.lvcp, o.bat_d, o.loc_d, nf, o.key_in,
		                                   o.ent_tmp, o.cnt);
	HIPCHK(hipGetLastError());
	tb = 0;
	HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, o.key_in, o.key_out, o.ent_tmp, o.ent_sorted, (size_t)nnz, 0, bits,
	                                 c->s));
	HIPCHK(rocprim::radix_sort_pairs(ov_tmp(o, tb), tb, o.key_in, o.key_out, o.ent_tmp, o.ent_sorted, (size_t)nnz, 0,
	                                 bits, c->s));
	tb = 0;
	const size_t ncnt = (size_t)nb * nf;
	HIPCHK(rocprim::exclusive_scan(nullptr, tb, o.cnt, o.gptr, (uint64_t)0, ncnt, rocprim::plus<uint64_t>(), c->s));
	HIPCHK(rocprim::exclusive_scan(ov_tmp(o, tb), tb, o.cnt, o.gptr, (uint64_t)0, ncnt, rocprim::plus<uint64_t>(),
	                               c->s));
	HIPCHK(hipMemcpyAsync(o.gptr + ncnt, &nnz, 8, hipMemcpyHostToDevice, c->s));
	// the level bases of every batch, for the per-batch level-ordered store
	const uint32_t L = nlevels(c);
	if (o.level_ptr_d && L) {
		k_ov_level_bases<<<grid_of((uint64_t)nb * (L + 1)), 256, 0, c->s>>>(o.gptr, o.level_ptr_d, L, nf, nb, o.lvl_d);
		HIPCHK(hipGetLastError());
		o.lvl_h.resize((size_t)nb * (L + 1));
		HIPCHK(d2h(c, o.lvl_h.data(), o.lvl_d, o.lvl_h.size() * 8));
	}
	sync(c);   // nnz (host) must outlive the copy
	o.batch_lord.assign(nb, 0);
	if (o.level_ptr_d && L)
		for (uint32_t b = 0; b < nb; b++) {
			const uint64_t n = o.rstart[b + 1] - o.rstart[b];
			bool ok = n > 0;
			for (uint32_t l = 0; l < L && ok; l++) ok = o.lvl_h[(size_t)b * (L + 1) + l + 1] - o.lvl_h[(size_t)b * (L + 1) + l] == n;
			o.batch_lord[b] = ok;
		}
	// the padded layout of levels >= 1: every workgroup run of the batch must fit its slot
	o.batch_pad.assign(nb, 0);
	if (o.cpw_d && L > 1) {
		HIPCHK(hipMemsetAsync(o.pad_bad_d, 0, (size_t)nb * 4, c->s));
		k_ov_pad_check<<<grid_of((uint64_t)nb * nf), 256, 0, c->s>>>(o.gptr, o.level_ptr_d, o.cpw_d, L, nf, nb,
		                                                          vbk::ov_pad_cap(), o.pad_bad_d);
		HIPCHK(hipGetLastError());
		std::vector<uint32_t> bad(nb);
		HIPCHK(d2h(c, bad.data(), o.pad_bad_d, (size_t)nb * 4));
		sync(c);
		for (uint32_t b = 0; b < nb; b++) o.batch_pad[b] = o.batch_lord[b] && !bad[b];
	}
}

// the per-batch store: positions of the batch's rows in every level and every entry's
// position in the next level; the records (predicted in row order) moved to level-0 order
void ov_lord_begin(vbfm_ctx *c, uint32_t b, uint32_t n, uint64_t nnz)
{
	OvState &o = *c->ov;
	const uint32_t L = nlevels(c);
	if (n > o.lord_cap_rows) {
		dfree(o.lpos); dfree(o.rows_b2);
		o.lpos = dalloc<uint32_t>((size_t)L * n);
		o.rows_b2 = dalloc<RowRec>(std::max<uint64_t>(n, o.pad_rows));
		o.lord_cap_rows = n;
	}
	const bool pad = !o.batch_pad.empty() && o.batch_pad[b];
	const uint64_t lnx_need = pad ? n + o.pad_prefix[L] : nnz;
	if (lnx_need > o.lord_cap_nnz) {
		dfree(o.lnx);
		o.lnx = dalloc<uint32_t>(lnx_need);
		o.lord_cap_nnz = lnx_need;
	}
	const uint64_t *base = o.lvl_d + (size_t)b * (L + 1);
	OvPad pd = {o.gptr + (size_t)b * c->tr.nf, o.level_ptr_d, o.cpw_d, 0u, o.lnx_off_d};
	{
		// each level's lnx region: packed (base[l] - base[0]) or, padded, level 0's n entries and
		// then every level's slots
		std::vector<uint64_t> off(L);
		for (uint32_t l = 0; l < L; l++)
			off[l] = pad ? (l == 0 ? 0 : n + o.pad_prefix[l]) : o.lvl_h[(size_t)b * (L + 1) + l] - o.lvl_h[(size_t)b * (L + 1)];
		HIPCHK(hipMemcpyAsync(o.lnx_off_d, off.data(), (size_t)L * 8, hipMemcpyHostToDevice, c->s));
		sync(c);   // (off is a host temporary)
		if (pad) pd.cap = vbk::ov_pad_cap();
	}
	if (pad) {
		const uint32_t groups = o.gbase_h[L];
		k_ov_pad_pos<false><<<groups, 256, 0, c->s>>>(o.ent_sorted, pd, o.gbase_d, L, n, o.lpos, o.lnx);
		HIPCHK(hipGetLastError());
		k_ov_pad_pos<true><<<groups, 256, 0, c->s>>>(o.ent_sorted, pd, o.gbase_d, L, n, o.lpos, o.lnx);
	} else {
		k_ov_lord_pos<<<grid_of(nnz), 256, 0, c->s>>>(o.ent_sorted, base, L, n, o.lpos);
		HIPCHK(hipGetLastError());
		k_ov_lord_next<<<grid_of(nnz), 256, 0, c->s>>>(o.ent_sorted, base, L, n, o.lpos, o.lnx);
	}
	HIPCHK(hipGetLastError());
	o.pad_on = pad;
	o.cur_n = n;
	HIPCHK(vbk::rows_scatter(o.rows_b2, c->rows, o.lpos, n, c->s));   // row r -> its level-0 position
	o.rows_other = c->rows;
	c->rows = o.rows_b2;
	o.lvl_cur = o.lvl_h.data() + (size_t)b * (L + 1);
	o.lord_on = true;
}

void ov_batch_capacity(vbfm_ctx *c, uint32_t n, uint64_t nnz)
{
	OvState &o = *c->ov;
	if (n > o.cap_rows) {
		dfree(o.rp_b); dfree(o.len_b); dfree(o.t_b); dfree(o.rows_b);
		o.rp_b = dalloc<uint64_t>((size_t)n + 1);
		o.len_b = dalloc<uint64_t>((size_t)n + 1);
		o.t_b = dalloc<float>(n);
		// also a padded level's buffer (ping-pong partner of rows_b2)
		o.rows_b = dalloc<RowRec>(std::max<uint64_t>(n, o.pad_rows));
		o.cap_rows = n;
	}
	if (nnz > o.cap_nnz) {
		dfree(o.csr_b);
		o.csr_b = dalloc<uint2>(nnz);
		o.cap_nnz = nnz;
	}
}

// update_w0 (fm_learn_vb_online.h:471-497) on the batch in c->rows / c->tr
void ov_step_w0(vbfm_ctx *c)
{
	OvState &o = *c->ov;
	const uint32_t n = c->tr.n;
	const double sigma_dash = c->s0d, mu_dash = c->mu0, mu_old = o.nat_mu0, sigma_old = o.nat_sig0;
	const double size = (double)o.n_total;
	// natural_sigma_0_dash is the same every row: the reference adds it n times
	const double nsig_i = ((1 - o.new_w0) * sigma_old) + o.new_w0 * (c->sigma_0 + o.n_total * c->alpha);
	double eta2 = 0.0;
	for (uint32_t i = 0; i < n; i++) eta2 += nsig_i;
	k_ov_w0_sum<256><<<c->RED_BLOCKS, 256, 0, c->s>>>(c->rows, n, (1 - o.new_w0) * mu_old, o.new_w0 * size * c->alpha,
	                                                  c->mu0, c->red_d);
	HIPCHK(hipGetLastError());
	const double eta1 = finish_sum(c, c->RED_BLOCKS);
	o.nat_mu0 = eta1 / n;
	o.nat_sig0 = eta2 / n;
	c->mu0 = o.nat_mu0 / o.nat_sig0;
	c->s0d = 1.0 / o.nat_sig0;
	HIPCHK(vbk::w0_apply(c->rows, n, mu_dash - c->mu0, c->s0d - sigma_dash, c->s));
}

// the hyper-parameter steps of update_all (fm_learn_vb_online.h:408-467); false on the early
// return of a NaN / inf alpha
bool ov_step_hyper(vbfm_ctx *c, uint32_t *nan_alpha, uint32_t *inf_alpha)
{
	OvState &o = *c->ov;
	const double alpha_temp = rows_energy(c);
	const double alpha_old = c->alpha;
	c->alpha = (1 - o.new_w0) * alpha_old + o.new_w0 * ((double)c->tr.n / alpha_temp);
	if (std::isnan(c->alpha)) { (*nan_alpha)++; c->alpha = alpha_old; return false; }
	if (std::isinf(c->alpha)) { (*inf_alpha)++; c->alpha = alpha_old; return false; }
	c->sigma_0 = (1 - o.new_w0) * c->sigma_0 + o.new_w0 * (1.0 / (c->mu0 * c->mu0 + c->s0d));
	std::vector<double> seg = param_sums(c, 0);
	for (uint32_t g = 0; g < c->G; g++)
		c->hyp_w[g] = (1 - o.new_w0) * c->hyp_w[g] + o.new_w0 * ((double)c->per_group[g] / seg[g]);
	for (int f = 0; f < c->k; f++)
		for (uint32_t g = 0; g < c->G; g++) {
			double &h = c->hyp_v[(size_t)g * c->k + f];
			h = (1 - o.new_w0) * h + o.new_w0 * ((double)c->per_group[g] / seg[(size_t)(f + 1) * c->G + g]);
		}
	upload_hyp(c);
	o.t_w0 += 1;
	o.new_w0 = std::pow((double)(T0 + o.t_w0), -LAMDA);
	return true;
}

}  // namespace

// =========================================================================================
extern "C" {

int vbfm_online_init(vbfm_ctx *c, const vbfm_online_config *cfg)
{
	if (!c || !cfg) return fail(c, "vbfm_online_init: null argument");
	return guarded(c, [&] {
		if (c->mc) throw std::string("an MCMC / ALS context cannot run the online VB learner");
		if (c->multi() || c->shard_mode == VBFM_SHARD_FEATURES)
			throw std::string("the online VB learner runs on one GPU (no communicator, no feature shards)");
		if (!c->rows) throw std::string("no train data set (vbfm_set_train)");
		if (!c->e_test) throw std::string("no test data set (vbfm_set_test)");
		if (cfg->init_mode != VBFM_ONLINE_INIT_HOST && cfg->init_mode != VBFM_ONLINE_INIT_REPLAY)
			throw std::string("unknown init mode");
		const uint32_t N = c->tr.n, nb = cfg->num_batch;
		if (nb == 0 || nb > 65536) throw std::string("num_batch must be in 1..65536");
		if (N == 0) throw std::string("empty train set");
		const uint32_t size = (uint32_t)std::ceil((double)N / nb);   // :56-57
		const uint32_t used = (uint32_t)std::ceil((double)N / size);
		if (used < nb)
			throw std::string("num_batch ") + std::to_string(nb) + " leaves batches " + std::to_string(used + 1) + ".." +
			    std::to_string(nb) + " of " + std::to_string(N) +
			    " rows empty (the reference divides by their zero size and crashes)";
		ov_free(c);
		c->ov = new OvState();
		try {
			OvState &o = *c->ov;
			// the column layout (one level sweep per batch, no level-ordered store)
			lord_release(c, false);
			c->sched_ready = false;
			require_train(c);
			for (hipEvent_t &e : o.ev) HIPCHK(hipEventCreate(&e));
			o.bev.resize((size_t)nb * 6);
			for (hipEvent_t &e : o.bev) HIPCHK(hipEventCreate(&e));
			o.num_batch = nb;
			o.n_total = N;
			o.size = size;
			// the initial draws (libfm.cpp:123-124, 259-274, 313; fm_learn_vb_online.h:736-741): the
			// VB learner's, then the stream continues into the epoch shuffles
			const size_t kd = (size_t)c->k * c->D;
			if (cfg->init_mode == VBFM_ONLINE_INIT_HOST) {
				std::vector<double> mw(c->D), sw(c->D, .02), mv(kd), sv(kd, .02), hw(c->G), hv((size_t)c->G * c->k);
				vbfm_params p = {mw.data(), sw.data(), mv.data(), sv.data(), hw.data(), hv.data(), 0, 0, 0, 0};
				vbrng::Glibc &rng = o.stream;
				rng.seed_with(cfg->seed);
				for (size_t i = 0; i < kd; i++) {                                              // fm.v (fm_model.h:97)
					const double v = rng.gaussian(0, cfg->init_stdev);
					if (cfg->fm_v) cfg->fm_v[i] = v;
				}
				for (uint32_t i = 0; i < c->D; i++) (void)rng.gaussian(0, cfg->init_stdev);   // fm.w (libfm.cpp:313)
				for (uint32_t i = 0; i < c->D; i++) mw[i] = 0.1 * rng.gaussian(0, 1);         // mu_w_dash.init_normal
				for (size_t i = 0; i < kd; i++) mv[i] = 0.1 * rng.gaussian(0, 1);            // mu_v_dash.init_normal
				std::fill(hw.begin(), hw.end(), 1.0);
				std::fill(hv.begin(), hv.end(), 1.0);
				p.alpha = 1.0; p.sigma_0 = 1.0; p.mu_0_dash = 0.0; p.sigma_0_dash = 0.02;
				if (vbfm_set_params(c, &p)) throw std::string(c->err);
			} else {
				if (vbfm_init_params_replay(c, cfg->seed, cfg->init_stdev, cfg->fm_v, nullptr)) throw std::string(c->err);
				uint32_t st[31];
				glibc_state_at(cfg->seed, c->init_stream_end, st);
				o.stream.set_chrono_state(st);
			}
			// fm_learn_vb_online::init (:686-758)
			const uint32_t D = c->D, nf = c->tr.nf;
			o.nat_w = dalloc<double2>(D);
			o.nat_v = dalloc<double2>(kd);
			o.new_wj = dalloc<double>(D);
			o.new_vj = dalloc<double>(D);
			o.t_wj = dalloc<uint32_t>(D);
			o.t_vj = dalloc<uint32_t>(D);
			o.ccount = dalloc<uint32_t>(D);
			HIPCHK(hipMemsetAsync(o.t_wj, 0, (size_t)D * 4, c->s));
			HIPCHK(hipMemsetAsync(o.t_vj, 0, (size_t)D * 4, c->s));
			const double rho0 = std::pow((double)(T0 + 0), -LAMDA);
			if (D) {
				k_ov_fill<<<grid_of(D), 256, 0, c->s>>>(o.new_wj, D, rho0);
				k_ov_fill<<<grid_of(D), 256, 0, c->s>>>(o.new_vj, D, rho0);
				k_ov_ccount<<<grid_of(D), 256, 0, c->s>>>(c->tr.col_ptr, nf, D, o.ccount);
				k_ov_nat_init<<<grid_of(D), 256, 0, c->s>>>(c->ms_w, D, o.nat_w);
			}
			if (kd) k_ov_nat_init_v<<<grid_of(kd), 256, 0, c->s>>>(c->ms_v, (uint32_t)c->k, c->D, o.nat_v);
			HIPCHK(hipGetLastError());
			o.t_w0 = 0;
			o.new_w0 = std::pow((double)(T0 + o.t_w0), -LAMDA);
			o.nat_mu0 = 0.0;
			o.nat_sig0 = 1 / c->s0d;
			o.shuffle.resize(N);
			for (uint32_t i = 0; i < N; i++) o.shuffle[i] = i + 1;
			// the epoch regrouping buffers
			const uint64_t nnz = c->tr.nnz;
			o.sh_d = dalloc<uint32_t>(N); o.bat_d = dalloc<uint32_t>(N); o.iota_d = dalloc<uint32_t>(N);
			o.rows_sorted = dalloc<uint32_t>(N); o.bat_sorted = dalloc<uint32_t>(N); o.loc_d = dalloc<uint32_t>(N);
			o.key_in = dalloc<uint16_t>(nnz); o.key_out = dalloc<uint16_t>(nnz);
			o.ent_tmp = dalloc<uint2>(nnz); o.ent_sorted = dalloc<uint2>(nnz);
			o.cnt = dalloc<uint32_t>((size_t)nb * nf);
			o.gptr = dalloc<uint64_t>((size_t)nb * nf + 1);
			// the per-batch level-ordered store: field-structured data (no row lists a feature
			// twice); factor 0's q-cache must come from the w sweep (k1), VBFM_LAYOUT=column or
			// vbfm_set_layout(VBFM_LAYOUT_COLUMN) keep the column kernels
			{
				const char *lay = getenv("VBFM_LAYOUT");
				bool want = c->layout_req != VBFM_LAYOUT_COLUMN && !(lay && !strcmp(lay, "column")) &&
				            (c->k1 || c->k == 0) && nlevels(c) > 0;
				if (want && nf) {
					std::vector<uint8_t> dup(nf);
					HIPCHK(hipMemcpy(dup.data(), c->dup, nf, hipMemcpyDeviceToHost));
					for (uint8_t d : dup) want = want && !d;
				}
				if (want) {
					const uint32_t L = nlevels(c);
					o.level_ptr_d = dalloc<uint32_t>((size_t)L + 1);
					HIPCHK(hipMemcpy(o.level_ptr_d, c->level_ptr.data(), ((size_t)L + 1) * 4, hipMemcpyHostToDevice));
					o.lvl_d = dalloc<uint64_t>((size_t)nb * (L + 1));
					uint32_t *cnt = dalloc<uint32_t>(1), ne1 = 1;
					HIPCHK(vbk::count_x_ne1(c->tr.csc, nnz, cnt, c->s));
					HIPCHK(d2h(c, &ne1, cnt, 4));
					sync(c);
					dfree(cnt);
					o.x_one = ne1 == 0;
					// the padded layout (VBFM_OV_PAD=0: packed runs at every level); the lanes per
					// column of a level's kernel follow its mean batch column (ov_level_args)
					const char *pe = getenv("VBFM_OV_PAD");
					const char *fe = getenv("VBFM_OV_FAST");   // A/B: 0 = the untagged arguments everywhere
					o.fast = !(fe && fe[0] == '0');
					const char *lg = getenv("VBFM_OV_LEGACY");
					o.legacy = lg && lg[0] == '1';
					if (!(pe && pe[0] == '0') && L > 1) {
						const uint32_t cap = vbk::ov_pad_cap();
						o.cpw_h.assign(L, 0);
						o.ngroups_h.assign(L, 0);
						o.pad_prefix.assign((size_t)L + 1, 0);
						for (uint32_t l = 0; l < L; l++) {
							const uint32_t nfl = c->level_ptr[l + 1] - c->level_ptr[l];
							o.cpw_h[l] = 256 / vbk::ov_lord_g(c->level_avg[l] / std::max(nb, 1u));
							o.ngroups_h[l] = (nfl + o.cpw_h[l] - 1) / o.cpw_h[l];
						}
						for (uint32_t l = 1; l < L; l++) {
							o.pad_prefix[l + 1] = o.pad_prefix[l] + (uint64_t)o.ngroups_h[l] * cap;
							o.pad_rows = std::max<uint64_t>(o.pad_rows, (uint64_t)o.ngroups_h[l] * cap);
						}
						o.gbase_h.assign((size_t)L + 1, 0);
						for (uint32_t l = 0; l < L; l++) o.gbase_h[l + 1] = o.gbase_h[l] + o.ngroups_h[l];
						o.cpw_d = dalloc<uint32_t>(L);
						HIPCHK(hipMemcpy(o.cpw_d, o.cpw_h.data(), (size_t)L * 4, hipMemcpyHostToDevice));
						o.gbase_d = dalloc<uint32_t>((size_t)L + 1);
						HIPCHK(hipMemcpy(o.gbase_d, o.gbase_h.data(), ((size_t)L + 1) * 4, hipMemcpyHostToDevice));
						o.pad_bad_d = dalloc<uint32_t>(nb);
					}
					o.lnx_off_d = dalloc<uint64_t>(L);
				}
			}
			{
				std::vector<uint64_t> cp((size_t)nf + 1), lv((size_t)nf + 1, 0);
				std::vector<uint32_t> feats(nf);
				HIPCHK(hipMemcpy(cp.data(), c->tr.col_ptr, cp.size() * 8, hipMemcpyDeviceToHost));
				if (nf) HIPCHK(hipMemcpy(feats.data(), c->level_feats, (size_t)nf * 4, hipMemcpyDeviceToHost));
				for (uint32_t i = 0; i < nf; i++) lv[i + 1] = lv[i] + (cp[feats[i] + 1] - cp[feats[i]]);
				o.lvcp = dalloc<uint64_t>(lv.size());
				HIPCHK(hipMemcpy(o.lvcp, lv.data(), lv.size() * 8, hipMemcpyHostToDevice));
			}
			o.rstart_d = dalloc<uint64_t>((size_t)nb + 1);
			c->q_ready[0] = c->q_ready[1] = -1;
			sync(c);
		} catch (...) {
			ov_free(c);
			throw;
		}
	});
}

int vbfm_online_epoch(vbfm_ctx *c, vbfm_online_stats *out)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (!c->ov) throw std::string("not an online VB context (vbfm_online_init)");
		OvState &o = *c->ov;
		vbfm_online_stats st;
		memset(&st, 0, sizeof(st));
		HIPCHK(hipMemsetAsync(c->counters, 0, CNT_N * 4, c->s));
		Range r_ep("vbfm_online_epoch");
		HIPCHK(hipEventRecord(o.ev[0], c->s));
		o.launches_v = 0;
		c->pev_used = 0;   // vbfm_set_profiling: the spans of this epoch only
		c->spans.clear();
		ov_regroup(c);
		HIPCHK(hipEventRecord(o.ev[1], c->s));
		const uint32_t nb = o.num_batch, nf = c->tr.nf;
		std::vector<uint64_t> eoff((size_t)nb + 1);
		for (uint32_t b = 0; b <= nb; b++)
			HIPCHK(d2h(c, &eoff[b], o.gptr + (size_t)b * nf, 8));
		sync(c);   // the permutation's copy to the device is done: draw the next one meanwhile
		ov_prefetch_shuffle(o);
		const DevData full = c->tr;
		RowRec *const rows_full = c->rows;
		const uint64_t n_global_full = c->n_global;
		auto restore = [&] {
			o.lord_on = false;
			o.pad_on = false;
			c->tr = full;
			c->rows = rows_full;
			c->n_global = n_global_full;
			c->q_ready[0] = c->q_ready[1] = -1;
		};
		try {
			for (uint32_t b = 0; b < nb; b++) {
				Range r_b("batch");
				hipEvent_t *bev = &o.bev[(size_t)b * 6];
				HIPCHK(hipEventRecord(bev[0], c->s));
				const uint32_t n = (uint32_t)(o.rstart[b + 1] - o.rstart[b]);
				const uint64_t nnz = eoff[b + 1] - eoff[b];
				ov_batch_capacity(c, n, nnz);
				const uint32_t *brows = o.rows_sorted + o.rstart[b];
				// the batch's CSR (rows ascending = the batch file's order)
				k_ov_rowlen<<<grid_of(n), 256, 0, c->s>>>(brows, n, full.row_ptr, o.len_b);
				HIPCHK(hipGetLastError());
				HIPCHK(hipMemsetAsync(o.len_b + n, 0, 8, c->s));
				size_t tb = 0;
				HIPCHK(vbk::exclusive_scan_u64(nullptr, &tb, o.len_b, o.rp_b, (size_t)n + 1, c->s));
				HIPCHK(vbk::exclusive_scan_u64(ov_tmp(o, tb), &tb, o.len_b, o.rp_b, (size_t)n + 1, c->s));
				k_ov_gather<<<grid_of(n, 4), 256, 0, c->s>>>(brows, n, full.row_ptr, full.csr, full.target, o.rp_b,
				                                            o.csr_b, o.t_b);
				HIPCHK(hipGetLastError());
				DevData bv = full;
				bv.n = n;
				bv.nnz = nnz;
				bv.col_ptr = o.gptr + (size_t)b * nf;
				bv.csc = o.ent_sorted;
				bv.row_ptr = o.rp_b;
				bv.csr = o.csr_b;
				bv.target = o.t_b;
				c->tr = bv;
				c->rows = o.rows_b;
				c->n_global = n;
				c->q_ready[0] = c->q_ready[1] = -1;
				// fresh caches of the batch (:111-139)
				const int bl = blocked_predict(c, c->tr);
				HIPCHK(vbk::predict_et(c->tr.row_ptr, c->tr.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, c->mu0, c->s0d,
				                       c->tr.target, c->scratch_n, c->rows, n, bl, c->s));
				o.lord_on = false;
				o.pad_on = false;
				if (o.batch_lord[b]) {
					ov_lord_begin(c, b, n, nnz);
					st.n_lord_batches++;
					if (o.pad_on) st.n_pad_batches++;
				}
				// update_all(train1, train.num_cases) (fm_learn_vb_online.h:354-469)
				HIPCHK(hipEventRecord(bev[1], c->s));
				if (c->k0) ov_step_w0(c);
				HIPCHK(hipEventRecord(bev[2], c->s));
				if (c->k1) step_w(c);
				HIPCHK(hipEventRecord(bev[3], c->s));
				if (c->D > 0) {
					for (int f = 0; f < c->k; f++) {
						step_qcache(c, f);
						step_v(c, f);
					}
					k_ov_steps<<<grid_of(c->D), 256, 0, c->s>>>(o.t_vj, o.new_vj, c->D);
					HIPCHK(hipGetLastError());
				}
				HIPCHK(hipEventRecord(bev[4], c->s));
				ov_step_hyper(c, &st.nan_alpha, &st.inf_alpha);
				// free energy of the first and the last batch (:143-146)
				if (b == 0 || b + 1 == nb) {
					const double fe = free_energy(c, rows_energy(c));
					if (b == 0) st.free_energy_first = fe;
					if (b + 1 == nb) st.free_energy_last = fe;
				}
				HIPCHK(hipEventRecord(bev[5], c->s));
				restore();
			}
		} catch (...) {
			restore();
			throw;
		}
		HIPCHK(hipEventRecord(o.ev[2], c->s));
		// test prediction and metrics (:190-245)
		test_predict(c, c->s);
		const double mn = c->min_target, mx = c->max_target;
		HIPCHK(vbk::test_metrics(c->e_test, c->te.target, c->te.n, mn, mx, c->pred_test, c->red_d, c->RED_BLOCKS, c->s));
		HIPCHK(d2h(c, c->red_h.data(), c->red_d, 2 * c->RED_BLOCKS * 8));
		HIPCHK(hipEventRecord(o.ev[3], c->s));
		sync(c);
		double tm[2] = {0.0, 0.0};
		for (uint32_t i = 0; i < c->RED_BLOCKS; i++) { tm[0] += c->red_h[2 * i]; tm[1] += c->red_h[2 * i + 1]; }
		st.rmse = std::sqrt(tm[0] / c->te.n);
		st.mae = tm[1] / c->te.n;
		st.alpha = c->alpha; st.sigma_0 = c->sigma_0; st.mu_0_dash = c->mu0; st.sigma_0_dash = c->s0d;
		vbfm_iter_stats it;
		memset(&it, 0, sizeof(it));
		read_counters(c, &it);
		st.nan_mu_w = it.nan_mu_w; st.nan_sigma_w = it.nan_sigma_w; st.inf_mu_w = it.inf_mu_w;
		st.nan_mu_v = it.nan_mu_v; st.nan_sigma_v = it.nan_sigma_v; st.inf_mu_v = it.inf_mu_v;
		st.num_batch = nb;
		st.num_levels = (int32_t)nlevels(c);
		float ms = 0.f;
		HIPCHK(hipEventElapsedTime(&ms, o.ev[0], o.ev[1])); st.ms_regroup = ms;
		HIPCHK(hipEventElapsedTime(&ms, o.ev[1], o.ev[2])); st.ms_batches = ms;
		HIPCHK(hipEventElapsedTime(&ms, o.ev[2], o.ev[3])); st.ms_test = ms;
		HIPCHK(hipEventElapsedTime(&ms, o.ev[0], o.ev[3])); st.ms_total = ms;
		double *ph[5] = {&st.ms_predict, &st.ms_w0, &st.ms_w, &st.ms_v, &st.ms_hyper};
		for (uint32_t b = 0; b < nb; b++)
			for (int q = 0; q < 5; q++) {
				HIPCHK(hipEventElapsedTime(&ms, o.bev[(size_t)b * 6 + q], o.bev[(size_t)b * 6 + q + 1]));
				*ph[q] += ms;
			}
		st.n_vlevel_launches = o.launches_v;
		st.nnz_train = c->tr.nnz;
		if (out) *out = st;
	});
}

int vbfm_online_get_state(vbfm_ctx *c, double *nat_mu_w, double *nat_sigma_w, double *nat_mu_v, double *nat_sigma_v,
                          double *new_wj, double *new_vj, double scalars[8])
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (!c->ov) throw std::string("not an online VB context (vbfm_online_init)");
		OvState &o = *c->ov;
		const size_t kd = (size_t)c->k * c->D;
		double *tmp = dalloc<double>(2 * std::max(kd, (size_t)c->D));
		HIPCHK(vbk::unpack_pairs(o.nat_w, tmp, tmp + c->D, 1, c->D, c->s));
		sync(c);
		if (nat_mu_w) HIPCHK(hipMemcpy(nat_mu_w, tmp, (size_t)c->D * 8, hipMemcpyDeviceToHost));
		if (nat_sigma_w) HIPCHK(hipMemcpy(nat_sigma_w, tmp + c->D, (size_t)c->D * 8, hipMemcpyDeviceToHost));
		if (kd) {
			HIPCHK(vbk::unpack_pairs(o.nat_v, tmp, tmp + kd, 1, kd, c->s));   // already [f][j]
			sync(c);
			if (nat_mu_v) HIPCHK(hipMemcpy(nat_mu_v, tmp, kd * 8, hipMemcpyDeviceToHost));
			if (nat_sigma_v) HIPCHK(hipMemcpy(nat_sigma_v, tmp + kd, kd * 8, hipMemcpyDeviceToHost));
		}
		dfree(tmp);
		if (new_wj) HIPCHK(hipMemcpy(new_wj, o.new_wj, (size_t)c->D * 8, hipMemcpyDeviceToHost));
		if (new_vj) HIPCHK(hipMemcpy(new_vj, o.new_vj, (size_t)c->D * 8, hipMemcpyDeviceToHost));
		if (scalars) {
			const double s[8] = {c->alpha, c->sigma_0, c->mu0, c->s0d, o.nat_mu0, o.nat_sig0, o.new_w0, (double)o.t_w0};
			memcpy(scalars, s, sizeof(s));
		}
	});
}

}  // extern "C"

// ---- checkpoint / resume of the online learner (vbfm_save_state / vbfm_load_state) ----------
// Between two epochs the online learner's state is the parameters, the hyper parameters and the
// four scalars (as VB's), the natural parameters and step sizes of every attribute and of w0
// (fm_learn_vb_online.h:686-758), and the epoch shuffle's inputs: the reference's rand() stream
// (its 31-word window) and the last permutation (the reference keeps it across epochs,
// fm_learn_vb_online_simultaneous.h:58-62). A batch's row caches are predicted afresh from the
// parameters (:111-139), so no records are kept. The next epoch's permutation, drawn ahead on a
// host thread, is not saved: the resumed context draws it from the same stream and permutation.
namespace vbi {

namespace {
constexpr size_t OV_HEAD_WORDS = 8 + 32;   // {num_batch, n_total, t_w0, 0...}, stream window + pad
}

bool ov_store_on(vbfm_ctx *c) { return c->ov && c->ov->level_ptr_d != nullptr; }

uint64_t ov_state_payload(vbfm_ctx *c)
{
	const uint64_t D = c->D, kd = (uint64_t)c->k * c->D, G = c->G, gk = G * (uint64_t)c->k;
	return OV_HEAD_WORDS * 4 + (uint64_t)c->tr.n * 4 + D * 16 + kd * 16 + (G + gk) * 8 + 4 * 8 + D * 16 + kd * 16 +
	       D * 8 * 2 + D * 4 * 2 + 3 * 8;
}

void ov_state_write(vbfm_ctx *c, CkptFile &f)
{
	OvState &o = *c->ov;
	// a prefetch thread still drawing the next permutation only reads the stream and the
	// permutation saved here (it writes sh_next / stream_next): no join, the draw stays usable
	uint32_t w[OV_HEAD_WORDS] = {};
	w[0] = o.num_batch; w[1] = o.n_total; w[2] = o.t_w0;
	o.stream.chrono_state(w + 8);
	f.write(w, sizeof(w));
	f.write(o.shuffle.data(), (size_t)o.n_total * 4);
	const size_t D = c->D, kd = (size_t)c->k * c->D;
	dev_to_file(c, f, c->ms_w, D * sizeof(double2));
	dev_to_file(c, f, c->ms_v, kd * sizeof(double2));
	f.write(c->hyp_w.data(), c->hyp_w.size() * 8);
	f.write(c->hyp_v.data(), c->hyp_v.size() * 8);
	const double sc[4] = {c->alpha, c->sigma_0, c->mu0, c->s0d};
	f.write(sc, sizeof(sc));
	dev_to_file(c, f, o.nat_w, D * sizeof(double2));
	dev_to_file(c, f, o.nat_v, kd * sizeof(double2));
	dev_to_file(c, f, o.new_wj, D * 8);
	dev_to_file(c, f, o.new_vj, D * 8);
	dev_to_file(c, f, o.t_wj, D * 4);
	dev_to_file(c, f, o.t_vj, D * 4);
	const double os[3] = {o.nat_mu0, o.nat_sig0, o.new_w0};
	f.write(os, sizeof(os));
}

void ov_state_read(vbfm_ctx *c, CkptFile &f)
{
	OvState &o = *c->ov;
	uint32_t w[OV_HEAD_WORDS];
	f.read(w, sizeof(w));
	if (w[0] != o.num_batch || w[1] != o.n_total)
		throw std::string("checkpoint of another mini-batch split (-batch): resume with the same num_batch");
	o.pre_join();   // a permutation drawn ahead from the state being replaced is dropped
	o.sh_next.clear();
	f.read(o.shuffle.data(), (size_t)o.n_total * 4);
	o.stream.set_chrono_state(w + 8);
	o.t_w0 = w[2];
	const size_t D = c->D, kd = (size_t)c->k * c->D;
	file_to_dev(c, f, c->ms_w, D * sizeof(double2));
	file_to_dev(c, f, c->ms_v, kd * sizeof(double2));
	f.read(c->hyp_w.data(), c->hyp_w.size() * 8);
	f.read(c->hyp_v.data(), c->hyp_v.size() * 8);
	upload_hyp(c);
	double sc[4];
	f.read(sc, sizeof(sc));
	c->alpha = sc[0]; c->sigma_0 = sc[1]; c->mu0 = sc[2]; c->s0d = sc[3];
	file_to_dev(c, f, o.nat_w, D * sizeof(double2));
	file_to_dev(c, f, o.nat_v, kd * sizeof(double2));
	file_to_dev(c, f, o.new_wj, D * 8);
	file_to_dev(c, f, o.new_vj, D * 8);
	file_to_dev(c, f, o.t_wj, D * 4);
	file_to_dev(c, f, o.t_vj, D * 4);
	double os[3];
	f.read(os, sizeof(os));
	o.nat_mu0 = os[0]; o.nat_sig0 = os[1]; o.new_w0 = os[2];
}

}  // namespace vbi
