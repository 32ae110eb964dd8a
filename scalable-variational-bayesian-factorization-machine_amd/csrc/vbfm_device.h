// vbfm_device.h -- device-side data layout shared by the kernels and the C-ABI layer.
//
// HBM layout (one context = one GPU = one row shard):
//   RowRec rows[N]      64-B aligned record per train row: the reference's two row caches
//                       e_q_term{e,q} (fm_learn_mcmc.h:52-55) and t_term{t,q,z}
//                       (fm_learn_vb.h:17-21) fused so that one 64-B line serves every
//                       gather of a row, plus a second q-cache slot: while factor f is swept
//                       from slot f%2, the q-cache of factor f+1 is accumulated into slot
//                       (f+1)%2 (the levels visit a row's features in ascending order, the
//                       order of add_main_q, so the fused sum is bit-exact).
//   CSC  col_ptr[nf+1] (u64), csc[nnz] (uint2 = {row, fp32 bits}) == sparse_entry<float>;
//                       bit 31 of the row id marks the entry that is its row's first
//                       (smallest-feature) entry: where the fused q-cache sum starts.
//   CSR  row_ptr[N+1]  (u64), csr[nnz] (uint2 = {feature, fp32 bits}), each row sorted by
//                       feature id: the order in which the reference's column-major loops
//                       visit a row, so per-row sums are bit-identical to the reference.
//   ms_v[D*k] (double2 = {mu, sigma}) of mu_v_dash/sigma_v_dash, FEATURE-major:
//             ms_v[j*k + f]; all factors of a feature are contiguous, so a prediction reads
//             one run per entry and mu_{f+1}[j] shares the line of mu_f[j];
//   ms_w[D]   (double2 = {mu, sigma}) of mu_w_dash/sigma_w_dash.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>

// The longest mean column of a level swept with the 64-thread x 2 workgroup shape (longer: see
// dispatch_shape). Every level kernel -- fused, deferred split, column-gather, entry store,
// MCMC -- takes its shape from the same thresholds: the same shape gives the same reduction tree,
// so the layouts and the fused / split forms stay bit-identical to each other. 128: a level of
// C4's per-rank shard on 8 GPUs (columns of ~100 entries) runs 2-5 % faster in the deferred split
// form with 64 x 2 than with 256 x 1 (one wave per column: more columns, and so more posterior
// gathers, in flight per CU; profiles/r05_split/), ~1-2 % slower fused -- a shape that only a
// row-sharded run meets among the BASELINE configurations (profiles/probes/ab_defer_small_shape.txt).
// VBFM_SMALL_MAX overrides (A/B).
inline uint32_t shape_small_max()
{
	static const uint32_t v = [] {
		const char *e = getenv("VBFM_SMALL_MAX");
		return e ? (uint32_t)atoi(e) : 128u;
	}();
	return v;
}

// A level's workgroup shape: BLOCK threads per column, R records per thread staged in LDS
// (CAP = BLOCK x R; a longer run is swept in chunks of CAP). f(BLOCK, R) is called with the shape
// as std::integral_constant values, so every kernel family launches its own template from one
// table. The reduction tree of a column depends on BLOCK only.
//   mean column <= shape_small_max():  64 x 2  (CAP 128)
//               <= 200:               256 x 1  (CAP 256)
//               <= 384:               128 x 3  (CAP 384: ~3 standard deviations above the mean
//                                     stay resident; 26 KB of LDS, 6 workgroups per CU, so a
//                                     level of <= 1,536 columns runs in one round. Multi-hot
//                                     bench +6 % against 256 x 2, field data of 250-entry columns
//                                     +2 % against 256 x 1: profiles/r05_multihot/shape_ab/)
//               <= 640:               256 x 2  (CAP 512)
//               longer:               512 x 2  (CAP 1024)
template <class F> inline void dispatch_shape(uint32_t avg, F &&f)
{
	typedef std::integral_constant<int, 64> B64;
	typedef std::integral_constant<int, 128> B128;
	typedef std::integral_constant<int, 256> B256;
	typedef std::integral_constant<int, 512> B512;
	typedef std::integral_constant<int, 1> R1;
	typedef std::integral_constant<int, 2> R2;
	typedef std::integral_constant<int, 3> R3;
	if (avg <= shape_small_max()) f(B64(), R2());
	else if (avg <= 200) f(B256(), R1());
	else if (avg <= 384) f(B128(), R3());
	else if (avg <= 640) f(B256(), R2());
	else f(B512(), R2());
}

// the BLOCK of dispatch_shape (kernels that take no R)
inline int shape_block(uint32_t avg)
{
	int b = 0;
	dispatch_shape(avg, [&](auto B, auto) { b = B(); });
	return b;
}

struct __attribute__((aligned(64))) RowRec {
	double e;    // cache[i].e      residual y - yhat (fm_learn_vb_simultaneous.h:42-44)
	double q;    // cache[i].q      q-cache slot 0: sum mu x
	double tq;   // cache_t[i].q    slot 0: sum sigma x^2
	double tz;   // cache_t[i].z    slot 0: sum mu^2 x^2
	double t;    // cache_t[i].t    variance term T_n (paper eq. 26)
	double q1, tq1, tz1;   // q-cache slot 1
};
#define ROW_MASK 0x7FFFFFFFu
#define ROW_FIRST 0x80000000u
static_assert(sizeof(RowRec) == 64, "RowRec must be one 64-B line");

enum {
	CNT_NAN_MU_W = 0, CNT_NAN_SIGMA_W, CNT_INF_MU_W,
	CNT_NAN_MU_V, CNT_NAN_SIGMA_V, CNT_INF_MU_V,
	CNT_RNG_SKIP,   // MCMC: draws not taken (non-finite or zero variance)
	CNT_N
};

// posterior of one feature of a level, as its entries' deferred correction needs it
// (row-sharded split on the level-ordered store): mu = NaN marks a skipped correction
struct __attribute__((aligned(32))) PostT {   // 32 B: two entries per 64-B line
	double mo, so, mu, sig;
};

// per-level launch description for the v / w sweeps
// a segment of a long column of one level (index of the column in the level's feature list,
// first entry and length within the column's run, the column's first segment and count)
struct LongSeg {
	uint32_t col, start, len, seg0, nseg;
};

struct LevelArgs {
#ifdef VBFM_OV_STAMPS
	unsigned long long *stamp;   // diagnostic build only (tools/ov_stamps.sh): per-workgroup phase stamps
#endif
	const uint64_t *col_ptr;
	const uint2 *csc;
	const uint32_t *feats;     // features of this level (ascending id)
	uint32_t nfeat;
	int feat_contig;           // the level's features are consecutive ids: feature i = feat_base + i
	uint32_t feat_base;        // (no feats[] load on the workgroup's path; field-structured data)
	RowRec *rows;
	double2 *ms;               // ms_v + f (stride k), or ms_w (stride 1)
	uint32_t ms_stride;
	const double *hyp;         // hyper prior: sigma_v(g, f) at hyp[g*stride], or sigma_w(g)
	uint32_t hyp_stride;
	const uint32_t *attr_group;
	const uint8_t *dup;        // column has a repeated row (sequential correction)
	double alpha;
	uint32_t *counters;
	double2 *stats;            // split mode: per-level-feature (sum1, sum2), or nullptr
	const double2 *ms_next;    // {mu, sigma} of factor f+1 (fused q-cache, stride ms_stride_next), or nullptr
	uint32_t ms_stride_next;
	int slot;                  // q-cache slot of the factor being swept (v) / of factor 0 (w)
	uint32_t avg_len;          // mean column length of the level (launch shape)
	uint32_t first_mask;       // ROW_FIRST: the fused q-cache restarts at a row's first entry;
	                           // 0 (feature shards): partial sums from a zeroed slot
	// level-ordered row store (vbfm_lorder.hip); unused by the column-gather kernels
	const uint64_t *lcp;       // global position of each level feature's run, indexed like feats [nfeat+1]
	const float *lx;           // x of every level-ordered entry (global position)
	const uint32_t *lnext;     // position of the entry's row in the next level's order
	uint64_t lbase;            // global position of the level's first entry (= level * rows)
	const RowRec *src;         // records in this level's order
	RowRec *dst;               // records in the next level's order
	int first_level;           // level 0: every row's smallest feature (q-cache restart)
	int ent;                   // the entry store: src == dst, lnext bit 31 = the row's first entry
	// deferred correction (row-sharded split on the level-ordered store)
	const uint32_t *lpidx;     // the entry's row: index of its previous-level feature in that level
	const float *lpx;          // ... and that entry's x
	PostT *tab;                // posteriors of the previous level (read) / of this level (written)
	const uint4 *lpay;         // {x bits, lnext, lpidx, lpx bits} per level-ordered entry (deferred split)
	const uint2 *lpay2;        // ... {lnext, lpidx} instead when every x is 1 (lpay null)
	int pending;               // bit 0: apply the previous level's correction first; bit 1: non-temporal record loads; bit 2: ... stores
	int first_prev;            // the previous level is level 0 (q-cache restart of its entries)
	int pend_kind;             // level 0 of a v sweep: the pending correction is the previous sweep's last
	                           // level (1: v of the other q-cache slot, 2: w); 0: this sweep's own
	uint32_t tab_base;         // the entry store: post writes tab[tab_base + i] (a table over every level
	                           // feature, tab_base = the level's first), the kernels read tab[global index]
	const uint32_t *lfirst;    // the entry store's flush: each row's first slot (nnz + r: no entries)
	uint64_t ent_nnz;          // ... and the number of entry slots
	// online VB (vbfm_online.hip): natural-gradient steps on a mini-batch; nat == nullptr: VB
	double2 *nat;              // natural parameters {mu, sigma} of each feature: nat[j * nat_stride]
	uint32_t nat_stride;       // 1: factor-major (nat_v + f * D), so a level's columns read one run
	double *rho;               // step size of each feature (new_wj / new_vj)
	const uint32_t *ccount;    // entries of each feature in the whole train set (col_count)
	uint32_t *tcount;          // w: t_wj (+= batch entries, rho refreshed); v of factor 0: t_vj; else nullptr
	int x_one;                 // online per-batch store: every train x is 1.0f (no per-entry x load)
	uint32_t pad_cap;          // online per-batch store, levels >= 1: workgroup w's run sits at record
	                           // w * pad_cap of the level's buffer (no column-bound load before the
	                           // run's loads); 0: runs packed (positions from the column bounds)
	int ov_fast;               // ... and a v level may take k_ov_lord's tagged-argument form
	// level-ordered store: the next level's column bounds (and feature list, or null), whose lines
	// each workgroup of this level touches once so that the next launch finds them in its L2
	const uint64_t *pf_lcp;
	const uint32_t *pf_feats;
	uint32_t pf_n;
	int hyp_uniform;           // one attribute group: the prior is hyp0 (no per-column lookup)
	double hyp0;
	// long columns of the level-ordered store (fused single-rank VB sweep): columns longer than
	// long_min are left by k_level_lord to segment workgroups (statistics partials, then a
	// posterior from the partials and the move); 0: none
	uint32_t long_min;
	const LongSeg *segs;       // the level's segments
	uint32_t nsegs;
	double2 *seg_part;         // per segment: (sum1, sum2), then the column's old {mu, sigma}
	int skew;                  // VBFM_DEBUG_SKEW (debug_skew)
};

// per-level launch description for the MCMC / ALS draws (vbfm_mcmc.hip); parameters are
// kept as double2 {value, 0} in the same feature-major layout as ms_v / ms_w so that the
// prediction kernels serve both learners
struct McArgs {
	const uint64_t *col_ptr;
	const uint2 *csc;
	const uint32_t *feats;
	uint32_t nfeat;
	int feat_contig;           // as LevelArgs
	uint32_t feat_base;
	RowRec *rows;
	double2 *par;              // v_f (at f, stride k) or w (stride 1)
	uint32_t stride;
	const double2 *par_next;   // v_{f+1} / v_0 for the fused q-cache, or nullptr
	uint32_t next_stride;
	const double *lambda;      // prior precision of (group g): lambda[g*hstride]
	const double *mu;          // prior mean of (group g): mu[g*hstride]
	uint32_t hstride;
	int hyp_uniform;           // one attribute group: the prior is {lambda0, mu0} by value
	double lambda0, mu0;
	const uint32_t *attr_group;
	const uint8_t *dup;
	double alpha;
	const double *z;           // reference-RNG mode: standard normal of feature j, or nullptr
	uint64_t rng_seed;         // device-RNG mode: counter-based normals keyed (seed, stream, j)
	uint64_t rng_stream;
	int sample;                // 0: ALS (conditional mean), 1: MCMC (draw)
	uint32_t *counters;
	double2 *stats;            // row-sharded mode: per-level-feature (sum h*e, sum h^2), or nullptr
	int slot;
	uint32_t avg_len;
	// level-ordered row store (as LevelArgs)
	const uint64_t *lcp;
	const float *lx;
	const uint32_t *lnext;
	uint64_t lbase;
	const RowRec *src;
	RowRec *dst;
	int first_level;
	// deferred correction (row-sharded split, as LevelArgs): the previous level's draws
	const uint32_t *lpidx;
	const float *lpx;
	PostT *tab;                // {mo = old value, mu = drawn value or NaN (no correction)}
	const uint4 *lpay;         // as LevelArgs::lpay
	const uint2 *lpay2;        // as LevelArgs::lpay2
	int pending;               // bit 0: apply the previous level's correction; bit 1: nt loads
	// the train re-prediction of draw_all's end (fm_learn_mcmc.h:117-348) accumulated inside the
	// v sweeps: while factor f is swept, v_{f-1} is final, so every entry the sweep visits adds
	// its factor-(f-1) terms to the row's record (mc_pred_acc); pk: 0 off, 1 sweep of factor 1
	// (the accumulators start), 2 a later factor; par_prev = v_{f-1} (stride next_stride)
	const double2 *par_prev;
	int pk;
	int ent;                   // the entry store (as LevelArgs::ent; fused sweeps only)
	int skew;                  // VBFM_DEBUG_SKEW (debug_skew)
};

// VBFM_DEBUG_SKEW=1 (tests/test_skew_gpu.py): in the kernels that read a column's parameter, then
// write its new value from one thread with no reduction between the two -- the split forms'
// posterior / draw kernels -- every wave but a workgroup's first sleeps ~50 us before it reads the
// old value. A missing barrier between the waves' reads and the write then shows on every run
// (the late waves read the new value as "old"), not on a lucky one; with the barrier the result
// is unchanged. The fused kernels reduce their statistics over the workgroup (a barrier) between
// the read and the write by construction. The compiler barrier keeps the read after the sleep.
__device__ __forceinline__ void debug_skew(int on)
{
	if (on && threadIdx.x >= 64) {
		for (int i = 0; i < 16; i++) __builtin_amdgcn_s_sleep(127);
		__asm__ __volatile__("" ::: "memory");
	}
}

// kernels launched from the C-ABI layer (vbfm_kernels.hip)
namespace vbk {
// test hook of the exchange's deadline (VBFM_FAULT=comm_stall): one wave that spins until *flag
// (coherent host memory) turns non-zero, at most ~100 s
hipError_t stall(const uint32_t *flag, hipStream_t s);
hipError_t v_level_fused(const LevelArgs &a, hipStream_t s);
hipError_t w_level_fused(const LevelArgs &a, hipStream_t s);
hipError_t v_level_stats(const LevelArgs &a, hipStream_t s);
hipError_t v_level_correct(const LevelArgs &a, hipStream_t s);
hipError_t w_level_stats(const LevelArgs &a, hipStream_t s);
hipError_t w_level_correct(const LevelArgs &a, hipStream_t s);
// pos: nullptr, or the record index of each row (level-ordered store: level-0 position)
hipError_t qcache(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_f, uint32_t stride, RowRec *rows,
                  uint32_t n, int slot, const uint32_t *pos, hipStream_t s);
// level-ordered row store (vbfm_lorder.hip): fused level, or split stats -> (all-reduce) -> move
hipError_t lord_level(const LevelArgs &a, int is_w, hipStream_t s);
// the long columns of a fused level (a.nsegs segments): statistics partials, then posterior + move
hipError_t lord_long(const LevelArgs &a, int is_w, hipStream_t s);
// the same for the column-gather layout's fused sweep (vbfm_kernels.hip)
hipError_t col_long(const LevelArgs &a, int is_w, hipStream_t s);
hipError_t lord_level_stats(const LevelArgs &a, int is_w, hipStream_t s);
hipError_t lord_level_move(const LevelArgs &a, int is_w, hipStream_t s);
// deferred form of the split (one pass over the records per level): previous level's
// correction + this level's statistics + move; posteriors into the table; final correction
hipError_t lord_defer_level(const LevelArgs &a, int is_w, hipStream_t s);
hipError_t lord_defer_post(const LevelArgs &a, int is_w, hipStream_t s);
hipError_t lord_defer_flush(const LevelArgs &a, int is_w, uint32_t n, hipStream_t s);
hipError_t lord_prev_map(const uint32_t *feats, uint32_t nfeat, const uint64_t *col_ptr, const uint2 *csc,
                         const float *dummy, uint32_t *prev_i, float *prev_x, hipStream_t s);
hipError_t lord_prev_fill(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, const uint64_t *col_ptr,
                          const uint2 *csc, const uint32_t *prev_i, const float *prev_x, uint32_t *lpidx, float *lpx,
                          hipStream_t s);
hipError_t lord_pos(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, uint64_t lbase, const uint64_t *col_ptr,
                    const uint2 *csc, uint32_t *pos, hipStream_t s);
hipError_t lord_fill(const uint32_t *feats, uint32_t nfeat, const uint64_t *lcp, uint64_t lbase, const uint64_t *col_ptr,
                     const uint2 *csc, const uint32_t *pos_next, float *lx, uint32_t *lnext, uint32_t *row0,
                     hipStream_t s);
// dst[p] = src[idx[p]] / dst[idx[p]] = src[p]
hipError_t rows_gather(RowRec *dst, const RowRec *src, const uint32_t *idx, uint32_t n, hipStream_t s);
// lpay[p] = {lx[p], lnext[p], lpidx[p], lpx[p]}
// entries of a CSC whose x is not 1.0f: *cnt = 0 iff every x is 1 (count of waves that saw one)
hipError_t count_x_ne1(const uint2 *csc, uint64_t nnz, uint32_t *cnt, hipStream_t s);
// lpay2[p] = {lnext[p], lpidx[p]} (every x 1)
hipError_t lord_pack2(const uint32_t *lnext, const uint32_t *lpidx, uint2 *lpay2, uint64_t nnz, hipStream_t s);
hipError_t lord_pack(const float *lx, const uint32_t *lnext, const uint32_t *lpidx, const float *lpx, uint4 *lpay,
                     uint64_t nnz, hipStream_t s);
// the entry store (levels that miss rows): per train row its entries' slots -> lnext [nnz] (bit 31:
// the row's first entry), lx [nnz] (or null), lfirst [n] (a row without entries: nnz + r);
// lvpos[j] = level position of feature j
hipError_t estore_build(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, const uint2 *csc,
                        const uint32_t *lvpos, const uint64_t *lcp, uint32_t n, uint64_t nnz, uint32_t *lnext,
                        float *lx, uint32_t *lfirst, hipStream_t s);
hipError_t estore_prev(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, const uint2 *csc,
                       const uint32_t *lvpos, const uint64_t *lcp, uint32_t n, uint32_t *lpidx, float *lpx, hipStream_t s);
hipError_t rows_scatter(RowRec *dst, const RowRec *src, const uint32_t *idx, uint32_t n, hipStream_t s);
// the level pattern without arithmetic: level 0's runs (lcp, nfeat columns) moved whole to their
// level-1 slots (lnext), src -> dst (placement probe of a record-buffer pair)
hipError_t place_move(const RowRec *src, RowRec *dst, const uint64_t *lcp, const uint32_t *lnext, uint32_t nfeat,
                      hipStream_t s);
hipError_t mark_first(const uint64_t *row_ptr, const uint2 *csr, const uint64_t *col_ptr, uint2 *csc,
                      uint32_t n, hipStream_t s);
// blocked = 0: the reference's summation order (bit-exact); 1: factors in blocks of 8
// (exact per-factor sums, the -1/2 sum v^2 x^2 term summed block-major: ~1 ulp apart);
// 2: one wave per row, lanes over factors (exact per-factor sums, cross-factor sums in a
// butterfly: ~1 ulp apart; k <= 256, else the blocked form)
hipError_t predict_e(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w,
                     int k, int k1, int k0, double mu0, double *out_e, uint32_t n, int blocked,
                     hipStream_t s);
hipError_t predict_t(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w,
                     int k, int k1, int k0, double sigma0_dash, RowRec *rows, uint32_t n, int blocked,
                     hipStream_t s);
hipError_t residual_init(RowRec *rows, const double *yhat, const float *target, uint32_t n, hipStream_t s);
// predict_e reading the factors' mu from a compact [j*k + f] copy vc (kd = k*D doubles; refresh:
// copy it from ms_v first); falls back to predict_e where the wave form does not apply
hipError_t predict_e_compact(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k,
                             int k1, int k0, double mu0, double *out, uint32_t n, int blocked, double *vc, size_t kd,
                             bool refresh, hipStream_t s);
hipError_t predict_et(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k, int k1,
                      int k0, double mu0, double s0d, const float *target, double *scratch, RowRec *rows, uint32_t n,
                      int blocked, hipStream_t s);
// per-block partial sums over rows; mode 0: e + mu0 ; mode 1: e*e + t ; out[nblocks]
hipError_t row_sums(const RowRec *rows, uint32_t n, int mode, double mu0, double *out, uint32_t nblocks,
                    hipStream_t s);
hipError_t w0_apply(RowRec *rows, uint32_t n, double de, double dt, hipStream_t s);
// test metrics: per block (sum err^2, sum |err|) of clipped predictions, and pred_this
hipError_t test_metrics(const double *e_test, const float *target, uint32_t n, double mn, double mx,
                        double *pred, double *out, uint32_t nblocks, hipStream_t s);
// train quirk: per block sum clip(e)^2
hipError_t train_quirk(const RowRec *rows, uint32_t n, double mn, double mx, double *out, uint32_t nblocks,
                       hipStream_t s);
// hyper-parameter / free-energy partial sums over attribute chunks (see vbfm_capi.hip)
struct Chunk { uint32_t begin, end; int32_t f; uint32_t g; };
hipError_t param_sums(const double2 *ms_w, const double2 *ms_v, const uint32_t *perm, uint32_t D,
                      const Chunk *chunks, uint32_t nchunks, int mode, const double *hyp_w,
                      const double *hyp_v, int k, double *out, hipStream_t s);
// the factors' segment sums in one coalesced pass over ms_v: chunks of one group's attributes
// (Chunk::f unused), gchunk[G+1] = each group's chunk range; part[nchunks * k] per-chunk
// partials, seg[f * G + g] the sums. model 0: VB (param_sums' modes), 1: MCMC (mc_param_sums')
hipError_t vsums(const double2 *ms_v, const uint32_t *perm, const Chunk *chunks, uint32_t nchunks,
                 const uint32_t *gchunk, uint32_t G, int model, int mode, const double *hv, int k, double *part,
                 double *seg, hipStream_t s);
// *out += an order-independent fingerprint of n words of 4 or 8 bytes (checkpoint data check)
hipError_t fingerprint(const void *a, uint64_t n, int word_bytes, uint64_t salt, unsigned long long *out,
                       hipStream_t s);
// level schedule
hipError_t level_init(uint32_t *level, uint32_t nf, hipStream_t s);
hipError_t level_relax(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t nf, uint32_t *level,
                       uint32_t *changed, hipStream_t s);
hipError_t mark_dups(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint8_t *dup, hipStream_t s);
// the same levels in Kahn's order: edge counts + the level-1 frontier (bounds[0..1]), then one
// frontier per round (round t: level t+1 in order[bounds[t]..bounds[t+1]), closes bounds[t+2])
hipError_t kahn_init(const uint64_t *row_ptr, const uint2 *csr, uint32_t n, uint32_t nf, uint32_t *indeg,
                     uint32_t *level, uint32_t *order, uint32_t *tail, uint32_t *bounds, hipStream_t s);
hipError_t kahn_round(const uint64_t *col_ptr, const uint2 *csc, const uint64_t *row_ptr, const uint2 *csr,
                      uint32_t *bounds, int t, uint32_t *indeg, uint32_t *level, uint32_t *order, uint32_t *tail,
                      hipStream_t s);
// feature-sharded passes (vbfm_capi.hip fs_pass): save e/t and zero the next q-cache slot;
// pack (or add) the shard's changes; unpack the summed changes; parameter exchange
hipError_t fs_begin(RowRec *rows, uint32_t n, double *base, int next_slot, hipStream_t s);
hipError_t fs_pack(const RowRec *rows, uint32_t n, const double *base, double *buf, int next_slot, int acc,
                   hipStream_t s);
hipError_t fs_unpack(RowRec *rows, uint32_t n, const double *base, const double *buf, int next_slot, hipStream_t s);
hipError_t fs_params(double2 *ms, uint32_t stride, const uint32_t *feats, uint32_t nfeat, double2 *pbuf, int to_buf,
                     hipStream_t s);
// synthetic generator (tests/synth.py is the specification)
hipError_t synth_csr(uint32_t n, uint32_t F, uint32_t S, uint64_t seed, int xmode, uint64_t model_seed,
                     uint64_t row0, uint64_t *row_ptr, uint2 *csr, float *target, hipStream_t s);
hipError_t synth_field_keys(const uint2 *csr, uint32_t n, uint32_t F, uint32_t S, uint32_t field,
                            uint32_t *keys, uint32_t *vals, hipStream_t s);
hipError_t synth_field_scatter(const uint32_t *sorted_rows, const uint2 *csr, uint32_t n, uint32_t F,
                               uint32_t field, uint2 *csc_field, hipStream_t s);
hipError_t synth_mh_len(uint32_t n, uint32_t lo, uint32_t hi, uint64_t seed, uint64_t row0, uint64_t *len,
                        hipStream_t s);
hipError_t synth_mh_fill(uint32_t n, uint32_t D, uint64_t seed, int xmode, uint64_t model_seed, uint64_t row0,
                         const double *gains, uint32_t lo, const uint64_t *row_ptr, uint2 *csr, uint32_t *row_of,
                         float *target, hipStream_t s);
hipError_t mh_keys(const uint2 *csr, uint64_t nnz, uint32_t *keys, uint32_t *vals, hipStream_t s);
hipError_t synth_mh_scatter(const uint32_t *sorted_p, const uint2 *csr, const uint32_t *row_of, uint64_t nnz,
                            uint2 *csc, hipStream_t s);
hipError_t count_features(const uint2 *csr, uint64_t nnz, uint64_t *counts, hipStream_t s);
// schedule check: owner[n] preset to ~0; *bad counts rows claimed by two columns of the level
hipError_t check_level(const uint32_t *feats, uint32_t nfeat, const uint64_t *col_ptr, const uint2 *csc,
                       const uint8_t *dup, uint32_t *owner, uint32_t *bad, hipStream_t s);
// row copy (row_ptr [n+1], feature-sorted csr [nnz]) of a CSC data set, built on the device
hipError_t build_csr(const uint64_t *col_ptr, const uint2 *csc, uint32_t nf, uint32_t n, uint64_t nnz,
                     uint64_t *row_ptr, uint2 *csr, hipStream_t s);
hipError_t sort_pairs_u32(void *tmp, size_t *tmp_bytes, const uint32_t *ki, uint32_t *ko, const uint32_t *vi,
                          uint32_t *vo, size_t n, int bits, hipStream_t s);
hipError_t exclusive_scan_u64(void *tmp, size_t *tmp_bytes, const uint64_t *in, uint64_t *out, size_t n,
                              hipStream_t s);
// ms[i] = {scale * N(0,1), second}, counter-based (seed, stream, i)
hipError_t init_normal_pairs(double2 *ms, size_t n, uint64_t seed, uint64_t stream, double scale, double second,
                             hipStream_t s);
// layout conversion between the reference's separate mu/sigma arrays ([f][j], f rows of
// D) and the device's feature-major double2 pairs ([j][f]); rows = 1 for the w arrays
hipError_t pack_pairs(const double *a, const double *b, double2 *out, uint32_t rows, size_t D, hipStream_t s);
hipError_t unpack_pairs(const double2 *in, double *a, double *b, uint32_t rows, size_t D, hipStream_t s);
// online VB (vbfm_online.hip): one level of the w / v sweep on a mini-batch (column layout)
hipError_t ov_level(const LevelArgs &a, int is_w, hipStream_t s);
// the same on the batch's level-ordered store (a.src / a.dst / a.lnext / a.lbase)
hipError_t ov_lord_level(const LevelArgs &a, int is_w, hipStream_t s);
// lanes per column of that kernel for a batch mean column length m; its padded slot size
uint32_t ov_lord_g(uint32_t m);
uint32_t ov_pad_cap();
// MCMC / ALS (vbfm_mcmc.hip); mode 0: fused, 1: statistics only (into a.stats),
// 2: draw + correction from the (all-reduced) a.stats
hipError_t mc_v_level(const McArgs &a, int mode, hipStream_t s);
hipError_t mc_w_level(const McArgs &a, int mode, hipStream_t s);
hipError_t mc_prior(const McArgs &a, uint32_t j0, uint32_t j1, int is_v, hipStream_t s);
hipError_t mc_qcache(const uint64_t *row_ptr, const uint2 *csr, const double2 *par_f, uint32_t stride, RowRec *rows,
                     uint32_t n, int slot, const uint32_t *pos, hipStream_t s);
// MCMC / ALS level on the level-ordered store; mode as mc_v_level (2 = draw + move)
hipError_t mc_lord_level(const McArgs &a, int mode, int is_w, hipStream_t s);
// MCMC / ALS deferred split on the level-ordered store: level l-1's correction, level l's
// statistics and the move in one pass; the draws after the all-reduce; the sweep's last correction
hipError_t mc_lord_defer_level(const McArgs &a, int is_w, hipStream_t s);
hipError_t mc_lord_defer_post(const McArgs &a, int is_w, hipStream_t s);
hipError_t mc_lord_defer_flush(const McArgs &a, int is_w, uint32_t n, hipStream_t s);
// per-block sums over rows; mode 0: e*e ; mode 1: e - w0
hipError_t mc_row_sums(const RowRec *rows, uint32_t n, int mode, double w0, double *out, uint32_t nblocks,
                       hipStream_t s);
// the end of the fused train re-prediction: the last factor's and the w terms from the rows'
// entries, yhat[row] = E + Q2 (+ w0) (mc_train_update follows); pk_done: the v sweeps
// accumulated factors 0..k-2 into the records; scratch [2 * D] receives compact copies of the
// last factor's v and of w
hipError_t mc_pred_final(const uint64_t *row_ptr, const uint2 *csr, const double2 *ms_v, const double2 *ms_w, int k,
                         int k1, int k0, double w0, int pk_done, const RowRec *rows, const uint32_t *pos, uint32_t n,
                         uint32_t D, double *scratch, double *yhat, hipStream_t s);
hipError_t mc_e_shift(RowRec *rows, uint32_t n, double d, hipStream_t s);
hipError_t mc_train_update(RowRec *rows, const double *yhat, const float *target, uint32_t n, double mn, double mx,
                           double *out, uint32_t nblocks, const uint32_t *pos, hipStream_t s);
// per block: (sum err_this^2, sum |err_this|, sum err_all^2, sum |err_all|) at out[4*b]
hipError_t mc_test_update(const double *e_test, const float *target, uint32_t n, double mn, double mx,
                          double inv_iters, double *pred_this, double *pred_sum, double *out, uint32_t nblocks,
                          hipStream_t s);
// mode 0: sum p ; mode 1: sum (p - c)^2 per (w | factor f, group g) chunk
hipError_t mc_param_sums(const double2 *pw, const double2 *pv, const uint32_t *perm, const Chunk *chunks,
                         uint32_t nchunks, int mode, const double *cw, const double *cv, int k, double *out,
                         hipStream_t s);
}  // namespace vbk

// feature id of the i-th feature of a level
template <class A> __device__ __forceinline__ uint32_t level_feat(const A &a, uint32_t i)
{
	return a.feat_contig ? a.feat_base + i : a.feats[i];
}
