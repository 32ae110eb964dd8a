// vbfm_capi.hip -- the C-ABI of include/vbfm.h: a VB learner context on one MI355X.
//
// It replaces fm_learn_vb / fm_learn_vb_simultaneous (src/libfm/src/fm_learn_vb.h,
// src/libfm/src/fm_learn_vb_simultaneous.h): the host keeps the reference's control flow
// (one iteration = update_all, test prediction, metrics) and the scalar hyper-parameter
// arithmetic; every O(nnz), O(N) and O(k*D) loop runs as a kernel of vbfm_kernels.hip on
// the context's stream. Device-side partial sums come back in a fixed order and are added
// on the host in that order, so results are deterministic run to run.
#include "vbfm_ctx.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <unistd.h>

using namespace vbi;

namespace vbi {

int fail(vbfm_ctx *c, const std::string &m)
{
	if (c) c->err = m; else vbfm_host_set_error(m.c_str());
	return -1;
}

// ---- the exchange's failure handling ------------------------------------------------------
// the rank, the phase, factor and level the path was in (XPhase), for every exchange message
static std::string x_where(vbfm_ctx *c)
{
	char b[160];
	int n = snprintf(b, sizeof(b), "rank %d/%d: %s", c->rank, c->nranks, c->x_phase);
	if (c->x_f >= 0 && n > 0 && n < (int)sizeof(b)) n += snprintf(b + n, sizeof(b) - n, ", factor %d", c->x_f);
	if (c->x_l >= 0 && n > 0 && n < (int)sizeof(b)) snprintf(b + n, sizeof(b) - n, ", level %d", c->x_l);
	return b;
}

// the stall kernel of VBFM_FAULT=comm_stall is released, and a stream that can still drain gets
// `grace_s` to do so before the communicator is aborted (an abort under a running collective is
// RCCL's prescribed way out of a dead peer, but a drained stream needs none of it)
static void stall_release(vbfm_ctx *c, double grace_s)
{
	if (!c->stall_flag) return;
	__atomic_store_n(c->stall_flag, 1u, __ATOMIC_SEQ_CST);
	const double end = wall_s() + grace_s;
	while (hipStreamQuery(c->s) == hipErrorNotReady && wall_s() < end) usleep(1000);
}

// abort the communicator and fail with `why`; every later exchange refuses with the same message
[[noreturn]] static void comm_fail(vbfm_ctx *c, const std::string &why)
{
	const std::string m = x_where(c) + ": " + why;
	stall_release(c, 5.0);
	if (c->comm) {
		(void)ncclCommAbort(c->comm);
		c->comm = nullptr;
	}
	c->comm_failed = true;
	c->comm_err = m + " (communicator aborted)";
	throw c->comm_err;
}

// VBFM_COMM_TRACE=1: a stderr line per RCCL call and wait of the exchange (time since the first)
static void comm_trace(vbfm_ctx *c, const char *what, double t)
{
	static const bool on = [] { const char *e = getenv("VBFM_COMM_TRACE"); return e && e[0] == '1'; }();
	static const double t0 = wall_s();
	if (on) fprintf(stderr, "[vbfm comm] %10.4f rank %d %s (%s) %.4f s\n", wall_s() - t0, c->rank, what, c->x_phase, t);
}

static ncclResult_t comm_async_error(vbfm_ctx *c)
{
	ncclResult_t ae = ncclSuccess;
	const ncclResult_t r = ncclCommGetAsyncError(c->comm, &ae);
	return r != ncclSuccess ? r : ae;
}

// an RCCL call's result: ncclInProgress (a non-blocking communicator still connecting) is polled
// until it settles or the deadline passes
static void comm_check(vbfm_ctx *c, ncclResult_t r, const char *what)
{
	comm_trace(c, r == ncclInProgress ? "in progress" : "returned", 0.0);
	if (r == ncclInProgress) {
		const double end = wall_s() + c->comm_timeout_s;
		for (;;) {
			r = comm_async_error(c);
			if (r != ncclInProgress) break;
			if (c->comm_timeout_s > 0 && wall_s() > end) {
				char b[160];
				snprintf(b, sizeof(b), "%s did not complete within %.0f s (VBFM_COMM_TIMEOUT_S)", what, c->comm_timeout_s);
				comm_fail(c, b);
			}
			usleep(200);
		}
	}
	if (r != ncclSuccess) comm_fail(c, std::string("RCCL ") + ncclGetErrorString(r) + " in " + what);
}

// wait for stream `st`: hipStreamSynchronize without a communicator; with one, poll the stream,
// RCCL's asynchronous error and the deadline (a rank that died leaves the others' all-reduce
// spinning: a blocking wait would never return)
static void comm_wait(vbfm_ctx *c, hipStream_t st)
{
	if (!c->comm) {
		HIPCHK(hipStreamSynchronize(st));
		return;
	}
	const double t0 = wall_s();
	comm_trace(c, "wait", 0.0);
	for (uint32_t spin = 0;; spin++) {
		const hipError_t e = hipStreamQuery(st);
		if (e == hipSuccess) {
			if (st == c->s) c->x_pending.clear();
			comm_trace(c, "waited", wall_s() - t0);
			return;
		}
		if (e != hipErrorNotReady) throw HipError{e, "hipStreamQuery"};
		const double ta = wall_s();
		const ncclResult_t ae = comm_async_error(c);
		if (wall_s() - ta > 0.5) comm_trace(c, "slow ncclCommGetAsyncError", wall_s() - ta);
		if (ae != ncclSuccess && ae != ncclInProgress)
			comm_fail(c, std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
		const double dt = wall_s() - t0;
		if (c->comm_timeout_s > 0 && dt > c->comm_timeout_s) {
			char b[200];
			snprintf(b, sizeof(b), "waiting for the stream, the all-reduces queued since the last wait did not "
			                       "complete within %.0f s (VBFM_COMM_TIMEOUT_S): a rank failed or stopped",
			         c->comm_timeout_s);
			comm_fail(c, std::string(b) + (c->x_pending.empty() ? "" : "; the first of them: " + c->x_pending));
		}
		// the first ~2 ms poll back to back (an all-reduce's usual wait), then sleep in steps of
		// up to 1 ms (a sweep's worth of queued levels)
		if (spin > 256) usleep(dt < 0.05 ? 50 : 1000);
	}
}

void sync(vbfm_ctx *c) { comm_wait(c, c->s); }

hipError_t d2h(vbfm_ctx *c, void *dst, const void *src, size_t bytes)
{
	if (c->comm) sync(c);
	return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->s);
}

void xs_reset(vbfm_ctx *c)
{
	const int32_t t = c->comm ? 1 : c->xfn ? 2 : 0;
	c->xs = vbfm_exchange_stats{};
	c->xs.transport = t;
	c->xs.timeout_s = c->comm ? c->comm_timeout_s : 0.0;
}

void xs_span(vbfm_ctx *c, float ms)
{
	c->xs.ms_timed += ms;
	c->xs.n_timed++;
}

// the fault hooks of the exchange (tests): VBFM_FAULT=comm makes rank VBFM_FAULT_RANK (default:
// the last) fail its first exchange inside a sweep as a failed collective would; comm_stall
// queues a kernel ahead of that exchange that spins until the deadline releases it (a peer that
// never arrives, on one GPU)
static void comm_fault_hooks(vbfm_ctx *c)
{
	if (c->x_l < 0) return;
	const char *fr = getenv("VBFM_FAULT_RANK");
	const int rank = fr ? atoi(fr) : c->nranks - 1;
	if (c->rank != rank) return;
	if (fault_at("comm")) {
		if (c->comm) comm_fail(c, "VBFM_FAULT=comm");
		throw x_where(c) + ": VBFM_FAULT=comm";
	}
	if (fault_at("comm_stall") && c->comm && !c->stall_done) {
		c->stall_done = true;
		if (!c->stall_flag) HIPCHK(hipHostMalloc((void **)&c->stall_flag, 4, hipHostMallocCoherent | hipHostMallocMapped));
		*c->stall_flag = 0;
		uint32_t *dflag = nullptr;
		HIPCHK(hipHostGetDevicePointer((void **)&dflag, c->stall_flag, 0));
		HIPCHK(vbk::stall(dflag, c->s));
	}
}

// in-place all-reduce of a device buffer across the ranks: RCCL on the context's stream, or
// (vbfm_comm_init_host) staged through host memory and handed to the caller's exchange
void allreduce_dev(vbfm_ctx *c, void *buf, size_t n, ncclDataType_t t, ncclRedOp_t op)
{
	if (c->comm_failed) throw c->comm_err;
	const size_t es = t == ncclDouble ? 8 : t == ncclUint32 ? 4 : 1;
	comm_fault_hooks(c);
	c->xs.n_calls++;
	c->xs.bytes += n * es;
	if (c->comm) {
		if (c->x_pending.empty()) c->x_pending = x_where(c);
		const size_t p = prof_begin(c, 3);
		const double ta = wall_s();
		const ncclResult_t r = ncclAllReduce(buf, buf, n, t, op, c->comm, c->s);
		if (wall_s() - ta > 0.5) comm_trace(c, "slow ncclAllReduce", wall_s() - ta);
		comm_check(c, r, "ncclAllReduce");
		prof_end(c, p);
		return;
	}
	if (!c->xfn) throw std::string("all-reduce without a communicator");
	const int32_t xt = t == ncclDouble ? VBFM_X_F64 : t == ncclUint32 ? VBFM_X_U32 : VBFM_X_U8;
	if (t != ncclDouble && t != ncclUint32 && t != ncclUint8) throw std::string("host exchange: unsupported type");
	const double t0 = wall_s();
	if (c->xbuf.size() < n * es) c->xbuf.resize(n * es);
	if (n) HIPCHK(d2h(c, c->xbuf.data(), buf, n * es));
	sync(c);
	if (c->xfn(c->xuser, c->xbuf.data(), n, xt, op == ncclMax ? VBFM_X_MAX : VBFM_X_SUM) != 0)
		throw x_where(c) + ": host exchange failed";
	if (n) HIPCHK(hipMemcpyAsync(buf, c->xbuf.data(), n * es, hipMemcpyHostToDevice, c->s));
	sync(c);
	xs_span(c, (float)((wall_s() - t0) * 1e3));
}

uint32_t ar_chunks(vbfm_ctx *c, uint32_t nfeat)
{
	if (!c->row_comm()) return 1;
	// default: one all-reduce per level. Cutting a level into chunks whose all-reduces overlap
	// the next chunk's statistics kernel is bit-identical, but each extra chunk costs a kernel
	// boundary, a second collective and two cross-stream events: 489 -> 516 -> 530 us per level
	// for 1 / 2 / 4 chunks at C4's per-rank size on 8 GPUs (one GPU, 1-rank RCCL,
	// profiles/r03_chunks/n8_shard), while it can hide at most t_ar(2 MB) - t_ar(1 MB) of a
	// latency-dominated ring all-reduce (~10-20 us on one xGMI node): a net loss there.
	// VBFM_AR_CHUNKS=n asks for n chunks of at least 64 columns (fabrics with slow collectives;
	// tests, A/B)
	const char *e = getenv("VBFM_AR_CHUNKS");
	const uint32_t want = e ? (uint32_t)std::max(atoi(e), 1) : 1u, floor = e ? 64u : 2048u;
	const uint32_t C = std::min<uint32_t>(want, nfeat / floor);
	return std::max<uint32_t>(1, std::min<uint32_t>(C, vbfm_ctx::AR_MAX_CHUNKS));
}

void allreduce_chunk(vbfm_ctx *c, double2 *buf, size_t n, uint32_t i)
{
	if (c->comm_failed) throw c->comm_err;
	if (!c->comm) {   // the host exchange is synchronous: nothing to overlap
		allreduce_dev(c, buf, n, ncclDouble, ncclSum);
		return;
	}
	if (!c->s_comm) {
		HIPCHK(hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking));
		for (auto &e : c->ev_ar) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
		HIPCHK(hipEventCreateWithFlags(&c->ev_arj, hipEventDisableTiming));
	}
	HIPCHK(hipEventRecord(c->ev_ar[i], c->s));
	HIPCHK(hipStreamWaitEvent(c->s_comm, c->ev_ar[i], 0));
	comm_fault_hooks(c);
	c->xs.n_calls++;
	c->xs.bytes += n * 8;
	if (c->x_pending.empty()) c->x_pending = x_where(c);
	const size_t p = prof_begin(c, 3, c->s_comm);
	comm_check(c, ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, c->comm, c->s_comm), "ncclAllReduce");
	prof_end(c, p, c->s_comm);
}

void allreduce_join(vbfm_ctx *c)
{
	if (!c->comm || !c->s_comm) return;
	HIPCHK(hipEventRecord(c->ev_arj, c->s_comm));
	HIPCHK(hipStreamWaitEvent(c->s, c->ev_arj, 0));
}

// all-reduce a few host doubles across the row shards (identity with one rank)
void allreduce_host(vbfm_ctx *c, double *v, int n)
{
	if (!c->row_comm()) return;   // feature shards hold every row: their sums are already global
	HIPCHK(hipMemcpyAsync(c->red_d, v, n * sizeof(double), hipMemcpyHostToDevice, c->s));
	allreduce_dev(c, c->red_d, n, ncclDouble, ncclSum);
	HIPCHK(d2h(c, v, c->red_d, n * sizeof(double)));
	sync(c);
}

// block partials of a row reduction, summed on the host in block order
double finish_sum(vbfm_ctx *c, uint32_t nblocks)
{
	HIPCHK(d2h(c, c->red_h.data(), c->red_d, nblocks * sizeof(double)));
	sync(c);
	double s = 0.0;
	for (uint32_t i = 0; i < nblocks; i++) s += c->red_h[i];
	return s;
}

void free_data(DevData &d)
{
	dfree(d.col_ptr); dfree(d.csc); dfree(d.row_ptr); dfree(d.csr); dfree(d.target);
	d = DevData();
}

void check_csc(const vbfm_csc *in)
{
	if (!in) throw std::string("null data set");
	if (in->nnz && (!in->col_ptr || !in->col_ent)) throw std::string("data set without entries");
	if (in->num_rows && !in->target) throw std::string("data set without targets");
	if (!in->col_ptr && in->num_feature) throw std::string("data set without col_ptr");
	if (in->num_feature && in->col_ptr[in->num_feature] != in->nnz) throw std::string("col_ptr does not end at nnz");
	for (uint32_t j = 0; j < in->num_feature; j++)
		if (in->col_ptr[j + 1] < in->col_ptr[j]) throw std::string("col_ptr is not monotone");
	for (uint64_t p = 0; p < in->nnz; p++)
		if (in->col_ent[p].id >= in->num_rows) throw std::string("row index out of range in col_ent");
}

// pad col_ptr to nf_pad columns (trailing empty columns), upload data set
void upload(vbfm_ctx *c, DevData &d, const vbfm_csc *in, uint32_t nf_pad)
{
	free_data(d);
	d.n = in->num_rows;
	d.nf_local = in->num_feature;
	d.nf = std::max(nf_pad, in->num_feature);
	d.nnz = in->nnz;
	std::vector<uint64_t> cp((size_t)d.nf + 1, in->nnz);
	if (in->num_feature) memcpy(cp.data(), in->col_ptr, ((size_t)in->num_feature + 1) * sizeof(uint64_t));
	else cp[0] = 0;
	d.col_ptr = dalloc<uint64_t>(cp.size());
	d.csc = dalloc<uint2>(d.nnz);
	d.row_ptr = dalloc<uint64_t>((size_t)d.n + 1);
	d.csr = dalloc<uint2>(d.nnz);
	d.target = dalloc<float>(d.n);
	HIPCHK(hipMemcpyAsync(d.col_ptr, cp.data(), cp.size() * 8, hipMemcpyHostToDevice, c->s));
	if (d.nnz) HIPCHK(hipMemcpyAsync(d.csc, in->col_ent, d.nnz * 8, hipMemcpyHostToDevice, c->s));
	HIPCHK(vbk::build_csr(d.col_ptr, d.csc, d.nf_local, d.n, d.nnz, d.row_ptr, d.csr, c->s));
	if (d.n) HIPCHK(hipMemcpyAsync(d.target, in->target, d.n * 4, hipMemcpyHostToDevice, c->s));
	float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
	for (uint32_t i = 0; i < d.n; i++) { mn = std::min(in->target[i], mn); mx = std::max(in->target[i], mx); }
	d.min_target = mn; d.max_target = mx;
	sync(c);
}

uint32_t nlevels(vbfm_ctx *c);
LevelArgs level_args(vbfm_ctx *c, uint32_t l, bool is_w, int f);

// ---- level-ordered row store (vbfm_lorder.hip) ------------------------------------------
void lord_release(vbfm_ctx *c, bool keep_rows)
{
	if (keep_rows) rows_row_order(c);   // (without keep_rows the records are discarded)
	sync(c);
	dfree(c->rows_alt); dfree(c->lcp); dfree(c->lx); dfree(c->lnext); dfree(c->lrow0); dfree(c->lpos0);
	dfree(c->lpidx); dfree(c->lpx); dfree(c->post_tab); dfree(c->lpay); dfree(c->lpay2);
	dfree(c->long_segs); dfree(c->seg_part);
	c->seg_ptr.clear();
	c->long_min_l.clear();
	c->place_ms.clear();
	c->place_pick[0] = c->place_pick[1] = -1;
	c->long_min = 0;
	c->lord = false;
	c->estore = false;
	c->rows_lorder = false;
}

static int layout_request(const vbfm_ctx *c)
{
	const char *env = getenv("VBFM_LAYOUT");
	if (env && !strcmp(env, "column")) return VBFM_LAYOUT_COLUMN;
	if (env && !strcmp(env, "level")) return VBFM_LAYOUT_LEVEL;
	if (env && !strcmp(env, "entry")) return VBFM_LAYOUT_ENTRY;
	if (env && !strcmp(env, "auto")) return VBFM_LAYOUT_AUTO;
	return c->layout_req;
}

// Long columns (skewed data): a column longer than its level's threshold is cut into segments of
// SEG_LEN = 1024 entries (one resident run of the 512-thread segment kernels), one workgroup each,
// in the fused single-rank sweep of either layout (lord_long / col_long); columns listing a row
// twice stay sequential. The threshold is max(1024, 4 x the level's mean column): the level's
// workgroup shape is sized for its mean (dispatch_shape), and a column far beyond it streams its
// run in many rounds while the rest of the launch has drained. ML-1M-shaped data (C2: items with
// popularity ~u^3, mean 228, longest 56,803): 2.79 -> 1.97 ms per iteration against the round-5
// rule (longer than 8192, in segments of 4096; profiles/r06_c2/seg_ab/). Uniform field data stays
// unsegmented (C4's longest column ~950 entries of a mean of 800). VBFM_SEG_MIN / VBFM_SEG_LEN
// override the threshold and the segment length, VBFM_LONG=0 turns segments off.
// lcp: prefix sums of the level features' column lengths (level_feats order).
static void build_long_segs(vbfm_ctx *c, const std::vector<uint64_t> &lcp, const std::vector<uint8_t> &dup,
                            const std::vector<uint32_t> &feats)
{
	const char *smn = getenv("VBFM_SEG_MIN"), *sln = getenv("VBFM_SEG_LEN");
	const uint32_t SEG_LEN = sln ? (uint32_t)std::max(atoi(sln), 64) : 1024u;
	const uint32_t L = nlevels(c);
	const char *lg = getenv("VBFM_LONG");
	const bool on = !(lg && lg[0] == '0');
	std::vector<LongSeg> segs;
	c->seg_ptr.assign((size_t)L + 1, 0);
	c->long_min_l.assign(L, 0);
	uint32_t maxs = 0;
	for (uint32_t l = 0; l < L; l++) {
		c->seg_ptr[l] = (uint32_t)segs.size();
		const uint32_t nfl = c->level_ptr[l + 1] - c->level_ptr[l];
		const uint64_t mean = nfl ? (lcp[c->level_ptr[l + 1]] - lcp[c->level_ptr[l]]) / nfl : 0;
		const uint32_t thr = smn ? (uint32_t)std::max(atoi(smn), 64)
		                         : (uint32_t)std::max<uint64_t>(1024u, std::min<uint64_t>(4 * mean, 1u << 30));
		for (uint32_t i = c->level_ptr[l]; on && i < c->level_ptr[l + 1]; i++) {
			const uint64_t len = lcp[i + 1] - lcp[i];
			if (len <= thr || dup[feats[i]]) continue;
			// seg0: the column's first segment, counted from the level's first (blockIdx)
			const uint32_t ns = (uint32_t)((len + SEG_LEN - 1) / SEG_LEN), s0 = (uint32_t)segs.size() - c->seg_ptr[l];
			for (uint32_t q = 0; q < ns; q++)
				segs.push_back({i - c->level_ptr[l], q * SEG_LEN,
				                (uint32_t)std::min<uint64_t>(SEG_LEN, len - (uint64_t)q * SEG_LEN), s0, ns});
		}
		if ((uint32_t)segs.size() > c->seg_ptr[l]) c->long_min_l[l] = thr;   // (0: nothing skipped)
		maxs = std::max(maxs, (uint32_t)segs.size() - c->seg_ptr[l]);
	}
	c->seg_ptr[L] = (uint32_t)segs.size();
	if (segs.empty()) return;
	c->long_min = 1;   // some level has segments (each level's threshold: long_min_l)
	c->long_segs = dalloc<LongSeg>(segs.size());
	HIPCHK(hipMemcpyAsync(c->long_segs, segs.data(), segs.size() * sizeof(LongSeg), hipMemcpyHostToDevice, c->s));
	c->seg_part = dalloc<double2>(2 * (size_t)maxs);
	sync(c);
}

// The entry store, for levels that miss rows (multi-hot rows without fields): one slot per
// train entry in the field store's order (level by level, the level's columns in ascending
// feature order, rows ascending in a column), nnz x 64 B; a row's record waits in the slot of
// the entry its next level sweeps, so a level streams its columns' runs and scatters each
// record to the row's next slot (k_level_lord<..., ENT>) instead of gathering and writing back
// rows in place (the column-gather layout: two random touches per entry).
// No row listing a feature twice (VB and MCMC / ALS); the store must fit in half the free
// memory. A row without entries parks its record in slot nnz + r. Row shards (split sweeps): the
// two-pass split (statistics, all-reduce, correction + move); VBFM_DEFER=1 takes the VB sweep's
// deferred form, which reads each slot's previous-entry payload (k_estore_prev: the global
// level-feature index and x of the row's previous entry) and a posterior table over all level
// features.
// Returns false when it does not apply (force: throw instead).
bool build_estore(vbfm_ctx *c, const std::vector<uint64_t> &lcp, const std::vector<uint8_t> &dup,
                  const std::vector<uint32_t> &feats, bool force)
{
	DevData &d = c->tr;
	const uint32_t n = d.n, nf = d.nf;
	std::string why;
	const char *env = getenv("VBFM_ESTORE");
	size_t fr = 0, tot = 0;
	HIPCHK(hipMemGetInfo(&fr, &tot));
	if (!force && env && env[0] == '0') why = "VBFM_ESTORE=0";
	else if (n == 0 || d.nnz == 0) why = "no train entries";
	else if (d.nnz + n >= 0x80000000ull) why = "more than 2^31 entries and rows";
	else if ((double)(d.nnz + n) * sizeof(RowRec) > 0.5 * (double)fr) why = "the store does not fit in half the free memory";
	for (uint32_t i = 0; i < nf && why.empty(); i++)
		if (dup[feats[i]]) why = "a row lists feature " + std::to_string(feats[i]) + " twice";
	if (!why.empty()) {
		if (force) throw std::string("entry store not possible: ") + why;
		return false;
	}
	std::vector<uint32_t> lvpos(nf);
	for (uint32_t i = 0; i < nf; i++) lvpos[feats[i]] = i;
	c->lcp = dalloc<uint64_t>(lcp.size());
	HIPCHK(hipMemcpyAsync(c->lcp, lcp.data(), lcp.size() * 8, hipMemcpyHostToDevice, c->s));
	uint32_t *lv = dalloc<uint32_t>(nf);
	HIPCHK(hipMemcpyAsync(lv, lvpos.data(), (size_t)nf * 4, hipMemcpyHostToDevice, c->s));
	{
		uint32_t *cnt = dalloc<uint32_t>(1), h = 1;
		HIPCHK(vbk::count_x_ne1(d.csc, d.nnz, cnt, c->s));
		HIPCHK(d2h(c, &h, cnt, 4));
		sync(c);
		dfree(cnt);
		const char *kx = getenv("VBFM_LX");
		if (h != 0 || (kx && kx[0] == '1')) c->lx = dalloc<float>(d.nnz);
	}
	c->lnext = dalloc<uint32_t>(d.nnz);
	c->lpos0 = dalloc<uint32_t>(n);
	// slots: the entries, then one parking slot per row (used by rows without entries)
	c->rows_alt = dalloc<RowRec>(d.nnz + n);
	HIPCHK(hipMemsetAsync(c->rows_alt, 0, (d.nnz + n) * sizeof(RowRec), c->s));
	HIPCHK(vbk::estore_build(d.row_ptr, d.csr, d.col_ptr, d.csc, lv, c->lcp, n, d.nnz, c->lnext, c->lx, c->lpos0,
	                         c->s));
	// the entry store's split is two-pass by default: its short levels' records are still in L2 /
	// MALL for the second pass, while the deferred form gathers a posterior per record from a
	// table over all features (one GPU, multi-hot bench: 23.9 vs 26.1 us per level without a
	// communicator, profiles/r03_multihot_split/); VBFM_DEFER=1 takes the deferred form
	const char *df = getenv("VBFM_DEFER");
	if ((c->row_comm() || c->force_split) && df && df[0] == '1') {
		uint32_t *pidx = dalloc<uint32_t>(d.nnz);
		float *px = dalloc<float>(d.nnz);
		HIPCHK(vbk::estore_prev(d.row_ptr, d.csr, d.col_ptr, d.csc, lv, c->lcp, n, pidx, px, c->s));
		if (c->lx) {
			c->lpay = dalloc<uint4>(d.nnz);
			HIPCHK(vbk::lord_pack(c->lx, c->lnext, pidx, px, c->lpay, d.nnz, c->s));
		} else {   // every x 1: 8 B per entry
			c->lpay2 = dalloc<uint2>(d.nnz);
			HIPCHK(vbk::lord_pack2(c->lnext, pidx, c->lpay2, d.nnz, c->s));
		}
		c->post_tab = dalloc<PostT>(std::max(nf, 1u));
		HIPCHK(hipMemsetAsync(c->post_tab, 0, (size_t)std::max(nf, 1u) * sizeof(PostT), c->s));
		sync(c);
		dfree(pidx);
		dfree(px);
	}
	sync(c);
	dfree(lv);
	c->lord = true;
	c->estore = true;
	c->rows_lorder = false;
	return true;
}

// Non-temporal record traffic of the deferred split kernels (LevelArgs::pending bits 2 = loads,
// 4 = stores). VBFM_DEFER_NT=0..3 (bit 0 loads, bit 1 stores) overrides; default both: the moved
// records then leave more of L2 to the posterior table the next level gathers from (one N = 8
// rank's shape, 1.25e7 rows: 426-427 -> 415-417 us per split level, profiles/r05_split/; alone,
// either half gained 0-1.5 %, profiles/probes/ab_defer_loads.txt, ab_defer_nt_store.txt)
static int defer_nt(const vbfm_ctx *)
{
	const char *e = getenv("VBFM_DEFER_NT");
	const int v = e ? atoi(e) : 3;
	return ((v & 1) ? 2 : 0) | ((v & 2) ? 4 : 0);
}

// Placement of the store's two record buffers (VBFM_PLACE, default 1). The level kernel's
// scattered whole-record writes run up to ~20 % faster or slower depending on where the driver
// placed the two buffers, persistently per allocation, while streaming copies do not change
// (tools/probe_place.hip, profiles/r04_short_columns/). A pair's time is close to the
// sum of a per-buffer part for each side (a slow source with a fast destination lands in between),
// so buffers are scored one at a time: the store's two buffers and up to VBFM_PLACE_TRIES - 2 fresh
// allocations, each moved to and from one reference buffer on level 0's real pattern (k_place_move,
// no arithmetic); the two best are kept (the records move with them), the rest freed. Only where a
// launch is long enough to time (>= 2e6 rows), within the caller's budget (vbfm_config
// place_candidates / place_budget_bytes) and half of the free memory. The results do not depend on
// the buffers (bit for bit).
static void tune_placement(vbfm_ctx *c)
{
	const uint32_t n = c->tr.n, L = nlevels(c);
	c->t_place = 0;
	c->place_bytes = 0;
	if (n < 2000000u || L < 2 || !c->lnext) return;
	const char *pe = getenv("VBFM_PLACE");
	if (pe && pe[0] == '0') return;
	const size_t bytes = (size_t)n * sizeof(RowRec);
	// stores under 2 GB (C3, one rank of N = 4 or 8) try 64 buffers, larger ones 16: the fast
	// allocations come in clusters along the allocation sequence and a few tries miss them on some
	// boxes (profiles/r04_short_columns/placement_tries/)
	const char *te = getenv("VBFM_PLACE_TRIES");
	int tries = bytes < ((size_t)2 << 30) ? 64 : 16;
	if (c->place_cands_cfg > 0) tries = c->place_cands_cfg;
	if (te) tries = atoi(te);
	if (tries <= 2) return;
	const char *be = getenv("VBFM_PLACE_BUDGET_GB");
	uint64_t budget = c->place_budget_cfg ? c->place_budget_cfg : VBFM_PLACE_BUDGET_DEFAULT;
	if (be) budget = (uint64_t)(atof(be) * (double)(1ull << 30));
	size_t fr = 0, tot = 0;
	HIPCHK(hipMemGetInfo(&fr, &tot));
	// no more than half of the free memory (a quarter with several ranks: rank processes rehearsed
	// on one GPU tune at the same time); the records' stash and the reference buffer come out of it
	const size_t cap = std::min<uint64_t>(budget, c->nranks > 1 ? fr / 4 : fr / 2);
	const size_t room = cap > 2 * bytes ? cap - 2 * bytes : 0;
	const int extra = (int)std::min<size_t>((size_t)tries - 2, room / (bytes + 1));
	if (extra < 1) return;
	const double t0 = wall_s();
	const uint64_t *lp = c->lcp + c->level_ptr[0];
	const uint32_t nfl = c->level_ptr[1] - c->level_ptr[0];
	// the records wait in a stash while every candidate is overwritten
	RowRec *keep = nullptr, *ref = nullptr;
	if (hipMalloc((void **)&keep, bytes) != hipSuccess || hipMalloc((void **)&ref, bytes) != hipSuccess) {
		(void)hipGetLastError();
		dfree(keep);
		return;
	}
	hipEvent_t e0 = nullptr, e1 = nullptr;
	// cand[0], cand[1]: the store's own pair; the rest fresh allocations this search owns until it
	// commits. On any failure the records go back into c->rows from the stash, every fresh candidate,
	// the stash and the reference buffer are freed, and the error propagates (build_schedule then
	// leaves the schedule to be rebuilt by the next call)
	std::vector<RowRec *> cand = {c->rows, c->rows_alt};
	bool stashed = false;
	try {
		HIPCHK(hipMemcpyAsync(keep, c->rows, bytes, hipMemcpyDeviceToDevice, c->s));
		stashed = true;
		HIPCHK(hipEventCreate(&e0));
		HIPCHK(hipEventCreate(&e1));
		auto score = [&](RowRec *x) {
			HIPCHK(vbk::place_move(ref, x, lp, c->lnext, nfl, c->s));   // warm-up
			HIPCHK(hipEventRecord(e0, c->s));
			for (int r = 0; r < 2; r++) {
				HIPCHK(vbk::place_move(ref, x, lp, c->lnext, nfl, c->s));
				HIPCHK(vbk::place_move(x, ref, lp, c->lnext, nfl, c->s));
			}
			HIPCHK(hipEventRecord(e1, c->s));
			HIPCHK(hipEventSynchronize(e1));
			float ms = 0.f;
			HIPCHK(hipEventElapsedTime(&ms, e0, e1));
			return ms;
		};
		// candidates: plain allocations (physically contiguous ones, hipDeviceMallocContiguous, probed
		// 14.1 ms against 11.5-11.8 ms for plain ones at C4 and no better at C3: not tried)
		// (an allocation the driver refuses ends the list: the tuning never fails the store)
		for (int i = 0; i < extra; i++) {
			void *q = nullptr;
			if (hipMalloc(&q, bytes) != hipSuccess) {
				(void)hipGetLastError();
				break;
			}
			cand.push_back((RowRec *)q);
		}
		c->place_bytes = (uint64_t)bytes * cand.size();   // the fresh candidates + the stash + the reference
		std::vector<float> ms(cand.size());
		for (size_t i = 0; i < cand.size(); i++) {
			ms[i] = score(cand[i]);
			if (i == 2 && fault_at("placement")) throw HipError{hipErrorOutOfMemory, "VBFM_FAULT=placement"};
		}
		std::vector<size_t> order(cand.size());
		for (size_t i = 0; i < order.size(); i++) order[i] = i;
		std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return ms[x] < ms[y]; });
		// the store ping-pongs between its two buffers, so the best few are also scored as pairs:
		// each level streams one and scatters into the other (VBFM_PLACE_PAIRS=<K>: the best K;
		// 0: keep the best two singles)
		const char *pp = getenv("VBFM_PLACE_PAIRS");
		const size_t K = std::min<size_t>(pp ? (size_t)atoi(pp) : 6, order.size());
		if (K > 2) {
			auto score_pair = [&](RowRec *x, RowRec *y) {
				HIPCHK(vbk::place_move(x, y, lp, c->lnext, nfl, c->s));   // warm-up
				HIPCHK(hipEventRecord(e0, c->s));
				for (int r = 0; r < 2; r++) {
					HIPCHK(vbk::place_move(x, y, lp, c->lnext, nfl, c->s));
					HIPCHK(vbk::place_move(y, x, lp, c->lnext, nfl, c->s));
				}
				HIPCHK(hipEventRecord(e1, c->s));
				HIPCHK(hipEventSynchronize(e1));
				float t = 0.f;
				HIPCHK(hipEventElapsedTime(&t, e0, e1));
				return t;
			};
			float best = 0.f;
			size_t ba = 0, bb = 1;
			c->place_pair_ms.clear();
			for (size_t a = 0; a < K; a++)
				for (size_t b = a + 1; b < K; b++) {
					const float t = score_pair(cand[order[a]], cand[order[b]]);
					c->place_pair_ms.push_back(t);
					if ((a == 0 && b == 1) || t < best) { best = t; ba = a; bb = b; }
				}
			std::swap(order[0], order[ba]);
			std::swap(order[1], order[bb]);   // bb > ba >= 0: untouched by the first swap
		}
		// commit (nothing below the frees can throw before c->rows names a live buffer again)
		for (size_t j = 2; j < order.size(); j++) dfree(cand[order[j]]);
		c->rows = cand[order[0]];
		c->rows_alt = cand[order[1]];
		cand.resize(2);   // every fresh buffer is now the store's or freed
		HIPCHK(hipMemcpyAsync(c->rows, keep, bytes, hipMemcpyDeviceToDevice, c->s));
		sync(c);
		stashed = false;
		c->place_ms.assign(ms.begin(), ms.end());
		c->place_pick[0] = (int)order[0];
		c->place_pick[1] = (int)order[1];
	} catch (...) {
		(void)hipStreamSynchronize(c->s);
		if (stashed) (void)hipMemcpy(c->rows, keep, bytes, hipMemcpyDeviceToDevice);
		for (size_t i = 2; i < cand.size(); i++) dfree(cand[i]);
		dfree(keep);
		dfree(ref);
		if (e0) (void)hipEventDestroy(e0);
		if (e1) (void)hipEventDestroy(e1);
		c->place_ms.clear();
		c->place_pick[0] = c->place_pick[1] = -1;
		throw;
	}
	dfree(keep);
	dfree(ref);
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	c->t_place = wall_s() - t0;
	const auto &ms = c->place_ms;
	const size_t order[2] = {(size_t)c->place_pick[0], (size_t)c->place_pick[1]};
	const char *lg = getenv("VBFM_PLACE_LOG");
	if (lg && lg[0] == '1') {
		fprintf(stderr, "vbfm placement: %u rows, level-0 pattern to and from a reference buffer x2:", n);
		for (size_t i = 0; i < ms.size(); i++)
			fprintf(stderr, " %.3f%s", ms[i], (i == order[0] || i == order[1]) ? "*" : "");
		fprintf(stderr, " ms");
		if (!c->place_pair_ms.empty()) {
			fprintf(stderr, "; the best as pairs, both directions x2:");
			for (float t : c->place_pair_ms) fprintf(stderr, " %.3f", t);
		}
		fprintf(stderr, " ms\n");
	}
}

// Level-ordered store of the train set when every level holds each row exactly once (no
// repeated feature in a row): per level l, positions [l*n, (l+1)*n) list the level's
// columns in ascending feature order, rows ascending within a column.
void build_lorder(vbfm_ctx *c, const std::vector<uint64_t> &cp, const std::vector<uint32_t> &feats)
{
	lord_release(c, true);
	const int req = layout_request(c);
	if (c->ov) return;   // the online learner sweeps mini-batch columns
	if (c->shard_mode == VBFM_SHARD_FEATURES) {
		if (req == VBFM_LAYOUT_LEVEL) throw std::string("the level-ordered row layout does not combine with feature shards");
		return;
	}
	DevData &d = c->tr;
	const uint32_t L = nlevels(c), n = d.n, nf = d.nf;
	std::string why;
	std::vector<uint8_t> dup(nf, 0);
	if (nf) HIPCHK(hipMemcpy(dup.data(), c->dup, nf, hipMemcpyDeviceToHost));
	std::vector<uint64_t> lcp((size_t)nf + 1, 0);
	for (uint32_t i = 0; i < nf; i++) lcp[i + 1] = lcp[i] + (cp[feats[i] + 1] - cp[feats[i]]);
	if (req == VBFM_LAYOUT_COLUMN) {
		build_long_segs(c, lcp, dup, feats);
		return;
	}
	if (n == 0 || L == 0) why = "no train rows";
	for (uint32_t l = 0; l < L && why.empty(); l++) {
		if (lcp[c->level_ptr[l + 1]] - lcp[c->level_ptr[l]] != n)
			why = "dependency level " + std::to_string(l + 1) + " does not hold every train row exactly once";
		for (uint32_t i = c->level_ptr[l]; i < c->level_ptr[l + 1] && why.empty(); i++)
			if (dup[feats[i]]) why = "a row lists feature " + std::to_string(feats[i]) + " twice";
	}
	if (!why.empty()) {
		if (req == VBFM_LAYOUT_LEVEL) throw std::string("level-ordered row layout not possible: ") + why;
		if (build_estore(c, lcp, dup, feats, req == VBFM_LAYOUT_ENTRY)) return;
		build_long_segs(c, lcp, dup, feats);   // the column-gather layout
		return;
	}
	if (req == VBFM_LAYOUT_ENTRY) {   // forced on complete levels too (tests)
		build_estore(c, lcp, dup, feats, true);
		return;
	}
	c->lcp = dalloc<uint64_t>(lcp.size());
	HIPCHK(hipMemcpyAsync(c->lcp, lcp.data(), lcp.size() * 8, hipMemcpyHostToDevice, c->s));
	build_long_segs(c, lcp, dup, feats);
	// x of every entry, unless all are 1.0f (one-hot libfm data): the level kernels then
	// read no x at all (VBFM_LX=1 keeps the array)
	{
		uint32_t *cnt = dalloc<uint32_t>(1), h = 1;
		HIPCHK(vbk::count_x_ne1(d.csc, d.nnz, cnt, c->s));
		HIPCHK(d2h(c, &h, cnt, 4));
		sync(c);
		dfree(cnt);
		const char *kx = getenv("VBFM_LX");
		if (h != 0 || (kx && kx[0] == '1')) c->lx = dalloc<float>(d.nnz);
	}
	c->lnext = dalloc<uint32_t>(d.nnz);
	c->lrow0 = dalloc<uint32_t>(n);
	c->lpos0 = dalloc<uint32_t>(n);
	c->rows_alt = dalloc<RowRec>(n);
	DevScratch<uint32_t> tmp_buf(n);   // freed on every path out, the placement search's failure included
	uint32_t *&tmp = tmp_buf.p;
	auto lev = [&](uint32_t l, uint32_t *&f, uint32_t &nfl, const uint64_t *&lp) {
		f = c->level_feats + c->level_ptr[l];
		nfl = c->level_ptr[l + 1] - c->level_ptr[l];
		lp = c->lcp + c->level_ptr[l];
	};
	uint32_t *f, nfl;
	const uint64_t *lp;
	lev(0, f, nfl, lp);
	HIPCHK(vbk::lord_pos(f, nfl, lp, 0, d.col_ptr, d.csc, c->lpos0, c->s));
	// backwards over the levels: level l needs the position map of level l+1 (level 0 for
	// the last level), held in tmp (or lpos0)
	for (uint32_t l = L; l-- > 0;) {
		lev(l, f, nfl, lp);
		const uint32_t *pos_next = (l + 1 == L) ? c->lpos0 : tmp;
		HIPCHK(vbk::lord_fill(f, nfl, lp, (uint64_t)l * n, d.col_ptr, d.csc, pos_next, c->lx, c->lnext,
		                      l == 0 ? c->lrow0 : nullptr, c->s));
		if (l > 0) HIPCHK(vbk::lord_pos(f, nfl, lp, (uint64_t)l * n, d.col_ptr, d.csc, tmp, c->s));
	}
	tune_placement(c);
	// split form (row shards): each entry's previous-level feature and x, for the deferred
	// correction (VBFM_DEFER=0 keeps the two-pass split)
	const char *df = getenv("VBFM_DEFER");
	if ((c->row_comm() || c->force_split) && !(df && df[0] == '0')) {
		c->lpidx = dalloc<uint32_t>(d.nnz);
		c->lpx = dalloc<float>(d.nnz);
		DevScratch<float> tmpx_buf(n);
		float *&tmpx = tmpx_buf.p;
		uint32_t maxlev = 0;
		for (uint32_t l = 0; l < L; l++) {
			const uint32_t pl = (l + L - 1) % L;
			maxlev = std::max(maxlev, c->level_ptr[l + 1] - c->level_ptr[l]);
			HIPCHK(vbk::lord_prev_map(c->level_feats + c->level_ptr[pl], c->level_ptr[pl + 1] - c->level_ptr[pl],
			                          d.col_ptr, d.csc, nullptr, tmp, tmpx, c->s));
			lev(l, f, nfl, lp);
			HIPCHK(vbk::lord_prev_fill(f, nfl, lp, d.col_ptr, d.csc, tmp, tmpx, c->lpidx, c->lpx, c->s));
		}
		c->post_tab = dalloc<PostT>(maxlev);
		sync(c);
		dfree(tmpx);
		// one 16-B record per entry for the deferred kernels; the separate arrays are not
		// read in this mode any more
		dfree(tmp);
		if (c->lx) {
			c->lpay = dalloc<uint4>(d.nnz);
			HIPCHK(vbk::lord_pack(c->lx, c->lnext, c->lpidx, c->lpx, c->lpay, d.nnz, c->s));
		} else {   // every x (and so every previous x) is 1: 8 B per entry
			c->lpay2 = dalloc<uint2>(d.nnz);
			HIPCHK(vbk::lord_pack2(c->lnext, c->lpidx, c->lpay2, d.nnz, c->s));
		}
		sync(c);
		dfree(c->lx); dfree(c->lnext); dfree(c->lpidx); dfree(c->lpx);
	}
	sync(c);
	dfree(tmp);
	c->lord = true;
}

// c->rows in level-0 order (before a sweep) / in row order (row-indexed kernels, readback)
void rows_level_order(vbfm_ctx *c)
{
	if (!c->lord || c->rows_lorder) return;
	if (c->estore) HIPCHK(vbk::rows_scatter(c->rows_alt, c->rows, c->lpos0, c->tr.n, c->s));   // row r -> its slot
	else HIPCHK(vbk::rows_gather(c->rows_alt, c->rows, c->lrow0, c->tr.n, c->s));
	std::swap(c->rows, c->rows_alt);
	c->rows_lorder = true;
}

void rows_row_order(vbfm_ctx *c)
{
	if (!c->rows_lorder) return;
	if (c->estore) HIPCHK(vbk::rows_gather(c->rows_alt, c->rows, c->lpos0, c->tr.n, c->s));
	else HIPCHK(vbk::rows_scatter(c->rows_alt, c->rows, c->lrow0, c->tr.n, c->s));
	std::swap(c->rows, c->rows_alt);
	c->rows_lorder = false;
}

// the data-set sums (w0, alpha / free energy, train quirk) read N consecutive records: the
// field store's level-0 order is such a permutation, the entry store's slots are not
void rows_dense(vbfm_ctx *c)
{
	if (c->estore) rows_row_order(c);
}

// ---- feature shards (vbfm_set_shard_mode) ------------------------------------------------
void fs_free(vbfm_ctx *c)
{
	dfree(c->fs_own); dfree(c->fs_base); dfree(c->fs_buf); dfree(c->fs_pbuf); dfree(c->fs_rows0);
	c->fs_own_n = 0;
	c->fs_lo.clear();
}

// chunk s of level l: level_feats[fs_lo[l*(P+1) + s], fs_lo[l*(P+1) + s + 1])
void build_fshards(vbfm_ctx *c)
{
	fs_free(c);
	if (c->shard_mode != VBFM_SHARD_FEATURES) return;
	if (c->multi() && c->fs_req > 1 && c->fs_req != c->nranks)
		throw std::string("feature shards: num_shards must equal the number of ranks (or 0)");
	const int P = c->multi() ? c->nranks : std::max(1, c->fs_req);
	c->fs_n = P;
	const uint32_t L = nlevels(c), n = c->tr.n;
	c->fs_lo.assign((size_t)L * (P + 1), 0);
	for (uint32_t l = 0; l < L; l++) {
		const uint32_t b = c->level_ptr[l], nl = c->level_ptr[l + 1] - b;
		for (int s = 0; s <= P; s++) c->fs_lo[(size_t)l * (P + 1) + s] = b + (uint32_t)((uint64_t)nl * s / P);
	}
	if (c->multi()) {
		std::vector<uint32_t> feats(c->tr.nf), own;
		if (c->tr.nf) HIPCHK(hipMemcpy(feats.data(), c->level_feats, (size_t)c->tr.nf * 4, hipMemcpyDeviceToHost));
		for (uint32_t l = 0; l < L; l++)
			for (uint32_t i = c->fs_lo[(size_t)l * (P + 1) + c->rank]; i < c->fs_lo[(size_t)l * (P + 1) + c->rank + 1]; i++)
				own.push_back(feats[i]);
		c->fs_own = dalloc<uint32_t>(own.size());
		c->fs_own_n = (uint32_t)own.size();
		if (!own.empty()) HIPCHK(hipMemcpy(c->fs_own, own.data(), own.size() * 4, hipMemcpyHostToDevice));
		c->fs_pbuf = dalloc<double2>(c->tr.nf);
	}
	c->fs_base = dalloc<double>(2 * (size_t)n);
	c->fs_buf = dalloc<double>(5 * (size_t)n);
	if (!c->multi() && P > 1) c->fs_rows0 = dalloc<RowRec>(n);
}

// one level of one shard: the shard's chunk of the level's columns (fused kernels; the fused
// q-cache does not restart at a row's first entry: each shard sums its own entries into the
// zeroed slot)
void sweep_level_shard(vbfm_ctx *c, uint32_t l, bool is_w, int f, int s)
{
	LevelArgs a = level_args(c, l, is_w, f);
	const size_t P1 = (size_t)c->fs_n + 1;
	const uint32_t lo = c->fs_lo[l * P1 + s], hi = c->fs_lo[l * P1 + s + 1];
	a.feats = c->level_feats + lo;
	a.nfeat = hi - lo;
	a.feat_base += lo - c->level_ptr[l];   // (used only when the level is consecutive ids)
	a.first_mask = 0;
	if (a.nfeat == 0) return;
	const size_t p = prof_begin(c, is_w ? 1 : 0);
	HIPCHK(is_w ? vbk::w_level_fused(a, c->s) : vbk::v_level_fused(a, c->s));
	prof_end(c, p);
}

// the w sweep (is_w) or the v sweep of factor f, feature-sharded: every shard starts from
// the same row caches and sweeps its chunks (fm_learn_vb.h:390-406 / :420-438 restricted to
// its columns), then the shards' changes are summed
void fs_pass(vbfm_ctx *c, bool is_w, int f)
{
	const uint32_t n = c->tr.n;
	const int next = is_w ? (c->k > 0 ? 0 : -1) : (f + 1 < c->k ? ((f + 1) & 1) : -1);
	const bool local = !c->multi();   // shards run here one after another
	const int s0 = local ? 0 : c->rank, s1 = local ? c->fs_n : c->rank + 1;
	HIPCHK(vbk::fs_begin(c->rows, n, c->fs_base, next, c->s));
	if (local && c->fs_n > 1)
		HIPCHK(hipMemcpyAsync(c->fs_rows0, c->rows, (size_t)n * sizeof(RowRec), hipMemcpyDeviceToDevice, c->s));
	for (int s = s0; s < s1; s++) {
		if (s > s0)
			HIPCHK(hipMemcpyAsync(c->rows, c->fs_rows0, (size_t)n * sizeof(RowRec), hipMemcpyDeviceToDevice, c->s));
		for (uint32_t l = 0; l < nlevels(c); l++) sweep_level_shard(c, l, is_w, f, s);
		HIPCHK(vbk::fs_pack(c->rows, n, c->fs_base, c->fs_buf, next, s > s0, c->s));
	}
	if (c->multi()) {
		// the pass's exchange follows its last level
		XPhase ph(c, is_w ? "w pass (feature shards)" : "v pass (feature shards)", is_w ? -1 : f,
		          (int)nlevels(c) - 1);
		allreduce_dev(c, c->fs_buf, (next < 0 ? 2 : 5) * (size_t)n, ncclDouble, ncclSum);
		// parameters: each rank contributes its own features, zero elsewhere
		double2 *ms = is_w ? c->ms_w : c->ms_v + f;
		const uint32_t stride = is_w ? 1 : (uint32_t)c->k;
		HIPCHK(hipMemsetAsync(c->fs_pbuf, 0, (size_t)c->tr.nf * 16, c->s));
		HIPCHK(vbk::fs_params(ms, stride, c->fs_own, c->fs_own_n, c->fs_pbuf, 1, c->s));
		allreduce_dev(c, c->fs_pbuf, 2 * (size_t)c->tr.nf, ncclDouble, ncclSum);
		HIPCHK(vbk::fs_params(ms, stride, c->level_feats, c->tr.nf, c->fs_pbuf, 0, c->s));
	}
	HIPCHK(vbk::fs_unpack(c->rows, n, c->fs_base, c->fs_buf, next, c->s));
}

// VBFM_CHECK=1: verify on the device that no level lets two columns touch one row (the
// property that makes the concurrent level kernels race-free and equal to the sequential sweep)
void check_schedule(vbfm_ctx *c)
{
	const uint32_t n = c->tr.n;
	uint32_t *owner = dalloc<uint32_t>(n), *bad = dalloc<uint32_t>(1);
	HIPCHK(hipMemsetAsync(bad, 0, 4, c->s));
	for (uint32_t l = 0; l < nlevels(c); l++) {
		HIPCHK(hipMemsetAsync(owner, 0xFF, (size_t)n * 4, c->s));
		HIPCHK(vbk::check_level(c->level_feats + c->level_ptr[l], c->level_ptr[l + 1] - c->level_ptr[l], c->tr.col_ptr,
		                        c->tr.csc, c->dup, owner, bad, c->s));
	}
	uint32_t nb = 0;
	HIPCHK(d2h(c, &nb, bad, 4));
	sync(c);
	dfree(owner);
	dfree(bad);
	if (nb) throw std::string("VBFM_CHECK: dependency schedule violated (") + std::to_string(nb) + " row claims)";
}

// The levels in Kahn's order (vbfm_kernels.hip k_kahn_*): rounds are queued 32 at a time; one
// read of the append counter per batch tells when every feature has its level.
static void kahn_levels(vbfm_ctx *c, uint32_t *level)
{
	DevData &d = c->tr;
	const uint32_t nf = d.nf;
	c->sched_kahn = true;
	if (nf == 0) return;
	const int batch = 32;
	const size_t nb = (size_t)nf + 2 * batch + 3;
	struct Bufs {   // freed on every exit, the error ones included
		uint32_t *indeg = nullptr, *order = nullptr, *tail = nullptr, *bounds = nullptr;
		~Bufs() { dfree(indeg); dfree(order); dfree(tail); dfree(bounds); }
	} b;
	uint32_t *indeg = b.indeg = dalloc<uint32_t>(nf), *order = b.order = dalloc<uint32_t>(nf);
	uint32_t *tail = b.tail = dalloc<uint32_t>(1), *bounds = b.bounds = dalloc<uint32_t>(nb);
	HIPCHK(vbk::kahn_init(d.row_ptr, d.csr, d.n, nf, indeg, level, order, tail, bounds, c->s));
	uint32_t prev = 0xFFFFFFFFu;
	for (int t = 0;; t += batch) {
		if ((size_t)t + batch + 2 >= nb) throw std::string("level schedule did not converge");
		for (int u = t; u < t + batch; u++)
			HIPCHK(vbk::kahn_round(d.col_ptr, d.csc, d.row_ptr, d.csr, bounds, u, indeg, level, order, tail, c->s));
		uint32_t tl = 0;
		HIPCHK(d2h(c, &tl, tail, 4));
		sync(c);
		c->sched_rounds += batch;
		if (tl == nf) break;
		if (tl == prev || tl > nf) throw std::string("level schedule did not converge (a feature cycle)");
		prev = tl;
	}
}

// Dependency levels of the train features (see vbfm_kernels.hip header). With several
// row shards every round's levels are max-reduced over the shards, so all ranks share one
// schedule: the one the un-sharded data set defines.
void build_schedule(vbfm_ctx *c)
{
	const double t0 = wall_s();
	c->t_schedule = c->t_store = c->t_place = 0;
	c->place_bytes = 0;
	DevData &d = c->tr;
	const uint32_t nf = d.nf;
	uint32_t *level = dalloc<uint32_t>(nf);
	uint32_t *changed = dalloc<uint32_t>(1);
	dfree(c->dup);
	c->dup = dalloc<uint8_t>(nf);
	HIPCHK(hipMemsetAsync(c->dup, 0, nf, c->s));
	HIPCHK(vbk::level_init(level, nf, c->s));
	HIPCHK(vbk::mark_dups(d.row_ptr, d.csr, d.n, c->dup, c->s));
	if (c->multi() && nf) allreduce_dev(c, c->dup, nf, ncclUint8, ncclMax);
	// VBFM_SCHEDULE: "relax" (rounds to the fixed point), "kahn" (one pass in Kahn's order), default:
	// relaxation rounds while they are cheap (field-structured data converges in two), then
	// Kahn's order; row shards relax (every round is max-reduced over the shards)
	const char *sm = getenv("VBFM_SCHEDULE");
	const int mode = c->multi() ? 0 : (sm && !strcmp(sm, "relax")) ? 0 : (sm && !strcmp(sm, "kahn")) ? 2 : 1;
	c->sched_rounds = 0;
	c->sched_kahn = false;
	for (int round = 0; mode != 2; round++) {
		if (mode == 1 && round == 3) {
			kahn_levels(c, level);
			break;
		}
		c->sched_rounds++;
		uint32_t ch = 0;
		HIPCHK(hipMemsetAsync(changed, 0, 4, c->s));
		HIPCHK(vbk::level_relax(d.row_ptr, d.csr, d.n, nf, level, changed, c->s));
		if (c->multi()) {
			if (nf) allreduce_dev(c, level, nf, ncclUint32, ncclMax);
			allreduce_dev(c, changed, 1, ncclUint32, ncclMax);
		}
		HIPCHK(d2h(c, &ch, changed, 4));
		sync(c);
		if (!ch) break;
		if (round > (int)nf + 2) throw std::string("level schedule did not converge");
	}
	if (mode == 2) kahn_levels(c, level);
	c->level_h.assign(nf, 0);
	if (nf) HIPCHK(hipMemcpy(c->level_h.data(), level, nf * 4, hipMemcpyDeviceToHost));
	dfree(level);
	dfree(changed);
	uint32_t L = 0;
	for (uint32_t j = 0; j < nf; j++) L = std::max(L, c->level_h[j]);
	c->level_ptr.assign((size_t)L + 1, 0);
	for (uint32_t j = 0; j < nf; j++) c->level_ptr[c->level_h[j]]++;
	for (uint32_t l = 0; l < L; l++) c->level_ptr[l + 1] += c->level_ptr[l];
	std::vector<uint32_t> feats(nf), pos(c->level_ptr.begin(), c->level_ptr.end() - 1);
	for (uint32_t j = 0; j < nf; j++) feats[pos[c->level_h[j] - 1]++] = j;   // ascending j per level
	dfree(c->level_feats);
	c->level_feats = dalloc<uint32_t>(nf);
	if (nf) HIPCHK(hipMemcpy(c->level_feats, feats.data(), nf * 4, hipMemcpyHostToDevice));
	std::vector<uint64_t> cp((size_t)nf + 1, 0);
	HIPCHK(hipMemcpy(cp.data(), d.col_ptr, ((size_t)nf + 1) * 8, hipMemcpyDeviceToHost));
	c->level_avg.assign(L, 0);
	c->level_base.assign(L, ~0u);
	for (uint32_t l = 0; l < L; l++) {
		const uint32_t lo = c->level_ptr[l], hi = c->level_ptr[l + 1];   // ascending, distinct ids
		if (hi > lo && feats[hi - 1] - feats[lo] == hi - lo - 1) c->level_base[l] = feats[lo];
	}
	for (uint32_t l = 0; l < L; l++) {
		uint64_t z = 0;
		for (uint32_t i = c->level_ptr[l]; i < c->level_ptr[l + 1]; i++) z += cp[feats[i] + 1] - cp[feats[i]];
		const uint32_t nfl = c->level_ptr[l + 1] - c->level_ptr[l];
		c->level_avg[l] = nfl ? (uint32_t)std::min<uint64_t>(z / nfl, 0xFFFFFFFFu) : 0;
	}
	uint32_t maxlev = 0;
	for (uint32_t l = 0; l < L; l++) maxlev = std::max(maxlev, c->level_ptr[l + 1] - c->level_ptr[l]);
	if ((c->row_comm() || c->force_split) && maxlev > c->stats_cap) {
		dfree(c->stats);
		c->stats = dalloc<double2>(maxlev);
		c->stats_cap = maxlev;
	}
	c->sched_ready = true;
	// a failure from here on (the store's allocations, the placement search) leaves the schedule to
	// be rebuilt by the next call instead of running on a half-built store
	try {
		const char *chk = getenv("VBFM_CHECK");
		if (chk && chk[0] == '1') check_schedule(c);
		build_fshards(c);
		const double t1 = wall_s();
		c->t_schedule = t1 - t0;
		build_lorder(c, cp, feats);
		c->t_store = wall_s() - t1;
	} catch (...) {
		c->sched_ready = false;
		// the half-built store goes too (the records are still in row order: the search puts them
		// back before it fails); the next call builds it from scratch
		try {
			lord_release(c, true);
		} catch (...) {
		}
		throw;
	}
}

// segments of the hyper / free-energy sums: (w or factor f) x group. The attributes are
// ordered by group (perm) and cut into chunks inside a group, ~2048 of them for a large D
// (256..4096 attributes each: enough workgroups to keep the loads in flight); one chunk list
// serves the w segments (one workgroup per chunk) and the factors (one workgroup per chunk for
// all k factors: k_vsums)
void build_chunks(vbfm_ctx *c)
{
	std::vector<uint32_t> perm(c->D), gptr((size_t)c->G + 1, 0);
	for (uint32_t i = 0; i < c->D; i++) gptr[c->group_h[i] + 1]++;
	for (uint32_t g = 0; g < c->G; g++) gptr[g + 1] += gptr[g];
	std::vector<uint32_t> pos(gptr.begin(), gptr.end() - 1);
	for (uint32_t i = 0; i < c->D; i++) perm[pos[c->group_h[i]]++] = i;
	c->chunks_h.clear();
	std::vector<uint32_t> gchunk((size_t)c->G + 1, 0);
	const uint32_t CH = std::min<uint32_t>(4096, std::max<uint32_t>(256, (c->D + 2047) / 2048));
	for (uint32_t g = 0; g < c->G; g++) {
		gchunk[g] = (uint32_t)c->chunks_h.size();
		for (uint32_t b = gptr[g]; b < gptr[g + 1]; b += CH)
			c->chunks_h.push_back(vbk::Chunk{b, std::min(b + CH, gptr[g + 1]), -1, g});
	}
	gchunk[c->G] = (uint32_t)c->chunks_h.size();
	const size_t nc = c->chunks_h.size();
	c->perm_d = dalloc<uint32_t>(c->D);
	if (c->D) HIPCHK(hipMemcpy(c->perm_d, perm.data(), c->D * 4, hipMemcpyHostToDevice));
	c->chunks_d = dalloc<vbk::Chunk>(nc);
	if (nc) HIPCHK(hipMemcpy(c->chunks_d, c->chunks_h.data(), nc * sizeof(vbk::Chunk), hipMemcpyHostToDevice));
	c->gchunk_d = dalloc<uint32_t>(gchunk.size());
	HIPCHK(hipMemcpy(c->gchunk_d, gchunk.data(), gchunk.size() * 4, hipMemcpyHostToDevice));
	c->chunk_out_d = dalloc<double>(nc + (size_t)c->k * c->G);   // w partials, then the factor sums
	c->vseg_d = c->chunk_out_d + nc;
	c->vpart_d = dalloc<double>(nc * (size_t)std::max(c->k, 1));
}

// w: chunk results summed per group in chunk order on the host; factors: k_vsums (fixed
// order on the device). seg index = (f+1)*G + g
std::vector<double> seg_sums(vbfm_ctx *c, int model, int mode, const double *hw, const double *hv, bool want_w,
                             bool want_v)
{
	const size_t nc = c->chunks_h.size();
	const size_t G = c->G, kg = (size_t)c->k * G;
	std::vector<double> out(nc + kg), seg((size_t)(c->k + 1) * G, 0.0);
	want_w = want_w && nc;
	want_v = want_v && nc && kg;
	if (want_w) {
		if (model == 0)
			HIPCHK(vbk::param_sums(c->ms_w, c->ms_v, c->perm_d, c->D, c->chunks_d, (uint32_t)nc, mode, hw, hv, c->k,
			                       c->chunk_out_d, c->s));
		else
			HIPCHK(vbk::mc_param_sums(c->ms_w, c->ms_v, c->perm_d, c->chunks_d, (uint32_t)nc, mode, hw, hv, c->k,
			                          c->chunk_out_d, c->s));
	}
	if (want_v)
		HIPCHK(vbk::vsums(c->ms_v, c->perm_d, c->chunks_d, (uint32_t)nc, c->gchunk_d, c->G, model, mode, hv, c->k,
		                  c->vpart_d, c->vseg_d, c->s));
	// one copy of what was computed: [w partials | factor sums]
	const size_t lo = want_w ? 0 : nc, hi = want_v ? nc + kg : nc;
	if (hi > lo) HIPCHK(d2h(c, out.data() + lo, c->chunk_out_d + lo, (hi - lo) * 8));
	sync(c);
	if (want_w)
		for (size_t i = 0; i < nc; i++) seg[c->chunks_h[i].g] += out[i];
	if (want_v) std::copy(out.begin() + nc, out.end(), seg.begin() + G);
	return seg;
}

std::vector<double> param_sums(vbfm_ctx *c, int mode)
{
	return seg_sums(c, 0, mode, c->hyp_w_d, c->hyp_v_d, true, true);
}

void upload_hyp(vbfm_ctx *c)
{
	HIPCHK(hipMemcpyAsync(c->hyp_w_d, c->hyp_w.data(), c->G * 8, hipMemcpyHostToDevice, c->s));
	if (c->k) HIPCHK(hipMemcpyAsync(c->hyp_v_d, c->hyp_v.data(), (size_t)c->G * c->k * 8, hipMemcpyHostToDevice, c->s));
}

void require_train(vbfm_ctx *c)
{
	if (!c->rows) throw std::string("no train data set (vbfm_set_train)");
	if (!c->sched_ready) build_schedule(c);
}

// VBFM_PREFETCH=0 (A/B): the level kernels do not touch the next level's column bounds (read once
// per context)
static bool pf_enabled(vbfm_ctx *c)
{
	if (c->prefetch < 0) {
		const char *e = getenv("VBFM_PREFETCH");
		c->prefetch = (e && e[0] == '0') ? 0 : 1;
	}
	return c->prefetch != 0;
}

LevelArgs level_args(vbfm_ctx *c, uint32_t l, bool is_w, int f)
{
	LevelArgs a = {};
	a.col_ptr = c->tr.col_ptr;
	a.csc = c->tr.csc;
	a.feats = c->level_feats + c->level_ptr[l];
	a.feat_contig = l < c->level_base.size() && c->level_base[l] != ~0u;
	a.feat_base = a.feat_contig ? c->level_base[l] : 0u;
	a.nfeat = c->level_ptr[l + 1] - c->level_ptr[l];
	a.rows = c->rows;
	a.ms = is_w ? c->ms_w : c->ms_v + f;
	a.ms_stride = is_w ? 1 : (uint32_t)c->k;
	a.ms_stride_next = (uint32_t)c->k;
	a.hyp = is_w ? c->hyp_w_d : c->hyp_v_d + f;
	a.hyp_stride = is_w ? 1 : (uint32_t)c->k;
	// one attribute group: the level kernels take the prior by value (hyp_w / hyp_v on the host
	// are the values last pushed to hyp_w_d / hyp_v_d)
	a.hyp_uniform = c->G == 1;
	a.hyp0 = c->G == 1 ? (is_w ? c->hyp_w[0] : c->hyp_v[f]) : 0.0;
	a.attr_group = c->group_d;
	a.dup = c->dup;
	a.alpha = c->alpha;
	a.counters = c->counters;
	a.stats = c->stats;
	a.skew = c->debug_skew;
	a.avg_len = c->level_avg[l];
	a.first_mask = ROW_FIRST;
	if (is_w) {
		a.slot = 0;                                          // fused q-cache of factor 0
		a.ms_next = c->k > 0 ? c->ms_v : nullptr;          // factor 0: ms_v[j*k + 0]
	} else {
		a.slot = f & 1;
		a.ms_next = f + 1 < c->k ? c->ms_v + (f + 1) : nullptr;
	}
	return a;
}

// event pair around one launch when profiling (the pool grows on first use)
size_t prof_begin(vbfm_ctx *c, int kind, hipStream_t st)
{
	if (!c->profiling) return NO_SPAN;
	if (c->prof_stride > 1 && c->prof_tick[kind]++ % (uint64_t)c->prof_stride != 0) return NO_SPAN;
	if (c->pev_used + 2 > c->pev.size()) {
		const size_t add = std::max<size_t>(256, c->pev.size());
		for (size_t i = 0; i < add; i++) {
			// timestamps only: no system-scope release / acquire (a default event's cache
			// writeback + invalidate costs ~4 us per record between short level launches)
			hipEvent_t e;
			HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
			c->pev.push_back(e);
		}
	}
	const size_t a = c->pev_used;
	c->pev_used += 2;
	HIPCHK(hipEventRecord(c->pev[a], st ? st : c->s));
	c->spans.push_back(vbfm_ctx::Span{a, kind});
	return a;
}

void prof_end(vbfm_ctx *c, size_t a, hipStream_t st)
{
	if (c->profiling && a != NO_SPAN) HIPCHK(hipEventRecord(c->pev[a + 1], st ? st : c->s));
}

void sweep_level(vbfm_ctx *c, uint32_t l, bool is_w, int f)
{
	LevelArgs a = level_args(c, l, is_w, f);
	if (a.nfeat == 0) return;
	Range r("level", 2);
	XPhase ph(c, is_w ? "w sweep" : "v sweep", is_w ? -1 : f, (int)l);
	const size_t p = prof_begin(c, is_w ? 1 : 0);
	if (c->ov) {
		// online VB: the level's columns restricted to the mini-batch (column layout, one GPU)
		ov_level_args(c, a, is_w, f);
		ov_launch_level(c, a, l, is_w);
		prof_end(c, p);
		return;
	}
	if (c->lord) {
		// level-ordered store: stream this level's records, move them to the next level's order
		a.lcp = c->lcp + c->level_ptr[l];
		{   // the level after this one in launch order: l + 1, or level 0 of the next sweep
			const uint32_t ln = l + 1 < nlevels(c) ? l + 1 : 0;
			a.pf_lcp = pf_enabled(c) ? c->lcp + c->level_ptr[ln] : nullptr;
			const bool contig = ln < c->level_base.size() && c->level_base[ln] != ~0u;
			a.pf_feats = contig ? nullptr : c->level_feats + c->level_ptr[ln];
			a.pf_n = a.pf_lcp ? c->level_ptr[ln + 1] - c->level_ptr[ln] : 0u;
		}
		a.lx = c->lx;
		a.lnext = c->lnext;
		a.lbase = (uint64_t)l * c->tr.n;
		a.src = c->rows;
		a.dst = c->rows_alt;
		a.first_level = l == 0;
		if (c->estore) {   // one store, global slots: records move to their rows' next slots in place
			a.lbase = 0;
			a.dst = c->rows;
			a.ent = 1;
			a.tab_base = c->level_ptr[l];
			a.lfirst = c->lpos0;
			a.ent_nnz = c->tr.nnz;
			if (!c->row_comm() && !c->force_split) {
				HIPCHK(vbk::lord_level(a, is_w, c->s));
				prof_end(c, p);
				return;
			}
		}
		if (!c->row_comm() && !c->force_split) {
			if (c->long_min) {
				a.long_min = c->long_min_l[l];
				a.segs = c->long_segs + c->seg_ptr[l];
				a.nsegs = c->seg_ptr[l + 1] - c->seg_ptr[l];
				a.seg_part = c->seg_part;
			}
			HIPCHK(vbk::lord_level(a, is_w, c->s));
			HIPCHK(vbk::lord_long(a, is_w, c->s));
		} else if (c->deferred()) {
			// deferred: level l-1's correction, level l's statistics and the move in one pass;
			// level l's correction after the all-reduce, by level l+1 (or the flush)
			a.lpay = c->lpay;
			a.lpay2 = c->lpay2;
			a.tab = c->post_tab;
			// level 0 of a v sweep may carry the previous sweep's last correction (vbfm_iterate);
			// in the entry store the rows' first entries -- which carry it -- lie in every level
			if (l == 0) {
				c->carry_in = (c->carry != 0 && !is_w) ? (c->carry == 3 ? 2 : 1) : 0;
				c->carry = 0;
			}
			const bool carried = (l == 0 || c->estore) && c->carry_in != 0;
			a.pend_kind = carried ? c->carry_in : 0;
			a.pending = (l > 0 || carried) ? 1 : 0;
			a.pending |= defer_nt(c);   // non-temporal record loads (2) / stores (4)
			a.first_prev = l == 1;
			stats_exchange(c, a, [&](const LevelArgs &b) { HIPCHK(vbk::lord_defer_level(b, is_w, c->s)); });
			HIPCHK(vbk::lord_defer_post(a, is_w, c->s));
			if (l + 1 == nlevels(c)) {
				// the sweep's last correction: left to level 0 of the next sweep when one follows
				// inside update_all (the w sweep -> factor 0, factor f -> f+1), else applied in
				// place on the level-0-ordered records
				const bool carry_out = c->carry_ok && (is_w ? c->k > 0 : f + 1 < c->k);
				if (carry_out) {
					c->carry = is_w ? 3 : 1 + (f & 1);
				} else {
					a.dst = c->estore ? c->rows : c->rows_alt;   // (the field store's: swapped below)
					a.first_prev = l == 0;
					HIPCHK(vbk::lord_defer_flush(a, is_w, c->tr.n, c->s));
				}
			}
		} else {
			stats_exchange(c, a, [&](const LevelArgs &b) { HIPCHK(vbk::lord_level_stats(b, is_w, c->s)); });
			HIPCHK(vbk::lord_level_move(a, is_w, c->s));
		}
		if (!c->estore) std::swap(c->rows, c->rows_alt);
		prof_end(c, p);
		return;
	}
	if (!c->row_comm() && !c->force_split) {
		if (c->long_min) {
			a.long_min = c->long_min_l[l];
			a.segs = c->long_segs + c->seg_ptr[l];
			a.nsegs = c->seg_ptr[l + 1] - c->seg_ptr[l];
			a.seg_part = c->seg_part;
		}
		HIPCHK(is_w ? vbk::w_level_fused(a, c->s) : vbk::v_level_fused(a, c->s));
		HIPCHK(vbk::col_long(a, is_w, c->s));
		prof_end(c, p);
		return;
	}
	// row-sharded form: per-feature sufficient statistics of this shard's rows, summed over
	// the shards, then every shard applies the identical posterior to its own rows
	stats_exchange(c, a, [&](const LevelArgs &b) {
		HIPCHK(is_w ? vbk::w_level_stats(b, c->s) : vbk::v_level_stats(b, c->s));
	});
	HIPCHK(is_w ? vbk::w_level_correct(a, c->s) : vbk::v_level_correct(a, c->s));
	prof_end(c, p);
}

uint32_t nlevels(vbfm_ctx *c) { return c->level_ptr.empty() ? 0 : (uint32_t)c->level_ptr.size() - 1; }

// ---- the steps of update_all ------------------------------------------------------------
void step_w0(vbfm_ctx *c)
{
	// update_w0 (fm_learn_vb.h:504-525)
	const double sigma_old = c->s0d;
	c->s0d = 1.0 / (c->sigma_0 + (double)c->n_global * c->alpha);
	rows_dense(c);
	HIPCHK(vbk::row_sums(c->rows, c->tr.n, 0, c->mu0, c->red_d, c->RED_BLOCKS, c->s));
	double w0_temp = finish_sum(c, c->RED_BLOCKS);
	allreduce_host(c, &w0_temp, 1);
	const double mu_old = c->mu0;
	c->mu0 = c->s0d * c->alpha * w0_temp;
	HIPCHK(vbk::w0_apply(c->rows, c->tr.n, mu_old - c->mu0, c->s0d - sigma_old, c->s));
}

// the w sweep; with factors it also leaves the q-cache of factor 0 in slot 0
void step_w(vbfm_ctx *c)
{
	rows_level_order(c);
	if (c->shard_mode == VBFM_SHARD_FEATURES) fs_pass(c, true, 0);
	else
		for (uint32_t l = 0; l < nlevels(c); l++) sweep_level(c, l, true, 0);
	if (c->k > 0) c->q_ready[0] = 0;
}

// make the q-cache of factor f current (zero + add_main_q, fm_learn_vb.h:411-418): a no-op
// when the previous sweep already accumulated it, else the row-parallel kernel
void step_qcache(vbfm_ctx *c, int f)
{
	const int slot = f & 1;
	if (c->q_ready[slot] != f) {
		const size_t p = prof_begin(c, 2);
		rows_level_order(c);
		HIPCHK(vbk::qcache(c->tr.row_ptr, c->tr.csr, c->ms_v + f, (uint32_t)c->k, c->rows, c->tr.n, slot,
		                   c->rows_lorder ? c->lpos0 : nullptr, c->s));
		prof_end(c, p);
		c->q_ready[slot] = f;
	}
	c->qslot = slot;
}

// the v sweep of factor f (which also accumulates the q-cache of factor f+1)
void step_v(vbfm_ctx *c, int f)
{
	rows_level_order(c);
	if (c->shard_mode == VBFM_SHARD_FEATURES) fs_pass(c, false, f);
	else
		for (uint32_t l = 0; l < nlevels(c); l++) sweep_level(c, l, false, f);
	c->qslot = f & 1;
	c->q_ready[f & 1] = -1;   // corrected in place, no longer the from-scratch sum add_main_q gives
	if (f + 1 < c->k) c->q_ready[(f + 1) & 1] = f + 1;
	else c->q_ready[(f + 1) & 1] = -1;
}

// ---- per-level steps (vbfm_step_w_level / vbfm_step_v_level) ----------------------------
void no_partial(vbfm_ctx *c)
{
	if (c->part_kind >= 0)
		throw std::string("a sweep driven level by level is in progress (finish it with vbfm_step_*_level)");
	if (c->part_kind == -2)
		throw std::string("a level of a sweep driven level by level failed: the row caches are undefined "
		                  "(vbfm_set_train or vbfm_load_state starts again)");
}

// level l of the w sweep (is_w) or of factor f's v sweep, exactly as the whole sweep runs it;
// levels must come in order 0..L-1. One rank's fused kernels or the two-pass split (the
// deferred split leaves a level's correction to the next level's kernel, so no per-level state
// would exist to compare)
void step_level(vbfm_ctx *c, bool is_w, int f, uint32_t l)
{
	const uint32_t L = nlevels(c);
	if (c->shard_mode == VBFM_SHARD_FEATURES) throw std::string("per-level steps: not with feature shards");
	if (c->deferred()) throw std::string("per-level steps: the deferred split keeps each level's correction pending (VBFM_DEFER=0)");
	if (l >= L) throw std::string("level out of range");
	const int kind = is_w ? 0 : 1;
	if (c->part_kind == -2) no_partial(c);
	if (c->part_kind < 0 ? l != 0 : (c->part_kind != kind || c->part_f != f || c->part_next != l))
		throw std::string("per-level steps: levels of a sweep must come in order from level 0");
	if (l == 0) {
		if (is_w) rows_level_order(c);
		else {
			step_qcache(c, f);   // a no-op when current
			rows_level_order(c);
		}
	}
	try {
		sweep_level(c, l, is_w, f);
		if (l == 1 && fault_at("level")) throw HipError{hipErrorLaunchFailure, "VBFM_FAULT=level"};
	} catch (...) {
		c->part_kind = -2;   // the records may be half moved: refuse everything until a restart
		throw;
	}
	c->part_kind = kind; c->part_f = f; c->part_next = l + 1;
	if (!is_w) c->qslot = f & 1;
	if (l + 1 < L) return;
	c->part_kind = -1;   // the sweep is complete: the bookkeeping of step_w / step_v
	if (is_w) {
		if (c->k > 0) c->q_ready[0] = 0;
	} else {
		c->q_ready[f & 1] = -1;
		c->q_ready[(f + 1) & 1] = f + 1 < c->k ? f + 1 : -1;
	}
}

// the records in row order while a level-by-level sweep of a level-ordered store is half done:
// the field store holds them in the order of the next level (position p = the p-th entry of
// that level's columns, features in schedule order, rows ascending), the entry store in the slot
// of each row's next entry of a later level (else its first slot; rows without entries park at
// nnz + r). Host-side debug readback.
std::vector<RowRec> rows_mid_sweep(vbfm_ctx *c)
{
	const uint32_t n = c->tr.n, nf = c->tr.nf, L = nlevels(c);
	const uint64_t nnz = c->tr.nnz;
	std::vector<uint64_t> cp((size_t)nf + 1);
	std::vector<uint2> ent(nnz);
	std::vector<uint32_t> feats(nf);
	HIPCHK(hipMemcpy(cp.data(), c->tr.col_ptr, cp.size() * 8, hipMemcpyDeviceToHost));
	if (nnz) HIPCHK(hipMemcpy(ent.data(), c->tr.csc, nnz * 8, hipMemcpyDeviceToHost));
	if (nf) HIPCHK(hipMemcpy(feats.data(), c->level_feats, (size_t)nf * 4, hipMemcpyDeviceToHost));
	const size_t nrec = c->estore ? nnz + n : n;
	std::vector<RowRec> store(nrec), out(n);
	if (nrec) HIPCHK(hipMemcpy(store.data(), c->rows, nrec * sizeof(RowRec), hipMemcpyDeviceToHost));
	const uint32_t done = c->part_next;   // levels 0 .. done-1 are swept
	if (!c->estore) {
		uint64_t p = 0;
		for (uint32_t i = c->level_ptr[done % L]; i < c->level_ptr[done % L + 1]; i++) {
			const uint32_t j = feats[i];
			for (uint64_t e = cp[j]; e < cp[j + 1]; e++) out[ent[e].x & ~ROW_FIRST] = store[p++];
		}
		if (p != n) throw std::string("internal: a level of the field store does not hold every row");
		return out;
	}
	std::vector<uint64_t> first(n, ~0ull), next(n, ~0ull);
	uint64_t s = 0;
	for (uint32_t l = 0; l < L; l++)
		for (uint32_t i = c->level_ptr[l]; i < c->level_ptr[l + 1]; i++) {
			const uint32_t j = feats[i];
			for (uint64_t e = cp[j]; e < cp[j + 1]; e++, s++) {
				const uint32_t r = ent[e].x & ~ROW_FIRST;
				if (first[r] == ~0ull) first[r] = s;
				if (l >= done && next[r] == ~0ull) next[r] = s;
			}
		}
	for (uint32_t r = 0; r < n; r++)
		out[r] = store[next[r] != ~0ull ? next[r] : first[r] != ~0ull ? first[r] : nnz + r];
	return out;
}

double rows_energy(vbfm_ctx *c)
{
	rows_dense(c);
	HIPCHK(vbk::row_sums(c->rows, c->tr.n, 1, 0.0, c->red_d, c->RED_BLOCKS, c->s));
	double s = finish_sum(c, c->RED_BLOCKS);
	allreduce_host(c, &s, 1);
	return s;
}

// fm_learn_vb.h:446-498; returns true on the early return of a NaN/inf alpha
bool step_hyper(vbfm_ctx *c, double *energy_out, uint32_t *nan_alpha, uint32_t *inf_alpha)
{
	const double energy = rows_energy(c);
	if (energy_out) *energy_out = energy;
	const double alpha_old = c->alpha;
	c->alpha = (double)c->n_global / energy;
	if (std::isnan(c->alpha)) { if (nan_alpha) (*nan_alpha)++; c->alpha = alpha_old; return true; }
	if (std::isinf(c->alpha)) { if (inf_alpha) (*inf_alpha)++; c->alpha = alpha_old; return true; }
	c->sigma_0 = 1.0 / (c->mu0 * c->mu0 + c->s0d);
	std::vector<double> seg = param_sums(c, 0);
	for (uint32_t g = 0; g < c->G; g++) c->hyp_w[g] = (double)c->per_group[g] / seg[g];
	for (int f = 0; f < c->k; f++)
		for (uint32_t g = 0; g < c->G; g++)
			c->hyp_v[(size_t)g * c->k + f] = (double)c->per_group[g] / seg[(size_t)(f + 1) * c->G + g];
	upload_hyp(c);
	return false;
}

// free_energy (fm_learn_vb.h:646-681), given sum(e^2 + t)
double free_energy(vbfm_ctx *c, double energy)
{
	const double temp1 = 2 * 3.14 * (1.0 / c->alpha);
	double fe = 0.0;
	fe += -0.5 * c->alpha * energy - .5 * (double)c->n_global * std::log(temp1);
	fe += -0.5 * c->sigma_0 * (c->mu0 * c->mu0 + c->s0d) + 0.5 * std::log(c->s0d * c->sigma_0) + .5;
	std::vector<double> seg = param_sums(c, 1);
	for (double v : seg) fe += v;
	return fe;
}

// the reference's exact summation order for small data sets, the wave-per-row form for
// large ones (VBFM_PREDICT=exact|blocked|wave overrides)
int blocked_predict(const vbfm_ctx *c, const DevData &d)
{
	const char *env = getenv("VBFM_PREDICT");
	if (env && !strcmp(env, "exact")) return 0;
	if (env && !strcmp(env, "blocked")) return 1;
	if (env && !strcmp(env, "wave")) return 2;
	return (double)d.nnz * c->k > 5e7 ? 2 : 0;
}

void test_predict(vbfm_ctx *c, hipStream_t s)
{
	HIPCHK(vbk::predict_e(c->te.row_ptr, c->te.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, c->mu0, c->e_test, c->te.n,
	                      blocked_predict(c, c->te), s));
}

// The per-iteration test prediction (fm_learn_vb_simultaneous.h:125) reads mu0, mu_w, mu_v,
// which are final once the factor sweeps end; the hyper-parameter step and the free energy
// (fm_learn_vb.h:446-498, :646-681) only read them. So the prediction runs on its own stream
// from the end of the sweeps, under the hyper step (its reductions, host arithmetic and
// syncs), and the metrics wait for it: the same kernel on the same inputs, bit-identical
// (VBFM_TEST_OVERLAP=0 runs it after the hyper step on the main stream).
bool test_overlap()
{
	const char *e = getenv("VBFM_TEST_OVERLAP");
	return !(e && e[0] == '0');
}

void read_counters(vbfm_ctx *c, vbfm_iter_stats *o)
{
	uint32_t h[CNT_N];
	HIPCHK(d2h(c, h, c->counters, sizeof(h)));
	sync(c);
	o->nan_mu_w = h[CNT_NAN_MU_W]; o->nan_sigma_w = h[CNT_NAN_SIGMA_W]; o->inf_mu_w = h[CNT_INF_MU_W];
	o->nan_mu_v = h[CNT_NAN_MU_V]; o->nan_sigma_v = h[CNT_NAN_SIGMA_V]; o->inf_mu_v = h[CNT_INF_MU_V];
}

float ev_ms(vbfm_ctx *c, int a, int b)
{
	float ms = 0.f;
	HIPCHK(hipEventElapsedTime(&ms, c->ev[a], c->ev[b]));
	return ms;
}

}  // namespace vbi

// =========================================================================================
extern "C" {

int vbfm_abi_version(void) { return VBFM_ABI_VERSION; }

int vbfm_device_count(int32_t *n)
{
	if (!n) return fail(nullptr, "vbfm_device_count: null argument");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
	*n = ndev;
	return 0;
}

const char *vbfm_last_error(const vbfm_ctx *ctx)
{
	if (ctx) return ctx->err.c_str();
	return vbfm_host_last_error();
}

int vbfm_create(vbfm_ctx **out, const vbfm_config *cfg)
{
	if (!out || !cfg) return fail(nullptr, "vbfm_create: null argument");
	*out = nullptr;
	if (cfg->task != 0) return fail(nullptr, "task not supported by the VB learner (regression only)");
	if (cfg->num_factor < 0) return fail(nullptr, "negative number of factors");
	if (cfg->num_attr_groups == 0) return fail(nullptr, "num_attr_groups must be >= 1");
	if (cfg->place_candidates < 0) return fail(nullptr, "place_candidates must be >= 0");
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(nullptr, "no HIP device available");
	if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, "device ordinal out of range");
	vbfm_ctx *c = new vbfm_ctx();
	c->dev = cfg->device;
	c->k0 = cfg->k0 != 0; c->k1 = cfg->k1 != 0; c->k = cfg->num_factor;
	c->D = cfg->num_attribute; c->G = cfg->num_attr_groups;
	c->min_target = cfg->min_target; c->max_target = cfg->max_target;
	c->place_cands_cfg = cfg->place_candidates;
	c->place_budget_cfg = cfg->place_budget_bytes;
	{
		const char *fs = getenv("VBFM_FORCE_SPLIT");
		c->force_split = fs && fs[0] == '1';
		const char *sk = getenv("VBFM_DEBUG_SKEW");
		c->debug_skew = sk && sk[0] == '1';
	}
	int rc = guarded(c, [&] {
		HIPCHK(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking));
		HIPCHK(hipStreamCreateWithFlags(&c->s_test, hipStreamNonBlocking));
		for (int i = 0; i < EV_N; i++) HIPCHK(hipEventCreate(&c->ev[i]));
		c->group_h.assign(c->D, 0);
		if (cfg->attr_group)
			for (uint32_t i = 0; i < c->D; i++) {
				if (cfg->attr_group[i] >= c->G) throw std::string("attr_group out of range");
				c->group_h[i] = cfg->attr_group[i];
			}
		c->per_group.assign(c->G, 0);
		for (uint32_t i = 0; i < c->D; i++) c->per_group[c->group_h[i]]++;
		c->group_d = dalloc<uint32_t>(c->D);
		if (c->D) HIPCHK(hipMemcpy(c->group_d, c->group_h.data(), c->D * 4, hipMemcpyHostToDevice));
		c->ms_v = dalloc<double2>((size_t)c->k * c->D);
		c->ms_w = dalloc<double2>(c->D);
		c->hyp_w_d = dalloc<double>(c->G);
		c->hyp_v_d = dalloc<double>((size_t)c->G * c->k);
		c->hyp_w.assign(c->G, 1.0);               // fm_learn_vb.h:707-708
		c->hyp_v.assign((size_t)c->G * c->k, 1.0);
		upload_hyp(c);
		// fm_learn_vb.h:693-712 defaults: mu 0 until set_params, sigma .02
		std::vector<double2> init((size_t)std::max<uint64_t>((uint64_t)c->k * c->D, c->D), make_double2(0.0, .02));
		if ((size_t)c->k * c->D)
			HIPCHK(hipMemcpy(c->ms_v, init.data(), (size_t)c->k * c->D * 16, hipMemcpyHostToDevice));
		if (c->D) HIPCHK(hipMemcpy(c->ms_w, init.data(), (size_t)c->D * 16, hipMemcpyHostToDevice));
		c->red_d = dalloc<double>(2 * vbfm_ctx::RED_BLOCKS);
		c->red_h.assign(2 * vbfm_ctx::RED_BLOCKS, 0.0);
		c->counters = dalloc<uint32_t>(CNT_N);
		HIPCHK(hipMemset(c->counters, 0, CNT_N * 4));
		build_chunks(c);
	});
	if (rc) {
		vbfm_host_set_error(c->err.c_str());
		vbfm_destroy(c);
		return rc;
	}
	*out = c;
	return 0;
}

void vbfm_destroy(vbfm_ctx *c)
{
	if (!c) return;
	(void)hipSetDevice(c->dev);
	if (c->comm_failed && c->s) {
		// an aborted communicator: RCCL's kernels leave on the abort, but a stream still busy after
		// 10 s is left to the process's exit (freeing under it would block in a device synchronise)
		const double end = wall_s() + 10.0;
		while (hipStreamQuery(c->s) == hipErrorNotReady && wall_s() < end) usleep(1000);
		if (hipStreamQuery(c->s) == hipErrorNotReady) {
			delete c;
			return;
		}
	}
	if (c->s) (void)hipStreamSynchronize(c->s);
	free_data(c->tr);
	free_data(c->te);
	dfree(c->rows); dfree(c->scratch_n); dfree(c->e_test); dfree(c->pred_test);
	dfree(c->ms_v); dfree(c->ms_w); dfree(c->hyp_w_d); dfree(c->hyp_v_d); dfree(c->group_d);
	dfree(c->level_feats); dfree(c->dup); dfree(c->red_d); dfree(c->perm_d); dfree(c->chunks_d);
	dfree(c->chunk_out_d); c->vseg_d = nullptr; dfree(c->gchunk_d); dfree(c->vpart_d); dfree(c->counters); dfree(c->stats);
	dfree(c->rows_alt); dfree(c->lcp); dfree(c->lx); dfree(c->lnext); dfree(c->lrow0); dfree(c->lpos0);
	fs_free(c);
	mc_free(c);
	ov_free(c);
	if (c->comm) ncclCommDestroy(c->comm);
	if (c->stall_flag) (void)hipHostFree(c->stall_flag);
	for (hipEvent_t e : c->ev_ar)
		if (e) (void)hipEventDestroy(e);
	if (c->ev_arj) (void)hipEventDestroy(c->ev_arj);
	if (c->s_comm) (void)hipStreamDestroy(c->s_comm);
	for (hipEvent_t e : c->pev) (void)hipEventDestroy(e);
	for (int i = 0; i < EV_N; i++)
		if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
	if (c->s) (void)hipStreamDestroy(c->s);
	if (c->s_test) (void)hipStreamDestroy(c->s_test);
	delete c;
}

static void alloc_rows(vbfm_ctx *c)
{
	lord_release(c, false);   // a new train set: the old records are discarded
	dfree(c->rows);
	dfree(c->scratch_n);
	c->rows = dalloc<RowRec>(c->tr.n);
	c->scratch_n = dalloc<double>(c->tr.n);
	HIPCHK(hipMemsetAsync(c->rows, 0, (size_t)std::max(c->tr.n, 1u) * sizeof(RowRec), c->s));
	uint64_t n = c->tr.n;
	c->n_global = n;
	c->q_ready[0] = c->q_ready[1] = -1;
	if (c->multi()) {
		double v = (double)n;
		allreduce_host(c, &v, 1);
		c->n_global = (uint64_t)v;
	}
	c->sched_ready = false;
}

// the train feature count every shard pads to (the max over shards)
static uint32_t global_nf(vbfm_ctx *c, uint32_t nf)
{
	if (!c->multi()) return nf;
	uint32_t *w = dalloc<uint32_t>(1);
	HIPCHK(hipMemcpyAsync(w, &nf, 4, hipMemcpyHostToDevice, c->s));
	allreduce_dev(c, w, 1, ncclUint32, ncclMax);
	uint32_t out = 0;
	HIPCHK(d2h(c, &out, w, 4));
	sync(c);
	dfree(w);
	return out;
}

int vbfm_set_train(vbfm_ctx *c, const vbfm_csc *in)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		const double t0 = wall_s();
		check_csc(in);
		const uint32_t nf = global_nf(c, in->num_feature);
		if (nf > c->D) throw std::string("train num_feature exceeds num_attribute");
		upload(c, c->tr, in, nf);
		if (c->tr.n > ROW_MASK) throw std::string("too many rows for one shard (max 2^31-1)");
		HIPCHK(vbk::mark_first(c->tr.row_ptr, c->tr.csr, c->tr.col_ptr, c->tr.csc, c->tr.n, c->s));
		alloc_rows(c);
		c->part_kind = -1;   // new records: no level-by-level sweep in progress
		c->t_set_train = wall_s() - t0;
	});
}

int vbfm_set_test(vbfm_ctx *c, const vbfm_csc *in)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		check_csc(in);
		if (in->num_feature > c->D) throw std::string("test num_feature exceeds num_attribute");
		upload(c, c->te, in, in->num_feature);
		dfree(c->e_test);
		dfree(c->pred_test);
		c->e_test = dalloc<double>(c->te.n);
		c->pred_test = dalloc<double>(c->te.n);
		double v = c->te.n;
		allreduce_host(c, &v, 1);
		c->test_n_global = (uint32_t)v;
	});
}

}  // extern "C"

namespace vbi {
// the end of a synthetic data set's construction: target range, then (train) the first-entry
// marks and the row records, (test) the prediction buffers
void synth_finish(vbfm_ctx *c, int32_t which)
{
	DevData &d = which ? c->te : c->tr;
	const uint32_t n = d.n;
	// target range (min/max over the targets: 1..5 by construction, computed exactly)
	std::vector<float> t(n);
	if (n) HIPCHK(hipMemcpy(t.data(), d.target, (size_t)n * 4, hipMemcpyDeviceToHost));
	float mn = 3.40282347e+38f, mx = -3.40282347e+38f;
	for (float v : t) { mn = std::min(v, mn); mx = std::max(v, mx); }
	d.min_target = mn; d.max_target = mx;
	if (which == 0) {
		if (n > ROW_MASK) throw std::string("too many rows for one shard (max 2^31-1)");
		HIPCHK(vbk::mark_first(d.row_ptr, d.csr, d.col_ptr, d.csc, n, c->s));
		alloc_rows(c);
	} else {
		dfree(c->e_test); dfree(c->pred_test);
		c->e_test = dalloc<double>(n);
		c->pred_test = dalloc<double>(n);
		double v = n;
		allreduce_host(c, &v, 1);
		c->test_n_global = (uint32_t)v;
	}
}
}  // namespace vbi

extern "C" {

int vbfm_synth_generate(vbfm_ctx *c, int32_t which, uint32_t n, uint32_t F, uint32_t S, uint64_t seed, int32_t xmode,
                        uint64_t model_seed, uint64_t row_offset)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		const double t0 = wall_s();
		if (which != 0 && which != 1) throw std::string("which must be 0 (train) or 1 (test)");
		const uint64_t nf64 = (uint64_t)F * S;
		if (nf64 >= 0xFFFFFFFFull || nf64 >= c->D || F == 0 || S == 0)
			throw std::string("synthetic shape does not fit num_attribute");
		DevData &d = which ? c->te : c->tr;
		free_data(d);
		d.n = n;
		d.nf_local = (uint32_t)nf64;
		d.nf = which ? d.nf_local : global_nf(c, d.nf_local);
		d.nnz = (uint64_t)n * F;
		d.row_ptr = dalloc<uint64_t>((size_t)n + 1);
		d.csr = dalloc<uint2>(d.nnz);
		d.target = dalloc<float>(n);
		d.col_ptr = dalloc<uint64_t>((size_t)d.nf + 1);
		d.csc = dalloc<uint2>(d.nnz);
		HIPCHK(vbk::synth_csr(n, F, S, seed, xmode, model_seed, row_offset, d.row_ptr, d.csr, d.target, c->s));
		// col_ptr: feature histogram + exclusive scan (padded columns stay empty)
		uint64_t *counts = dalloc<uint64_t>((size_t)d.nf + 1);
		HIPCHK(hipMemsetAsync(counts, 0, ((size_t)d.nf + 1) * 8, c->s));
		HIPCHK(vbk::count_features(d.csr, d.nnz, counts, c->s));
		size_t tb = 0;
		HIPCHK(vbk::exclusive_scan_u64(nullptr, &tb, counts, d.col_ptr, (size_t)d.nf + 1, c->s));
		void *tmp = dalloc<uint8_t>(tb);
		HIPCHK(vbk::exclusive_scan_u64(tmp, &tb, counts, d.col_ptr, (size_t)d.nf + 1, c->s));
		dfree(tmp);
		dfree(counts);
		// CSC per field: stable radix sort of (id within field, row) keeps rows ascending
		uint32_t *ki = dalloc<uint32_t>(n), *ko = dalloc<uint32_t>(n), *vi = dalloc<uint32_t>(n),
		         *vo = dalloc<uint32_t>(n);
		int bits = 1;
		while ((1ull << bits) < S) bits++;
		tb = 0;
		HIPCHK(vbk::sort_pairs_u32(nullptr, &tb, ki, ko, vi, vo, n, bits, c->s));
		void *stmp = dalloc<uint8_t>(tb);
		for (uint32_t fl = 0; fl < F; fl++) {
			HIPCHK(vbk::synth_field_keys(d.csr, n, F, S, fl, ki, vi, c->s));
			size_t tb2 = tb;
			HIPCHK(vbk::sort_pairs_u32(stmp, &tb2, ki, ko, vi, vo, n, bits, c->s));
			HIPCHK(vbk::synth_field_scatter(vo, d.csr, n, F, fl, d.csc + (uint64_t)fl * n, c->s));
		}
		sync(c);
		dfree(stmp); dfree(ki); dfree(ko); dfree(vi); dfree(vo);
		synth_finish(c, which);
		if (which == 0) c->t_set_train = wall_s() - t0;
	});
}

int vbfm_synth_multihot(vbfm_ctx *c, int32_t which, uint32_t n, uint32_t D, uint32_t lo, uint32_t hi, uint64_t seed,
                        int32_t xmode, uint64_t model_seed, uint64_t row_offset)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		const double t0 = wall_s();
		if (which != 0 && which != 1) throw std::string("which must be 0 (train) or 1 (test)");
		if (lo < 1 || hi < lo || hi > 64 || D < hi || D >= c->D)
			throw std::string("multi-hot shape: need 1 <= lo <= hi <= 64, hi <= num_features < num_attribute");
		DevData &d = which ? c->te : c->tr;
		free_data(d);
		d.n = n;
		d.nf_local = D;
		d.nf = which ? d.nf_local : global_nf(c, d.nf_local);
		d.row_ptr = dalloc<uint64_t>((size_t)n + 1);
		HIPCHK(vbk::synth_mh_len(n, lo, hi, seed, row_offset, d.row_ptr, c->s));
		size_t tb = 0;
		HIPCHK(vbk::exclusive_scan_u64(nullptr, &tb, d.row_ptr, d.row_ptr, (size_t)n + 1, c->s));
		void *tmp = dalloc<uint8_t>(tb);
		HIPCHK(vbk::exclusive_scan_u64(tmp, &tb, d.row_ptr, d.row_ptr, (size_t)n + 1, c->s));
		HIPCHK(d2h(c, &d.nnz, d.row_ptr + n, 8));
		sync(c);
		dfree(tmp);
		if (d.nnz >= 0xFFFFFFFFull) throw std::string("multi-hot data set too large (nnz >= 2^32)");
		// bias / interaction gains per row length L (host sqrt: correctly rounded, as tests/synth.py)
		std::vector<double> gh(2 * (size_t)(hi - lo + 1));
		for (uint32_t L = lo; L <= hi; L++) {
			gh[2 * (L - lo)] = std::sqrt(12.0 / (double)L);
			gh[2 * (L - lo) + 1] = L >= 2 ? std::sqrt(72.0 / ((double)L * (double)(L - 1) / 2.0)) : 0.0;
		}
		double *gains = dalloc<double>(gh.size());
		HIPCHK(hipMemcpy(gains, gh.data(), gh.size() * 8, hipMemcpyHostToDevice));
		d.csr = dalloc<uint2>(d.nnz);
		d.target = dalloc<float>(n);
		uint32_t *row_of = dalloc<uint32_t>(d.nnz);
		HIPCHK(vbk::synth_mh_fill(n, D, seed, xmode, model_seed, row_offset, gains, lo, d.row_ptr, d.csr, row_of,
		                          d.target, c->s));
		// CSC: entries stably sorted by feature (rows stay ascending inside a column)
		d.col_ptr = dalloc<uint64_t>((size_t)d.nf + 1);
		d.csc = dalloc<uint2>(d.nnz);
		uint64_t *counts = dalloc<uint64_t>((size_t)d.nf + 1);
		HIPCHK(hipMemsetAsync(counts, 0, ((size_t)d.nf + 1) * 8, c->s));
		HIPCHK(vbk::count_features(d.csr, d.nnz, counts, c->s));
		tb = 0;
		HIPCHK(vbk::exclusive_scan_u64(nullptr, &tb, counts, d.col_ptr, (size_t)d.nf + 1, c->s));
		tmp = dalloc<uint8_t>(tb);
		HIPCHK(vbk::exclusive_scan_u64(tmp, &tb, counts, d.col_ptr, (size_t)d.nf + 1, c->s));
		sync(c);
		dfree(tmp);
		dfree(counts);
		uint32_t *ki = dalloc<uint32_t>(d.nnz), *ko = dalloc<uint32_t>(d.nnz), *vi = dalloc<uint32_t>(d.nnz),
		         *vo = dalloc<uint32_t>(d.nnz);
		HIPCHK(vbk::mh_keys(d.csr, d.nnz, ki, vi, c->s));
		int bits = 1;
		while ((1ull << bits) < D) bits++;
		tb = 0;
		HIPCHK(vbk::sort_pairs_u32(nullptr, &tb, ki, ko, vi, vo, d.nnz, bits, c->s));
		void *stmp = dalloc<uint8_t>(tb);
		HIPCHK(vbk::sort_pairs_u32(stmp, &tb, ki, ko, vi, vo, d.nnz, bits, c->s));
		HIPCHK(vbk::synth_mh_scatter(vo, d.csr, row_of, d.nnz, d.csc, c->s));
		sync(c);
		dfree(stmp); dfree(ki); dfree(ko); dfree(vi); dfree(vo); dfree(row_of); dfree(gains);
		synth_finish(c, which);
		if (which == 0) c->t_set_train = wall_s() - t0;
	});
}

int vbfm_get_shape(vbfm_ctx *c, int32_t which, uint32_t *n, uint32_t *nf, uint64_t *nnz)
{
	if (!c) return fail(nullptr, "null context");
	const DevData &d = which ? c->te : c->tr;
	if (n) *n = d.n;
	if (nf) *nf = d.nf_local;
	if (nnz) *nnz = d.nnz;
	return 0;
}

int vbfm_get_csc(vbfm_ctx *c, int32_t which, uint64_t *col_ptr, vbfm_entry *col_ent, float *target)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		const DevData &d = which ? c->te : c->tr;
		if (col_ptr) HIPCHK(hipMemcpy(col_ptr, d.col_ptr, ((size_t)d.nf_local + 1) * 8, hipMemcpyDeviceToHost));
		if (col_ent && d.nnz) {
			HIPCHK(hipMemcpy(col_ent, d.csc, d.nnz * 8, hipMemcpyDeviceToHost));
			for (uint64_t p = 0; p < d.nnz; p++) col_ent[p].id &= ROW_MASK;   // first-entry flags
		}
		if (target && d.n) HIPCHK(hipMemcpy(target, d.target, (size_t)d.n * 4, hipMemcpyDeviceToHost));
	});
}

int vbfm_get_levels(vbfm_ctx *c, uint32_t *level, uint32_t *num_levels)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		if (level) std::copy(c->level_h.begin(), c->level_h.begin() + c->tr.nf_local, level);
		if (num_levels) *num_levels = nlevels(c);
	});
}

int vbfm_set_params(vbfm_ctx *c, const vbfm_params *p)
{
	if (!c || !p) return fail(c, "null argument");
	return guarded(c, [&] {
		const size_t kd = (size_t)c->k * c->D;
		if (!p->mu_w || !p->sigma_w || (kd && (!p->mu_v || !p->sigma_v)))
			throw std::string("vbfm_set_params: parameter arrays missing");
		double *tmp = dalloc<double>(2 * std::max(kd, (size_t)c->D));
		HIPCHK(hipMemcpyAsync(tmp, p->mu_w, c->D * 8, hipMemcpyHostToDevice, c->s));
		HIPCHK(hipMemcpyAsync(tmp + c->D, p->sigma_w, c->D * 8, hipMemcpyHostToDevice, c->s));
		HIPCHK(vbk::pack_pairs(tmp, tmp + c->D, c->ms_w, 1, c->D, c->s));
		sync(c);
		if (kd) {
			HIPCHK(hipMemcpyAsync(tmp, p->mu_v, kd * 8, hipMemcpyHostToDevice, c->s));
			HIPCHK(hipMemcpyAsync(tmp + kd, p->sigma_v, kd * 8, hipMemcpyHostToDevice, c->s));
			HIPCHK(vbk::pack_pairs(tmp, tmp + kd, c->ms_v, (uint32_t)c->k, c->D, c->s));
			sync(c);
		}
		dfree(tmp);
		if (p->hyp_sigma_w) std::copy(p->hyp_sigma_w, p->hyp_sigma_w + c->G, c->hyp_w.begin());
		if (p->hyp_sigma_v) std::copy(p->hyp_sigma_v, p->hyp_sigma_v + (size_t)c->G * c->k, c->hyp_v.begin());
		upload_hyp(c);
		c->alpha = p->alpha; c->sigma_0 = p->sigma_0; c->mu0 = p->mu_0_dash; c->s0d = p->sigma_0_dash;
		c->q_ready[0] = c->q_ready[1] = -1;
		sync(c);
	});
}

int vbfm_get_params(vbfm_ctx *c, vbfm_params *p)
{
	if (!c || !p) return fail(c, "null argument");
	return guarded(c, [&] {
		const size_t kd = (size_t)c->k * c->D;
		double *tmp = dalloc<double>(2 * std::max(kd, (size_t)c->D));
		HIPCHK(vbk::unpack_pairs(c->ms_w, tmp, tmp + c->D, 1, c->D, c->s));
		if (p->mu_w) HIPCHK(d2h(c, p->mu_w, tmp, c->D * 8));
		if (p->sigma_w) HIPCHK(d2h(c, p->sigma_w, tmp + c->D, c->D * 8));
		sync(c);
		if (kd) {
			HIPCHK(vbk::unpack_pairs(c->ms_v, tmp, tmp + kd, (uint32_t)c->k, c->D, c->s));
			if (p->mu_v) HIPCHK(d2h(c, p->mu_v, tmp, kd * 8));
			if (p->sigma_v) HIPCHK(d2h(c, p->sigma_v, tmp + kd, kd * 8));
			sync(c);
		}
		dfree(tmp);
		if (p->hyp_sigma_w) std::copy(c->hyp_w.begin(), c->hyp_w.end(), p->hyp_sigma_w);
		if (p->hyp_sigma_v) std::copy(c->hyp_v.begin(), c->hyp_v.end(), p->hyp_sigma_v);
		p->alpha = c->alpha; p->sigma_0 = c->sigma_0; p->mu_0_dash = c->mu0; p->sigma_0_dash = c->s0d;
	});
}

int vbfm_init_params_device(vbfm_ctx *c, uint64_t seed)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		HIPCHK(vbk::init_normal_pairs(c->ms_w, c->D, seed, 11, 0.1, .02, c->s));
		HIPCHK(vbk::init_normal_pairs(c->ms_v, (size_t)c->k * c->D, seed, 12, 0.1, .02, c->s));
		std::fill(c->hyp_w.begin(), c->hyp_w.end(), 1.0);
		std::fill(c->hyp_v.begin(), c->hyp_v.end(), 1.0);
		upload_hyp(c);
		c->alpha = 1.0; c->sigma_0 = 1.0; c->mu0 = 0.0; c->s0d = 0.02;
		c->q_ready[0] = c->q_ready[1] = -1;
		sync(c);
	});
}

int vbfm_init_caches(vbfm_ctx *c)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->mc) throw std::string("an MCMC / ALS context: use the vbfm_mcmc_* entry points");
		if (c->ov) throw std::string("an online VB context: use vbfm_online_epoch");
		require_train(c);
		no_partial(c);
		// fm_learn_vb_simultaneous.h:37-44: yhat of train and test, T of train, e = y - yhat
		rows_row_order(c);
		const int bl = blocked_predict(c, c->tr);
		HIPCHK(vbk::predict_et(c->tr.row_ptr, c->tr.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, c->mu0, c->s0d,
		                       c->tr.target, c->scratch_n, c->rows, c->tr.n, bl, c->s));
		if (c->e_test) test_predict(c, c->s);
		sync(c);
	});
}

int vbfm_step_w0(vbfm_ctx *c)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] { require_train(c); no_partial(c); if (c->k0) step_w0(c); sync(c); });
}

int vbfm_step_w(vbfm_ctx *c)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] { require_train(c); no_partial(c); if (c->k1) step_w(c); sync(c); });
}

int vbfm_step_qcache(vbfm_ctx *c, int32_t f)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		if (f < 0 || f >= c->k) throw std::string("factor out of range");
		no_partial(c);
		step_qcache(c, f);
		sync(c);
	});
}

int vbfm_step_v(vbfm_ctx *c, int32_t f)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		if (f < 0 || f >= c->k) throw std::string("factor out of range");
		no_partial(c);
		if (c->q_ready[f & 1] != f) throw std::string("vbfm_step_v: q-cache of this factor is not current (vbfm_step_qcache)");
		step_v(c, f);
		sync(c);
	});
}

int vbfm_step_w_level(vbfm_ctx *c, int32_t level)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		if (!c->k1) throw std::string("k1 = 0: there is no w sweep");
		step_level(c, true, 0, (uint32_t)level);
		sync(c);
	});
}

int vbfm_step_v_level(vbfm_ctx *c, int32_t f, int32_t level)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		if (f < 0 || f >= c->k) throw std::string("factor out of range");
		step_level(c, false, f, (uint32_t)level);
		sync(c);
	});
}

int vbfm_step_hyper(vbfm_ctx *c, int32_t *early)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		no_partial(c);
		const bool e = step_hyper(c, nullptr, nullptr, nullptr);
		if (early) *early = e ? 1 : 0;
		sync(c);
	});
}

int vbfm_free_energy(vbfm_ctx *c, double *F)
{
	if (!c || !F) return fail(c, "null argument");
	return guarded(c, [&] { require_train(c); no_partial(c); *F = free_energy(c, rows_energy(c)); });
}

int vbfm_get_rows(vbfm_ctx *c, double *e, double *t, double *q, double *tq, double *tz)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->part_kind == -2) no_partial(c);   // a failed level: the records may be half moved
		std::vector<RowRec> h;
		if (c->part_kind >= 0 && c->lord) {   // half a level-by-level sweep on a level-ordered store
			sync(c);
			h = rows_mid_sweep(c);
		} else {
			rows_row_order(c);
			sync(c);   // the readback below runs on the null stream, which does not wait for c->s
			h.resize(c->tr.n);
			if (c->tr.n) HIPCHK(hipMemcpy(h.data(), c->rows, (size_t)c->tr.n * sizeof(RowRec), hipMemcpyDeviceToHost));
		}
		const bool s1 = c->qslot == 1;
		for (uint32_t i = 0; i < c->tr.n; i++) {
			if (e) e[i] = h[i].e;
			if (t) t[i] = h[i].t;
			if (q) q[i] = s1 ? h[i].q1 : h[i].q;
			if (tq) tq[i] = s1 ? h[i].tq1 : h[i].tq;
			if (tz) tz[i] = s1 ? h[i].tz1 : h[i].tz;
		}
	});
}

int vbfm_get_test_e(vbfm_ctx *c, double *e)
{
	if (!c || !e) return fail(c, "null argument");
	return guarded(c, [&] {
		if (c->te.n) HIPCHK(hipMemcpy(e, c->e_test, (size_t)c->te.n * 8, hipMemcpyDeviceToHost));
	});
}

int vbfm_get_test_pred(vbfm_ctx *c, double *pred)
{
	if (!c || !pred) return fail(c, "null argument");
	return guarded(c, [&] {
		if (c->te.n) HIPCHK(hipMemcpy(pred, c->pred_test, (size_t)c->te.n * 8, hipMemcpyDeviceToHost));
	});
}

}  // extern "C"

// ---- checkpoint / resume ---------------------------------------------------------------------
// The reference always starts from its initial draws (num_complete_iter = 0,
// fm_learn_vb_simultaneous.h:20) and keeps no state on disk. Between two vbfm_iterate calls the
// VB learner's state is the parameters, the hyper parameters, the four scalars and the train
// row records (row order; their q-cache slots are rebuilt inside the next sweeps, they are kept
// only so that a resumed context holds the same bytes). An MCMC / ALS context writes its own
// payload behind the same header (vbi::mc_state_*, vbfm_mcmc_capi.hip).
namespace vbi {

struct StateHeader {
	char magic[8];        // "VBFMST01"
	uint32_t version;
	int32_t k0, k1, k;
	uint32_t D, G;
	uint32_t n_train, nf_train;
	uint64_t nnz_train;
	uint64_t data_fp;     // fingerprint of the train CSC (col_ptr, entries) and targets
	int32_t nranks, rank;
	uint32_t iter;
	uint32_t level_order; // the records were in level-0 order (data-set sums add them in that order)
	uint64_t layout;      // version 2: row layout (VBFM_LAYOUT_*) | shard mode << 8: both decide the
	                      // order of the data-set sums, so a resume must use the same ones
	uint64_t flags;       // STATE_FLAG_* (0 in files of libvbfm before round 5: was reserved)
	uint64_t shapes;      // the workgroup shape table the sums ran with (state_shapes; 0 before round 6:
	                      // was reserved)
	uint64_t reserved;
};
// the layout word of an online checkpoint says whether its batches ran on the per-batch level store
// (written since round 5; before, an online learner always wrote COLUMN, whichever it used)
constexpr uint64_t STATE_FLAG_OV_LAYOUT = 1;
// a column's reduction tree follows its workgroup shape (dispatch_shape, vbfm_device.h) and, for a
// long column, its segments (build_long_segs), so a resume continues bit for bit only under the same
// tables: their revision (4: round 6's -- the round-5 shapes with 128 x 3 and the small-shape cutoff
// at 128, and segments of 1024 beyond max(1024, 4 x the level's mean)), an id of any segment
// override in force (VBFM_LONG / VBFM_SEG_MIN / VBFM_SEG_LEN; 0: none) and the small-shape cutoff
// (VBFM_SMALL_MAX): revision << 48 | segment id << 32 | cutoff
constexpr uint64_t SHAPE_TABLE_REVISION = 4;
static uint64_t seg_rule_id()
{
	const char *v[3] = {getenv("VBFM_LONG"), getenv("VBFM_SEG_MIN"), getenv("VBFM_SEG_LEN")};
	if (!v[0] && !v[1] && !v[2]) return 0;
	uint64_t h = 1469598103934665603ull;   // FNV-1a over the three settings
	for (const char *p : v) {
		for (const char *q = p ? p : "-"; *q; q++) h = (h ^ (uint8_t)*q) * 1099511628211ull;
		h = (h ^ 0xffu) * 1099511628211ull;
	}
	return (h & 0xfffeu) | 1u;
}
static uint64_t state_shapes() { return SHAPE_TABLE_REVISION << 48 | seg_rule_id() << 32 | shape_small_max(); }
static_assert(sizeof(StateHeader) == 104, "checkpoint header layout");
constexpr char STATE_MAGIC[8] = {'V', 'B', 'F', 'M', 'S', 'T', '0', '1'};
constexpr char MC_STATE_MAGIC[8] = {'V', 'B', 'F', 'M', 'M', 'C', '0', '1'};   // MCMC / ALS payload
constexpr char OV_STATE_MAGIC[8] = {'V', 'B', 'F', 'M', 'O', 'V', '0', '1'};   // online VB payload

// the learner a checkpoint belongs to: 0 VB, 1 MCMC / ALS, 2 online VB
int state_kind(const vbfm_ctx *c) { return c->mc ? 1 : c->ov ? 2 : 0; }
const char *state_magic(int kind) { return kind == 1 ? MC_STATE_MAGIC : kind == 2 ? OV_STATE_MAGIC : STATE_MAGIC; }
constexpr size_t IO_CHUNK = (size_t)64 << 20;

uint64_t train_fingerprint(vbfm_ctx *c)
{
	unsigned long long *d = dalloc<unsigned long long>(1);
	HIPCHK(hipMemsetAsync(d, 0, 8, c->s));
	HIPCHK(vbk::fingerprint(c->tr.col_ptr, (uint64_t)c->tr.nf + 1, 8, 1, d, c->s));
	HIPCHK(vbk::fingerprint(c->tr.csc, c->tr.nnz, 8, 2, d, c->s));
	HIPCHK(vbk::fingerprint(c->tr.target, c->tr.n, 4, 3, d, c->s));
	unsigned long long h = 0;
	HIPCHK(d2h(c, &h, d, 8));
	sync(c);
	dfree(d);
	return h;
}

uint64_t state_layout(vbfm_ctx *c)
{
	// the online learner: whether its batches run on the per-batch level-ordered store (the
	// store's data-set sums add a batch's rows in level-0 order)
	const int lay = c->ov ? (ov_store_on(c) ? VBFM_LAYOUT_LEVEL : VBFM_LAYOUT_COLUMN)
	                      : c->estore ? VBFM_LAYOUT_ENTRY : c->lord ? VBFM_LAYOUT_LEVEL : VBFM_LAYOUT_COLUMN;
	return (uint64_t)lay | (uint64_t)c->shard_mode << 8;
}

StateHeader state_header(vbfm_ctx *c, uint32_t iter)
{
	StateHeader h;
	memset(&h, 0, sizeof(h));
	memcpy(h.magic, STATE_MAGIC, 8);
	h.version = 2;
	h.k0 = c->k0; h.k1 = c->k1; h.k = c->k;
	h.D = c->D; h.G = c->G;
	h.n_train = c->tr.n; h.nf_train = c->tr.nf; h.nnz_train = c->tr.nnz;
	h.data_fp = train_fingerprint(c);
	h.nranks = c->nranks; h.rank = c->rank;
	h.iter = iter;
	h.layout = state_layout(c);
	h.flags = STATE_FLAG_OV_LAYOUT;
	h.shapes = state_shapes();
	return h;
}

// bytes that follow the header: ms_w, ms_v, hyper parameters, four scalars, the row records
uint64_t state_payload(vbfm_ctx *c)
{
	return (uint64_t)c->D * 16 + (uint64_t)c->k * c->D * 16 + (uint64_t)c->G * 8 + (uint64_t)c->G * c->k * 8 + 32 +
	       (uint64_t)c->tr.n * sizeof(RowRec);
}


void dev_to_file(vbfm_ctx *c, CkptFile &f, const void *d, size_t bytes)
{
	std::vector<uint8_t> buf(std::min(bytes, IO_CHUNK));
	for (size_t o = 0; o < bytes; o += IO_CHUNK) {
		const size_t n = std::min(IO_CHUNK, bytes - o);
		HIPCHK(d2h(c, buf.data(), (const uint8_t *)d + o, n));
		sync(c);
		f.write(buf.data(), n);
	}
}

void file_to_dev(vbfm_ctx *c, CkptFile &f, void *d, size_t bytes)
{
	std::vector<uint8_t> buf(std::min(bytes, IO_CHUNK));
	for (size_t o = 0; o < bytes; o += IO_CHUNK) {
		const size_t n = std::min(IO_CHUNK, bytes - o);
		f.read(buf.data(), n);
		HIPCHK(hipMemcpyAsync((uint8_t *)d + o, buf.data(), n, hipMemcpyHostToDevice, c->s));
		sync(c);
	}
}


}  // namespace vbi

extern "C" {

int vbfm_save_state(vbfm_ctx *c, const char *path, uint32_t iter)
{
	if (!c || !path) return fail(c, "null argument");
	return guarded(c, [&] {
		require_train(c);
		no_partial(c);
		StateHeader h = state_header(c, iter);
		memcpy(h.magic, state_magic(state_kind(c)), 8);
		h.level_order = c->rows_lorder ? 1 : 0;
		rows_row_order(c);
		// written beside the target and renamed over it once complete and on disk: a failed
		// or interrupted save never destroys the previous checkpoint (-resume X -save_state X)
		const std::string tmp = std::string(path) + ".tmp";
		try {
			CkptFile f(tmp.c_str(), "wb");
			f.write(&h, sizeof(h));
			if (c->mc) {
				mc_state_write(c, f);
			} else if (c->ov) {
				ov_state_write(c, f);
			} else {
				dev_to_file(c, f, c->ms_w, (size_t)c->D * sizeof(double2));
				dev_to_file(c, f, c->ms_v, (size_t)c->k * c->D * sizeof(double2));
				f.write(c->hyp_w.data(), c->hyp_w.size() * 8);
				f.write(c->hyp_v.data(), c->hyp_v.size() * 8);
				const double sc[4] = {c->alpha, c->sigma_0, c->mu0, c->s0d};
				f.write(sc, sizeof(sc));
				dev_to_file(c, f, c->rows, (size_t)c->tr.n * sizeof(RowRec));
			}
			if (fflush(f.f) != 0 || fsync(fileno(f.f)) != 0) throw std::string("short write to ") + tmp;
			if (fclose(f.f) != 0) { f.f = nullptr; throw std::string("short write to ") + tmp; }
			f.f = nullptr;
			if (rename(tmp.c_str(), path) != 0) throw std::string("cannot rename ") + tmp + " to " + path;
		} catch (...) {
			unlink(tmp.c_str());
			if (h.level_order) rows_level_order(c);
			throw;
		}
		if (h.level_order) rows_level_order(c);   // the run goes on exactly as without the save
	});
}

int vbfm_load_state(vbfm_ctx *c, const char *path, uint32_t *iter)
{
	if (!c || !path) return fail(c, "null argument");
	return guarded(c, [&] {
		require_train(c);
		if (c->part_kind >= 0) no_partial(c);   // (a failed level, -2, is what a restore repairs)
		CkptFile f(path, "rb");
		StateHeader h;
		f.read(&h, sizeof(h));
		int kind = -1;
		for (int q = 0; q < 3; q++)
			if (memcmp(h.magic, state_magic(q), 8) == 0) kind = q;
		if (kind < 0 || h.version != 2) throw std::string("not a libvbfm checkpoint (version 2): ") + path;
		static const char *const learner[3] = {"a VB checkpoint: resume it in a VB context",
		                                       "an MCMC / ALS checkpoint: resume it in an MCMC / ALS context",
		                                       "an online VB checkpoint: resume it in an online VB context"};
		if (kind != state_kind(c)) throw std::string(learner[kind]);
		if (h.k0 != c->k0 || h.k1 != c->k1 || h.k != c->k || h.D != c->D || h.G != c->G)
			throw std::string("checkpoint of another model configuration (-dim / num_attribute / groups)");
		if (h.nranks != c->nranks || h.rank != c->rank)
			throw std::string("checkpoint of another rank (each rank resumes from its own file)");
		if (h.n_train != c->tr.n || h.nf_train != c->tr.nf || h.nnz_train != c->tr.nnz ||
		    h.data_fp != train_fingerprint(c))
			throw std::string("checkpoint of another train data set");
		if (kind == 2 && !(h.flags & STATE_FLAG_OV_LAYOUT))
			throw std::string("an online VB checkpoint written by an older libvbfm, whose layout word does not record "
			                  "whether the batches ran on the per-batch level store (the order of the batches' data-set "
			                  "sums): resume it with the libvbfm that wrote it");
		if (h.shapes != state_shapes()) {
			char b[512];
			auto desc = [](uint64_t w) {
				return "revision " + std::to_string(w >> 48) + ", segment override " +
				       std::to_string((w >> 32) & 0xffffu) + ", VBFM_SMALL_MAX " + std::to_string(w & 0xffffffffu);
			};
			snprintf(b, sizeof(b), "checkpoint written under another workgroup shape table (%s; this library: %s): the "
			         "column sums would change order and the run would not continue bit for bit; resume with the "
			         "libvbfm and settings that wrote it",
			         h.shapes ? desc(h.shapes).c_str() : "a libvbfm before round 6, unrecorded", desc(state_shapes()).c_str());
			throw std::string(b);
		}
		if (h.layout != state_layout(c))
			throw std::string("checkpoint of another row layout or shard mode (the data-set sums would add the rows in "
			                  "another order): resume with the same VBFM_LAYOUT / vbfm_set_layout and shard mode");
		if (h.level_order && !c->lord) throw std::string("checkpoint of a level-ordered run: resume with the same row layout");
		// the whole file is there before any state is replaced
		const uint64_t payload = kind == 1 ? mc_state_payload(c) : kind == 2 ? ov_state_payload(c) : state_payload(c);
		if (fseek(f.f, 0, SEEK_END) != 0 || (uint64_t)ftell(f.f) != sizeof(h) + payload ||
		    fseek(f.f, (long)sizeof(h), SEEK_SET) != 0)
			throw std::string("checkpoint file truncated or of another size: ") + path;
		rows_row_order(c);
		if (kind == 1) {
			mc_state_read(c, f);
		} else if (kind == 2) {
			ov_state_read(c, f);
		} else {
			file_to_dev(c, f, c->ms_w, (size_t)c->D * sizeof(double2));
			file_to_dev(c, f, c->ms_v, (size_t)c->k * c->D * sizeof(double2));
			f.read(c->hyp_w.data(), c->hyp_w.size() * 8);
			f.read(c->hyp_v.data(), c->hyp_v.size() * 8);
			upload_hyp(c);
			double sc[4];
			f.read(sc, sizeof(sc));
			c->alpha = sc[0]; c->sigma_0 = sc[1]; c->mu0 = sc[2]; c->s0d = sc[3];
			file_to_dev(c, f, c->rows, (size_t)c->tr.n * sizeof(RowRec));
		}
		c->rows_lorder = false;
		if (h.level_order) rows_level_order(c);
		c->q_ready[0] = c->q_ready[1] = -1;
		c->carry = 0;
		c->part_kind = -1;   // every record restored
		sync(c);
		if (iter) *iter = h.iter;
	});
}

int vbfm_factor_sweep(vbfm_ctx *c, double *ms_device)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		require_train(c);
		no_partial(c);
		HIPCHK(hipEventRecord(c->ev[EV_BEGIN], c->s));
		for (int f = 0; f < c->k; f++) { step_qcache(c, f); step_v(c, f); }
		HIPCHK(hipEventRecord(c->ev[EV_V], c->s));
		sync(c);
		if (ms_device) *ms_device = ev_ms(c, EV_BEGIN, EV_V);
	});
}

int vbfm_iterate(vbfm_ctx *c, vbfm_iter_stats *o)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->mc) throw std::string("an MCMC / ALS context: use the vbfm_mcmc_* entry points");
		if (c->ov) throw std::string("an online VB context: use vbfm_online_epoch");
		require_train(c);
		no_partial(c);
		if (!c->e_test) throw std::string("no test data set (vbfm_set_test)");
		vbfm_iter_stats st;
		memset(&st, 0, sizeof(st));
		HIPCHK(hipMemsetAsync(c->counters, 0, CNT_N * 4, c->s));
		c->pev_used = 0;
		c->spans.clear();
		xs_reset(c);
		Range r_it("vbfm_iterate");
		HIPCHK(hipEventRecord(c->ev[EV_BEGIN], c->s));
		// update_all (fm_learn_vb.h:383-501)
		if (c->k0) { Range r("update_w0"); XPhase ph(c, "update_w0"); step_w0(c); }
		HIPCHK(hipEventRecord(c->ev[EV_W0], c->s));
		// the sweeps follow each other directly: a deferred split may carry a sweep's last
		// correction into the next sweep's first level (sweep_level); the last sweep flushes
		c->carry = 0;
		c->carry_ok = c->deferred() && c->D > 0 && c->k > 0;
		try {
			if (c->k1) { Range r("update_w sweep"); step_w(c); }
			HIPCHK(hipEventRecord(c->ev[EV_W], c->s));
			if (c->D > 0)
				for (int f = 0; f < c->k; f++) {
					char nm[32];
					snprintf(nm, sizeof(nm), "factor %d", f);
					Range r(nm);
					step_qcache(c, f);
					step_v(c, f);
				}
		} catch (...) {
			c->carry_ok = c->carry = 0;
			throw;
		}
		c->carry_ok = 0;
		if (c->carry) throw std::string("internal: a deferred correction was left pending");
		HIPCHK(hipEventRecord(c->ev[EV_V], c->s));
		const bool overlap = test_overlap();
		if (overlap) {
			HIPCHK(hipStreamWaitEvent(c->s_test, c->ev[EV_V], 0));
			HIPCHK(hipEventRecord(c->ev[EV_TP0], c->s_test));
			test_predict(c, c->s_test);
			HIPCHK(hipEventRecord(c->ev[EV_TP1], c->s_test));
		}
		double energy = 0.0;
		bool early;
		try {
			Range r("hyper + free energy");
			XPhase ph(c, "hyper-parameters + free energy");
			early = step_hyper(c, &energy, &st.nan_alpha, &st.inf_alpha);
			st.free_energy_valid = early ? 0 : 1;
			st.free_energy = early ? NAN : free_energy(c, energy);
		} catch (...) {
			// the overlapped prediction is still queued on s_test: later calls on c->s (the next
			// sweeps write ms_v, get_test_pred reads e_test) must not race it
			if (overlap) (void)hipStreamWaitEvent(c->s, c->ev[EV_TP1], 0);
			throw;
		}
		HIPCHK(hipEventRecord(c->ev[EV_HYPER], c->s));
		// test prediction and metrics (fm_learn_vb_simultaneous.h:125-222)
		Range r_test("test prediction");
		XPhase ph_test(c, "test metrics");
		if (overlap) {
			HIPCHK(hipStreamWaitEvent(c->s, c->ev[EV_TP1], 0));
		} else {
			HIPCHK(hipEventRecord(c->ev[EV_TP0], c->s));
			test_predict(c, c->s);
			HIPCHK(hipEventRecord(c->ev[EV_TP1], c->s));
		}
		const double mn = c->min_target, mx = c->max_target;
		HIPCHK(vbk::test_metrics(c->e_test, c->te.target, c->te.n, mn, mx, c->pred_test, c->red_d, c->RED_BLOCKS, c->s));
		HIPCHK(d2h(c, c->red_h.data(), c->red_d, 2 * c->RED_BLOCKS * 8));
		sync(c);
		double tm[3] = {0.0, 0.0, 0.0};
		for (uint32_t i = 0; i < c->RED_BLOCKS; i++) { tm[0] += c->red_h[2 * i]; tm[1] += c->red_h[2 * i + 1]; }
		rows_dense(c);
		HIPCHK(vbk::train_quirk(c->rows, c->tr.n, mn, mx, c->red_d, c->RED_BLOCKS, c->s));
		tm[2] = finish_sum(c, c->RED_BLOCKS);
		allreduce_host(c, tm, 3);
		HIPCHK(hipEventRecord(c->ev[EV_TEST], c->s));
		sync(c);
		st.rmse = std::sqrt(tm[0] / c->test_n_global);
		st.mae = tm[1] / c->test_n_global;
		st.train_quirk = std::sqrt(tm[2] / (double)c->n_global);
		st.num_levels = (int32_t)nlevels(c);
		st.alpha = c->alpha; st.sigma_0 = c->sigma_0; st.mu_0_dash = c->mu0; st.sigma_0_dash = c->s0d;
		read_counters(c, &st);
		st.ms_w0 = ev_ms(c, EV_BEGIN, EV_W0);
		st.ms_w = ev_ms(c, EV_W0, EV_W);
		st.ms_v = ev_ms(c, EV_W, EV_V);
		st.ms_qcache = 0.0;
		st.ms_hyper = ev_ms(c, EV_V, EV_HYPER);
		st.ms_test = ev_ms(c, EV_HYPER, EV_TEST);
		st.ms_test_predict = ev_ms(c, EV_TP0, EV_TP1);
		st.ms_total = ev_ms(c, EV_BEGIN, EV_TEST);
		st.nnz_train = c->tr.nnz;
		for (const auto &sp : c->spans) {
			float ms = 0.f;
			HIPCHK(hipEventElapsedTime(&ms, c->pev[sp.a], c->pev[sp.a + 1]));
			if (sp.kind == 0) { st.ms_vlevel_kernels += ms; st.n_vlevel_launches++; }
			else if (sp.kind == 1) { st.ms_wlevel_kernels += ms; st.n_wlevel_launches++; }
			else if (sp.kind == 2) { st.ms_qcache_kernels += ms; st.n_qcache_launches++; }
			else xs_span(c, ms);
		}
		st.ms_qcache = st.ms_qcache_kernels;
		if (o) *o = st;
	});
}

int vbfm_set_shard_mode(vbfm_ctx *c, int32_t mode, int32_t num_shards)
{
	if (!c) return fail(nullptr, "null context");
	if (mode != VBFM_SHARD_ROWS && mode != VBFM_SHARD_FEATURES) return fail(c, "unknown shard mode");
	if (num_shards < 0) return fail(c, "negative number of shards");
	if (c->rows) return fail(c, "vbfm_set_shard_mode must precede vbfm_set_train");
	if (c->mc && mode == VBFM_SHARD_FEATURES) return fail(c, "feature shards are implemented for the VB learner only");
	c->shard_mode = mode;
	c->fs_req = mode == VBFM_SHARD_FEATURES ? num_shards : 1;
	return 0;
}

int vbfm_set_layout(vbfm_ctx *c, int32_t layout)
{
	if (!c) return fail(nullptr, "null context");
	if (layout < VBFM_LAYOUT_AUTO || layout > VBFM_LAYOUT_ENTRY) return fail(c, "unknown row layout");
	if (c->rows) return fail(c, "vbfm_set_layout must precede vbfm_set_train");
	c->layout_req = layout;
	return 0;
}

int vbfm_get_layout(vbfm_ctx *c, int32_t *layout)
{
	if (!c || !layout) return fail(c, "null argument");
	return guarded(c, [&] {
		require_train(c);
		*layout = c->estore ? VBFM_LAYOUT_ENTRY : c->lord ? VBFM_LAYOUT_LEVEL : VBFM_LAYOUT_COLUMN;
	});
}

int vbfm_set_profiling(vbfm_ctx *c, int32_t on)
{
	if (!c) return fail(nullptr, "null context");
	c->profiling = on != 0;
	c->prof_stride = on > 1 ? on : 1;
	for (auto &t : c->prof_tick) t = 0;
	return 0;
}

int vbfm_comm_unique_id(uint8_t out[128])
{
	ncclUniqueId id;
	if (ncclGetUniqueId(&id) != ncclSuccess) return fail(nullptr, "ncclGetUniqueId failed");
	static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
	memcpy(out, &id, 128);
	return 0;
}

int vbfm_comm_init(vbfm_ctx *c, int32_t nranks, int32_t rank, const uint8_t uid[128])
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->rows) throw std::string("vbfm_comm_init must precede vbfm_set_train");
		if (c->multi()) throw c->comm_failed ? c->comm_err : std::string("the context already has a communicator");
		if (nranks < 1 || rank < 0 || rank >= nranks) throw std::string("bad rank / nranks");
		// one rank needs no communicator; VBFM_FORCE_COMM=1 creates it anyway so that every
		// RCCL call of the sharded path runs (the 1-GPU test box cannot host two ranks)
		const char *fc = getenv("VBFM_FORCE_COMM");
		if (nranks == 1 && !(fc && fc[0] == '1')) return;
		ncclUniqueId id;
		memcpy(&id, uid, 128);
		c->nranks = nranks;
		c->rank = rank;
		const char *to = getenv("VBFM_COMM_TIMEOUT_S");
		c->comm_timeout_s = to ? std::max(atof(to), 0.0) : 300.0;
		const char *bl = getenv("VBFM_COMM_BLOCKING");
		const bool blocking = bl && bl[0] == '1';
		// non-blocking: the set-up returns at once (ncclInProgress) and is polled against the
		// deadline like every later wait on a collective (comm_check / comm_wait)
		ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
		cfg.blocking = blocking ? 1 : 0;
		XPhase ph(c, "communicator set-up");
		const ncclResult_t r = ncclCommInitRankConfig(&c->comm, nranks, id, rank, &cfg);
		if (r != ncclSuccess && r != ncclInProgress) {
			if (c->comm) (void)ncclCommAbort(c->comm);
			c->comm = nullptr;
			throw x_where(c) + ": RCCL " + ncclGetErrorString(r) + " in ncclCommInitRankConfig";
		}
		if (!c->comm) throw x_where(c) + ": ncclCommInitRankConfig returned no communicator";
		comm_check(c, r, "ncclCommInitRankConfig");
		comm_check(c, comm_async_error(c), "ncclCommInitRankConfig");
		if (blocking) c->comm_timeout_s = 0.0;   // no deadline: every wait blocks
		xs_reset(c);
	});
}

int vbfm_placement_info(vbfm_ctx *c, float *ms, int32_t *count, int32_t *kept)
{
	if (!c || !count || !kept) return fail(c, "null argument");
	return guarded(c, [&] {
		const int32_t cap = *count;
		*count = (int32_t)c->place_ms.size();
		kept[0] = c->place_pick[0];
		kept[1] = c->place_pick[1];
		for (int32_t i = 0; ms && i < std::min(cap, *count); i++) ms[i] = c->place_ms[(size_t)i];
	});
}

int vbfm_setup_info(vbfm_ctx *c, vbfm_setup_stats *o)
{
	if (!c || !o) return fail(c, "null argument");
	return guarded(c, [&] {
		memset(o, 0, sizeof(*o));
		o->s_set_train = c->t_set_train;
		o->s_schedule = c->t_schedule;
		o->s_store = c->t_store;
		o->s_placement = c->t_place;
		o->place_bytes = c->place_bytes;
		o->place_candidates = (int32_t)c->place_ms.size();
		o->place_kept[0] = c->place_pick[0];
		o->place_kept[1] = c->place_pick[1];
	});
}

int vbfm_comm_info(vbfm_ctx *c, int32_t *nranks, int32_t *rank, int32_t *transport)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->comm_failed) throw c->comm_err;
		int n = c->nranks, r = c->rank, t = 0;
		if (c->comm) {          // ask RCCL itself, not the context's copy
			comm_check(c, ncclCommCount(c->comm, &n), "ncclCommCount");
			comm_check(c, ncclCommUserRank(c->comm, &r), "ncclCommUserRank");
			t = 1;
		} else if (c->xfn) {
			t = 2;
		} else {
			n = 1;
			r = 0;
		}
		if (nranks) *nranks = n;
		if (rank) *rank = r;
		if (transport) *transport = t;
	});
}

int vbfm_exchange_info(vbfm_ctx *c, vbfm_exchange_stats *o)
{
	if (!c || !o) return fail(c, "null argument");
	*o = c->xs;
	o->ms_estimated = o->transport == 1 && o->n_timed ? o->ms_timed / o->n_timed * (double)o->n_calls : o->ms_timed;
	return 0;
}

int vbfm_comm_init_host(vbfm_ctx *c, int32_t nranks, int32_t rank, vbfm_exchange_fn fn, void *user)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		if (c->rows) throw std::string("vbfm_comm_init_host must precede vbfm_set_train");
		if (c->multi()) throw std::string("the context already has a communicator");
		if (nranks < 1 || rank < 0 || rank >= nranks) throw std::string("bad rank / nranks");
		if (!fn) throw std::string("null exchange function");
		c->xfn = fn;
		c->xuser = user;
		c->nranks = nranks;
		c->rank = rank;
		xs_reset(c);
	});
}

}  // extern "C"
