// vbfm_ctx.h -- the learner context behind include/vbfm.h and the host-side helpers its
// two front ends share: the VB learner (vbfm_capi.hip) and the MCMC / ALS learner
// (vbfm_mcmc_capi.hip). Internal to libvbfm; not part of the ABI.
#pragma once
#include "vbfm_device.h"
#include "../../include/vbfm.h"

#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <string>
#include <vector>

extern "C" const char *vbfm_host_last_error(void);
extern "C" void vbfm_host_set_error(const char *msg);

struct McState;   // vbfm_mcmc_capi.hip
struct OvState;   // vbfm_online.hip

namespace vbi {

struct DevData {
	uint32_t n = 0, nf = 0;        // rows; columns of the transposed copy (padded to the global nf)
	uint32_t nf_local = 0;
	uint64_t nnz = 0;
	uint64_t *col_ptr = nullptr;   // [nf+1]
	uint2 *csc = nullptr;          // [nnz]
	uint64_t *row_ptr = nullptr;   // [n+1]
	uint2 *csr = nullptr;          // [nnz] feature-sorted rows
	float *target = nullptr;       // [n]
	float min_target = 0, max_target = 0;
};

struct HipError {
	hipError_t e;
	const char *what;
};

#define HIPCHK(x)                                                   \
	do {                                                            \
		hipError_t _e = (x);                                        \
		if (_e != hipSuccess) throw HipError{_e, #x};               \
	} while (0)

#define NCCLCHK(x)                                                  \
	do {                                                            \
		ncclResult_t _r = (x);                                      \
		if (_r != ncclSuccess) throw std::string("RCCL: ") + ncclGetErrorString(_r) + " in " #x; \
	} while (0)

template <class T> inline T *dalloc(size_t n)
{
	void *p = nullptr;
	HIPCHK(hipMalloc(&p, (n ? n : 1) * sizeof(T)));
	return (T *)p;
}

template <class T> inline void dfree(T *&p)
{
	if (p) (void)hipFree((void *)p);
	p = nullptr;
}

// a device buffer freed when its scope ends, normally or by an exception (dfree(buf.p) frees it early)
template <class T> struct DevScratch {
	T *p = nullptr;
	explicit DevScratch(size_t n) : p(dalloc<T>(n)) {}
	~DevScratch() { dfree(p); }
	DevScratch(const DevScratch &) = delete;
	DevScratch &operator=(const DevScratch &) = delete;
};

enum { EV_BEGIN, EV_W0, EV_W, EV_V, EV_HYPER, EV_TEST, EV_TP0, EV_TP1, EV_N };

// host wall clock (s) of the set-up steps vbfm_setup_info reports
inline double wall_s()
{
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the deferred MCMC / ALS split kernel's record stores non-temporal (VBFM_DEFER_NT bit 1, default
// on; its loads always are), as the VB one's (vbfm_capi.hip defer_nt)
inline bool defer_nt_stores()
{
	const char *e = getenv("VBFM_DEFER_NT");
	return ((e ? atoi(e) : 3) & 2) != 0;
}

// test hook: VBFM_FAULT=<where> makes the named step throw as a failed HIP call would (the error
// paths of the store build and the per-level steps, tests/test_placement_gpu.py)
inline bool fault_at(const char *where)
{
	const char *e = getenv("VBFM_FAULT");
	return e && !strcmp(e, where);
}

// roctx ranges around the phases of an iteration (VBFM_ROCTX=1; 2 adds one per level launch)
// for rocprofv3 --marker-trace timelines
inline int roctx_level()
{
	const char *e = getenv("VBFM_ROCTX");
	return e ? atoi(e) : 0;
}

struct Range {
	bool on;
	Range(const char *name, int lvl = 1) : on(roctx_level() >= lvl) { if (on) roctxRangePushA(name); }
	~Range() { if (on) roctxRangePop(); }
};

}  // namespace vbi

struct vbfm_ctx {
	using DevData = vbi::DevData;
	std::string err;
	int dev = 0;
	hipStream_t s = nullptr;
	hipStream_t s_test = nullptr;   // the test prediction, overlapping the hyper-parameter step
	// row shards over RCCL: the per-level all-reduce of chunk i of a level's statistics runs on
	// s_comm while chunk i+1 computes on s (stats_exchange); events order the two
	hipStream_t s_comm = nullptr;
	static constexpr int AR_MAX_CHUNKS = 8;
	hipEvent_t ev_ar[AR_MAX_CHUNKS] = {};
	hipEvent_t ev_arj = nullptr;
	int k0 = 1, k1 = 1, k = 0;
	uint32_t D = 0, G = 1;
	std::vector<uint32_t> group_h, per_group;
	uint32_t *group_d = nullptr;
	float min_target = 0, max_target = 0;
	DevData tr, te;
	RowRec *rows = nullptr;
	double *scratch_n = nullptr;   // yhat of train at init
	double *e_test = nullptr, *pred_test = nullptr;
	double2 *ms_v = nullptr, *ms_w = nullptr;
	double *hyp_w_d = nullptr, *hyp_v_d = nullptr;
	std::vector<double> hyp_w, hyp_v;
	double alpha = 1.0, sigma_0 = 1.0, mu0 = 0.0, s0d = 0.02;
	// schedule
	std::vector<uint32_t> level_ptr, level_h, level_avg;
	std::vector<uint32_t> level_base;   // first id of a level of consecutive feature ids, else ~0u
	int q_ready[2] = {-1, -1};     // factor whose q-cache each slot holds (-1: none)
	int qslot = 0;                 // slot reported by vbfm_get_rows
	int carry_in = 0;              // the pending kind carried into the current sweep (deferred split)
	// a sweep driven level by level (vbfm_step_w_level / vbfm_step_v_level): kind -1 none, 0 the
	// w sweep, 1 the v sweep of factor part_f; part_next = the level expected next
	int part_kind = -1, part_f = 0;
	std::vector<float> place_ms;    // tune_placement: each candidate buffer's score (ms), [0], [1] = the first pair
	int place_pick[2] = {-1, -1};   // ... and the two kept (records, alternate)
	std::vector<float> place_pair_ms;   // ... the best few scored as pairs (a < b in score order)
	int prefetch = -1;              // the level kernels touch the next level's column bounds (VBFM_PREFETCH; -1: not read yet)
	int place_cands_cfg = 0;        // vbfm_config::place_candidates / place_budget_bytes (0: defaults)
	uint64_t place_budget_cfg = 0;
	uint64_t place_bytes = 0;       // device memory the last search held at its peak
	// host wall seconds of the set-up steps (vbfm_setup_info)
	double t_set_train = 0, t_schedule = 0, t_store = 0, t_place = 0;
	uint32_t part_next = 0;
	uint32_t *level_feats = nullptr;
	uint8_t *dup = nullptr;
	bool sched_ready = false;
	int sched_rounds = 0;          // relaxation rounds (+ Kahn rounds queued) of the last schedule
	bool sched_kahn = false;       // the last schedule came from Kahn's order
	// reductions
	static constexpr uint32_t RED_BLOCKS = 512;
	double *red_d = nullptr;
	std::vector<double> red_h;
	uint32_t *perm_d = nullptr;
	vbk::Chunk *chunks_d = nullptr;
	std::vector<vbk::Chunk> chunks_h;   // attribute chunks, group by group (build_chunks)
	uint32_t *gchunk_d = nullptr;       // [G+1] each group's chunk range
	double *chunk_out_d = nullptr;      // [chunks] w partials
	double *vpart_d = nullptr;          // [chunks * k] factor partials
	double *vseg_d = nullptr;           // [k * G] factor sums (inside chunk_out_d)
	uint32_t *counters = nullptr;
	// row-sharded multi-GPU
	int nranks = 1, rank = 0;
	bool force_split = false;      // VBFM_FORCE_SPLIT=1: the multi-rank kernels on one rank
	int debug_skew = 0;            // VBFM_DEBUG_SKEW=1: late waves in the split forms' posterior kernels
	ncclComm_t comm = nullptr;
	// communicator health: RCCL runs non-blocking (its errors surface through
	// ncclCommGetAsyncError), polled against a deadline wherever the host waits on work that holds a
	// collective (comm_wait); a failure or a missed deadline aborts the communicator, and every
	// later exchange refuses with the first message (comm_err)
	double comm_timeout_s = 300.0;   // VBFM_COMM_TIMEOUT_S
	bool comm_failed = false;
	std::string comm_err;
	// where the path is when it exchanges (the messages name it): a phase, the factor (-1: none)
	// and the level (-1: not in a sweep)
	const char *x_phase = "set-up";
	int x_f = -1, x_l = -1;
	std::string x_pending;           // the first exchange issued since the last completed wait (x_where)
	vbfm_exchange_stats xs = {};     // this iteration's exchanges (vbfm_exchange_info)
	uint32_t *stall_flag = nullptr;  // VBFM_FAULT=comm_stall: host flag that releases the stall kernel
	bool stall_done = false;
	double2 *stats = nullptr;
	uint32_t stats_cap = 0;
	uint64_t n_global = 0;
	uint32_t test_n_global = 0;
	hipEvent_t ev[vbi::EV_N] = {};
	// per-launch profiling (vbfm_set_profiling)
	bool profiling = false;
	int prof_stride = 1;             // event pair around every prof_stride-th launch of a kind
	uint64_t prof_tick[4] = {0, 0, 0, 0};
	std::vector<hipEvent_t> pev;
	size_t pev_used = 0;
	struct Span { size_t a; int kind; };   // kind 0 = v level, 1 = w level, 2 = qcache, 3 = exchange
	std::vector<Span> spans;
	// level-ordered row store (vbfm_lorder.hip)
	int layout_req = VBFM_LAYOUT_AUTO;
	bool lord = false;             // built for the current train set and in use
	bool estore = false;           // ... as the entry store (levels that miss rows: build_estore);
	                               // lpos0 then holds each row's slot between sweeps, lrow0 is unused
	bool rows_lorder = false;      // rows currently hold level-0 order (else row order)
	RowRec *rows_alt = nullptr;    // second record buffer (each level moves rows -> rows_alt)
	uint64_t *lcp = nullptr;       // [nf+1] global position of each level feature's run
	float *lx = nullptr;           // [nnz] x per level-ordered entry
	uint32_t *lnext = nullptr;     // [nnz] position of the entry's row in the next level
	uint32_t *lrow0 = nullptr;     // [n] row at each level-0 position
	uint32_t *lpos0 = nullptr;     // [n] level-0 position of each row
	uint32_t *lpidx = nullptr;     // [nnz] split form: the row's previous-level feature (index in its level)
	float *lpx = nullptr;          // [nnz] ... and its x (deferred correction)
	uint2 *lpay2 = nullptr;        // [nnz] ... {lnext, lpidx} instead when every x is 1 (no lx)
	uint4 *lpay = nullptr;         // [nnz] deferred split: {x, lnext, lpidx, lpx} of every entry in one
	                               // 16-B load (lx / lnext / lpidx / lpx are freed once packed)
	PostT *post_tab = nullptr;     // [max level width] posteriors of the last level swept
	// long columns of the level store (fused single-rank sweep): segments of every level
	uint32_t long_min = 0;         // nonzero: some level has long columns split into segments
	std::vector<uint32_t> long_min_l;  // [L] each level's threshold (0: no segments in the level)
	std::vector<uint32_t> seg_ptr; // [L+1] each level's segments in long_segs
	LongSeg *long_segs = nullptr;
	double2 *seg_part = nullptr;   // [2 * max segments of a level]
	// deferred split across sweeps (vbfm_iterate only): the last level's correction of a sweep is
	// left to level 0 of the next one instead of a flush pass. carry: 0 none, 1 / 2 = v sweep of
	// q-cache slot 0 / 1, 3 = w sweep
	int carry_ok = 0, carry = 0;
	// feature-sharded mode (vbfm_set_shard_mode): shards own column chunks of every level
	int shard_mode = VBFM_SHARD_ROWS;
	int fs_req = 1;                // shards requested (no communicator: run one after another here)
	int fs_n = 1;                  // shards in use
	std::vector<uint32_t> fs_lo;   // [L * (fs_n + 1)] chunk bounds of each level in level_feats
	uint32_t *fs_own = nullptr;    // this rank's features (all levels) for the parameter exchange
	uint32_t fs_own_n = 0;
	double *fs_base = nullptr;     // [2n] e, t at the start of a pass
	double *fs_buf = nullptr;      // [5n] summed changes / partial q-caches
	double2 *fs_pbuf = nullptr;    // [nf] parameter exchange
	RowRec *fs_rows0 = nullptr;    // in-process shards: the rows at the start of a pass
	vbfm_exchange_fn xfn = nullptr; // vbfm_comm_init_host: all-reduces through the caller
	void *xuser = nullptr;
	std::vector<uint8_t> xbuf;      // host staging of a host-exchange all-reduce
	bool deferred() const { return lpay || lpay2; }
	bool multi() const { return comm || xfn || comm_failed; }
	bool row_comm() const { return multi() && shard_mode == VBFM_SHARD_ROWS; }
	McState *mc = nullptr;         // set by vbfm_mcmc_init: the context runs the MCMC / ALS learner
	OvState *ov = nullptr;         // set by vbfm_online_init: the context runs the online VB learner
	// vbfm_init_params_replay: the draws' seed and the glibc outputs they consumed (after the
	// warm-up), so that a learner can continue the reference's stream (UINT64_MAX: unknown)
	uint32_t init_stream_seed = 0;
	uint64_t init_stream_end = ~0ull;
};


namespace vbi {

int fail(vbfm_ctx *c, const std::string &m);

template <class F> int guarded(vbfm_ctx *c, F &&fn)
{
	try {
		if (c) HIPCHK(hipSetDevice(c->dev));
		fn();
		return 0;
	} catch (const HipError &e) {
		return fail(c, std::string("HIP error ") + hipGetErrorString(e.e) + " in " + e.what);
	} catch (const std::string &m) {
		return fail(c, m);
	} catch (const char *m) {
		return fail(c, m);
	} catch (const std::bad_alloc &) {
		return fail(c, "host out of memory");
	}
}

void sync(vbfm_ctx *c);
// a copy from the device into host memory, queued on the context's stream. A copy into pageable
// memory holds the calling thread until the stream reaches it, so with an RCCL communicator the
// stream is waited for first through sync's deadline and error polling, not inside the copy
hipError_t d2h(vbfm_ctx *c, void *dst, const void *src, size_t bytes);
// the phase the next exchanges belong to (restored on scope exit), for comm_fail's message
struct XPhase {
	vbfm_ctx *c;
	const char *p;
	int f, l;
	XPhase(vbfm_ctx *c_, const char *phase, int f_ = -1, int l_ = -1) : c(c_), p(c_->x_phase), f(c_->x_f), l(c_->x_l)
	{
		c->x_phase = phase; c->x_f = f_; c->x_l = l_;
	}
	~XPhase() { c->x_phase = p; c->x_f = f; c->x_l = l; }
};
// a new iteration's exchange accounting (vbfm_exchange_info)
void xs_reset(vbfm_ctx *c);
// fold the timed exchange spans of the iteration into c->xs (vbfm_iterate / vbfm_mcmc_iterate)
void xs_span(vbfm_ctx *c, float ms);
void allreduce_host(vbfm_ctx *c, double *v, int n);
// in-place all-reduce of a device buffer over the ranks (RCCL on c->s, or the host exchange)
void allreduce_dev(vbfm_ctx *c, void *buf, size_t n, ncclDataType_t t, ncclRedOp_t op);
double finish_sum(vbfm_ctx *c, uint32_t nblocks);
// chunks the per-level exchange is cut into (1: one all-reduce after the level's statistics)
uint32_t ar_chunks(vbfm_ctx *c, uint32_t nfeat);
// in-place fp64 sum over the ranks of n doubles of chunk i (< ar_chunks) of a level, issued after
// the work queued on c->s so far; RCCL: on s_comm, so that c->s can go on with the next chunk
void allreduce_chunk(vbfm_ctx *c, double2 *buf, size_t n, uint32_t i);
// c->s waits for every chunk's all-reduce issued since the last join
void allreduce_join(vbfm_ctx *c);

// chunk [c0, c1) of a level's features as a launch of its own (LevelArgs / McArgs): the
// kernels index their columns, runs and statistics by the launch's feature index
template <class A>
A level_chunk(const A &a, uint32_t c0, uint32_t c1)
{
	A b = a;
	b.nfeat = c1 - c0;
	if (b.feat_contig) b.feat_base += c0;
	else b.feats += c0;
	if (b.lcp) b.lcp += c0;
	b.stats += c0;
	return b;
}

// a level's statistics kernel(s) and their all-reduce over the row shards: the level's columns
// in ar_chunks() chunks, chunk i's all-reduce overlapping chunk i+1's kernel; every chunk sums
// the same columns' entries as one launch would, so the results are bit-identical
template <class A, class F>
void stats_exchange(vbfm_ctx *c, const A &a, F launch)
{
	const uint32_t C = ar_chunks(c, a.nfeat);
	if (C <= 1) {
		launch(a);
		if (c->row_comm()) allreduce_dev(c, a.stats, 2 * (size_t)a.nfeat, ncclDouble, ncclSum);
		return;
	}
	for (uint32_t i = 0; i < C; i++) {
		const uint32_t c0 = (uint32_t)((uint64_t)a.nfeat * i / C), c1 = (uint32_t)((uint64_t)a.nfeat * (i + 1) / C);
		const A b = level_chunk(a, c0, c1);
		launch(b);
		allreduce_chunk(c, b.stats, 2 * (size_t)b.nfeat, i);
	}
	allreduce_join(c);
}
void require_train(vbfm_ctx *c);
uint32_t nlevels(vbfm_ctx *c);
constexpr size_t NO_SPAN = ~(size_t)0;   // prof_begin: this launch is not timed
size_t prof_begin(vbfm_ctx *c, int kind, hipStream_t st = nullptr);
void prof_end(vbfm_ctx *c, size_t a, hipStream_t st = nullptr);
int blocked_predict(const vbfm_ctx *c, const DevData &d);
float ev_ms(vbfm_ctx *c, int a, int b);
void mc_free(vbfm_ctx *c);   // vbfm_mcmc_capi.hip
void ov_free(vbfm_ctx *c);   // vbfm_online.hip
void glibc_state_at(uint32_t seed, uint64_t pos, uint32_t st[31]);   // vbfm_replay.hip
// online VB: the per-feature fields of LevelArgs for the w sweep or factor f (vbfm_online.hip)
void ov_level_args(vbfm_ctx *c, LevelArgs &a, bool is_w, int f);
void ov_launch_level(vbfm_ctx *c, LevelArgs &a, uint32_t l, bool is_w);
// steps of update_all shared with the online learner (vbfm_capi.hip)
void step_w(vbfm_ctx *c);
void step_qcache(vbfm_ctx *c, int f);
void step_v(vbfm_ctx *c, int f);
double rows_energy(vbfm_ctx *c);
std::vector<double> param_sums(vbfm_ctx *c, int mode);
// the per-(w | factor f, group g) segment sums at [(f + 1) * G + g]; model 0: VB, 1: MCMC
// (their modes: param_sums / mc_param_sums; hw [G] / hv [G*k] their mode-1 constants); a
// segment not wanted is left 0
std::vector<double> seg_sums(vbfm_ctx *c, int model, int mode, const double *hw, const double *hv, bool want_w,
                             bool want_v);
double free_energy(vbfm_ctx *c, double energy);
void test_predict(vbfm_ctx *c, hipStream_t s);
void read_counters(vbfm_ctx *c, vbfm_iter_stats *o);
void upload_hyp(vbfm_ctx *c);
void lord_release(vbfm_ctx *c, bool keep_rows);
void rows_level_order(vbfm_ctx *c);   // records in level-0 order before a sweep (no-op without the store)
void rows_dense(vbfm_ctx *c);         // records N-dense for the data-set sums (row order from the entry store)
void rows_row_order(vbfm_ctx *c);     // records back in row order (row-indexed kernels, readback)   // level-ordered store freed (rows back to row order)

// checkpoint files (vbfm_save_state / vbfm_load_state, vbfm_capi.hip): whole-buffer I/O that
// throws on a short read or write, device buffers staged through the host in 64 MB pieces
struct CkptFile {
	FILE *f;
	std::string path;
	CkptFile(const char *p, const char *mode) : f(fopen(p, mode)), path(p)
	{
		if (!f) throw std::string("cannot open checkpoint file ") + p;
	}
	~CkptFile() { if (f) fclose(f); }
	void write(const void *p, size_t n)
	{
		if (n && fwrite(p, 1, n, f) != n) throw std::string("short write to ") + path;
	}
	void read(void *p, size_t n)
	{
		if (n && fread(p, 1, n, f) != n) throw std::string("checkpoint file truncated: ") + path;
	}
};
void dev_to_file(vbfm_ctx *c, CkptFile &f, const void *d, size_t bytes);
void file_to_dev(vbfm_ctx *c, CkptFile &f, void *d, size_t bytes);
// the MCMC / ALS learner's part of a checkpoint (vbfm_mcmc_capi.hip): its payload size, and the
// payload written / read behind the common header (the caller has put the records in row order)
uint64_t mc_state_payload(vbfm_ctx *c);
void mc_state_write(vbfm_ctx *c, CkptFile &f);
void mc_state_read(vbfm_ctx *c, CkptFile &f);
// ... and the online learner's (vbfm_online.hip)
uint64_t ov_state_payload(vbfm_ctx *c);
// the online learner sweeps its batches on the per-batch level-ordered store (k_ov_lord)
bool ov_store_on(vbfm_ctx *c);
void ov_state_write(vbfm_ctx *c, CkptFile &f);
void ov_state_read(vbfm_ctx *c, CkptFile &f);

}  // namespace vbi
