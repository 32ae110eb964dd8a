/* include/vbfm.h -- C-ABI of libvbfm.so, the MI355X-native VB factorization-machine learner.
 *
 * Drop-in boundary for the reference's learner seam: the abstract `fm_learn`
 * (src/libfm/src/fm_learn.h:38-265) as specialised by `fm_learn_vb` /
 * `fm_learn_vb_simultaneous` (src/libfm/src/fm_learn_vb.h:25-793,
 * src/libfm/src/fm_learn_vb_simultaneous.h:15-309) and selected by `-method vb` in
 * src/libfm/libfm.cpp:306-311. The reference has no FFI; the entry points below are what
 * a host (the libFM-compatible CLI in host/, or any C/ctypes caller) binds in place of
 * `new fm_learn_vb_simultaneous()` + `init()` + `learn(train, test)`.
 *
 * Conventions
 *  - plain C types only; every array is caller-owned host memory unless a name says
 *    `_device`; the library copies what it needs and never keeps a caller pointer.
 *  - every function returns 0 on success, nonzero on failure; the message is then in
 *    vbfm_last_error(ctx) (or vbfm_last_error(NULL) for failures without a context).
 *    The reference signals errors by throwing `const char*` / `std::string`, which main()
 *    prints as "ERROR: <msg>" (src/libfm/libfm.cpp:521-525); a host maps a nonzero return
 *    to exactly that.
 *  - one host thread per context; calls are synchronous (they return after the device
 *    work they enqueue has completed), like the reference's single-threaded learner.
 *  - arithmetic is IEEE fp64 for all state, fp32 for design-matrix values and targets
 *    (FM_FLOAT, src/fm_core/fm_data.h:25), uint32 row / feature ids.
 */
#ifndef VBFM_H_
#define VBFM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: vbfm_synth_generate's model_seed / row_offset, vbfm_synth_multihot, VBFM_LAYOUT_ENTRY,
 *    vbfm_iter_stats::ms_test_predict, checkpoints, vbfm_comm_info, vbfm_device_count and the
 *    per-level step entry points.
 * 3: vbfm_config's placement budget (place_candidates, place_budget_bytes) and vbfm_setup_info.
 * 4: vbfm_exchange_info; RCCL communicators are non-blocking with a deadline (VBFM_COMM_TIMEOUT_S).
 * A binding checks vbfm_abi_version() against the value it was built for and refuses a mismatch
 * (struct sizes and argument lists differ). */
#define VBFM_ABI_VERSION 4

typedef struct vbfm_ctx vbfm_ctx;

/* == sparse_entry<float> (src/util/fmatrix.h:36-39): 8 bytes, id then value. In a
 * transposed (column) matrix `id` is the row index. */
typedef struct {
	uint32_t id;
	float value;
} vbfm_entry;

/* A data set as the reference's learner sees it: the transposed copy `data_t` built by
 * Data::create_data_t (src/libfm/src/Data.h:457-509) -- column j lists its rows in
 * ascending order -- plus the targets (Data::target). */
typedef struct {
	uint32_t num_rows;        /* Data::num_cases */
	uint32_t num_feature;     /* data_t->getNumRows(): max feature id + 1 */
	uint64_t nnz;
	const uint64_t *col_ptr;  /* [num_feature + 1] */
	const vbfm_entry *col_ent;/* [nnz] */
	const float *target;      /* [num_rows] */
} vbfm_csc;

/* Learner configuration: the fields main() sets on the model and learner before init()
 * (src/libfm/libfm.cpp:215-274, 306-311, 331-334). */
typedef struct {
	int32_t k0;               /* -dim k0: use bias w0 */
	int32_t k1;               /* -dim k1: use 1-way interactions w */
	int32_t num_factor;       /* -dim k2 */
	uint32_t num_attribute;   /* D = max(train.num_feature, test.num_feature) + 1 (libfm.cpp:215) */
	uint32_t num_attr_groups; /* DataMetaInfo::num_attr_groups (1 without -meta) */
	const uint32_t *attr_group; /* [num_attribute] group of each attribute, or NULL = all 0 */
	float min_target;         /* train.min_target (libfm.cpp:333) */
	float max_target;         /* train.max_target (libfm.cpp:332) */
	int32_t device;           /* HIP device ordinal */
	int32_t task;             /* 0 = regression (the only task the VB learner evaluates) */
	/* Placement search of the level-ordered store's two record buffers (no reference counterpart;
	 * DESIGN.md §5b): the scattered record writes of a level run up to ~20 % faster or slower
	 * depending on where the driver placed the buffers, so at store build (>= 2e6 rows) the library
	 * scores candidate buffers on level 0's pattern and keeps the two fastest. Results do not depend
	 * on it (bit for bit). Zero-initialised fields take the defaults.
	 *   place_candidates:   buffers scored, the store's own two included (0 = default: 64 for a
	 *                       store under 2 GB of records, 16 above; 1 or 2 = no search);
	 *   place_budget_bytes: device memory the search may hold at once on top of the store -- the
	 *                       records' stash, a reference buffer and the fresh candidates (0 = default,
	 *                       VBFM_PLACE_BUDGET_DEFAULT).
	 * The search also never takes more than half of the device memory free when it starts (a quarter
	 * with several ranks); when that leaves room for fewer candidates it scores fewer, or none: it
	 * never fails the store. VBFM_PLACE=0 / VBFM_PLACE_TRIES=n / VBFM_PLACE_BUDGET_GB=x in the
	 * environment override the two fields. vbfm_setup_info reports what the search held and took. */
	int32_t place_candidates;
	uint64_t place_budget_bytes;
} vbfm_config;
/* 96 GiB: 16 candidates at C4 (6.4 GB buffers). Fast regions can first appear past the first
 * ~50 GB of allocations (profiles/r06_placement/README.md, calls 1 and wide_search) */
#define VBFM_PLACE_BUDGET_DEFAULT ((uint64_t)96 << 30)

/* Variational and hyper parameters (fm_learn_vb.h:36-46). Arrays are caller-allocated. */
typedef struct {
	double *mu_w, *sigma_w;         /* [D]   mu_w_dash, sigma_w_dash            */
	double *mu_v, *sigma_v;         /* [k*D] mu_v_dash[f][j], sigma_v_dash[f][j] */
	double *hyp_sigma_w;            /* [G]   sigma_w(g)                          */
	double *hyp_sigma_v;            /* [G*k] sigma_v(g, f), row-major [g][f]     */
	double alpha, sigma_0, mu_0_dash, sigma_0_dash;
} vbfm_params;

/* What one pass of the reference's iteration loop reports
 * (fm_learn_vb_simultaneous.h:86-222, fm_learn_vb.h:646-681). */
typedef struct {
	double rmse, mae;           /* test, on predictions clipped to the train range */
	double train_quirk;         /* the "Train=" value: sqrt(mean(clip(e)^2)) */
	double free_energy;         /* F; valid only if free_energy_valid */
	int32_t free_energy_valid;  /* 0 when update_all returned early on a NaN/inf alpha */
	int32_t num_levels;         /* dependency levels of the train schedule */
	double alpha, sigma_0, mu_0_dash, sigma_0_dash;
	uint32_t nan_mu_w, nan_sigma_w, inf_mu_w;
	uint32_t nan_mu_v, nan_sigma_v, inf_mu_v;
	uint32_t nan_alpha, inf_alpha;
	/* device time of the phases of this iteration (hipEvents on the context stream), ms */
	double ms_w0, ms_w, ms_qcache, ms_v, ms_hyper, ms_test, ms_total;
	/* with vbfm_set_profiling(ctx, 1): summed device time of the individual kernel launches
	 * (an event pair around every launch), and the launch counts */
	double ms_vlevel_kernels, ms_wlevel_kernels, ms_qcache_kernels;
	int32_t n_vlevel_launches, n_wlevel_launches, n_qcache_launches;
	uint64_t nnz_train;         /* nnz of this shard's train data */
	/* device time of the test prediction itself; it runs on a second stream under the
	 * hyper-parameter step (ms_test then covers only what follows it: metrics, train quirk) */
	double ms_test_predict;
} vbfm_iter_stats;

/* ---- lifecycle ---------------------------------------------------------------------- */
int vbfm_create(vbfm_ctx **out, const vbfm_config *cfg);   /* fm_learn_vb::init (fm_learn_vb.h:685-743) */
void vbfm_destroy(vbfm_ctx *ctx);
const char *vbfm_last_error(const vbfm_ctx *ctx);
int vbfm_abi_version(void);
/* HIP devices visible to this process (0 without a GPU). No reference counterpart: the
 * reference is single-threaded on the host; the multi-rank CLI (-devices) maps ranks to
 * ordinals with it. It initialises the HIP runtime: call it only in the process that will
 * use the GPU (never before a fork). */
int vbfm_device_count(int32_t *n);

/* ---- data (DataSubset hand-over, fm_learn_vb::learn, fm_learn_vb.h:746-786) ----------- */
int vbfm_set_train(vbfm_ctx *ctx, const vbfm_csc *train);
int vbfm_set_test(vbfm_ctx *ctx, const vbfm_csc *test);
/* Field-structured synthetic data generated directly in HBM (tests/synth.py defines it):
 * rows x n_fields one-hot fields of ids_per_field ids each. which: 0 = train, 1 = test.
 * seed draws the rows, model_seed the planted model (bias + rank-2 interaction) that the
 * train set, the test set and every rank's shard share; the rows generated are rows
 * [row_offset, row_offset + num_rows) of the one-rank data set (a row shard). */
int vbfm_synth_generate(vbfm_ctx *ctx, int32_t which, uint32_t num_rows, uint32_t n_fields,
                        uint32_t ids_per_field, uint64_t seed, int32_t xmode, uint64_t model_seed,
                        uint64_t row_offset);
/* Multi-hot rows WITHOUT field structure (tests/synth.py generate_multihot defines it): row R
 * holds lo..hi (<= 64) distinct ids out of num_features, one per stratum of the id range, and
 * the same planted model; the levels of such data miss rows, so the sweeps take the
 * column-gather layout. Rows [row_offset, row_offset + num_rows) of the one-rank data set. */
int vbfm_synth_multihot(vbfm_ctx *ctx, int32_t which, uint32_t num_rows, uint32_t num_features, uint32_t lo,
                        uint32_t hi, uint64_t seed, int32_t xmode, uint64_t model_seed, uint64_t row_offset);
/* Copy back the device copy of a data set (parity of the device transpose / generator). */
int vbfm_get_csc(vbfm_ctx *ctx, int32_t which, uint64_t *col_ptr /*[nf+1]*/, vbfm_entry *col_ent /*[nnz]*/,
                 float *target /*[rows]*/);
int vbfm_get_shape(vbfm_ctx *ctx, int32_t which, uint32_t *num_rows, uint32_t *num_feature, uint64_t *nnz);
/* level of each train feature (1-based; [train.num_feature]) and the number of levels */
int vbfm_get_levels(vbfm_ctx *ctx, uint32_t *level, uint32_t *num_levels);

/* ---- parameters ----------------------------------------------------------------------- */
int vbfm_set_params(vbfm_ctx *ctx, const vbfm_params *p);
int vbfm_get_params(vbfm_ctx *ctx, vbfm_params *p);

/* Bench-scale random init on the device: mu_w_dash, mu_v_dash = 0.1 * N(0,1) from a
 * counter-based generator (splitmix64 + Box-Muller; NOT the reference's glibc stream),
 * sigma_* = .02, hyper parameters and scalars at their fm_learn_vb::init values. */
int vbfm_init_params_device(vbfm_ctx *ctx, uint64_t seed);

/* The reference's initial draws -- exactly what vbfm_init_params_host + vbfm_set_params
 * produce (srand(seed); fm.v, fm.w ~ N(0, init_stdev); mu_w_dash, mu_v_dash = 0.1 N(0,1);
 * glibc rand() with Leva normals) -- generated on the device: the glibc stream split into
 * chunks by jump-ahead, Leva's rejection as a stream compaction. fm_v [k*D] (f-major) and
 * fm_w [D] receive the model draws (v_file.txt) when not NULL. */
int vbfm_init_params_replay(vbfm_ctx *ctx, uint32_t seed, double init_stdev, double *fm_v, double *fm_w);

/* ---- learning (fm_learn_vb_simultaneous::_learn, fm_learn_vb_simultaneous.h:18-259) ---- */
int vbfm_init_caches(vbfm_ctx *ctx);                     /* :37-44 */
int vbfm_iterate(vbfm_ctx *ctx, vbfm_iter_stats *out);   /* one pass of :75-258 */
int vbfm_get_test_pred(vbfm_ctx *ctx, double *pred /*[test rows]*/); /* pred_this (clipped) */

/* ---- the steps of update_all (fm_learn_vb.h:383-501), for step-level parity ---------- */
int vbfm_step_w0(vbfm_ctx *ctx);                  /* update_w0, :504-525 */
int vbfm_step_w(vbfm_ctx *ctx);                   /* the w sweep, :390-406 / :527-574 */
int vbfm_step_qcache(vbfm_ctx *ctx, int32_t f);   /* zero + add_main_q, :411-418 / :354-381 */
int vbfm_step_v(vbfm_ctx *ctx, int32_t f);        /* the v sweep of factor f, :420-438 / :577-644 */
/* One dependency level of a sweep, for localising a parity miss below one
 * sweep: level l (0-based, in order 0..L-1, L from vbfm_get_levels) of the w sweep, or of factor
 * f's v sweep (its q-cache is made current at level 0). After level l the caches and parameters
 * equal the reference's after its update_w / update_v of every feature of levels 0..l, features
 * of a level in ascending id order (fm_learn_vb.h:390-406, 409-440; ref_driver levels). Same
 * kernels as the whole sweep; one rank or the two-pass split (VBFM_DEFER=0), not the deferred
 * split or feature shards. vbfm_get_rows / vbfm_get_params read the state between two levels;
 * other steps are refused until the sweep's last level has run. */
int vbfm_step_w_level(vbfm_ctx *ctx, int32_t level);
int vbfm_step_v_level(vbfm_ctx *ctx, int32_t f, int32_t level);
int vbfm_step_hyper(vbfm_ctx *ctx, int32_t *early_return); /* :446-498 */
int vbfm_free_energy(vbfm_ctx *ctx, double *F);   /* :646-681 (value only, no file) */
/* row caches: e (cache[].e), t/q/z of cache_t, q of cache (the factor q-cache) */
int vbfm_get_rows(vbfm_ctx *ctx, double *e, double *t, double *q, double *tq, double *tz);
int vbfm_get_test_e(vbfm_ctx *ctx, double *e /*[test rows]*/);

/* Layout of the row caches in HBM during the sweeps (no reference counterpart: the
 * reference keeps cache[] / cache_t[] in row order, fm_learn_vb.h:17-21,746-786).
 *   VBFM_LAYOUT_AUTO   (default) level-ordered when every dependency level holds each train
 *                      row exactly once (field-structured one-hot data), else column-gather;
 *   VBFM_LAYOUT_COLUMN row order, columns gather their rows;
 *   VBFM_LAYOUT_LEVEL  records kept in the current level's column order and streamed
 *                      (vbfm_set_layout fails at the first sweep when the data does not
 *                      allow it). Results are identical up to the summation order of the
 *                      data-set sums (w0, alpha, free energy).
 *   VBFM_LAYOUT_ENTRY  for levels that miss rows (multi-hot rows without fields): one slot per
 *                      train entry in the level order, a row's record in the slot of the entry
 *                      its next level sweeps; levels stream their runs and move each record to
 *                      its row's next slot (nnz x 64 B of HBM; one rank). AUTO picks it
 *                      where LEVEL does not apply and it fits (VBFM_ESTORE=0: COLUMN instead).
 * Set before vbfm_set_train; VBFM_LAYOUT=auto|column|level|entry in the environment overrides.
 * vbfm_get_layout reports the layout in use (COLUMN, LEVEL or ENTRY) once the train set is known. */
#define VBFM_LAYOUT_AUTO 0
#define VBFM_LAYOUT_COLUMN 1
#define VBFM_LAYOUT_LEVEL 2
#define VBFM_LAYOUT_ENTRY 3
int vbfm_set_layout(vbfm_ctx *ctx, int32_t layout);
int vbfm_get_layout(vbfm_ctx *ctx, int32_t *layout);

/* per-launch event timing of the sweep kernels inside vbfm_iterate (off by default) */
int vbfm_set_profiling(vbfm_ctx *ctx, int32_t on);   /* on > 1: time every on-th launch of a kind */

/* ---- checkpoint / resume ----------------------------------------------------------------
 * No reference counterpart: the reference always starts from its initial draws
 * (num_complete_iter = 0, fm_learn_vb_simultaneous.h:20) and keeps no state on disk. The VB
 * learner's state between two vbfm_iterate calls -- {mu, sigma} of w and v, the hyper
 * parameters, alpha, sigma_0, mu_0_dash, sigma_0_dash and this rank's train row caches -- goes
 * to one file. vbfm_load_state, on a context created with the same configuration, rank and
 * train data (checked: shape and a fingerprint of the train CSC and targets; the test set is
 * free), replaces vbfm_init_caches and the run continues bit for bit. iter: the caller's
 * iteration count, stored and returned. An MCMC / ALS context (vbfm_mcmc_init) writes its
 * chain instead -- the RNG (mode, seed, completed iterations, the reference stream's position),
 * the parameters, hyper-priors, w0, alpha, the test predictions and their running sum, the
 * train row caches -- and vbfm_load_state on a context initialised the same way (vbfm_mcmc_init
 * with the same method and RNG mode; it replaces vbfm_mcmc_init_caches) continues the chain bit
 * for bit. An online context (vbfm_online_init with the same -batch) saves between epochs:
 * parameters, natural parameters, step sizes, the rand() stream and the last permutation. */
int vbfm_save_state(vbfm_ctx *ctx, const char *path, uint32_t iter);
int vbfm_load_state(vbfm_ctx *ctx, const char *path, uint32_t *iter);

/* ---- the factor sweep alone (the metric's timed unit: q-cache + v sweep, all factors) -- */
int vbfm_factor_sweep(vbfm_ctx *ctx, double *ms_device);

/* ---- multi-GPU: row-sharded exact mode over RCCL ----------------------------------------
 * Each rank owns a slice of the train rows; per dependency level the per-feature
 * sufficient statistics are all-reduced, so every rank computes identical posteriors. */
int vbfm_comm_unique_id(uint8_t out[128]);
int vbfm_comm_init(vbfm_ctx *ctx, int32_t nranks, int32_t rank, const uint8_t uid[128]);

/* The same row- / feature-sharded modes with a caller-supplied exchange instead of RCCL:
 * every all-reduce of the path stages its buffer in host memory and calls
 * fn(user, buf, count, dtype, op), which must all-reduce buf in place across the ranks and
 * return 0 (non-zero: the call fails with "host exchange failed"). dtype: VBFM_X_F64 /
 * VBFM_X_U32 / VBFM_X_U8; op: VBFM_X_SUM / VBFM_X_MAX. Test transport (e.g. a gloo
 * all-reduce from Python): it lets several ranks share one GPU, which RCCL refuses, so the
 * multi-rank kernels run on a one-GPU box exactly as over RCCL, minus the collective itself. */
#define VBFM_X_F64 0
#define VBFM_X_U32 1
#define VBFM_X_U8 2
#define VBFM_X_SUM 0
#define VBFM_X_MAX 1
typedef int (*vbfm_exchange_fn)(void *user, void *buf, uint64_t count, int32_t dtype, int32_t op);
int vbfm_comm_init_host(vbfm_ctx *ctx, int32_t nranks, int32_t rank, vbfm_exchange_fn fn, void *user);
/* The communicator as RCCL reports it (ncclCommCount / ncclCommUserRank): transport 0 = none
 * (one rank), 1 = RCCL, 2 = host exchange (nranks / rank as given to vbfm_comm_init_host). */
int vbfm_comm_info(vbfm_ctx *ctx, int32_t *nranks, int32_t *rank, int32_t *transport);
/* Failure handling of the exchange (no reference counterpart: the reference is one process).
 * vbfm_comm_init creates a non-blocking RCCL communicator (ncclCommInitRankConfig, blocking = 0).
 * Wherever the library waits for work that holds a collective -- the communicator's set-up, an
 * RCCL call that returns ncclInProgress, a stream synchronisation after an all-reduce -- it polls
 * ncclCommGetAsyncError and a deadline of VBFM_COMM_TIMEOUT_S seconds (default 300) instead of
 * blocking. On an RCCL error or a missed deadline it aborts the communicator (ncclCommAbort) and
 * the call fails; vbfm_last_error names the rank, the phase, factor and level of the exchange and
 * the cause, and every later call that exchanges fails with the same message. A host exchange
 * (vbfm_comm_init_host) fails when the caller's function returns non-zero; its transport owns the
 * timeout. VBFM_COMM_BLOCKING=1 creates a blocking communicator instead (no deadline). */
/* The exchanges of the last vbfm_iterate / vbfm_mcmc_iterate (since vbfm_comm_init before the
 * first): every all-reduce of the path counted with its payload, and its time -- RCCL: an event
 * pair on the stream that runs it around every all-reduce vbfm_set_profiling's stride samples
 * (device time from the call's enqueue to its completion: the wait for the slowest rank
 * included), scaled to all calls; host exchange: the host wall time of every call (copies
 * included). Zero without a communicator. */
typedef struct {
	int32_t transport;        /* as vbfm_comm_info */
	int32_t n_timed;          /* all-reduces timed */
	uint64_t n_calls;         /* all-reduces issued */
	uint64_t bytes;           /* their payload per rank */
	double ms_timed;          /* summed time of the timed ones */
	double ms_estimated;      /* ms_timed / n_timed * n_calls (host exchange: = ms_timed) */
	double timeout_s;         /* the deadline in force (0: blocking communicator or none) */
} vbfm_exchange_stats;
int vbfm_exchange_info(vbfm_ctx *ctx, vbfm_exchange_stats *out);
/* The level store's record-buffer placement (VBFM_PLACE): the score (ms, level 0's pattern to and
 * from a reference buffer) of each candidate record buffer, [0] and [1] being the pair allocated
 * first, and in kept[0], kept[1] the indices of the two buffers kept (records, alternate).
 * *count = 0 when no placement was tuned. ms holds up to *count on entry (in: capacity). */
int vbfm_placement_info(vbfm_ctx *ctx, float *ms, int32_t *count, int32_t *kept);
/* What setting up the train set cost (no reference counterpart; the reference's load and
 * create_data_t are the host's, Data.h:106-283, 457-509): host wall seconds of the last
 * vbfm_set_train (copy to the device + the device CSR build) and of the first sweep's set-up of that
 * train set -- the dependency levels, the row store (level / entry store, long-column segments,
 * split-form payloads) and, inside it, the placement search with the device memory it held at its
 * peak and the candidates it scored (0: no search). Zero until the step has run. */
typedef struct {
	double s_set_train;       /* vbfm_set_train / vbfm_synth_generate of the train set */
	double s_schedule;        /* dependency levels */
	double s_store;           /* row store build, the placement search included */
	double s_placement;       /* ... of which the placement search */
	uint64_t place_bytes;     /* device memory the search held at its peak */
	int32_t place_candidates; /* buffers scored (0: no search) */
	int32_t place_kept[2];    /* the two kept, as vbfm_placement_info's kept */
} vbfm_setup_stats;
int vbfm_setup_info(vbfm_ctx *ctx, vbfm_setup_stats *out);

/* Partition of the VB sweep over ranks (set before vbfm_set_train).
 *   VBFM_SHARD_ROWS (default): the exact row-sharded mode above.
 *   VBFM_SHARD_FEATURES: the north star's feature-column partition. Every rank holds ALL train
 *     rows; the columns of every dependency level are split into num_shards contiguous chunks
 *     and each rank sweeps its chunk; after the w sweep and after every factor pass the ranks'
 *     changes of the e / t row caches, their partial q-caches of the next factor and their
 *     updated parameters are summed with one ncclAllReduce each. Shards do not see each
 *     other's updates within a pass (Jacobi across shards), so results differ from the
 *     reference's sequential sweep when num_shards > 1 (exact for num_shards = 1). Without a
 *     communicator num_shards > 1 runs the shards one after another in this process (same
 *     arithmetic; for tests). num_shards = 0: one shard per rank. VB learner only. */
#define VBFM_SHARD_ROWS 0
#define VBFM_SHARD_FEATURES 1
int vbfm_set_shard_mode(vbfm_ctx *ctx, int32_t mode, int32_t num_shards);

/* ---- online VB learner (-method vb_online, OVBFM) -------------------------------------
 * Replaces fm_learn_vb_online + fm_learn_vb_online_simultaneous (src/libfm/src/
 * fm_learn_vb_online.h, fm_learn_vb_online_simultaneous.h:20-290; selected at
 * src/libfm/libfm.cpp:312-320). vbfm_online_init turns a context made by vbfm_create that holds
 * its train and test sets into the online learner: the VB learner's initial draws (host or
 * device replay, the same values), then fm_learn_vb_online::init (natural parameters, step
 * sizes, col_count). Each vbfm_online_epoch is one iteration of _learn's loop: a
 * std::random_shuffle of the rows on the reference's rand() stream, num_batch mini-batches
 * (row r in batch ceil(shuffle[r] / ceil(N / num_batch))), update_all on each batch in turn,
 * then the test RMSE. num_attribute follows the online CLI: largest feature id of train and
 * test + 1 (find_max_feature, libfm.cpp:167-170, 528-600). One GPU. A num_batch that leaves a
 * batch empty is refused (the reference divides by its zero size). */
#define VBFM_ONLINE_INIT_HOST 0    /* draws on the host (glibc restatement) */
#define VBFM_ONLINE_INIT_REPLAY 1  /* the same draws on the device (vbfm_init_params_replay) */
typedef struct {
	uint32_t num_batch;       /* -batch (libfm.cpp:320; default 50) */
	uint32_t seed;            /* srand(seed) (libfm.cpp:123-124) */
	double init_stdev;        /* -init_stdev (draws of fm.v / fm.w that precede the learner's) */
	int32_t init_mode;        /* VBFM_ONLINE_INIT_* */
	double *fm_v;             /* [k*D] f-major or NULL: receives the fm.v draws (v_file.txt, fm_model.h:98) */
} vbfm_online_config;

typedef struct {
	double rmse, mae;                              /* test, clipped (:206-245) */
	double free_energy_first, free_energy_last;    /* "free energy" of batch 1 and batch num_batch (:143-146) */
	double alpha, sigma_0, mu_0_dash, sigma_0_dash;
	uint32_t nan_mu_w, nan_sigma_w, inf_mu_w;
	uint32_t nan_mu_v, nan_sigma_v, inf_mu_v;
	uint32_t nan_alpha, inf_alpha;
	uint32_t num_batch;
	int32_t num_levels;
	/* device time: regrouping into batches, the batches' update_all, test; ms */
	double ms_regroup, ms_batches, ms_test, ms_total;
	/* ... and the batches' phases summed over the epoch: batch CSR + predictions, update_w0,
	 * the w sweep, the factor sweeps, the hyper-parameters + free energy */
	double ms_predict, ms_w0, ms_w, ms_v, ms_hyper;
	uint32_t n_vlevel_launches;   /* level launches of the factor sweeps */
	uint64_t nnz_train;
	uint32_t n_lord_batches;      /* batches swept on their level-ordered store (complete levels) */
	uint32_t n_pad_batches;       /* ... of which with the padded layout of levels >= 1 (fills the
	                               * struct's tail padding: its size is unchanged) */
} vbfm_online_stats;

int vbfm_online_init(vbfm_ctx *ctx, const vbfm_online_config *cfg);
int vbfm_online_epoch(vbfm_ctx *ctx, vbfm_online_stats *out);
/* the learner's own state: natural parameters ([D], [k*D] f-major as vbfm_params), step sizes
 * new_wj / new_vj [D], scalars {alpha, sigma_0, mu_0_dash, sigma_0_dash, natural_mu_0_dash,
 * natural_sigma_0_dash, new_w0, t_w0}; NULL arrays are skipped. vbfm_get_params and
 * vbfm_get_test_pred serve the online learner as the VB one. */
int vbfm_online_get_state(vbfm_ctx *ctx, double *nat_mu_w, double *nat_sigma_w, double *nat_mu_v,
                          double *nat_sigma_v, double *new_wj, double *new_vj, double scalars[8]);

/* ---- MCMC / ALS learner (-method mcmc | als) -------------------------------------------
 * Replaces fm_learn_mcmc / fm_learn_mcmc_simultaneous (src/libfm/src/fm_learn_mcmc.h,
 * src/libfm/src/fm_learn_mcmc_simultaneous.h), regression, without relation blocks.
 * vbfm_mcmc_init turns a context made by vbfm_create into an MCMC/ALS learner; the data
 * hand-over (vbfm_set_train / vbfm_set_test / vbfm_synth_generate), vbfm_comm_init and the
 * level schedule are the VB learner's. State is the model's point values fm.w0 / fm.w /
 * fm.v and the hyper-priors; the row cache holds e = yhat - y (the MCMC sign, :76-80). */
#define VBFM_RNG_REFERENCE 0  /* every draw from the reference's stream: srand(seed), glibc
                                 rand(), Leva normals, Marsaglia-Tsang gammas (random.h),
                                 consumed in the reference's order: the draws the reference
                                 makes on the same inputs */
#define VBFM_RNG_DEVICE 1     /* hyper-prior draws from that stream; the per-attribute
                                 normals of draw_w / draw_v from a counter-based generator
                                 keyed (seed, iteration, factor, attribute), identical on
                                 every shard; fm.w / fm.v initialised on the device */

typedef struct {
	int32_t do_sample;        /* fm_learn_mcmc::do_sample: 1 mcmc, 0 als (libfm.cpp:131-135, 303) */
	int32_t do_multilevel;    /* fm_learn_mcmc::do_multilevel (libfm.cpp:304) */
	int32_t rng;              /* VBFM_RNG_* */
	uint32_t seed;            /* srand(seed) (libfm.cpp:123-124) */
	double init_stdev;        /* -init_stdev: fm.v, fm.w ~ N(0, init_stdev) (fm_model.h:97, libfm.cpp:298) */
	const double *regular;    /* -regular values: 0, 1, 3 or 1 + 2*num_attr_groups of them (libfm.cpp:367-411) */
	int32_t num_regular;
} vbfm_mcmc_config;

typedef struct {
	double *w;                /* [D]   fm.w */
	double *v;                /* [k*D] fm.v[f][j] */
	double *w_mu, *w_lambda;  /* [G]   fm_learn_mcmc::w_mu, w_lambda */
	double *v_mu, *v_lambda;  /* [G*k] v_mu(g, f), v_lambda(g, f), row-major [g][f] */
	double w0, alpha, reg0;   /* fm.w0, fm_learn_mcmc::alpha, fm.reg0 */
} vbfm_mcmc_params;

typedef struct {
	double rmse_all, mae_all;   /* test, on the running mean of the clipped predictions: "Test=" */
	double rmse_this, mae_this; /* test, this iteration's predictions */
	double train_rmse;          /* "Train=" (fm_learn_mcmc_simultaneous.h:153-162) */
	double alpha, w0;
	uint32_t nan_alpha, inf_alpha, nan_w0, inf_w0, nan_w, inf_w, nan_v, inf_v;
	uint32_t nan_w_mu, inf_w_mu, nan_w_lambda, inf_w_lambda, nan_v_mu, inf_v_mu, nan_v_lambda, inf_v_lambda;
	uint32_t rng_skipped;       /* VBFM_RNG_REFERENCE: attributes whose draw / no-draw decision
	                               (the reference draws no normal for a zero or non-finite
	                               variance) differed from the host's, i.e. 0 while the stream
	                               is the reference's; VBFM_RNG_DEVICE: such attributes */
	int32_t num_levels;
	/* device time of the phases (hipEvents), ms; per-launch sums with vbfm_set_profiling */
	double ms_hyper, ms_w, ms_v, ms_predict, ms_total;
	double ms_vlevel_kernels;
	int32_t n_vlevel_launches;
	uint64_t nnz_train;
} vbfm_mcmc_stats;

int vbfm_mcmc_init(vbfm_ctx *ctx, const vbfm_mcmc_config *cfg);  /* fm_learn_mcmc::init (fm_learn_mcmc.h:1092-1151),
                                                                    parameter draws and -regular (libfm.cpp:123-124, 273-304, 367-411) */
int vbfm_mcmc_set_params(vbfm_ctx *ctx, const vbfm_mcmc_params *p);
int vbfm_mcmc_get_params(vbfm_ctx *ctx, vbfm_mcmc_params *p);      /* NULL arrays are skipped */
int vbfm_mcmc_init_caches(vbfm_ctx *ctx);                          /* _learn prologue, fm_learn_mcmc_simultaneous.h:64-81 */
int vbfm_mcmc_iterate(vbfm_ctx *ctx, vbfm_mcmc_stats *out);        /* one pass of :83-304: draw_all, re-predict, evaluate */
/* fm_learn_mcmc::predict (fm_learn_mcmc.h:355-381): sampling -> pred_sum_all / num_iter,
 * else the last iteration's predictions; clipped to the train target range */
int vbfm_mcmc_get_test_pred(vbfm_ctx *ctx, int32_t num_iter, double *pred /*[test rows]*/);
/* the v draws of all factors alone (q-cache + draw_v sweeps, :501-621), for the bench */
int vbfm_mcmc_factor_sweep(vbfm_ctx *ctx, double *ms_device);

/* ---- host side of the reference's CLI path (loader, RNG init) -------------------------- */
typedef struct {
	uint32_t num_rows, num_feature;
	uint64_t nnz;
	float min_target, max_target;
	float *target;                  /* [num_rows] */
	uint64_t *row_ptr; vbfm_entry *row_ent;   /* CSR in file order   (Data.h:233-278) */
	uint64_t *col_ptr; vbfm_entry *col_ent;   /* transposed copy     (Data.h:457-509) */
} vbfm_host_data;
/* Data::load (Data.h:106-283): libfm text, or the binary triple <name>.x/.xt/.y
 * (fmatrix.h:46-52, matrix.h:296-312) when those files exist. Text is parsed in parallel
 * (VBFM_LOADER_THREADS, default min(cores, 16)) with the reference's sscanf semantics; the
 * transpose (Data::create_data_t) is a parallel stable counting sort. */
int vbfm_load_data(const char *filename, vbfm_host_data *out);
/* The reference's binary triple of a loaded data set: <base>.x (CSR rows in file order),
 * <base>.xt (the transposed copy) and <base>.y, as tools/convert + tools/transpose write them
 * (fmatrix.h:67-86, matrix.h:280-293). vbfm_load_data(<base>) then reads it back. */
int vbfm_save_data(const char *basename, const vbfm_host_data *d);
void vbfm_free_host_data(vbfm_host_data *d);
/* srand(seed) then the reference's draw order: fm.v (k*D) ~ N(0, init_stdev)
 * (fm_model.h:97), fm.w (D) (libfm.cpp:307), mu_w_dash (D), mu_v_dash (k*D) as 0.1*N(0,1)
 * (fm_learn_vb.h:709-711); sigma_* and hyper parameters at their init values.
 * fm_v / fm_w may be NULL (they are drawn either way, to keep the stream aligned). */
int vbfm_init_params_host(uint32_t seed, double init_stdev, int32_t num_factor, uint32_t num_attribute,
                          uint32_t num_attr_groups, vbfm_params *out, double *fm_v, double *fm_w);

#ifdef __cplusplus
}
#endif
#endif /* VBFM_H_ */
