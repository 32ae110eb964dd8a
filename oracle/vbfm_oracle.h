/* oracle/vbfm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * C restatement of the reference's libFM `-method vb` (and `-method als`) path, used only
 * as the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Never linked into, or called by, the product (libvbfm). Pinned against the compiled
 * reference (oracle/_ref/ref_driver) through the fixtures in tests/golden/.
 *
 * Citations are relative to /root/reference.
 */
#ifndef VBFM_ORACLE_H_
#define VBFM_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A loaded libfm data set: CSR in file order (Data.h:233-278) and the transposed copy
 * built by Data::create_data_t (Data.h:457-509). */
typedef struct {
	uint32_t num_rows;
	uint32_t num_feature;     /* max feature id + 1, 0 without features (Data.h:220-222) */
	uint64_t nnz;
	float min_target, max_target;
	float *target;
	uint64_t *row_ptr; uint32_t *row_feat; float *row_val;
	uint64_t *col_ptr; uint32_t *col_row; float *col_val;
} or_data;

/* glibc rand() TYPE_3 restatement (the reference draws through rand(): random.h:174-176) */
void or_srand(uint32_t seed);
int32_t or_rand(void);
double or_ran_gaussian(void);                       /* random.h:150-164 (Leva) */
double or_ran_gaussian_ms(double mean, double stdev); /* random.h:166-172 */

int or_load_libfm(const char *path, or_data *out, char *err, int errlen); /* Data.h:106-283 */
int or_data_from_csr(uint32_t num_rows, uint64_t nnz, const uint64_t *row_ptr,
                     const uint32_t *row_feat, const float *row_val, const float *target,
                     or_data *out);                 /* create_data_t on given CSR */
void or_free_data(or_data *d);

/* VB learner state (fm_learn_vb.h:36-59) */
typedef struct {
	int k0, k1, k;
	uint32_t D;                 /* num_all_attribute (libfm.cpp:215) */
	uint32_t G;                 /* num_attr_groups */
	uint32_t *attr_group;       /* [D] */
	uint32_t *num_attr_per_group; /* [G] */
	double alpha, sigma_0, mu_0_dash, sigma_0_dash;
	double *sigma_w;            /* [G]   */
	double *sigma_v;            /* [G*k] row-major [g][f] */
	double *mu_w, *sig_w;       /* [D]   */
	double *mu_v, *sig_v;       /* [k*D] row-major [f][j] */
	double *fm_v, *fm_w;        /* fm_model draws (v_file.txt), only for RNG parity */
	/* row caches (fm_learn_mcmc.h:52-55, fm_learn_vb.h:17-21) */
	uint32_t n_train, n_test;
	double *e, *q, *t, *tq, *tz;
	double *e_test, *q_test;
	double *pred_test;
	float min_target, max_target;
	uint32_t nan_mu_w, nan_sigma_w, inf_mu_w, nan_mu_v, nan_sigma_v, inf_mu_v, nan_alpha, inf_alpha;
	double last_free_energy;
	int hyper_skipped;          /* update_all returned early (fm_learn_vb.h:456-469) */
} or_vb;

int or_vb_create(or_vb *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group /*D or NULL*/);
void or_vb_destroy(or_vb *st);
/* libfm.cpp:123-124 + 273 + 307 + fm_learn_vb.h:693-712, in the reference's draw order */
void or_vb_init_params(or_vb *st, uint32_t seed, double init_stdev);
int or_vb_attach(or_vb *st, const or_data *train, const or_data *test);
/* fm_learn_vb.h:70-203 on one data set: writes prediction into e_out */
void or_vb_predict_eterms(const or_vb *st, const or_data *d, double *e_out, double *q_scratch);
/* fm_learn_vb.h:207-312 */
void or_vb_predict_t(const or_vb *st, const or_data *d, double *t_out, double *q_scratch, double *z_scratch);
/* fm_learn_vb_simultaneous.h:37-44 */
void or_vb_init_caches(or_vb *st, const or_data *train, const or_data *test);
void or_vb_update_w0(or_vb *st, const or_data *train);                 /* fm_learn_vb.h:504-525 */
void or_vb_update_w_all(or_vb *st, const or_data *train);              /* fm_learn_vb.h:390-406,527-574 */
void or_vb_add_main_q(or_vb *st, const or_data *train, int f);         /* fm_learn_vb.h:411-418,354-381 */
void or_vb_update_v_all(or_vb *st, const or_data *train, int f);       /* fm_learn_vb.h:420-438,577-644 */
int or_vb_hyper(or_vb *st, const or_data *train);                      /* fm_learn_vb.h:446-498; 1 = early return */
double or_vb_free_energy(or_vb *st, const or_data *train);             /* fm_learn_vb.h:646-681 */
void or_vb_update_all(or_vb *st, const or_data *train);                /* fm_learn_vb.h:383-501 */
/* one iteration of fm_learn_vb_simultaneous.h:75-258 (regression) */
void or_vb_iterate(or_vb *st, const or_data *train, const or_data *test,
                   double *rmse, double *mae, double *train_quirk);

/* Row-sharded restatement of update_all: the rows of `train` are this shard's rows only;
 * every per-feature / per-data-set sum goes through `allreduce(buf, n, user)` (in-place sum
 * over shards). With one shard it is update_all itself up to summation order. */
typedef void (*or_allreduce_fn)(double *buf, int n, void *user);
void or_vb_update_all_sharded(or_vb *st, const or_data *train, uint32_t n_train_global,
                              uint32_t nf_train_global, or_allreduce_fn allreduce, void *user);

/* Feature-sharded update_all: libvbfm's VBFM_SHARD_FEATURES mode (the north star's column
 * partition; NOT an algorithm of the reference, so its parity is unpinned against it and
 * equals or_vb_update_all only for nshards = 1, up to the e0 + (e - e0) rounding). Each
 * shard updates its own features (shard[j] for j < train->num_feature, ascending id) from
 * the same row caches; then the shards' changes of e / t and their partial q-caches of the
 * next factor are summed in shard order. */
void or_vb_update_all_fsharded(or_vb *st, const or_data *train, int nshards, const int32_t *shard);

/* Online VB (OVBFM, -method vb_online): fm_learn_vb_online (fm_learn_vb_online.h) driven by
 * fm_learn_vb_online_simultaneous::_learn (fm_learn_vb_online_simultaneous.h:20-270): per
 * epoch the rows are shuffled into num_batch mini-batches (libstdc++ random_shuffle on the
 * rand() stream), every batch gets its own caches and one Robbins-Monro natural-gradient
 * update_all with step sizes (t0 + t)^-0.5. */
typedef struct {
	or_vb vb;                        /* parameters, hyper parameters, row caches of the batch */
	double *nat_mu_w, *nat_sig_w;    /* [D] natural_mu_w_dash, natural_sigma_w_dash */
	double *nat_mu_v, *nat_sig_v;    /* [k*D] [f][j] */
	double nat_mu0, nat_sig0;
	double new_w0, lamda;
	double *new_wj, *new_vj;         /* [D] */
	uint32_t *t_wj, *t_vj;           /* [D] */
	uint32_t t_w0, t0_w0, t0_wj, t0_vj;
	uint32_t *col_count;             /* [D] entries of each attribute in the whole train file */
	uint32_t num_batch, n_total, size_except_last;
	uint32_t *shuffle;               /* [n_total], kept across epochs like the reference's */
	double fe_first, fe_last;        /* free energy of the epoch's first / last batch */
	int hyper_skipped_any;
} or_ovb;

int or_ovb_create(or_ovb *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group, uint32_t num_batch);
void or_ovb_destroy(or_ovb *st);
/* srand(seed) + the draws of or_vb_init_params, then fm_learn_vb_online::init
 * (fm_learn_vb_online.h:668-760): natural parameters, step sizes, col_count of `train`.
 * test sizes the test caches. */
void or_ovb_init(or_ovb *st, uint32_t seed, double init_stdev, const or_data *train, const or_data *test);
/* one epoch: shuffle, batches, update_all per batch, test RMSE / MAE */
void or_ovb_epoch(or_ovb *st, const or_data *train, const or_data *test, double *rmse, double *mae);

/* MCMC / ALS learner state (fm_learn_mcmc.h); ALS = mcmc without sampling / multilevel
 * (libfm.cpp:131-135). Draws come from the or_srand stream, as the reference's rand(). */
typedef struct {
	int k0, k1, k;
	uint32_t D, G;
	uint32_t *attr_group, *num_attr_per_group;
	double w0, alpha;
	double *w, *v;              /* fm_model w [D], v [k*D] */
	double *w_lambda, *v_lambda, *w_mu, *v_mu; /* [G], [G*k], [G], [G*k] */
	uint32_t n_train, n_test;
	double *e, *q, *e_test, *q_test;
	double *pred_sum_all, *pred_this;
	float min_target, max_target;
	uint32_t iter_done;
	int do_sample, do_multilevel;   /* fm_learn_mcmc.h:92-93 */
	double reg0;                    /* fm.reg0 (libfm.cpp:367-411) */
	uint32_t nan_w, inf_w, nan_v, inf_v;
	double *tmp_g;                  /* cache_for_group_values */
} or_als;

int or_als_create(or_als *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group);
void or_als_destroy(or_als *st);
void or_als_configure(or_als *st, int do_sample, int do_multilevel, double reg0);
double or_ran_gamma(double a);                 /* random.h:118-144 */
double or_ran_gamma_ab(double a, double b);    /* random.h:146-148 */
void or_als_init_params(or_als *st, uint32_t seed, double init_stdev); /* libfm.cpp:123,273,298 */
int or_als_attach(or_als *st, const or_data *train, const or_data *test);
void or_als_iterate(or_als *st, const or_data *train, const or_data *test,
                    double *rmse_all, double *rmse_this, double *train_rmse);

#ifdef __cplusplus
}
#endif
#endif
