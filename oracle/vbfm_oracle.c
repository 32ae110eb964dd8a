/* oracle/vbfm_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker; never the product).
 *
 * Plain-C restatement of the reference's libFM VB path and of its MCMC / ALS learner. Every function follows the reference's arithmetic expression by
 * expression, in the reference's loop order, so that on the same inputs it reproduces the
 * reference bit for bit (pinned by tests/test_oracle_golden.py against dumps of the
 * compiled reference, oracle/_ref/ref_driver).
 *
 * Type discipline that matters for bit-exactness: design-matrix values are fp32
 * (FM_FLOAT, src/fm_core/fm_data.h:25) and a product of two fp32 values stays fp32 before it
 * meets a double (e.g. `x_li * x_li * h` at fm_learn_vb.h:595). Build with
 * -ffp-contract=off.
 *
 * Citations are relative to /root/reference.
 */
#define _GNU_SOURCE
#include "vbfm_oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* glibc rand(): TYPE_3 additive feedback generator (degree 31, separation 3), seeded by
 * the Park-Miller LCG and warmed up by 310 discarded outputs. Restated from the published
 * glibc algorithm (stdlib/random_r.c); the reference reaches it through ran_uniform()
 * (src/util/random.h:174-176) after srand(seed) (src/libfm/libfm.cpp:123-124).          */
static int32_t g_r[34];
static int g_f, g_b; /* front / rear indices into the 31-word ring (stored in g_r[0..30]) */

void or_srand(uint32_t seed)
{
	int32_t word;
	int i;
	if (seed == 0) seed = 1;
	g_r[0] = (int32_t)seed;
	word = (int32_t)seed;
	for (i = 1; i < 31; i++) {
		long hi = word / 127773, lo = word % 127773;
		word = (int32_t)(16807 * lo - 2836 * hi);
		if (word < 0) word += 2147483647;
		g_r[i] = word;
	}
	g_f = 3; g_b = 0;
	for (i = 0; i < 310; i++) (void)or_rand();
}

int32_t or_rand(void)
{
	uint32_t val = (uint32_t)g_r[g_f] + (uint32_t)g_r[g_b];
	g_r[g_f] = (int32_t)val;
	g_f = (g_f + 1) % 31;
	g_b = (g_b + 1) % 31;
	return (int32_t)(val >> 1);
}

static double or_uniform(void) { return or_rand() / ((double)2147483647 + 1); } /* random.h:174-176 */

/* Leva's ratio-of-uniforms normal generator (random.h:150-164). */
double or_ran_gaussian(void)
{
	double u, v, x, y, Q;
	for (;;) {
		do { u = or_uniform(); } while (u == 0.0);
		v = 1.7156 * (or_uniform() - 0.5);
		x = u - 0.449871;
		y = fabs(v) + 0.386595;
		Q = x * x + y * (0.19600 * y - 0.25472 * x);
		if (Q < 0.27597) break;
		if (!((Q > 0.27846) || ((v * v) > (-4.0 * u * u * log(u))))) break;
	}
	return v / u;
}

double or_ran_gaussian_ms(double mean, double stdev) /* random.h:166-172 */
{
	if (stdev == 0.0 || isnan(stdev)) return mean;
	return mean + stdev * or_ran_gaussian();
}

/* ------------------------------------------------------------------------------------ */
/* libfm text loader: Data::load (src/libfm/src/Data.h:106-283). Two passes, sscanf
 * semantics ("%f%n" for the target, "%d:%f%n" for features), blank lines and lines
 * starting with '#' skipped, anything left after the features is an error.             */
static int parse_line(const char *line, float *target, uint32_t *feat, float *val,
                      uint32_t *n, int *maxf, int fill)
{
	const char *p = line;
	float v;
	int nchar, fid;
	while (*p == ' ' || *p == '\t') p++;
	if (*p == 0 || *p == '#') return 0;
	if (sscanf(p, "%f%n", &v, &nchar) < 1) return -1;
	p += nchar;
	*target = v;
	*n = 0;
	while (sscanf(p, "%d:%f%n", &fid, &v, &nchar) >= 2) {
		p += nchar;
		if (fid < 0) return -2;
		if (fid > *maxf) *maxf = fid;
		if (fill) { feat[*n] = (uint32_t)fid; val[*n] = v; }
		(*n)++;
	}
	while (*p != 0 && (*p == ' ' || *p == '\t')) p++;
	if (*p != 0 && *p != '#') return -1;
	return 1;
}

static int transpose_csr(or_data *d)
{
	/* Data::create_data_t (Data.h:457-509): column j lists (row, value) in ascending row
	 * order, entries of one row in their file order. */
	uint32_t nf = d->num_feature;
	uint64_t *cnt = (uint64_t *)calloc((size_t)nf + 1, sizeof(uint64_t));
	uint32_t i;
	uint64_t j;
	if (!cnt) return -1;
	d->col_ptr = (uint64_t *)malloc(((size_t)nf + 1) * sizeof(uint64_t));
	d->col_row = (uint32_t *)malloc((d->nnz ? d->nnz : 1) * sizeof(uint32_t));
	d->col_val = (float *)malloc((d->nnz ? d->nnz : 1) * sizeof(float));
	if (!d->col_ptr || !d->col_row || !d->col_val) { free(cnt); return -1; }
	for (j = 0; j < d->nnz; j++) cnt[d->row_feat[j]]++;
	d->col_ptr[0] = 0;
	for (i = 0; i < nf; i++) d->col_ptr[i + 1] = d->col_ptr[i] + cnt[i];
	for (i = 0; i < nf; i++) cnt[i] = d->col_ptr[i];
	for (i = 0; i < d->num_rows; i++)
		for (j = d->row_ptr[i]; j < d->row_ptr[i + 1]; j++) {
			uint32_t f = d->row_feat[j];
			d->col_row[cnt[f]] = i;
			d->col_val[cnt[f]] = d->row_val[j];
			cnt[f]++;
		}
	free(cnt);
	return 0;
}

int or_load_libfm(const char *path, or_data *out, char *err, int errlen)
{
	FILE *fp;
	char *line = NULL;
	size_t cap = 0;
	ssize_t len;
	int pass, maxf = -1, has_feature = 0;
	size_t scratch_cap = 0;
	uint32_t rows = 0, *feat = NULL;
	uint64_t nnz = 0;
	float *val = NULL;
	memset(out, 0, sizeof(*out));
	out->min_target = 3.40282347e+38f;
	out->max_target = -3.40282347e+38f;
	for (pass = 0; pass < 2; pass++) {
		uint32_t r = 0;
		uint64_t c = 0;
		fp = fopen(path, "r");
		if (!fp) { snprintf(err, errlen, "unable to open %s", path); return -1; }
		if (pass == 1) {
			out->num_rows = rows;
			out->nnz = nnz;
			out->num_feature = has_feature ? (uint32_t)maxf + 1 : 0;
			out->target = (float *)malloc((rows ? rows : 1) * sizeof(float));
			out->row_ptr = (uint64_t *)malloc(((size_t)rows + 1) * sizeof(uint64_t));
			out->row_feat = (uint32_t *)malloc((nnz ? nnz : 1) * sizeof(uint32_t));
			out->row_val = (float *)malloc((nnz ? nnz : 1) * sizeof(float));
			out->row_ptr[0] = 0;
		}
		while ((len = getline(&line, &cap, fp)) >= 0) {
			float tgt;
			uint32_t n;
			int rc;
			if (len > 0 && line[len - 1] == '\n') line[len - 1] = 0;
			if (pass == 0) {
				/* the counting pass parses into a scratch row sized by the line length */
				size_t maxn = (size_t)len / 2 + 1;
				if (maxn > scratch_cap) {
					free(feat); free(val);
					feat = (uint32_t *)malloc(maxn * sizeof(uint32_t));
					val = (float *)malloc(maxn * sizeof(float));
					scratch_cap = maxn;
				}
				rc = parse_line(line, &tgt, feat, val, &n, &maxf, 1);
			} else {
				rc = parse_line(line, &tgt, out->row_feat + c, out->row_val + c, &n, &maxf, 1);
			}
			if (rc < 0) {
				snprintf(err, errlen, "cannot parse line \"%s\"", line);
				fclose(fp); free(line); free(feat); free(val);
				return -1;
			}
			if (rc == 0) continue;
			if (pass == 0) {
				/* std::min(_value, min_target) / std::max(_value, max_target) (Data.h:200-201):
				 * a NaN target resets both, as the reference's std::min / std::max do */
				out->min_target = (out->min_target < tgt) ? out->min_target : tgt;
				out->max_target = (tgt < out->max_target) ? out->max_target : tgt;
				rows++;
				nnz += n;
				if (n) has_feature = 1;
			} else {
				out->target[r] = tgt;
				c += n;
				r++;
				out->row_ptr[r] = c;
			}
		}
		fclose(fp);
		if (pass == 0) { free(feat); free(val); feat = NULL; val = NULL; }
	}
	free(line);
	if (transpose_csr(out)) { snprintf(err, errlen, "out of memory"); return -1; }
	return 0;
}

int or_data_from_csr(uint32_t num_rows, uint64_t nnz, const uint64_t *row_ptr,
                     const uint32_t *row_feat, const float *row_val, const float *target,
                     or_data *out)
{
	uint64_t j;
	uint32_t i;
	int maxf = -1;
	memset(out, 0, sizeof(*out));
	out->num_rows = num_rows;
	out->nnz = nnz;
	out->target = (float *)malloc((num_rows ? num_rows : 1) * sizeof(float));
	out->row_ptr = (uint64_t *)malloc(((size_t)num_rows + 1) * sizeof(uint64_t));
	out->row_feat = (uint32_t *)malloc((nnz ? nnz : 1) * sizeof(uint32_t));
	out->row_val = (float *)malloc((nnz ? nnz : 1) * sizeof(float));
	memcpy(out->row_ptr, row_ptr, ((size_t)num_rows + 1) * sizeof(uint64_t));
	memcpy(out->row_feat, row_feat, nnz * sizeof(uint32_t));
	memcpy(out->row_val, row_val, nnz * sizeof(float));
	memcpy(out->target, target, num_rows * sizeof(float));
	out->min_target = 3.40282347e+38f;
	out->max_target = -3.40282347e+38f;
	for (i = 0; i < num_rows; i++) {
		out->min_target = (out->min_target < target[i]) ? out->min_target : target[i];   /* Data.h:164-165 */
		out->max_target = (target[i] < out->max_target) ? out->max_target : target[i];
	}
	for (j = 0; j < nnz; j++) if ((int)row_feat[j] > maxf) maxf = (int)row_feat[j];
	out->num_feature = (uint32_t)(maxf + 1);
	return transpose_csr(out);
}

void or_free_data(or_data *d)
{
	free(d->target); free(d->row_ptr); free(d->row_feat); free(d->row_val);
	free(d->col_ptr); free(d->col_row); free(d->col_val);
	memset(d, 0, sizeof(*d));
}

/* ------------------------------------------------------------------------------------ */
/* VB learner                                                                           */
static void *xcalloc(size_t n, size_t s) { return calloc(n ? n : 1, s); }

int or_vb_create(or_vb *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group)
{
	uint32_t i;
	memset(st, 0, sizeof(*st));
	st->k0 = k0; st->k1 = k1; st->k = k; st->D = D;
	st->attr_group = (uint32_t *)xcalloc(D, sizeof(uint32_t));
	st->G = 1;
	if (attr_group) {   /* DataMetaInfo::loadGroupsFromFile (Data.h:49-61) */
		st->G = 0;
		for (i = 0; i < D; i++) {
			st->attr_group[i] = attr_group[i];
			if (attr_group[i] + 1 > st->G) st->G = attr_group[i] + 1;
		}
	}
	st->num_attr_per_group = (uint32_t *)xcalloc(st->G, sizeof(uint32_t));
	for (i = 0; i < D; i++) st->num_attr_per_group[st->attr_group[i]]++;
	st->sigma_w = (double *)xcalloc(st->G, sizeof(double));
	st->sigma_v = (double *)xcalloc((size_t)st->G * k, sizeof(double));
	st->mu_w = (double *)xcalloc(D, sizeof(double));
	st->sig_w = (double *)xcalloc(D, sizeof(double));
	st->mu_v = (double *)xcalloc((size_t)k * D, sizeof(double));
	st->sig_v = (double *)xcalloc((size_t)k * D, sizeof(double));
	st->fm_v = (double *)xcalloc((size_t)k * D, sizeof(double));
	st->fm_w = (double *)xcalloc(D, sizeof(double));
	/* fm_learn_vb::init (fm_learn_vb.h:693-712) */
	st->alpha = 1.0; st->sigma_0 = 1.0; st->mu_0_dash = 0.0; st->sigma_0_dash = 0.02;
	for (i = 0; i < st->G; i++) st->sigma_w[i] = 1;
	for (i = 0; i < st->G * (uint32_t)k; i++) st->sigma_v[i] = 1;
	for (i = 0; i < D; i++) st->sig_w[i] = .02;
	for (i = 0; i < (uint32_t)k * D; i++) st->sig_v[i] = .02;
	return 0;
}

void or_vb_destroy(or_vb *st)
{
	free(st->attr_group); free(st->num_attr_per_group); free(st->sigma_w); free(st->sigma_v);
	free(st->mu_w); free(st->sig_w); free(st->mu_v); free(st->sig_v); free(st->fm_v); free(st->fm_w);
	free(st->e); free(st->q); free(st->t); free(st->tq); free(st->tz);
	free(st->e_test); free(st->q_test); free(st->pred_test);
	memset(st, 0, sizeof(*st));
}

void or_vb_init_params(or_vb *st, uint32_t seed, double init_stdev)
{
	uint32_t i;
	uint32_t kd = (uint32_t)st->k * st->D;
	or_srand(seed);                                                   /* libfm.cpp:123-124 */
	for (i = 0; i < kd; i++) st->fm_v[i] = or_ran_gaussian_ms(0, init_stdev); /* fm_model.h:97 */
	for (i = 0; i < st->D; i++) st->fm_w[i] = or_ran_gaussian_ms(0, init_stdev); /* libfm.cpp:307 */
	for (i = 0; i < st->D; i++) st->mu_w[i] = 0.1 * or_ran_gaussian_ms(0, 1);   /* fm_learn_vb.h:709, matrix.h:358-363 */
	for (i = 0; i < kd; i++) st->mu_v[i] = 0.1 * or_ran_gaussian_ms(0, 1);      /* fm_learn_vb.h:711, matrix.h:375-381 */
}

int or_vb_attach(or_vb *st, const or_data *train, const or_data *test)
{
	st->n_train = train->num_rows;
	st->n_test = test->num_rows;
	st->e = (double *)xcalloc(train->num_rows, sizeof(double));
	st->q = (double *)xcalloc(train->num_rows, sizeof(double));
	st->t = (double *)xcalloc(train->num_rows, sizeof(double));
	st->tq = (double *)xcalloc(train->num_rows, sizeof(double));
	st->tz = (double *)xcalloc(train->num_rows, sizeof(double));
	st->e_test = (double *)xcalloc(test->num_rows, sizeof(double));
	st->q_test = (double *)xcalloc(test->num_rows, sizeof(double));
	st->pred_test = (double *)xcalloc(test->num_rows, sizeof(double));
	st->min_target = train->min_target;   /* libfm.cpp:332-333 */
	st->max_target = train->max_target;
	return 0;
}

/* fm_learn_vb.h:70-203 (one data set; iterates that data set's own transposed copy) */
void or_vb_predict_eterms(const or_vb *st, const or_data *d, double *e, double *q)
{
	uint32_t i, c;
	uint64_t p;
	int f;
	for (i = 0; i < d->num_rows; i++) { e[i] = 0.0; q[i] = 0.0; }
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++)
				q[d->col_row[p]] += v[i] * d->col_val[p];
		for (c = 0; c < d->num_rows; c++) { double qa = q[c]; e[c] += 0.5 * qa * qa; q[c] = 0.0; }
	}
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) {
				float x = d->col_val[p];
				q[d->col_row[p]] -= 0.5 * v[i] * v[i] * x * x;
			}
	}
	if (st->k1)
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++)
				q[d->col_row[p]] += st->mu_w[i] * d->col_val[p];
	for (c = 0; c < d->num_rows; c++) {
		double qa = q[c];
		e[c] = e[c] + qa;
		if (st->k0) e[c] += st->mu_0_dash;
		q[c] = 0.0;
	}
}

/* fm_learn_vb.h:207-312 */
void or_vb_predict_t(const or_vb *st, const or_data *d, double *t, double *q, double *z)
{
	uint32_t i, c;
	uint64_t p;
	int f;
	for (i = 0; i < d->num_rows; i++) { q[i] = 0.0; z[i] = 0.0; t[i] = 0.0; }
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D;
		const double *vs = st->sig_v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) {
				uint32_t r = d->col_row[p];
				float x = d->col_val[p];
				q[r] += v[i] * x * v[i] * x;
				z[r] += vs[i] * x * x;
			}
		for (c = 0; c < d->num_rows; c++) {
			double qa = q[c], za = z[c];
			t[c] += (0.5 * za * za + za * qa);
			q[c] = 0.0; z[c] = 0.0;
		}
	}
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D;
		const double *vs = st->sig_v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) {
				float x = d->col_val[p];
				q[d->col_row[p]] -= (v[i] * v[i] * x * x * x * x * vs[i] +
				                     0.5 * x * x * x * x * vs[i] * vs[i]);
			}
	}
	if (st->k1)
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) {
				float x = d->col_val[p];
				q[d->col_row[p]] += st->sig_w[i] * x * x;
			}
	for (c = 0; c < d->num_rows; c++) {
		double qa = q[c];
		t[c] = t[c] + qa;
		if (st->k0) t[c] += st->sigma_0_dash;
		q[c] = 0.0;
	}
}

void or_vb_init_caches(or_vb *st, const or_data *train, const or_data *test)
{
	uint32_t c;
	or_vb_predict_eterms(st, train, st->e, st->q);
	or_vb_predict_eterms(st, test, st->e_test, st->q_test);
	or_vb_predict_t(st, train, st->t, st->tq, st->tz);
	for (c = 0; c < train->num_rows; c++) st->e[c] = train->target[c] - st->e[c];
}

void or_vb_update_w0(or_vb *st, const or_data *train)
{
	double sigma_old = st->sigma_0_dash, mu_old, w0_temp = 0.0;
	uint32_t i;
	st->sigma_0_dash = 1.0 / (st->sigma_0 + train->num_rows * st->alpha);
	mu_old = st->mu_0_dash;
	for (i = 0; i < train->num_rows; i++) w0_temp += st->e[i] + st->mu_0_dash;
	st->mu_0_dash = st->sigma_0_dash * st->alpha * w0_temp;
	for (i = 0; i < train->num_rows; i++) {
		st->e[i] = st->e[i] + (mu_old - st->mu_0_dash);
		st->t[i] = st->t[i] + (st->sigma_0_dash - sigma_old);
	}
}

/* update_w (fm_learn_vb.h:527-574) for one feature column */
static void vb_update_w(or_vb *st, double *mu, double *sigma, double sigma_w,
                        const uint32_t *rows, const float *vals, uint64_t n)
{
	double w_sigma_sqr = 0, w_mean = 0, mu_old = *mu, sigma_old = *sigma;
	uint64_t p;
	for (p = 0; p < n; p++) {
		float x = vals[p];
		w_mean += x * (st->e[rows[p]] + x * *mu);
		w_sigma_sqr += x * x;            /* fp32 product */
	}
	*sigma = (double)1.0 / (sigma_w + st->alpha * w_sigma_sqr);
	*mu = *sigma * st->alpha * w_mean;
	if (isnan(*sigma) || isinf(*sigma)) { st->nan_sigma_w++; *sigma = sigma_old; }
	if (isnan(*mu)) { st->nan_mu_w++; *mu = mu_old; return; }
	if (isinf(*mu)) { st->inf_mu_w++; *mu = mu_old; return; }
	for (p = 0; p < n; p++) {
		double h = vals[p];
		uint32_t r = rows[p];
		st->e[r] += h * (mu_old - *mu);
		st->t[r] += h * h * (*sigma - sigma_old);
	}
}

void or_vb_update_w_all(or_vb *st, const or_data *train)
{
	uint32_t i;
	if (!st->k1) return;
	for (i = 0; i < train->num_feature; i++) {
		uint64_t b = train->col_ptr[i], n = train->col_ptr[i + 1] - b;
		vb_update_w(st, &st->mu_w[i], &st->sig_w[i], st->sigma_w[st->attr_group[i]],
		            train->col_row + b, train->col_val + b, n);
	}
}

void or_vb_add_main_q(or_vb *st, const or_data *train, int f)
{
	uint32_t c, i;
	uint64_t p;
	const double *v = st->mu_v + (size_t)f * st->D;
	const double *vs = st->sig_v + (size_t)f * st->D;
	for (c = 0; c < train->num_rows; c++) { st->q[c] = 0.0; st->tq[c] = 0.0; st->tz[c] = 0.0; }
	for (i = 0; i < train->num_feature; i++)
		for (p = train->col_ptr[i]; p < train->col_ptr[i + 1]; p++) {
			uint32_t r = train->col_row[p];
			float x = train->col_val[p];
			st->q[r] += v[i] * x;
			st->tq[r] += vs[i] * x * x;
			st->tz[r] += v[i] * v[i] * x * x;
		}
}

/* update_v (fm_learn_vb.h:577-644) for one feature column */
static void vb_update_v(or_vb *st, double *mu, double *sigma, double sigma_v_g,
                        const uint32_t *rows, const float *vals, uint64_t n)
{
	double v_sigma_sqr = 0, v_mean = 0, mu_old = *mu, sigma_old = *sigma;
	uint64_t p;
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		float xx = x * x;
		double h = st->q[r] - x * *mu;
		double h1 = st->tq[r] - xx * *sigma;
		v_mean += x * h * (st->e[r] + x * *mu * h);
		v_sigma_sqr += xx * h * h + xx * h1;
	}
	*sigma = (double)1.0 / (sigma_v_g + st->alpha * v_sigma_sqr);
	*mu = *sigma * st->alpha * v_mean;
	if (isnan(*sigma) || isinf(*sigma)) { *sigma = sigma_old; st->nan_sigma_v++; }
	if (isnan(*mu)) { st->nan_mu_v++; *mu = mu_old; return; }
	if (isinf(*mu)) { st->inf_mu_v++; *mu = mu_old; return; }
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		float xx = x * x;
		double h = x * (st->q[r] - x * mu_old);
		double h1 = xx * (st->tq[r] - xx * sigma_old);
		double h2 = xx * (st->tz[r] - xx * mu_old * mu_old);
		st->q[r] += x * (*mu - mu_old);
		st->tq[r] += xx * (*sigma - sigma_old);
		st->tz[r] += xx * (*mu * *mu - mu_old * mu_old);
		st->e[r] += h * (mu_old - *mu);
		st->t[r] += (h1 + h2) * (*sigma - sigma_old);
		st->t[r] += h1 * (*mu * *mu - mu_old * mu_old);
	}
}

void or_vb_update_v_all(or_vb *st, const or_data *train, int f)
{
	uint32_t i;
	double *v = st->mu_v + (size_t)f * st->D;
	double *vs = st->sig_v + (size_t)f * st->D;
	for (i = 0; i < train->num_feature; i++) {
		uint64_t b = train->col_ptr[i], n = train->col_ptr[i + 1] - b;
		vb_update_v(st, &v[i], &vs[i], st->sigma_v[(size_t)st->attr_group[i] * st->k + f],
		            train->col_row + b, train->col_val + b, n);
	}
}

static void vb_hyper_groups(or_vb *st)
{
	/* fm_learn_vb.h:472-498 */
	uint32_t i, g;
	int f;
	double *tmp = (double *)xcalloc(st->G, sizeof(double));
	st->sigma_0 = 1.0 / (st->mu_0_dash * st->mu_0_dash + st->sigma_0_dash);
	for (i = 0; i < st->D; i++) tmp[st->attr_group[i]] += st->mu_w[i] * st->mu_w[i] + st->sig_w[i];
	for (g = 0; g < st->G; g++) st->sigma_w[g] = (double)st->num_attr_per_group[g] / tmp[g];
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D, *v1 = st->sig_v + (size_t)f * st->D;
		for (g = 0; g < st->G; g++) tmp[g] = 0.0;
		for (i = 0; i < st->D; i++) tmp[st->attr_group[i]] += v[i] * v[i] + v1[i];
		for (g = 0; g < st->G; g++) st->sigma_v[(size_t)g * st->k + f] = (double)st->num_attr_per_group[g] / tmp[g];
	}
	free(tmp);
}

int or_vb_hyper(or_vb *st, const or_data *train)
{
	/* fm_learn_vb.h:446-470: alpha, early return on NaN/inf */
	double alpha_temp = 0.0, alpha_old;
	uint32_t i;
	for (i = 0; i < train->num_rows; i++) alpha_temp += st->e[i] * st->e[i] + st->t[i];
	alpha_old = st->alpha;
	st->alpha = (double)train->num_rows / alpha_temp;
	if (isnan(st->alpha)) { st->nan_alpha++; st->alpha = alpha_old; return 1; }
	if (isinf(st->alpha)) { st->inf_alpha++; st->alpha = alpha_old; return 1; }
	vb_hyper_groups(st);
	return 0;
}

static double vb_free_energy_from(or_vb *st, double temp, uint32_t n)
{
	/* fm_learn_vb.h:662-677 (note 3.14, not pi) */
	double fe = 0.0, temp1 = 2 * 3.14 * (1.0 / st->alpha);
	uint32_t i;
	int f;
	fe += -0.5 * st->alpha * temp - .5 * n * log(temp1);
	fe += -0.5 * st->sigma_0 * (st->mu_0_dash * st->mu_0_dash + st->sigma_0_dash) +
	      0.5 * log(st->sigma_0_dash * st->sigma_0) + .5;
	for (i = 0; i < st->D; i++) {
		uint32_t g = st->attr_group[i];
		fe += -0.5 * st->sigma_w[g] * (st->mu_w[i] * st->mu_w[i] + st->sig_w[i]) +
		      0.5 * log(st->sig_w[i] * st->sigma_w[g]) + .5;
	}
	for (f = 0; f < st->k; f++) {
		const double *v = st->mu_v + (size_t)f * st->D, *v1 = st->sig_v + (size_t)f * st->D;
		for (i = 0; i < st->D; i++) {
			double sv = st->sigma_v[(size_t)st->attr_group[i] * st->k + f];
			fe += -0.5 * sv * (v[i] * v[i] + v1[i]) + 0.5 * log(v1[i] * sv) + .5;
		}
	}
	st->last_free_energy = fe;
	return fe;
}

double or_vb_free_energy(or_vb *st, const or_data *train)
{
	double temp = 0.0;
	uint32_t i;
	for (i = 0; i < train->num_rows; i++) temp += st->e[i] * st->e[i] + st->t[i];
	return vb_free_energy_from(st, temp, train->num_rows);
}

void or_vb_update_all(or_vb *st, const or_data *train)
{
	int f;
	if (st->k0) or_vb_update_w0(st, train);
	if (st->k1) or_vb_update_w_all(st, train);
	if (st->D > 0)
		for (f = 0; f < st->k; f++) {
			or_vb_add_main_q(st, train, f);
			or_vb_update_v_all(st, train, f);
		}
	st->hyper_skipped = or_vb_hyper(st, train);
	if (!st->hyper_skipped) or_vb_free_energy(st, train);
}

/* ---- OVBFM (see vbfm_oracle.h) ------------------------------------------------------------ */
int or_ovb_create(or_ovb *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group, uint32_t num_batch)
{
	memset(st, 0, sizeof(*st));
	or_vb_create(&st->vb, k0, k1, k, D, attr_group);
	st->num_batch = num_batch;
	st->nat_mu_w = (double *)xcalloc(D, 8); st->nat_sig_w = (double *)xcalloc(D, 8);
	st->nat_mu_v = (double *)xcalloc((size_t)k * D, 8); st->nat_sig_v = (double *)xcalloc((size_t)k * D, 8);
	st->new_wj = (double *)xcalloc(D, 8); st->new_vj = (double *)xcalloc(D, 8);
	st->t_wj = (uint32_t *)xcalloc(D, 4); st->t_vj = (uint32_t *)xcalloc(D, 4);
	st->col_count = (uint32_t *)xcalloc(D, 4);
	return 0;
}

void or_ovb_destroy(or_ovb *st)
{
	or_vb_destroy(&st->vb);
	free(st->nat_mu_w); free(st->nat_sig_w); free(st->nat_mu_v); free(st->nat_sig_v);
	free(st->new_wj); free(st->new_vj); free(st->t_wj); free(st->t_vj); free(st->col_count); free(st->shuffle);
	memset(st, 0, sizeof(*st));
}

void or_ovb_init(or_ovb *st, uint32_t seed, double init_stdev, const or_data *train, const or_data *test)
{
	or_vb *vb = &st->vb;
	uint32_t i, D = vb->D;
	uint64_t p;
	size_t kd = (size_t)vb->k * D;
	or_vb_init_params(vb, seed, init_stdev);     /* same draws and order as fm_learn_vb */
	/* fm_learn_vb_online.h:686-700: learning rates */
	st->lamda = 0.5;
	st->t0_w0 = 1; st->t0_wj = 1; st->t0_vj = 1; st->t_w0 = 0;
	st->new_w0 = pow((double)(st->t0_w0 + st->t_w0), -st->lamda);
	for (i = 0; i < D; i++) {
		st->new_wj[i] = pow((double)(st->t0_wj + 0), -st->lamda);
		st->new_vj[i] = pow((double)(st->t0_vj + 0), -st->lamda);
		st->t_wj[i] = 0; st->t_vj[i] = 0;
	}
	st->nat_mu0 = 0.0;
	st->nat_sig0 = 1 / vb->sigma_0_dash;
	/* :706-730: col_count over the train file (every "%u:%lf" entry) */
	for (i = 0; i < D; i++) st->col_count[i] = 0;
	for (p = 0; p < train->nnz; p++)
		if (train->row_feat[p] < D) st->col_count[train->row_feat[p]] += 1;
	/* :745-758: natural parameters */
	for (i = 0; i < D; i++) { st->nat_mu_w[i] = vb->mu_w[i] / 0.02; st->nat_sig_w[i] = 1 / vb->sig_w[i]; }
	for (p = 0; p < kd; p++) { st->nat_mu_v[p] = vb->mu_v[p] / 0.02; st->nat_sig_v[p] = 1 / vb->sig_v[p]; }
	/* _learn (fm_learn_vb_online_simultaneous.h:55-62) */
	st->n_total = train->num_rows;
	st->size_except_last = (uint32_t)ceil((double)train->num_rows / st->num_batch);
	st->shuffle = (uint32_t *)xcalloc(train->num_rows, 4);
	for (i = 0; i < train->num_rows; i++) st->shuffle[i] = i + 1;
	vb->n_test = test->num_rows;
	vb->e_test = (double *)xcalloc(test->num_rows, 8);
	vb->q_test = (double *)xcalloc(test->num_rows, 8);
	vb->pred_test = (double *)xcalloc(test->num_rows, 8);
	vb->min_target = train->min_target;
	vb->max_target = train->max_target;
}

/* update_w0 (fm_learn_vb_online.h:471-497) */
static void ovb_update_w0(or_ovb *st, const or_data *b, uint32_t size)
{
	or_vb *vb = &st->vb;
	double sigma_dash = vb->sigma_0_dash, mu_dash = vb->mu_0_dash, mu_old = st->nat_mu0, sigma_old = st->nat_sig0;
	double eta1 = 0.0, eta2 = 0.0, w0_temp;
	uint32_t i;
	for (i = 0; i < b->num_rows; i++) {
		w0_temp = vb->e[i] + vb->mu_0_dash;
		st->nat_sig0 = ((1 - st->new_w0) * sigma_old) + st->new_w0 * (vb->sigma_0 + size * vb->alpha);
		st->nat_mu0 = ((1 - st->new_w0) * mu_old) + st->new_w0 * size * vb->alpha * w0_temp;
		eta1 += st->nat_mu0;
		eta2 += st->nat_sig0;
	}
	st->nat_mu0 = eta1 / b->num_rows;
	st->nat_sig0 = eta2 / b->num_rows;
	vb->mu_0_dash = st->nat_mu0 / st->nat_sig0;
	vb->sigma_0_dash = 1.0 / st->nat_sig0;
	for (i = 0; i < b->num_rows; i++) {
		vb->e[i] = vb->e[i] + (mu_dash - vb->mu_0_dash);
		vb->t[i] = vb->t[i] + (vb->sigma_0_dash - sigma_dash);
	}
}

/* update_w (fm_learn_vb_online.h:499-556) for one non-empty column of the batch */
static void ovb_update_w(or_ovb *st, uint32_t col, double sigma_w, const uint32_t *rows, const float *vals, uint64_t n)
{
	or_vb *vb = &st->vb;
	double *mu = &vb->mu_w[col], *sigma = &vb->sig_w[col];
	double mu_dash = *mu, sigma_dash = *sigma, mu_old = st->nat_mu_w[col], sigma_old = st->nat_sig_w[col];
	double eta1 = 0.0, eta2 = 0.0, w_mean, w_sigma_sqr;
	uint64_t p;
	for (p = 0; p < n; p++) {
		float x = vals[p];
		w_mean = x * (vb->e[rows[p]] + x * *mu);
		w_sigma_sqr = x * x;
		st->nat_sig_w[col] = ((1 - st->new_wj[col]) * sigma_old) +
		                     st->new_wj[col] * (sigma_w + vb->alpha * st->col_count[col] * w_sigma_sqr);
		st->nat_mu_w[col] = ((1 - st->new_wj[col]) * mu_old) + st->new_wj[col] * st->col_count[col] * vb->alpha * w_mean;
		eta1 += st->nat_mu_w[col];
		eta2 += st->nat_sig_w[col];
	}
	st->t_wj[col] += (uint32_t)n;
	st->new_wj[col] = pow((double)(st->t0_wj + st->t_wj[col]), -st->lamda);
	st->nat_mu_w[col] = eta1 / (uint32_t)n;
	st->nat_sig_w[col] = eta2 / (uint32_t)n;
	*mu = st->nat_mu_w[col] / st->nat_sig_w[col];
	*sigma = 1 / st->nat_sig_w[col];
	if (isnan(*sigma) || isinf(*sigma)) { vb->nan_sigma_w++; *sigma = sigma_dash; }
	if (isnan(*mu)) { vb->nan_mu_w++; *mu = mu_dash; return; }
	if (isinf(*mu)) { vb->inf_mu_w++; *mu = mu_dash; return; }
	for (p = 0; p < n; p++) {
		double h = vals[p];
		uint32_t r = rows[p];
		vb->e[r] += h * (mu_dash - *mu);
		vb->t[r] += h * h * (*sigma - sigma_dash);
	}
}

/* update_v (fm_learn_vb_online.h:558-627) for one non-empty column of the batch */
static void ovb_update_v(or_ovb *st, int f, uint32_t col, double sigma_v_g, const uint32_t *rows, const float *vals,
                         uint64_t n)
{
	or_vb *vb = &st->vb;
	const size_t ix = (size_t)f * vb->D + col;
	double *mu = &vb->mu_v[ix], *sigma = &vb->sig_v[ix];
	double mu_dash = *mu, sigma_dash = *sigma, mu_old = st->nat_mu_v[ix], sigma_old = st->nat_sig_v[ix];
	double eta1 = 0.0, eta2 = 0.0, v_mean, v_sigma_sqr;
	uint64_t p;
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		double h = vb->q[r] - x * *mu;
		double h1 = vb->tq[r] - x * x * *sigma;
		v_mean = x * h * (vb->e[r] + x * *mu * h);
		v_sigma_sqr = x * x * h * h + x * x * h1;
		st->nat_sig_v[ix] = (1 - st->new_vj[col]) * sigma_old +
		                    st->new_vj[col] * (sigma_v_g + vb->alpha * st->col_count[col] * v_sigma_sqr);
		st->nat_mu_v[ix] = ((1 - st->new_vj[col]) * mu_old) + st->new_vj[col] * st->col_count[col] * vb->alpha * v_mean;
		eta1 += st->nat_mu_v[ix];
		eta2 += st->nat_sig_v[ix];
	}
	st->nat_mu_v[ix] = eta1 / (uint32_t)n;
	st->nat_sig_v[ix] = eta2 / (uint32_t)n;
	*mu = st->nat_mu_v[ix] / st->nat_sig_v[ix];
	*sigma = 1 / st->nat_sig_v[ix];
	if (isnan(*sigma) || isinf(*sigma)) { *sigma = sigma_dash; vb->nan_sigma_v++; }
	if (isnan(*mu)) { vb->nan_mu_v++; *mu = mu_dash; return; }
	if (isinf(*mu)) { vb->inf_mu_v++; *mu = mu_dash; return; }
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		double h = x * (vb->q[r] - x * mu_dash);
		double h1 = x * x * (vb->tq[r] - x * x * sigma_dash);
		double h2 = x * x * (vb->tz[r] - x * x * mu_dash * mu_dash);
		vb->q[r] += x * (*mu - mu_dash);
		vb->tq[r] += x * x * (*sigma - sigma_dash);
		vb->tz[r] += x * x * (*mu * *mu - mu_dash * mu_dash);
		vb->e[r] += h * (mu_dash - *mu);
		vb->t[r] += (h1 + h2) * (*sigma - sigma_dash);
		vb->t[r] += h1 * (*mu * *mu - mu_dash * mu_dash);
	}
}

/* update_all (fm_learn_vb_online.h:354-469) on one batch; _size = all train rows */
static void ovb_update_all(or_ovb *st, const or_data *b, uint32_t size)
{
	or_vb *vb = &st->vb;
	uint32_t i, g, c;
	int f;
	if (vb->k0) ovb_update_w0(st, b, size);
	if (vb->k1)
		for (i = 0; i < b->num_feature; i++) {
			uint64_t cb = b->col_ptr[i], n = b->col_ptr[i + 1] - cb;
			if (n == 0) continue;
			ovb_update_w(st, i, vb->sigma_w[vb->attr_group[i]], b->col_row + cb, b->col_val + cb, n);
		}
	if (vb->D > 0) {
		for (f = 0; f < vb->k; f++) {
			or_vb_add_main_q(vb, b, f);   /* zeroes q, tq, tz first */
			for (i = 0; i < b->num_feature; i++) {
				uint64_t cb = b->col_ptr[i], n = b->col_ptr[i + 1] - cb;
				if (n == 0) continue;
				ovb_update_v(st, f, i, vb->sigma_v[(size_t)vb->attr_group[i] * vb->k + f], b->col_row + cb,
				             b->col_val + cb, n);
				if (f == 0) st->t_vj[i] += (uint32_t)n;
			}
		}
		for (i = 0; i < b->num_feature; i++) st->new_vj[i] = pow((double)(st->t0_vj + st->t_vj[i]), -st->lamda);
	}
	{   /* alpha (:413-433) */
		double alpha_temp = 0.0, alpha_old;
		for (c = 0; c < b->num_rows; c++) alpha_temp += vb->e[c] * vb->e[c] + vb->t[c];
		alpha_old = vb->alpha;
		vb->alpha = (1 - st->new_w0) * alpha_old + st->new_w0 * ((double)b->num_rows / alpha_temp);
		if (isnan(vb->alpha)) { vb->nan_alpha++; vb->alpha = alpha_old; st->hyper_skipped_any = 1; return; }
		if (isinf(vb->alpha)) { vb->inf_alpha++; vb->alpha = alpha_old; st->hyper_skipped_any = 1; return; }
	}
	vb->sigma_0 = (1 - st->new_w0) * vb->sigma_0 + st->new_w0 * (1.0 / (vb->mu_0_dash * vb->mu_0_dash + vb->sigma_0_dash));
	{
		double *tmp = (double *)xcalloc(vb->G, 8);
		for (i = 0; i < vb->D; i++) tmp[vb->attr_group[i]] += vb->mu_w[i] * vb->mu_w[i] + vb->sig_w[i];
		for (g = 0; g < vb->G; g++)
			vb->sigma_w[g] = (1 - st->new_w0) * vb->sigma_w[g] + st->new_w0 * ((double)vb->num_attr_per_group[g] / tmp[g]);
		for (f = 0; f < vb->k; f++) {
			const double *v = vb->mu_v + (size_t)f * vb->D, *v1 = vb->sig_v + (size_t)f * vb->D;
			for (g = 0; g < vb->G; g++) tmp[g] = 0.0;
			for (i = 0; i < vb->D; i++) tmp[vb->attr_group[i]] += v[i] * v[i] + v1[i];
			for (g = 0; g < vb->G; g++)
				vb->sigma_v[(size_t)g * vb->k + f] = (1 - st->new_w0) * vb->sigma_v[(size_t)g * vb->k + f] +
				                                     st->new_w0 * ((double)vb->num_attr_per_group[g] / tmp[g]);
		}
		free(tmp);
	}
	st->t_w0 += 1;
	st->new_w0 = pow((double)(st->t0_w0 + st->t_w0), -st->lamda);
}

/* the rows of one batch (ascending, the order they are written to the batch file) as a data
 * set with num_attribute columns (Data::load(file, num_attribute), Data.h:287-454) */
static void ovb_batch_data(const or_data *train, const uint32_t *rows, uint32_t n, uint32_t D, or_data *out)
{
	uint64_t nnz = 0, p, q;
	uint32_t i, *feat;
	uint64_t *rp = (uint64_t *)xcalloc((size_t)n + 1, 8);
	float *val, *y = (float *)xcalloc(n, 4);
	for (i = 0; i < n; i++) nnz += train->row_ptr[rows[i] + 1] - train->row_ptr[rows[i]];
	feat = (uint32_t *)xcalloc(nnz, 4);
	val = (float *)xcalloc(nnz, 4);
	for (i = 0, q = 0; i < n; i++) {
		y[i] = train->target[rows[i]];
		for (p = train->row_ptr[rows[i]]; p < train->row_ptr[rows[i] + 1]; p++, q++) {
			feat[q] = train->row_feat[p];
			val[q] = train->row_val[p];
		}
		rp[i + 1] = q;
	}
	or_data_from_csr(n, nnz, rp, feat, val, y, out);
	if (out->num_feature < D) {   /* pad the transposed copy to num_attribute columns */
		uint64_t *cp = (uint64_t *)xcalloc((size_t)D + 1, 8);
		memcpy(cp, out->col_ptr, ((size_t)out->num_feature + 1) * 8);
		for (i = out->num_feature + 1; i <= D; i++) cp[i] = cp[out->num_feature];
		free(out->col_ptr);
		out->col_ptr = cp;
		out->num_feature = D;
	}
	free(rp); free(feat); free(val); free(y);
}

void or_ovb_epoch(or_ovb *st, const or_data *train, const or_data *test, double *rmse, double *mae)
{
	or_vb *vb = &st->vb;
	const uint32_t N = st->n_total;
	uint32_t i, j, c, *rows = (uint32_t *)xcalloc(N, 4);
	double s_rmse = 0.0, s_mae = 0.0, mx = vb->max_target, mn = vb->min_target;
	/* std::random_shuffle (libstdc++ stl_algo.h): i from 1, j = rand() % (i + 1) */
	for (i = 1; i < N; i++) {
		uint32_t k2 = (uint32_t)(or_rand() % (int32_t)(i + 1));
		if (k2 != i) { uint32_t t = st->shuffle[i]; st->shuffle[i] = st->shuffle[k2]; st->shuffle[k2] = t; }
	}
	for (j = 1; j <= st->num_batch; j++) {
		uint32_t n = 0;
		or_data b;
		for (i = 0; i < N; i++)
			if ((uint32_t)ceil((double)st->shuffle[i] / st->size_except_last) == j) rows[n++] = i;
		ovb_batch_data(train, rows, n, vb->D, &b);
		free(vb->e); free(vb->q); free(vb->t); free(vb->tq); free(vb->tz);
		vb->e = (double *)xcalloc(n, 8); vb->q = (double *)xcalloc(n, 8); vb->t = (double *)xcalloc(n, 8);
		vb->tq = (double *)xcalloc(n, 8); vb->tz = (double *)xcalloc(n, 8);
		vb->n_train = n;
		or_vb_predict_eterms(vb, &b, vb->e, vb->q);
		or_vb_predict_t(vb, &b, vb->t, vb->tq, vb->tz);
		for (c = 0; c < n; c++) vb->e[c] = b.target[c] - vb->e[c];
		ovb_update_all(st, &b, N);
		if (j == st->num_batch || j == 1) {
			const double fe = or_vb_free_energy(vb, &b);
			if (j == 1) st->fe_first = fe;
			if (j == st->num_batch) st->fe_last = fe;
		}
		or_free_data(&b);
	}
	free(rows);
	or_vb_predict_eterms(vb, test, vb->e_test, vb->q_test);
	for (c = 0; c < test->num_rows; c++) {
		double p = vb->e_test[c];
		p = p < mx ? p : mx;
		p = mn > p ? mn : p;
		vb->pred_test[c] = p;
		p = vb->pred_test[c] * 1.0;
		p = p < mx ? p : mx;
		p = mn > p ? mn : p;
		{
			double err = p - test->target[c];
			s_rmse += err * err;
			s_mae += fabs(err);
		}
	}
	*rmse = sqrt(s_rmse / test->num_rows);
	*mae = s_mae / test->num_rows;
}

/* ---- feature-sharded update_all (see vbfm_oracle.h) ----------------------------------- */
/* partial q-cache of factor f over the features of one shard, ascending id (the order the
 * fused kernels add a row's own entries in), from 0.0 */
static void fs_partial_q(const or_vb *st, const or_data *train, int f, int s, const int32_t *shard,
                         double *q, double *tq, double *tz)
{
	uint32_t i, c;
	uint64_t p;
	const double *v = st->mu_v + (size_t)f * st->D, *vs = st->sig_v + (size_t)f * st->D;
	for (c = 0; c < train->num_rows; c++) { q[c] = 0.0; tq[c] = 0.0; tz[c] = 0.0; }
	for (i = 0; i < train->num_feature; i++) {
		if (shard[i] != s) continue;
		for (p = train->col_ptr[i]; p < train->col_ptr[i + 1]; p++) {
			uint32_t r = train->col_row[p];
			float x = train->col_val[p];
			q[r] += v[i] * x;
			tq[r] += vs[i] * x * x;
			tz[r] += v[i] * v[i] * x * x;
		}
	}
}

/* one pass (f < 0: the w sweep) over all shards, then the sums of their changes */
static void fs_pass(or_vb *st, const or_data *train, int f, int P, const int32_t *shard)
{
	const uint32_t n = train->num_rows;
	const int next = f < 0 ? (st->k > 0 ? 0 : -1) : (f + 1 < st->k ? f + 1 : -1);
	double *e0 = (double *)xcalloc(n, 8), *t0 = (double *)xcalloc(n, 8);
	double *q0 = (double *)xcalloc(n, 8), *tq0 = (double *)xcalloc(n, 8), *tz0 = (double *)xcalloc(n, 8);
	double *de = (double *)xcalloc(n, 8), *dt = (double *)xcalloc(n, 8);
	double *nq = (double *)xcalloc(n, 8), *ntq = (double *)xcalloc(n, 8), *ntz = (double *)xcalloc(n, 8);
	double *pq = (double *)xcalloc(n, 8), *ptq = (double *)xcalloc(n, 8), *ptz = (double *)xcalloc(n, 8);
	uint32_t c, i;
	int s;
	memcpy(e0, st->e, n * 8); memcpy(t0, st->t, n * 8);
	memcpy(q0, st->q, n * 8); memcpy(tq0, st->tq, n * 8); memcpy(tz0, st->tz, n * 8);
	for (s = 0; s < P; s++) {
		memcpy(st->e, e0, n * 8); memcpy(st->t, t0, n * 8);
		memcpy(st->q, q0, n * 8); memcpy(st->tq, tq0, n * 8); memcpy(st->tz, tz0, n * 8);
		for (i = 0; i < train->num_feature; i++) {
			uint64_t b = train->col_ptr[i], m = train->col_ptr[i + 1] - b;
			if (shard[i] != s) continue;
			if (f < 0)
				vb_update_w(st, &st->mu_w[i], &st->sig_w[i], st->sigma_w[st->attr_group[i]], train->col_row + b,
				            train->col_val + b, m);
			else
				vb_update_v(st, &st->mu_v[(size_t)f * st->D + i], &st->sig_v[(size_t)f * st->D + i],
				            st->sigma_v[(size_t)st->attr_group[i] * st->k + f], train->col_row + b, train->col_val + b, m);
		}
		if (next >= 0) fs_partial_q(st, train, next, s, shard, pq, ptq, ptz);
		for (c = 0; c < n; c++) {
			double a = st->e[c] - e0[c], b = st->t[c] - t0[c];
			de[c] = s ? de[c] + a : a;
			dt[c] = s ? dt[c] + b : b;
			if (next >= 0) {
				nq[c] = s ? nq[c] + pq[c] : pq[c];
				ntq[c] = s ? ntq[c] + ptq[c] : ptq[c];
				ntz[c] = s ? ntz[c] + ptz[c] : ptz[c];
			}
		}
	}
	for (c = 0; c < n; c++) {
		st->e[c] = e0[c] + de[c];
		st->t[c] = t0[c] + dt[c];
		if (next >= 0) { st->q[c] = nq[c]; st->tq[c] = ntq[c]; st->tz[c] = ntz[c]; }
	}
	free(e0); free(t0); free(q0); free(tq0); free(tz0); free(de); free(dt);
	free(nq); free(ntq); free(ntz); free(pq); free(ptq); free(ptz);
}

void or_vb_update_all_fsharded(or_vb *st, const or_data *train, int P, const int32_t *shard)
{
	int f, have_q = 0;
	if (st->k0) or_vb_update_w0(st, train);
	if (st->k1) { fs_pass(st, train, -1, P, shard); have_q = st->k > 0; }
	if (st->D > 0)
		for (f = 0; f < st->k; f++) {
			if (!have_q) or_vb_add_main_q(st, train, f);   /* factor 0 without a w sweep */
			fs_pass(st, train, f, P, shard);
			have_q = 1;
		}
	st->hyper_skipped = or_vb_hyper(st, train);
	if (!st->hyper_skipped) or_vb_free_energy(st, train);
}

void or_vb_iterate(or_vb *st, const or_data *train, const or_data *test,
                   double *rmse, double *mae, double *train_quirk)
{
	/* fm_learn_vb_simultaneous.h:82-222 (regression) */
	uint32_t c;
	double mx = st->max_target, mn = st->min_target, s = 0.0, s_rmse = 0.0, s_mae = 0.0;
	st->nan_mu_w = st->nan_sigma_w = st->inf_mu_w = 0;
	st->nan_mu_v = st->nan_sigma_v = st->inf_mu_v = 0;
	st->nan_alpha = 0;
	or_vb_update_all(st, train);
	or_vb_predict_eterms(st, test, st->e_test, st->q_test);
	for (c = 0; c < test->num_rows; c++) {
		double p = st->e_test[c];
		p = p < mx ? p : mx;     /* std::min(max_target, p) */
		p = mn > p ? mn : p;     /* std::max(min_target, p) */
		st->pred_test[c] = p;
	}
	for (c = 0; c < train->num_rows; c++) {
		double p = st->e[c];
		p = p < mx ? p : mx;
		p = mn > p ? mn : p;
		s += p * p;
	}
	*train_quirk = sqrt(s / train->num_rows);
	for (c = 0; c < test->num_rows; c++) {   /* _evaluate (fm_learn_vb_simultaneous.h:261-279) */
		double p = st->pred_test[c] * 1.0, err;
		p = p < mx ? p : mx;
		p = mn > p ? mn : p;
		err = p - test->target[c];
		s_rmse += err * err;
		s_mae += fabs(err);
	}
	*rmse = sqrt(s_rmse / test->num_rows);
	*mae = s_mae / test->num_rows;
}

/* Row-sharded update_all: the exchange pattern a row-sharded multi-device run uses. Each
 * feature's (v_mean, v_ss) sums and each whole-data-set sum are reduced over shards; the
 * posterior is then computed identically on every shard. */
#define COLB(d, i) ((i) < (d)->num_feature ? (d)->col_ptr[i] : 0)
#define COLE(d, i) ((i) < (d)->num_feature ? (d)->col_ptr[(i) + 1] : 0)

void or_vb_update_all_sharded(or_vb *st, const or_data *train, uint32_t n_global,
                              uint32_t nf_global, or_allreduce_fn allreduce, void *user)
{
	uint32_t i, c;
	uint64_t p;
	int f;
	double buf[2];
	if (st->k0) {   /* update_w0 with a reduced sum */
		double sigma_old = st->sigma_0_dash, mu_old = st->mu_0_dash;
		st->sigma_0_dash = 1.0 / (st->sigma_0 + n_global * st->alpha);
		buf[0] = 0.0;
		for (c = 0; c < train->num_rows; c++) buf[0] += st->e[c] + st->mu_0_dash;
		allreduce(buf, 1, user);
		st->mu_0_dash = st->sigma_0_dash * st->alpha * buf[0];
		for (c = 0; c < train->num_rows; c++) {
			st->e[c] = st->e[c] + (mu_old - st->mu_0_dash);
			st->t[c] = st->t[c] + (st->sigma_0_dash - sigma_old);
		}
	}
	if (st->k1)
		for (i = 0; i < nf_global; i++) {
			double *mu = &st->mu_w[i], *sigma = &st->sig_w[i], mo = *mu, so = *sigma;
			buf[0] = 0.0; buf[1] = 0.0;
			for (p = COLB(train, i); p < COLE(train, i); p++) {
				float x = train->col_val[p];
				buf[0] += x * (st->e[train->col_row[p]] + x * *mu);
				buf[1] += x * x;
			}
			allreduce(buf, 2, user);
			*sigma = (double)1.0 / (st->sigma_w[st->attr_group[i]] + st->alpha * buf[1]);
			*mu = *sigma * st->alpha * buf[0];
			if (isnan(*sigma) || isinf(*sigma)) { st->nan_sigma_w++; *sigma = so; }
			if (isnan(*mu) || isinf(*mu)) { st->nan_mu_w++; *mu = mo; continue; }
			for (p = COLB(train, i); p < COLE(train, i); p++) {
				double h = train->col_val[p];
				uint32_t r = train->col_row[p];
				st->e[r] += h * (mo - *mu);
				st->t[r] += h * h * (*sigma - so);
			}
		}
	for (f = 0; f < st->k; f++) {
		double *v = st->mu_v + (size_t)f * st->D, *vs = st->sig_v + (size_t)f * st->D;
		or_vb_add_main_q(st, train, f);
		for (i = 0; i < nf_global; i++) {
			double mo = v[i], so = vs[i];
			buf[0] = 0.0; buf[1] = 0.0;
			for (p = COLB(train, i); p < COLE(train, i); p++) {
				uint32_t r = train->col_row[p];
				float x = train->col_val[p], xx = x * x;
				double h = st->q[r] - x * mo, h1 = st->tq[r] - xx * so;
				buf[0] += x * h * (st->e[r] + x * mo * h);
				buf[1] += xx * h * h + xx * h1;
			}
			allreduce(buf, 2, user);
			vs[i] = (double)1.0 / (st->sigma_v[(size_t)st->attr_group[i] * st->k + f] + st->alpha * buf[1]);
			v[i] = vs[i] * st->alpha * buf[0];
			if (isnan(vs[i]) || isinf(vs[i])) { vs[i] = so; st->nan_sigma_v++; }
			if (isnan(v[i]) || isinf(v[i])) { v[i] = mo; st->nan_mu_v++; continue; }
			for (p = COLB(train, i); p < COLE(train, i); p++) {
				uint32_t r = train->col_row[p];
				float x = train->col_val[p], xx = x * x;
				double h = x * (st->q[r] - x * mo);
				double h1 = xx * (st->tq[r] - xx * so);
				double h2 = xx * (st->tz[r] - xx * mo * mo);
				st->q[r] += x * (v[i] - mo);
				st->tq[r] += xx * (vs[i] - so);
				st->tz[r] += xx * (v[i] * v[i] - mo * mo);
				st->e[r] += h * (mo - v[i]);
				st->t[r] += (h1 + h2) * (vs[i] - so);
				st->t[r] += h1 * (v[i] * v[i] - mo * mo);
			}
		}
	}
	buf[0] = 0.0;
	for (c = 0; c < train->num_rows; c++) buf[0] += st->e[c] * st->e[c] + st->t[c];
	allreduce(buf, 1, user);
	{
		double alpha_old = st->alpha;
		st->alpha = (double)n_global / buf[0];
		st->hyper_skipped = 0;
		if (isnan(st->alpha) || isinf(st->alpha)) { st->nan_alpha++; st->alpha = alpha_old; st->hyper_skipped = 1; return; }
	}
	vb_hyper_groups(st);
	buf[0] = 0.0;
	for (c = 0; c < train->num_rows; c++) buf[0] += st->e[c] * st->e[c] + st->t[c];
	allreduce(buf, 1, user);
	vb_free_energy_from(st, buf[0], n_global);
}

/* ------------------------------------------------------------------------------------ */
/* MCMC / ALS: fm_learn_mcmc + fm_learn_mcmc_simultaneous (regression, no relations).
 * ALS is the same learner with do_sample = do_multilevel = 0 (libfm.cpp:131-135).        */

/* random.h:118-148: Marsaglia-Tsang for a >= 1, the U^(1/a) boost below 1 */
double or_ran_gamma(double a)
{
	if (a < 1.0) {
		double u;
		do { u = or_uniform(); } while (u == 0.0);
		return or_ran_gamma(a + 1.0) * pow(u, 1.0 / a);
	} else {
		double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d), x, v, u;
		do {
			do {
				x = or_ran_gaussian();
				v = 1.0 + c * x;
			} while (v <= 0.0);
			v = v * v * v;
			u = or_uniform();
		} while ((u >= (1.0 - 0.0331 * (x * x) * (x * x))) && (log(u) >= (0.5 * x * x + d * (1.0 - v + log(v)))));
		return d * v;
	}
}

double or_ran_gamma_ab(double a, double b) { return or_ran_gamma(a) / b; } /* random.h:146-148 */

int or_als_create(or_als *st, int k0, int k1, int k, uint32_t D, const uint32_t *attr_group)
{
	uint32_t i;
	memset(st, 0, sizeof(*st));
	st->k0 = k0; st->k1 = k1; st->k = k; st->D = D;
	st->attr_group = (uint32_t *)xcalloc(D, sizeof(uint32_t));
	st->G = 1;
	if (attr_group) {
		st->G = 0;
		for (i = 0; i < D; i++) {
			st->attr_group[i] = attr_group[i];
			if (attr_group[i] + 1 > st->G) st->G = attr_group[i] + 1;
		}
	}
	st->num_attr_per_group = (uint32_t *)xcalloc(st->G, sizeof(uint32_t));
	for (i = 0; i < D; i++) st->num_attr_per_group[st->attr_group[i]]++;
	st->w = (double *)xcalloc(D, sizeof(double));
	st->v = (double *)xcalloc((size_t)k * D, sizeof(double));
	st->w_lambda = (double *)xcalloc(st->G, sizeof(double));
	st->w_mu = (double *)xcalloc(st->G, sizeof(double));
	st->v_lambda = (double *)xcalloc((size_t)st->G * k, sizeof(double));
	st->v_mu = (double *)xcalloc((size_t)st->G * k, sizeof(double));
	st->alpha = 1;   /* fm_learn_mcmc::init (fm_learn_mcmc.h:1100-1117) */
	st->w0 = 0;
	st->do_sample = 0; st->do_multilevel = 0; st->reg0 = 0.0;
	return 0;
}

void or_als_configure(or_als *st, int do_sample, int do_multilevel, double reg0)
{
	st->do_sample = do_sample; st->do_multilevel = do_multilevel; st->reg0 = reg0;
}

void or_als_destroy(or_als *st)
{
	free(st->attr_group); free(st->num_attr_per_group); free(st->w); free(st->v);
	free(st->w_lambda); free(st->w_mu); free(st->v_lambda); free(st->v_mu);
	free(st->e); free(st->q); free(st->e_test); free(st->q_test);
	free(st->pred_sum_all); free(st->pred_this); free(st->tmp_g);
	memset(st, 0, sizeof(*st));
}

void or_als_init_params(or_als *st, uint32_t seed, double init_stdev)
{
	uint32_t i, kd = (uint32_t)st->k * st->D;
	or_srand(seed);
	for (i = 0; i < kd; i++) st->v[i] = or_ran_gaussian_ms(0, init_stdev);   /* fm_model.h:97 */
	for (i = 0; i < st->D; i++) st->w[i] = or_ran_gaussian_ms(0, init_stdev); /* libfm.cpp:298 */
}

/* fm_learn_mcmc.h:117-348 without relations, on the fm_model parameters */
static void als_predict(const or_als *st, const or_data *d, double *e, double *q)
{
	uint32_t i, c;
	uint64_t p;
	int f;
	for (i = 0; i < d->num_rows; i++) { e[i] = 0.0; q[i] = 0.0; }
	for (f = 0; f < st->k; f++) {
		const double *v = st->v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) q[d->col_row[p]] += v[i] * d->col_val[p];
		for (c = 0; c < d->num_rows; c++) { double qa = q[c]; e[c] += 0.5 * qa * qa; q[c] = 0.0; }
	}
	for (f = 0; f < st->k; f++) {
		const double *v = st->v + (size_t)f * st->D;
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) {
				float x = d->col_val[p];
				q[d->col_row[p]] -= 0.5 * v[i] * v[i] * x * x;
			}
	}
	if (st->k1)
		for (i = 0; i < d->num_feature; i++)
			for (p = d->col_ptr[i]; p < d->col_ptr[i + 1]; p++) q[d->col_row[p]] += st->w[i] * d->col_val[p];
	for (c = 0; c < d->num_rows; c++) {
		e[c] = e[c] + q[c];
		if (st->k0) e[c] += st->w0;
		q[c] = 0.0;
	}
}

int or_als_attach(or_als *st, const or_data *train, const or_data *test)
{
	uint32_t c;
	st->n_train = train->num_rows; st->n_test = test->num_rows;
	st->e = (double *)xcalloc(train->num_rows, sizeof(double));
	st->q = (double *)xcalloc(train->num_rows, sizeof(double));
	st->e_test = (double *)xcalloc(test->num_rows, sizeof(double));
	st->q_test = (double *)xcalloc(test->num_rows, sizeof(double));
	st->pred_sum_all = (double *)xcalloc(test->num_rows, sizeof(double));
	st->pred_this = (double *)xcalloc(test->num_rows, sizeof(double));
	st->min_target = train->min_target; st->max_target = train->max_target;
	/* fm_learn_mcmc_simultaneous.h:71-80: predict train and test, e = yhat - y */
	als_predict(st, train, st->e, st->q);
	als_predict(st, test, st->e_test, st->q_test);
	for (c = 0; c < train->num_rows; c++) st->e[c] = st->e[c] - train->target[c];
	st->iter_done = 0;
	return 0;
}

/* draw_w (fm_learn_mcmc.h:671-718) */
static void als_draw_w(or_als *st, double *w, double w_mu, double w_lambda,
                       const uint32_t *rows, const float *vals, uint64_t n)
{
	double w_sigma_sqr = 0, w_mean = 0, w_old;
	uint64_t p;
	for (p = 0; p < n; p++) {
		float x = vals[p];
		w_mean += x * (st->e[rows[p]] - *w * x);
		w_sigma_sqr += x * x;
	}
	w_sigma_sqr = (double)1.0 / (w_lambda + st->alpha * w_sigma_sqr);
	w_mean = -w_sigma_sqr * (st->alpha * w_mean - w_mu * w_lambda);
	w_old = *w;
	if (isnan(w_sigma_sqr) || isinf(w_sigma_sqr)) *w = 0.0;
	else *w = st->do_sample ? or_ran_gaussian_ms(w_mean, sqrt(w_sigma_sqr)) : w_mean;
	if (isnan(*w)) { st->nan_w++; *w = w_old; return; }
	if (isinf(*w)) { st->inf_w++; *w = w_old; return; }
	for (p = 0; p < n; p++) {
		double h = vals[p];
		st->e[rows[p]] -= h * (w_old - *w);
	}
}

/* draw_v (fm_learn_mcmc.h:780-835) */
static void als_draw_v(or_als *st, double *v, double v_mu, double v_lambda,
                       const uint32_t *rows, const float *vals, uint64_t n)
{
	double v_sigma_sqr = 0, v_mean = 0, v_old;
	uint64_t p;
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		double h = x * (st->q[r] - x * *v);
		v_mean += h * st->e[r];
		v_sigma_sqr += h * h;
	}
	v_mean -= *v * v_sigma_sqr;
	v_sigma_sqr = (double)1.0 / (v_lambda + st->alpha * v_sigma_sqr);
	v_mean = -v_sigma_sqr * (st->alpha * v_mean - v_mu * v_lambda);
	v_old = *v;
	if (isnan(v_sigma_sqr) || isinf(v_sigma_sqr)) *v = 0.0;
	else *v = st->do_sample ? or_ran_gaussian_ms(v_mean, sqrt(v_sigma_sqr)) : v_mean;
	if (isnan(*v)) { st->nan_v++; *v = v_old; return; }
	if (isinf(*v)) { st->inf_v++; *v = v_old; return; }
	for (p = 0; p < n; p++) {
		uint32_t r = rows[p];
		float x = vals[p];
		double h = x * (st->q[r] - x * v_old);
		st->q[r] -= x * (v_old - *v);
		st->e[r] -= h * (v_old - *v);
	}
}

/* hyper-prior constants of fm_learn_mcmc::init (fm_learn_mcmc.h:1100-1103) */
#define MC_ALPHA_0 1.0
#define MC_GAMMA_0 1.0
#define MC_BETA_0 1.0
#define MC_MU_0 0.0

/* draw_alpha (fm_learn_mcmc.h:901-929) */
static void mc_draw_alpha(or_als *st, uint32_t n)
{
	double alpha_n, gamma_n, alpha_old;
	uint32_t i;
	if (!st->do_multilevel) { st->alpha = MC_ALPHA_0; return; }
	alpha_n = MC_ALPHA_0 + n;
	gamma_n = MC_GAMMA_0;
	for (i = 0; i < n; i++) gamma_n += st->e[i] * st->e[i];
	alpha_old = st->alpha;
	st->alpha = or_ran_gamma_ab(alpha_n / 2.0, gamma_n / 2.0);
	if (isnan(st->alpha) || isinf(st->alpha)) st->alpha = alpha_old;
}

/* draw_w_lambda / draw_w_mu (fm_learn_mcmc.h:931-1008); the early `return` on a NaN/inf
 * draw skips the remaining groups, as in the reference */
static void mc_draw_w_lambda(or_als *st)
{
	double *gam = st->tmp_g;
	uint32_t g, i;
	if (!st->do_multilevel) return;
	for (g = 0; g < st->G; g++) gam[g] = MC_BETA_0 * (st->w_mu[g] - MC_MU_0) * (st->w_mu[g] - MC_MU_0) + MC_GAMMA_0;
	for (i = 0; i < st->D; i++) {
		g = st->attr_group[i];
		gam[g] += (st->w[i] - st->w_mu[g]) * (st->w[i] - st->w_mu[g]);
	}
	for (g = 0; g < st->G; g++) {
		double a = MC_ALPHA_0 + st->num_attr_per_group[g] + 1, old = st->w_lambda[g];
		st->w_lambda[g] = st->do_sample ? or_ran_gamma_ab(a / 2.0, gam[g] / 2.0) : a / gam[g];
		if (isnan(st->w_lambda[g]) || isinf(st->w_lambda[g])) { st->w_lambda[g] = old; return; }
	}
}

static void mc_draw_w_mu(or_als *st)
{
	double *mean = st->tmp_g;
	uint32_t g, i;
	if (!st->do_multilevel) { for (g = 0; g < st->G; g++) st->w_mu[g] = MC_MU_0; return; }
	for (g = 0; g < st->G; g++) mean[g] = 0.0;
	for (i = 0; i < st->D; i++) mean[st->attr_group[i]] += st->w[i];
	for (g = 0; g < st->G; g++) {
		double s2, old = st->w_mu[g];
		mean[g] = (mean[g] + MC_BETA_0 * MC_MU_0) / (st->num_attr_per_group[g] + MC_BETA_0);
		s2 = (double)1.0 / ((st->num_attr_per_group[g] + MC_BETA_0) * st->w_lambda[g]);
		st->w_mu[g] = st->do_sample ? or_ran_gaussian_ms(mean[g], sqrt(s2)) : mean[g];
		if (isnan(st->w_mu[g]) || isinf(st->w_mu[g])) { st->w_mu[g] = old; return; }
	}
}

/* draw_v_lambda / draw_v_mu (fm_learn_mcmc.h:1011-1089); v_mu, v_lambda at [g*k + f] */
static void mc_draw_v_lambda(or_als *st)
{
	double *gam = st->tmp_g;
	uint32_t g, i;
	int f, k = st->k;
	if (!st->do_multilevel) return;
	for (f = 0; f < k; f++) {
		const double *v = st->v + (size_t)f * st->D;
		for (g = 0; g < st->G; g++) {
			double m = st->v_mu[(size_t)g * k + f];
			gam[g] = MC_BETA_0 * (m - MC_MU_0) * (m - MC_MU_0) + MC_GAMMA_0;
		}
		for (i = 0; i < st->D; i++) {
			double m;
			g = st->attr_group[i];
			m = st->v_mu[(size_t)g * k + f];
			gam[g] += (v[i] - m) * (v[i] - m);
		}
		for (g = 0; g < st->G; g++) {
			double a = MC_ALPHA_0 + st->num_attr_per_group[g] + 1, *lam = &st->v_lambda[(size_t)g * k + f], old = *lam;
			*lam = st->do_sample ? or_ran_gamma_ab(a / 2.0, gam[g] / 2.0) : a / gam[g];
			if (isnan(*lam) || isinf(*lam)) { *lam = old; return; }
		}
	}
}

static void mc_draw_v_mu(or_als *st)
{
	double *mean = st->tmp_g;
	uint32_t g, i;
	int f, k = st->k;
	if (!st->do_multilevel) { for (i = 0; i < st->G * (uint32_t)k; i++) st->v_mu[i] = MC_MU_0; return; }
	for (f = 0; f < k; f++) {
		const double *v = st->v + (size_t)f * st->D;
		for (g = 0; g < st->G; g++) mean[g] = 0.0;
		for (i = 0; i < st->D; i++) mean[st->attr_group[i]] += v[i];
		for (g = 0; g < st->G; g++) {
			double s2, *mu = &st->v_mu[(size_t)g * k + f], old = *mu;
			mean[g] = (mean[g] + MC_BETA_0 * MC_MU_0) / (st->num_attr_per_group[g] + MC_BETA_0);
			s2 = (double)1.0 / ((st->num_attr_per_group[g] + MC_BETA_0) * st->v_lambda[(size_t)g * k + f]);
			*mu = st->do_sample ? or_ran_gaussian_ms(mean[g], sqrt(s2)) : mean[g];
			if (isnan(*mu) || isinf(*mu)) { *mu = old; return; }
		}
	}
}

void or_als_iterate(or_als *st, const or_data *train, const or_data *test,
                    double *rmse_all, double *rmse_this, double *train_rmse)
{
	uint32_t i, c;
	uint64_t p;
	int f;
	double mx = st->max_target, mn = st->min_target, s = 0.0, s1 = 0.0, s2 = 0.0;
	if (!st->tmp_g) st->tmp_g = (double *)xcalloc(st->G, sizeof(double));
	/* draw_all (fm_learn_mcmc.h:411-623) */
	mc_draw_alpha(st, train->num_rows);
	if (st->k0) {   /* draw_w0 (fm_learn_mcmc.h:628-668), w0_mean_0 = 0 */
		double w0_mean = 0, w0_sigma_sqr, w0_old = st->w0;
		for (c = 0; c < train->num_rows; c++) w0_mean += st->e[c] - st->w0;
		w0_sigma_sqr = (double)1.0 / (st->reg0 + st->alpha * train->num_rows);
		w0_mean = -w0_sigma_sqr * (st->alpha * w0_mean - 0.0 * st->reg0);
		st->w0 = st->do_sample ? or_ran_gaussian_ms(w0_mean, sqrt(w0_sigma_sqr)) : w0_mean;
		if (isnan(st->w0) || isinf(st->w0)) st->w0 = w0_old;
		else for (c = 0; c < train->num_rows; c++) st->e[c] -= (w0_old - st->w0);
	}
	if (st->k1) {
		mc_draw_w_lambda(st);
		mc_draw_w_mu(st);
		for (i = 0; i < train->num_feature; i++) {
			uint32_t g = st->attr_group[i];
			uint64_t b = train->col_ptr[i];
			als_draw_w(st, &st->w[i], st->w_mu[g], st->w_lambda[g], train->col_row + b,
			           train->col_val + b, train->col_ptr[i + 1] - b);
		}
		for (i = train->num_feature; i < st->D; i++) {
			uint32_t g = st->attr_group[i];
			als_draw_w(st, &st->w[i], st->w_mu[g], st->w_lambda[g], NULL, NULL, 0);
		}
	}
	if (st->k > 0) {
		mc_draw_v_lambda(st);
		mc_draw_v_mu(st);
	}
	for (f = 0; f < st->k; f++) {
		double *v = st->v + (size_t)f * st->D;
		for (c = 0; c < train->num_rows; c++) st->q[c] = 0.0;
		for (i = 0; i < train->num_feature; i++)   /* add_main_q (fm_learn_mcmc.h:384-409) */
			for (p = train->col_ptr[i]; p < train->col_ptr[i + 1]; p++)
				st->q[train->col_row[p]] += v[i] * train->col_val[p];
		for (i = 0; i < train->num_feature; i++) {
			uint32_t g = st->attr_group[i];
			uint64_t b = train->col_ptr[i];
			als_draw_v(st, &v[i], st->v_mu[(size_t)g * st->k + f], st->v_lambda[(size_t)g * st->k + f],
			           train->col_row + b, train->col_val + b, train->col_ptr[i + 1] - b);
		}
		for (i = train->num_feature; i < st->D; i++) {
			uint32_t g = st->attr_group[i];
			als_draw_v(st, &v[i], st->v_mu[(size_t)g * st->k + f], st->v_lambda[(size_t)g * st->k + f],
			           NULL, NULL, 0);
		}
	}
	/* fm_learn_mcmc_simultaneous.h:134-175 */
	als_predict(st, train, st->e, st->q);
	als_predict(st, test, st->e_test, st->q_test);
	for (c = 0; c < test->num_rows; c++) {
		double pp = st->e_test[c];
		st->pred_this[c] = pp;
		pp = pp < mx ? pp : mx;      /* std::min(max_target, p) */
		pp = mn < pp ? pp : mn;      /* std::max(min_target, p) */
		st->pred_sum_all[c] += pp;
	}
	for (c = 0; c < train->num_rows; c++) {
		double pp = st->e[c], err;
		pp = pp < mx ? pp : mx;
		pp = mn < pp ? pp : mn;
		err = pp - train->target[c];
		s += err * err;
		st->e[c] = st->e[c] - train->target[c];
	}
	*train_rmse = sqrt(s / train->num_rows);
	for (c = 0; c < test->num_rows; c++) {   /* _evaluate (fm_learn_mcmc_simultaneous.h:261-279) */
		double pp = st->pred_this[c] * 1.0, err;
		pp = pp < mx ? pp : mx; pp = mn < pp ? pp : mn;
		err = pp - test->target[c];
		s1 += err * err;
		pp = st->pred_sum_all[c] * (1.0 / (st->iter_done + 1));
		pp = pp < mx ? pp : mx; pp = mn < pp ? pp : mn;
		err = pp - test->target[c];
		s2 += err * err;
	}
	*rmse_this = sqrt(s1 / test->num_rows);
	*rmse_all = sqrt(s2 / test->num_rows);
	st->iter_done++;
}
