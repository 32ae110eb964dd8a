// tests/cli_stub.cpp -- TEST INFRASTRUCTURE: a host-only stand-in for the GPU half of
// include/vbfm.h, so that bin/libFM's own host logic (flag handling, the fork of one process per
// rank, the row slices, the shared-memory exchange, rank 0's files, the -out gather, failure
// handling) runs under AddressSanitizer / UBSan on a CPU (tests/test_host_sanitizers.py). The
// loader and the initial draws are the product's own (csrc/vbfm_host.cpp, linked beside).
//
// A "learner" here keeps its rank's test targets; vbfm_iterate exchanges (through the rank's
// host exchange) the sums of the targets and the row counts, plus a buffer larger than one
// exchange slot whose sum every rank checks, and reports rmse = mean test target over all
// ranks, free energy = -(train rows over all ranks); vbfm_get_test_pred returns the rank's test
// targets, so a gathered -out file must list the whole test set's targets in row order.
#include "vbfm.h"

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" const char *vbfm_host_last_error(void);
extern "C" void vbfm_host_set_error(const char *m);

struct vbfm_ctx {
	std::string err;
	int32_t k = 0;
	uint32_t D = 0, n_train = 0, n_test = 0;
	std::vector<float> test_y;
	vbfm_exchange_fn fn = nullptr;
	void *user = nullptr;
	int32_t nranks = 1, rank = 0;
	uint32_t iter = 0;
};

static int fail(vbfm_ctx *c, const char *m)
{
	if (c) c->err = m;
	else vbfm_host_set_error(m);
	return -1;
}

extern "C" {

int vbfm_abi_version(void) { return VBFM_ABI_VERSION; }
const char *vbfm_last_error(const vbfm_ctx *c) { return c ? c->err.c_str() : vbfm_host_last_error(); }
int vbfm_device_count(int32_t *n)
{
	*n = 1;
	return 0;
}
int vbfm_create(vbfm_ctx **out, const vbfm_config *cfg)
{
	if (cfg->device != 0) return fail(nullptr, "device ordinal out of range");
	vbfm_ctx *c = new vbfm_ctx();
	c->k = cfg->num_factor;
	c->D = cfg->num_attribute;
	*out = c;
	return 0;
}
void vbfm_destroy(vbfm_ctx *c) { delete c; }
int vbfm_setup_info(vbfm_ctx *, vbfm_setup_stats *o)
{
	memset(o, 0, sizeof(*o));
	o->place_kept[0] = o->place_kept[1] = -1;
	return 0;
}
int vbfm_set_shard_mode(vbfm_ctx *, int32_t, int32_t) { return 0; }
int vbfm_exchange_info(vbfm_ctx *c, vbfm_exchange_stats *o)
{
	memset(o, 0, sizeof(*o));
	o->transport = c->fn ? 2 : 0;
	return 0;
}
int vbfm_comm_unique_id(uint8_t *) { return fail(nullptr, "no RCCL in the sanitizer build"); }
int vbfm_comm_init(vbfm_ctx *c, int32_t, int32_t, const uint8_t *) { return fail(c, "no RCCL in the sanitizer build"); }
int vbfm_comm_init_host(vbfm_ctx *c, int32_t nranks, int32_t rank, vbfm_exchange_fn fn, void *user)
{
	c->fn = fn;
	c->user = user;
	c->nranks = nranks;
	c->rank = rank;
	return 0;
}
int vbfm_set_train(vbfm_ctx *c, const vbfm_csc *d)
{
	for (uint64_t p = 0; p < d->nnz; p++)
		if (d->col_ent[p].id >= d->num_rows) return fail(c, "row index out of range in col_ent");
	c->n_train = d->num_rows;
	return 0;
}
int vbfm_set_test(vbfm_ctx *c, const vbfm_csc *d)
{
	c->n_test = d->num_rows;
	c->test_y.assign(d->target, d->target + d->num_rows);
	return 0;
}
int vbfm_init_params_replay(vbfm_ctx *c, uint32_t, double, double *fm_v, double *fm_w)
{
	if (fm_v) memset(fm_v, 0, sizeof(double) * (size_t)c->k * c->D);
	if (fm_w) memset(fm_w, 0, sizeof(double) * c->D);
	return 0;
}
int vbfm_set_params(vbfm_ctx *, const vbfm_params *) { return 0; }
int vbfm_init_caches(vbfm_ctx *) { return 0; }

int vbfm_iterate(vbfm_ctx *c, vbfm_iter_stats *st)
{
	memset(st, 0, sizeof(*st));
	double s[3] = {0.0, (double)c->n_test, (double)c->n_train};
	for (float y : c->test_y) s[0] += y;
	uint32_t mx = (uint32_t)c->rank;
	if (c->fn) {
		if (c->fn(c->user, s, 3, VBFM_X_F64, VBFM_X_SUM)) return fail(c, "host exchange failed");
		if (c->fn(c->user, &mx, 1, VBFM_X_U32, VBFM_X_MAX)) return fail(c, "host exchange failed");
		if (mx != (uint32_t)(c->nranks - 1)) return fail(c, "max exchange wrong");
		std::vector<double> big((size_t)700000, (double)(c->rank + 1));   // > one 4 MB slot
		if (c->fn(c->user, big.data(), big.size(), VBFM_X_F64, VBFM_X_SUM)) return fail(c, "host exchange failed");
		const double want = c->nranks * (c->nranks + 1) / 2.0;
		for (double v : big)
			if (v != want) return fail(c, "chunked exchange wrong");
	}
	st->rmse = s[0] / s[1];
	st->mae = 0.0;
	st->train_quirk = s[2];
	st->free_energy = -s[2];
	st->free_energy_valid = 1;
	c->iter++;
	return 0;
}
int vbfm_get_test_pred(vbfm_ctx *c, double *pred)
{
	for (uint32_t i = 0; i < c->n_test; i++) pred[i] = c->test_y[i];
	return 0;
}
int vbfm_save_state(vbfm_ctx *c, const char *path, uint32_t iter)
{
	FILE *f = fopen(path, "wb");
	if (!f) return fail(c, "cannot open checkpoint file");
	fwrite(&iter, 4, 1, f);
	fwrite(&c->rank, 4, 1, f);
	fclose(f);
	return 0;
}
int vbfm_load_state(vbfm_ctx *c, const char *path, uint32_t *iter)
{
	FILE *f = fopen(path, "rb");
	if (!f) return fail(c, "cannot open checkpoint file");
	int32_t r = -1;
	const bool ok = fread(iter, 4, 1, f) == 1 && fread(&r, 4, 1, f) == 1;
	fclose(f);
	if (!ok || r != c->rank) return fail(c, "checkpoint of another rank");
	return 0;
}
int vbfm_mcmc_init(vbfm_ctx *c, const vbfm_mcmc_config *) { return fail(c, "no MCMC in the sanitizer build"); }
int vbfm_mcmc_get_params(vbfm_ctx *c, vbfm_mcmc_params *) { return fail(c, "no MCMC"); }
int vbfm_mcmc_init_caches(vbfm_ctx *c) { return fail(c, "no MCMC"); }
int vbfm_mcmc_iterate(vbfm_ctx *c, vbfm_mcmc_stats *) { return fail(c, "no MCMC"); }
int vbfm_mcmc_get_test_pred(vbfm_ctx *c, int32_t, double *) { return fail(c, "no MCMC"); }
int vbfm_online_init(vbfm_ctx *c, const vbfm_online_config *) { return fail(c, "no online learner"); }
int vbfm_online_epoch(vbfm_ctx *c, vbfm_online_stats *) { return fail(c, "no online learner"); }

}  // extern "C"
