// vbfm_mcmc_capi.hip -- the MCMC / ALS learner of include/vbfm.h (-method mcmc | als).
//
// Replaces fm_learn_mcmc / fm_learn_mcmc_simultaneous (src/libfm/src/fm_learn_mcmc.h,
// src/libfm/src/fm_learn_mcmc_simultaneous.h) for regression without relation blocks. The
// host keeps draw_all's control flow and every scalar / per-group hyper-prior draw, in the
// reference's order on the reference's random stream (vbfm_rng.h); the sweeps over the
// attributes (draw_w, draw_v with their e / q corrections), the q-cache, the prior draws of
// attributes without train rows, the full re-prediction of train and test and all O(N) /
// O(k*D) sums run as the kernels of vbfm_mcmc.hip on the context's stream, scheduled by the
// same dependency levels as the VB sweep (exact Gauss-Seidel order).
#include "vbfm_ctx.h"
#include "vbfm_rng.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

using namespace vbi;

namespace {

// hyper-prior constants of fm_learn_mcmc::init (fm_learn_mcmc.h:1100-1103)
constexpr double ALPHA_0 = 1.0, GAMMA_0 = 1.0, BETA_0 = 1.0, MU_0 = 0.0;

enum { MEV_BEGIN, MEV_HYPER, MEV_W, MEV_V, MEV_PRED, MEV_N };
enum { HC_NAN_ALPHA, HC_INF_ALPHA, HC_NAN_W0, HC_INF_W0, HC_NAN_WMU, HC_INF_WMU, HC_NAN_WL, HC_INF_WL,
       HC_NAN_VMU, HC_INF_VMU, HC_NAN_VL, HC_INF_VL, HC_N };

constexpr uint32_t MC_RED_BLOCKS = 512;

}  // namespace

struct McState {
	int sample = 0, multilevel = 0, rng = VBFM_RNG_REFERENCE;
	uint32_t seed = 1;
	vbrng::Glibc stream;
	double w0 = 0.0, alpha = 1.0, reg0 = 0.0;
	std::vector<double> w_mu, w_lambda, v_mu, v_lambda;   // [G], [G], [G*k], [G*k] ([g][f])
	double *hyp_d = nullptr;                              // the four arrays, in that order
	double *z_d = nullptr;                                // [D] normals of one sweep (reference RNG)
	std::vector<double> z_h;
	std::vector<uint8_t> col_nonempty;                    // [train nf] over all shards
	double *pred_this = nullptr, *pred_sum = nullptr;     // [test rows]
	double *vc = nullptr;                                 // [k*D] compact v for the re-prediction
	double *pc = nullptr;                                 // [2*D] last factor's v and w (fused re-prediction)
	double *red_d = nullptr;                              // [4 * MC_RED_BLOCKS]
	std::vector<double> red_h;
	uint32_t iter = 0;
	bool caches = false;
	bool pred_acc = false;                                // v sweeps accumulate the train re-prediction
	uint32_t hc[HC_N] = {};
	hipEvent_t ev[MEV_N] = {};
};

namespace vbi {

void mc_free(vbfm_ctx *c)
{
	McState *m = c->mc;
	if (!m) return;
	dfree(m->hyp_d); dfree(m->z_d); dfree(m->pred_this); dfree(m->pred_sum); dfree(m->red_d); dfree(m->vc); dfree(m->pc);
	for (int i = 0; i < MEV_N; i++)
		if (m->ev[i]) (void)hipEventDestroy(m->ev[i]);
	delete m;
	c->mc = nullptr;
}

}  // namespace vbi

namespace {

McState &mc(vbfm_ctx *c)
{
	if (!c->mc) throw std::string("not an MCMC / ALS context (vbfm_mcmc_init)");
	return *c->mc;
}

size_t G_(vbfm_ctx *c) { return c->G; }
size_t GK(vbfm_ctx *c) { return (size_t)c->G * c->k; }
double *d_w_mu(vbfm_ctx *c) { return c->mc->hyp_d; }
double *d_w_lambda(vbfm_ctx *c) { return c->mc->hyp_d + G_(c); }
double *d_v_mu(vbfm_ctx *c) { return c->mc->hyp_d + 2 * G_(c); }
double *d_v_lambda(vbfm_ctx *c) { return c->mc->hyp_d + 2 * G_(c) + GK(c); }

void upload_hyper(vbfm_ctx *c)
{
	McState &m = *c->mc;
	const size_t G = G_(c), gk = GK(c);
	HIPCHK(hipMemcpyAsync(d_w_mu(c), m.w_mu.data(), G * 8, hipMemcpyHostToDevice, c->s));
	HIPCHK(hipMemcpyAsync(d_w_lambda(c), m.w_lambda.data(), G * 8, hipMemcpyHostToDevice, c->s));
	if (gk) {
		HIPCHK(hipMemcpyAsync(d_v_mu(c), m.v_mu.data(), gk * 8, hipMemcpyHostToDevice, c->s));
		HIPCHK(hipMemcpyAsync(d_v_lambda(c), m.v_lambda.data(), gk * 8, hipMemcpyHostToDevice, c->s));
	}
	sync(c);   // the host vectors may change right after
}

// -regular for mcmc / als (libfm.cpp:367-411)
void apply_regular(vbfm_ctx *c, const double *reg, int n)
{
	McState &m = *c->mc;
	const size_t G = c->G, k = c->k;
	if (n < 0 || (n > 0 && !reg)) throw std::string("-regular: bad value list");
	if (n == 0 || n == 1 || n == 3) {
		const double r0 = n == 0 ? 0.0 : reg[0], rw = n == 3 ? reg[1] : r0, rv = n == 3 ? reg[2] : r0;
		m.reg0 = r0;
		std::fill(m.w_lambda.begin(), m.w_lambda.end(), rw);
		std::fill(m.v_lambda.begin(), m.v_lambda.end(), rv);
		return;
	}
	if ((size_t)n != 1 + 2 * G)
		throw std::string("-regular: expected 0, 1, 3 or 1 + 2 * num_attr_groups values");
	m.reg0 = reg[0];
	for (size_t g = 0; g < G; g++) m.w_lambda[g] = reg[1 + g];
	for (size_t g = 0; g < G; g++)
		for (size_t f = 0; f < k; f++) m.v_lambda[g * k + f] = reg[1 + G + g];
}

// per-(w | factor f, group g) sums of the parameters, mode 0: sum p, 1: sum (p - mu)^2;
// segment index (f + 1) * G + g (seg_sums); only the w or only the factor segments
std::vector<double> mc_param_sums(vbfm_ctx *c, int mode, bool is_v)
{
	return seg_sums(c, 1, mode, d_w_mu(c), d_v_mu(c), !is_v, is_v);
}

double mc_row_sum(vbfm_ctx *c, int mode, double w0)
{
	rows_dense(c);
	HIPCHK(vbk::mc_row_sums(c->rows, c->tr.n, mode, w0, c->red_d, c->RED_BLOCKS, c->s));
	double s = finish_sum(c, c->RED_BLOCKS);
	allreduce_host(c, &s, 1);
	return s;
}

// ---- host-side draws, in draw_all's order (fm_learn_mcmc.h:411-623) ---------------------
void draw_alpha(vbfm_ctx *c)   // :901-929
{
	McState &m = *c->mc;
	if (!m.multilevel) { m.alpha = ALPHA_0; return; }
	const double alpha_n = ALPHA_0 + (double)c->n_global;
	const double gamma_n = GAMMA_0 + mc_row_sum(c, 0, 0.0);
	const double old = m.alpha;
	m.alpha = m.stream.gamma(alpha_n / 2.0, gamma_n / 2.0);
	if (std::isnan(m.alpha)) { m.hc[HC_NAN_ALPHA]++; m.alpha = old; }
	else if (std::isinf(m.alpha)) { m.hc[HC_INF_ALPHA]++; m.alpha = old; }
}

void draw_w0(vbfm_ctx *c)   // :628-668 (w0_mean_0 = 0)
{
	McState &m = *c->mc;
	const double sum = mc_row_sum(c, 1, m.w0);
	const double s2 = (double)1.0 / (m.reg0 + m.alpha * (double)c->n_global);
	const double mean = -s2 * (m.alpha * sum - 0.0 * m.reg0);
	const double old = m.w0;
	m.w0 = m.sample ? m.stream.gaussian(mean, std::sqrt(s2)) : mean;
	if (std::isnan(m.w0)) { m.hc[HC_NAN_W0]++; m.w0 = old; return; }
	if (std::isinf(m.w0)) { m.hc[HC_INF_W0]++; m.w0 = old; return; }
	rows_dense(c);
	HIPCHK(vbk::mc_e_shift(c->rows, c->tr.n, old - m.w0, c->s));
}

// gamma draws of the precisions (draw_w_lambda :970-1008, draw_v_lambda :1051-1089); an
// out-of-range draw restores the old value and ends the draw, as the reference's return
bool draw_lambda(McState &m, double shape, double gam, double &lam, uint32_t *nan_c, uint32_t *inf_c)
{
	const double old = lam;
	lam = m.sample ? m.stream.gamma(shape / 2.0, gam / 2.0) : shape / gam;
	if (std::isnan(lam)) { (*nan_c)++; lam = old; return false; }
	if (std::isinf(lam)) { (*inf_c)++; lam = old; return false; }
	return true;
}

bool draw_mu(McState &m, double mean, double s2, double &mu, uint32_t *nan_c, uint32_t *inf_c)
{
	const double old = mu;
	mu = m.sample ? m.stream.gaussian(mean, std::sqrt(s2)) : mean;
	if (std::isnan(mu)) { (*nan_c)++; mu = old; return false; }
	if (std::isinf(mu)) { (*inf_c)++; mu = old; return false; }
	return true;
}

void draw_w_hyper(vbfm_ctx *c)
{
	McState &m = *c->mc;
	if (!m.multilevel) {   // draw_w_lambda returns, draw_w_mu sets mu_0
		std::fill(m.w_mu.begin(), m.w_mu.end(), MU_0);
		upload_hyper(c);
		return;
	}
	const std::vector<double> sq = mc_param_sums(c, 1, false);   // sum (w - w_mu(g))^2
	for (uint32_t g = 0; g < c->G; g++) {
		const double gam = BETA_0 * (m.w_mu[g] - MU_0) * (m.w_mu[g] - MU_0) + GAMMA_0 + sq[g];
		const double shape = ALPHA_0 + c->per_group[g] + 1;
		if (!draw_lambda(m, shape, gam, m.w_lambda[g], &m.hc[HC_NAN_WL], &m.hc[HC_INF_WL])) break;
	}
	const std::vector<double> sum = mc_param_sums(c, 0, false);  // sum w
	for (uint32_t g = 0; g < c->G; g++) {
		const double mean = (sum[g] + BETA_0 * MU_0) / (c->per_group[g] + BETA_0);
		const double s2 = (double)1.0 / ((c->per_group[g] + BETA_0) * m.w_lambda[g]);
		if (!draw_mu(m, mean, s2, m.w_mu[g], &m.hc[HC_NAN_WMU], &m.hc[HC_INF_WMU])) break;
	}
	upload_hyper(c);
}

void draw_v_hyper(vbfm_ctx *c)
{
	McState &m = *c->mc;
	const int k = c->k;
	if (!m.multilevel) {
		std::fill(m.v_mu.begin(), m.v_mu.end(), MU_0);
		upload_hyper(c);
		return;
	}
	const std::vector<double> sq = mc_param_sums(c, 1, true);   // sum (v_f - v_mu(g, f))^2
	[&] {
		for (int f = 0; f < k; f++)
			for (uint32_t g = 0; g < c->G; g++) {
				const double mu = m.v_mu[(size_t)g * k + f];
				const double gam = BETA_0 * (mu - MU_0) * (mu - MU_0) + GAMMA_0 + sq[(size_t)(f + 1) * c->G + g];
				const double shape = ALPHA_0 + c->per_group[g] + 1;
				if (!draw_lambda(m, shape, gam, m.v_lambda[(size_t)g * k + f], &m.hc[HC_NAN_VL], &m.hc[HC_INF_VL]))
					return;
			}
	}();
	const std::vector<double> sum = mc_param_sums(c, 0, true);
	[&] {
		for (int f = 0; f < k; f++)
			for (uint32_t g = 0; g < c->G; g++) {
				const double mean = (sum[(size_t)(f + 1) * c->G + g] + BETA_0 * MU_0) / (c->per_group[g] + BETA_0);
				const double s2 = (double)1.0 / ((c->per_group[g] + BETA_0) * m.v_lambda[(size_t)g * k + f]);
				if (!draw_mu(m, mean, s2, m.v_mu[(size_t)g * k + f], &m.hc[HC_NAN_VMU], &m.hc[HC_INF_VMU])) return;
			}
	}();
	upload_hyper(c);
}

// the reference's normals of one attribute sweep, attribute by attribute: an attribute takes
// one iff its conditional variance is finite and nonzero, i.e. unless its prior precision is
// 0 and its column is empty in every shard (NaN marks "no draw"; the kernels count any
// attribute where the data disagree, vbfm_mcmc_stats::rng_skipped)
void fill_normals(vbfm_ctx *c, const double *lambda, size_t hstride)
{
	McState &m = *c->mc;
	if (!m.sample || m.rng != VBFM_RNG_REFERENCE) return;
	m.z_h.resize(c->D);
	for (uint32_t j = 0; j < c->D; j++) {
		const double lam = lambda[(size_t)c->group_h[j] * hstride];
		const bool nonempty = j < m.col_nonempty.size() && m.col_nonempty[j];
		const bool draws = !std::isnan(lam) && (lam != 0.0 || nonempty) && !std::isinf(lam);
		m.z_h[j] = draws ? m.stream.gaussian() : NAN;
	}
	HIPCHK(hipMemcpyAsync(m.z_d, m.z_h.data(), (size_t)c->D * 8, hipMemcpyHostToDevice, c->s));
	sync(c);
}

McArgs mc_args(vbfm_ctx *c, uint32_t l, bool is_w, int f)
{
	McState &m = *c->mc;
	McArgs a;
	memset(&a, 0, sizeof(a));
	a.col_ptr = c->tr.col_ptr;
	a.csc = c->tr.csc;
	if (l < nlevels(c)) {
		a.feats = c->level_feats + c->level_ptr[l];
		a.feat_contig = c->level_base[l] != ~0u;
		a.feat_base = c->level_base[l];
		a.nfeat = c->level_ptr[l + 1] - c->level_ptr[l];
		a.avg_len = c->level_avg[l];
	}
	a.rows = c->rows;
	a.par = is_w ? c->ms_w : c->ms_v + f;
	a.stride = is_w ? 1 : (uint32_t)c->k;
	a.next_stride = (uint32_t)c->k;
	if (is_w) a.par_next = c->k > 0 ? c->ms_v : nullptr;
	else a.par_next = f + 1 < c->k ? c->ms_v + (f + 1) : nullptr;
	a.lambda = is_w ? d_w_lambda(c) : d_v_lambda(c) + f;
	a.mu = is_w ? d_w_mu(c) : d_v_mu(c) + f;
	a.hstride = is_w ? 1 : (uint32_t)c->k;
	// one attribute group: the prior by value (the host copies are what was pushed to hyp_d)
	a.hyp_uniform = c->G == 1;
	if (c->G == 1) {
		a.lambda0 = is_w ? m.w_lambda[0] : m.v_lambda[f];
		a.mu0 = is_w ? m.w_mu[0] : m.v_mu[f];
	}
	a.attr_group = c->group_d;
	a.dup = c->dup;
	a.alpha = m.alpha;
	a.z = (m.sample && m.rng == VBFM_RNG_REFERENCE) ? m.z_d : nullptr;
	a.rng_seed = m.seed;
	a.rng_stream = (uint64_t)m.iter * (uint64_t)(c->k + 1) + (uint64_t)(is_w ? 0 : f + 1);
	a.sample = m.sample;
	a.counters = c->counters;
	a.stats = c->stats;
	a.skew = c->debug_skew;
	a.slot = is_w ? 0 : (f & 1);
	if (m.pred_acc && !is_w && f >= 1) {   // factor f-1 is final: its re-prediction terms ride along
		a.par_prev = c->ms_v + (f - 1);
		a.pk = f == 1 ? 1 : 2;
	}
	return a;
}

// The train re-prediction after draw_all fused into the v sweeps (McArgs::pk) and one final
// row pass (k_mc_pred_final) instead of a separate prediction of every entry's k factors:
// the same operations in the same order, so e is bit-identical (VBFM_MC_FUSED_PREDICT=0: the
// separate prediction)
bool fused_predict()
{
	const char *e = getenv("VBFM_MC_FUSED_PREDICT");
	return !(e && e[0] == '0');
}

void mc_sweep(vbfm_ctx *c, bool is_w, int f)
{
	rows_level_order(c);
	for (uint32_t l = 0; l < nlevels(c); l++) {
		McArgs a = mc_args(c, l, is_w, f);
		if (a.nfeat == 0) continue;
		XPhase ph(c, is_w ? "draw_w sweep" : "draw_v sweep", is_w ? -1 : f, (int)l);
		const size_t p = prof_begin(c, is_w ? 1 : 0);
		if (c->lord) {   // level-ordered store: stream the runs, move the records to level l+1
			a.lcp = c->lcp + c->level_ptr[l];
			a.lx = c->lx;
			a.lnext = c->lnext;
			a.lbase = (uint64_t)l * c->tr.n;
			a.src = c->rows;
			a.dst = c->rows_alt;
			a.first_level = l == 0;
			if (c->estore) {   // one store, global slots: each record to its row's next slot
				a.lbase = 0;
				a.dst = c->rows;
				a.ent = 1;
				if (!c->row_comm() && !c->force_split) {
					HIPCHK(vbk::mc_lord_level(a, 0, is_w, c->s));
				} else {   // row shards: the two-pass split (statistics, all-reduce, draw + move)
					stats_exchange(c, a, [&](const McArgs &b) { HIPCHK(vbk::mc_lord_level(b, 1, is_w, c->s)); });
					HIPCHK(vbk::mc_lord_level(a, 2, is_w, c->s));
				}
				prof_end(c, p);
				continue;
			}
			if (!c->row_comm() && !c->force_split) {
				HIPCHK(vbk::mc_lord_level(a, 0, is_w, c->s));
			} else if (c->deferred()) {
				// deferred: level l-1's correction, level l's statistics and the move in one pass;
				// the draws after the all-reduce, applied by level l+1 (or the flush)
				a.lpay = c->lpay;
				a.lpay2 = c->lpay2;
				a.tab = c->post_tab;
				a.pending = (l > 0 ? 3 : 0) | (defer_nt_stores() ? 4 : 0);
				stats_exchange(c, a, [&](const McArgs &b) { HIPCHK(vbk::mc_lord_defer_level(b, is_w, c->s)); });
				HIPCHK(vbk::mc_lord_defer_post(a, is_w, c->s));
				if (l + 1 == nlevels(c)) {   // the sweep's last correction, on level-0-ordered records
					a.dst = c->rows_alt;      // (swapped below)
					HIPCHK(vbk::mc_lord_defer_flush(a, is_w, c->tr.n, c->s));
				}
			} else {
				stats_exchange(c, a, [&](const McArgs &b) { HIPCHK(vbk::mc_lord_level(b, 1, is_w, c->s)); });
				HIPCHK(vbk::mc_lord_level(a, 2, is_w, c->s));
			}
			std::swap(c->rows, c->rows_alt);
			prof_end(c, p);
			continue;
		}
		if (!c->row_comm() && !c->force_split) {
			HIPCHK(is_w ? vbk::mc_w_level(a, 0, c->s) : vbk::mc_v_level(a, 0, c->s));
		} else {   // row-sharded: statistics of this shard, summed over shards, identical draws
			stats_exchange(c, a, [&](const McArgs &b) {
				HIPCHK(is_w ? vbk::mc_w_level(b, 1, c->s) : vbk::mc_v_level(b, 1, c->s));
			});
			HIPCHK(is_w ? vbk::mc_w_level(a, 2, c->s) : vbk::mc_v_level(a, 2, c->s));
		}
		prof_end(c, p);
	}
	// attributes beyond the train data: drawn from their prior (:449-457 / :569-577)
	McArgs a = mc_args(c, nlevels(c), is_w, f);
	HIPCHK(vbk::mc_prior(a, c->tr.nf, c->D, is_w ? 0 : 1, c->s));
}

void mc_step_w(vbfm_ctx *c)
{
	draw_w_hyper(c);
	fill_normals(c, c->mc->w_lambda.data(), 1);
	mc_sweep(c, true, 0);
	if (c->k > 0) c->q_ready[0] = 0;
}

// q-cache of factor f, then the draw_v sweep (which leaves the q-cache of f+1)
void mc_step_v(vbfm_ctx *c, int f)
{
	const int slot = f & 1;
	if (c->q_ready[slot] != f) {
		const size_t p = prof_begin(c, 2);
		rows_level_order(c);
		HIPCHK(vbk::mc_qcache(c->tr.row_ptr, c->tr.csr, c->ms_v + f, (uint32_t)c->k, c->rows, c->tr.n, slot,
		                      c->rows_lorder ? c->lpos0 : nullptr, c->s));
		prof_end(c, p);
	}
	fill_normals(c, c->mc->v_lambda.data() + f, (size_t)c->k);
	mc_sweep(c, false, f);
	c->q_ready[slot] = -1;
	c->q_ready[(f + 1) & 1] = f + 1 < c->k ? f + 1 : -1;
}

// full prediction of train (into scratch; unless train = false) and test (fm_learn_mcmc.h:117-348)
void mc_predict(vbfm_ctx *c, bool train = true)
{
	McState &m = *c->mc;
	// the parameters are {v, 0} pairs: the wave-form prediction reads a compact copy of v
	// (half the bytes of every entry's k factors), refreshed once per re-prediction
	const size_t kd = (size_t)c->k * c->D;
	const int btr = blocked_predict(c, c->tr), bte = c->e_test ? blocked_predict(c, c->te) : 0;
	if ((btr == 2 || bte == 2) && c->k <= 256 && kd && !m.vc) m.vc = dalloc<double>(kd);
	bool fresh = false;
	if (train) {
		HIPCHK(vbk::predict_e_compact(c->tr.row_ptr, c->tr.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, m.w0,
		                              c->scratch_n, c->tr.n, btr, m.vc, kd, !fresh, c->s));
		fresh = fresh || (btr == 2 && m.vc);
	}
	if (c->e_test)
		HIPCHK(vbk::predict_e_compact(c->te.row_ptr, c->te.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, m.w0, c->e_test,
		                              c->te.n, bte, m.vc, kd, !fresh, c->s));
}

void require_test(vbfm_ctx *c)
{
	if (!c->e_test) throw std::string("no test data set (vbfm_set_test)");
	McState &m = *c->mc;
	dfree(m.pred_this);
	dfree(m.pred_sum);
	m.pred_this = dalloc<double>(c->te.n);
	m.pred_sum = dalloc<double>(c->te.n);
	HIPCHK(hipMemsetAsync(m.pred_sum, 0, (size_t)std::max(c->te.n, 1u) * 8, c->s));
	HIPCHK(hipMemsetAsync(m.pred_this, 0, (size_t)std::max(c->te.n, 1u) * 8, c->s));
}

// which train columns hold an entry in some shard (decides the reference's draw count)
void scan_columns(vbfm_ctx *c)
{
	McState &m = *c->mc;
	const uint32_t nf = c->tr.nf;
	std::vector<uint64_t> cp((size_t)nf + 1, 0);
	HIPCHK(hipMemcpy(cp.data(), c->tr.col_ptr, ((size_t)nf + 1) * 8, hipMemcpyDeviceToHost));
	m.col_nonempty.assign(nf, 0);
	for (uint32_t j = 0; j < nf; j++) m.col_nonempty[j] = cp[j + 1] > cp[j];
	if (c->multi() && nf) {
		uint8_t *d = dalloc<uint8_t>(nf);
		HIPCHK(hipMemcpyAsync(d, m.col_nonempty.data(), nf, hipMemcpyHostToDevice, c->s));
		allreduce_dev(c, d, nf, ncclUint8, ncclMax);
		HIPCHK(d2h(c, m.col_nonempty.data(), d, nf));
		sync(c);
		dfree(d);
	}
}

}  // namespace

// =========================================================================================
extern "C" {

int vbfm_mcmc_init(vbfm_ctx *c, const vbfm_mcmc_config *cfg)
{
	if (!c || !cfg) return fail(c, "vbfm_mcmc_init: null argument");
	return guarded(c, [&] {
		if (cfg->rng != VBFM_RNG_REFERENCE && cfg->rng != VBFM_RNG_DEVICE) throw std::string("unknown rng mode");
		if (c->shard_mode == VBFM_SHARD_FEATURES)
			throw std::string("feature shards are implemented for the VB learner only");
		mc_free(c);
		c->mc = new McState();
		McState &m = *c->mc;
		for (int i = 0; i < MEV_N; i++) HIPCHK(hipEventCreate(&m.ev[i]));
		m.sample = cfg->do_sample != 0;
		m.multilevel = cfg->do_multilevel != 0;
		m.rng = cfg->rng;
		m.seed = cfg->seed;
		m.w_mu.assign(c->G, 0.0);              // fm_learn_mcmc::init (:1105-1113)
		m.w_lambda.assign(c->G, 0.0);
		m.v_mu.assign(GK(c), 0.0);
		m.v_lambda.assign(GK(c), 0.0);
		m.alpha = 1.0;
		m.w0 = 0.0;
		apply_regular(c, cfg->regular, cfg->num_regular);
		m.hyp_d = dalloc<double>(2 * G_(c) + 2 * GK(c));
		m.z_d = dalloc<double>(c->D);
		m.red_d = dalloc<double>(4 * MC_RED_BLOCKS);
		m.red_h.assign(4 * MC_RED_BLOCKS, 0.0);
		upload_hyper(c);
		// srand(seed); fm.v ~ N(0, init_stdev) (fm_model.h:97), then fm.w (libfm.cpp:298)
		m.stream.seed_with(cfg->seed);
		const size_t kd = (size_t)c->k * c->D;
		if (m.rng == VBFM_RNG_REFERENCE) {
			std::vector<double> v(kd), w(c->D), zero(std::max(kd, (size_t)c->D), 0.0);
			for (double &x : v) x = m.stream.gaussian(0.0, cfg->init_stdev);
			for (double &x : w) x = m.stream.gaussian(0.0, cfg->init_stdev);
			double *tmp = dalloc<double>(2 * std::max(kd, (size_t)c->D));
			const size_t half = std::max(kd, (size_t)c->D);
			HIPCHK(hipMemcpyAsync(tmp + half, zero.data(), half * 8, hipMemcpyHostToDevice, c->s));
			if (kd) {
				HIPCHK(hipMemcpyAsync(tmp, v.data(), kd * 8, hipMemcpyHostToDevice, c->s));
				HIPCHK(vbk::pack_pairs(tmp, tmp + half, c->ms_v, (uint32_t)c->k, c->D, c->s));
			}
			if (c->D) {
				sync(c);
				HIPCHK(hipMemcpyAsync(tmp, w.data(), (size_t)c->D * 8, hipMemcpyHostToDevice, c->s));
				HIPCHK(vbk::pack_pairs(tmp, tmp + half, c->ms_w, 1, c->D, c->s));
			}
			sync(c);
			dfree(tmp);
		} else {
			HIPCHK(vbk::init_normal_pairs(c->ms_v, kd, cfg->seed, 21, cfg->init_stdev, 0.0, c->s));
			HIPCHK(vbk::init_normal_pairs(c->ms_w, c->D, cfg->seed, 22, cfg->init_stdev, 0.0, c->s));
			sync(c);
		}
		c->q_ready[0] = c->q_ready[1] = -1;
	});
}

int vbfm_mcmc_set_params(vbfm_ctx *c, const vbfm_mcmc_params *p)
{
	if (!c || !p) return fail(c, "null argument");
	return guarded(c, [&] {
		McState &m = mc(c);
		const size_t kd = (size_t)c->k * c->D, half = std::max(kd, (size_t)c->D);
		if (!p->w || (kd && !p->v)) throw std::string("vbfm_mcmc_set_params: parameter arrays missing");
		double *tmp = dalloc<double>(2 * half);
		HIPCHK(hipMemsetAsync(tmp + half, 0, half * 8, c->s));
		HIPCHK(hipMemcpyAsync(tmp, p->w, (size_t)c->D * 8, hipMemcpyHostToDevice, c->s));
		HIPCHK(vbk::pack_pairs(tmp, tmp + half, c->ms_w, 1, c->D, c->s));
		sync(c);
		if (kd) {
			HIPCHK(hipMemcpyAsync(tmp, p->v, kd * 8, hipMemcpyHostToDevice, c->s));
			HIPCHK(vbk::pack_pairs(tmp, tmp + half, c->ms_v, (uint32_t)c->k, c->D, c->s));
			sync(c);
		}
		dfree(tmp);
		if (p->w_mu) std::copy(p->w_mu, p->w_mu + G_(c), m.w_mu.begin());
		if (p->w_lambda) std::copy(p->w_lambda, p->w_lambda + G_(c), m.w_lambda.begin());
		if (p->v_mu) std::copy(p->v_mu, p->v_mu + GK(c), m.v_mu.begin());
		if (p->v_lambda) std::copy(p->v_lambda, p->v_lambda + GK(c), m.v_lambda.begin());
		m.w0 = p->w0;
		m.alpha = p->alpha;
		m.reg0 = p->reg0;
		upload_hyper(c);
		c->q_ready[0] = c->q_ready[1] = -1;
	});
}

int vbfm_mcmc_get_params(vbfm_ctx *c, vbfm_mcmc_params *p)
{
	if (!c || !p) return fail(c, "null argument");
	return guarded(c, [&] {
		McState &m = mc(c);
		const size_t kd = (size_t)c->k * c->D, half = std::max(kd, (size_t)c->D);
		double *tmp = dalloc<double>(2 * half);
		HIPCHK(vbk::unpack_pairs(c->ms_w, tmp, tmp + half, 1, c->D, c->s));
		if (p->w) HIPCHK(d2h(c, p->w, tmp, (size_t)c->D * 8));
		sync(c);
		if (kd && p->v) {
			HIPCHK(vbk::unpack_pairs(c->ms_v, tmp, tmp + half, (uint32_t)c->k, c->D, c->s));
			HIPCHK(d2h(c, p->v, tmp, kd * 8));
			sync(c);
		}
		dfree(tmp);
		if (p->w_mu) std::copy(m.w_mu.begin(), m.w_mu.end(), p->w_mu);
		if (p->w_lambda) std::copy(m.w_lambda.begin(), m.w_lambda.end(), p->w_lambda);
		if (p->v_mu) std::copy(m.v_mu.begin(), m.v_mu.end(), p->v_mu);
		if (p->v_lambda) std::copy(m.v_lambda.begin(), m.v_lambda.end(), p->v_lambda);
		p->w0 = m.w0;
		p->alpha = m.alpha;
		p->reg0 = m.reg0;
	});
}

int vbfm_mcmc_init_caches(vbfm_ctx *c)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		McState &m = mc(c);
		require_train(c);
		require_test(c);
		scan_columns(c);
		// fm_learn_mcmc_simultaneous.h:71-80: predict train and test, e = yhat - y
		mc_predict(c);
		HIPCHK(vbk::mc_train_update(c->rows, c->scratch_n, c->tr.target, c->tr.n, c->min_target, c->max_target,
		                            m.red_d, MC_RED_BLOCKS, c->rows_lorder ? c->lpos0 : nullptr, c->s));
		sync(c);
		m.iter = 0;
		m.caches = true;
		c->q_ready[0] = c->q_ready[1] = -1;
	});
}

int vbfm_mcmc_iterate(vbfm_ctx *c, vbfm_mcmc_stats *o)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		McState &m = mc(c);
		require_train(c);
		if (!m.caches) throw std::string("vbfm_mcmc_init_caches first");
		vbfm_mcmc_stats st;
		memset(&st, 0, sizeof(st));
		memset(m.hc, 0, sizeof(m.hc));
		HIPCHK(hipMemsetAsync(c->counters, 0, CNT_N * 4, c->s));
		c->pev_used = 0;
		c->spans.clear();
		xs_reset(c);
		c->q_ready[0] = c->q_ready[1] = -1;
		HIPCHK(hipEventRecord(m.ev[MEV_BEGIN], c->s));
		// draw_all (fm_learn_mcmc.h:411-623)
		draw_alpha(c);
		if (c->k0) draw_w0(c);
		HIPCHK(hipEventRecord(m.ev[MEV_HYPER], c->s));
		if (c->k1) mc_step_w(c);
		HIPCHK(hipEventRecord(m.ev[MEV_W], c->s));
		const bool fused = fused_predict();
		if (c->k > 0) {
			draw_v_hyper(c);
			struct Acc {
				McState &m;
				Acc(McState &m_, bool on) : m(m_) { m.pred_acc = on; }
				~Acc() { m.pred_acc = false; }
			} acc(m, fused);
			for (int f = 0; f < c->k; f++) mc_step_v(c, f);
		}
		HIPCHK(hipEventRecord(m.ev[MEV_V], c->s));
		// re-predict and evaluate (fm_learn_mcmc_simultaneous.h:134-175, 238-245)
		mc_predict(c, !fused);
		const double mn = c->min_target, mx = c->max_target;
		HIPCHK(vbk::mc_test_update(c->e_test, c->te.target, c->te.n, mn, mx, 1.0 / (m.iter + 1), m.pred_this,
		                           m.pred_sum, m.red_d, MC_RED_BLOCKS, c->s));
		HIPCHK(d2h(c, m.red_h.data(), m.red_d, 4 * MC_RED_BLOCKS * 8));
		sync(c);
		double tm[5] = {0, 0, 0, 0, 0};
		for (uint32_t b = 0; b < MC_RED_BLOCKS; b++)
			for (int q = 0; q < 4; q++) tm[q] += m.red_h[4 * b + q];
		if (fused) {   // yhat of train from the sweeps' accumulators + the last factor and w
			if (!m.pc) m.pc = dalloc<double>(2 * (size_t)c->D);
			HIPCHK(vbk::mc_pred_final(c->tr.row_ptr, c->tr.csr, c->ms_v, c->ms_w, c->k, c->k1, c->k0, m.w0, c->k >= 2,
			                          c->rows, c->rows_lorder ? c->lpos0 : nullptr, c->tr.n, c->D, m.pc, c->scratch_n,
			                          c->s));
		}
		HIPCHK(vbk::mc_train_update(c->rows, c->scratch_n, c->tr.target, c->tr.n, mn, mx, c->red_d, c->RED_BLOCKS,
		                            c->rows_lorder ? c->lpos0 : nullptr, c->s));
		tm[4] = finish_sum(c, c->RED_BLOCKS);
		allreduce_host(c, tm, 5);
		HIPCHK(hipEventRecord(m.ev[MEV_PRED], c->s));
		sync(c);
		m.iter++;
		const double nt = (double)c->test_n_global;
		st.rmse_this = std::sqrt(tm[0] / nt);
		st.mae_this = tm[1] / nt;
		st.rmse_all = std::sqrt(tm[2] / nt);
		st.mae_all = tm[3] / nt;
		st.train_rmse = std::sqrt(tm[4] / (double)c->n_global);
		st.alpha = m.alpha;
		st.w0 = m.w0;
		uint32_t h[CNT_N];
		HIPCHK(hipMemcpy(h, c->counters, sizeof(h), hipMemcpyDeviceToHost));
		st.nan_w = h[CNT_NAN_MU_W]; st.inf_w = h[CNT_INF_MU_W];
		st.nan_v = h[CNT_NAN_MU_V]; st.inf_v = h[CNT_INF_MU_V];
		st.rng_skipped = h[CNT_RNG_SKIP];
		st.nan_alpha = m.hc[HC_NAN_ALPHA]; st.inf_alpha = m.hc[HC_INF_ALPHA];
		st.nan_w0 = m.hc[HC_NAN_W0]; st.inf_w0 = m.hc[HC_INF_W0];
		st.nan_w_mu = m.hc[HC_NAN_WMU]; st.inf_w_mu = m.hc[HC_INF_WMU];
		st.nan_w_lambda = m.hc[HC_NAN_WL]; st.inf_w_lambda = m.hc[HC_INF_WL];
		st.nan_v_mu = m.hc[HC_NAN_VMU]; st.inf_v_mu = m.hc[HC_INF_VMU];
		st.nan_v_lambda = m.hc[HC_NAN_VL]; st.inf_v_lambda = m.hc[HC_INF_VL];
		st.num_levels = (int32_t)nlevels(c);
		auto ms = [&](int a, int b) {
			float t = 0.f;
			HIPCHK(hipEventElapsedTime(&t, m.ev[a], m.ev[b]));
			return (double)t;
		};
		st.ms_hyper = ms(MEV_BEGIN, MEV_HYPER);
		st.ms_w = ms(MEV_HYPER, MEV_W);
		st.ms_v = ms(MEV_W, MEV_V);
		st.ms_predict = ms(MEV_V, MEV_PRED);
		st.ms_total = ms(MEV_BEGIN, MEV_PRED);
		for (const auto &sp : c->spans) {
			if (sp.kind != 0 && sp.kind != 3) continue;
			float t = 0.f;
			HIPCHK(hipEventElapsedTime(&t, c->pev[sp.a], c->pev[sp.a + 1]));
			if (sp.kind == 3) {
				xs_span(c, t);
				continue;
			}
			st.ms_vlevel_kernels += t;
			st.n_vlevel_launches++;
		}
		st.nnz_train = c->tr.nnz;
		if (o) *o = st;
	});
}

int vbfm_mcmc_get_test_pred(vbfm_ctx *c, int32_t num_iter, double *pred)
{
	if (!c || !pred) return fail(c, "null argument");
	return guarded(c, [&] {
		McState &m = mc(c);
		if (!m.pred_sum) throw std::string("no predictions yet");
		const uint32_t n = c->te.n;
		std::vector<double> h(n);
		if (n) HIPCHK(hipMemcpy(h.data(), m.sample ? m.pred_sum : m.pred_this, (size_t)n * 8, hipMemcpyDeviceToHost));
		const double mn = c->min_target, mx = c->max_target;
		for (uint32_t i = 0; i < n; i++) {
			double p = m.sample ? h[i] / num_iter : h[i];
			p = std::min(mx, p);
			p = std::max(mn, p);
			pred[i] = p;
		}
	});
}

int vbfm_mcmc_factor_sweep(vbfm_ctx *c, double *ms_device)
{
	if (!c) return fail(nullptr, "null context");
	return guarded(c, [&] {
		McState &m = mc(c);
		require_train(c);
		if (m.col_nonempty.empty()) scan_columns(c);
		c->q_ready[0] = c->q_ready[1] = -1;
		HIPCHK(hipEventRecord(m.ev[MEV_W], c->s));
		for (int f = 0; f < c->k; f++) mc_step_v(c, f);
		HIPCHK(hipEventRecord(m.ev[MEV_V], c->s));
		sync(c);
		float t = 0.f;
		HIPCHK(hipEventElapsedTime(&t, m.ev[MEV_W], m.ev[MEV_V]));
		if (ms_device) *ms_device = t;
	});
}

}  // extern "C"

// ---- checkpoint / resume of the MCMC / ALS learner (vbfm_save_state / vbfm_load_state) ------
// The reference keeps no state on disk (num_complete_iter = 0, fm_learn_mcmc_simultaneous.h:
// 50-83). Between two vbfm_mcmc_iterate calls the chain's state is: the RNG (mode, seed, the
// completed iterations, which key the device streams, and the reference stream's 31-word
// window), the parameters as stored ({value, 0} pairs), the hyper-priors, w0, alpha, reg0, the
// test predictions of the last iteration and their running sum (pred_this / pred_sum: "Test="
// is the mean over all iterations, :152-175) and the train row records (e = yhat - y of the
// last re-prediction; the q-caches are rebuilt inside the next sweep). The RNG block comes
// first so that a file of another method or RNG mode is refused before any state is replaced.
namespace vbi {

namespace {
constexpr size_t MC_RNG_WORDS = 8 + 32;   // {sample, multilevel, rng, seed, iter, 0, 0, 0}, window + pad
}

uint64_t mc_state_payload(vbfm_ctx *c)
{
	const uint64_t D = c->D, kd = (uint64_t)c->k * c->D, G = c->G, gk = G * (uint64_t)c->k;
	return MC_RNG_WORDS * 4 + D * 16 + kd * 16 + (2 * G + 2 * gk) * 8 + 3 * 8 + 2 * (uint64_t)c->te.n * 8 +
	       (uint64_t)c->tr.n * sizeof(RowRec);
}

void mc_state_write(vbfm_ctx *c, CkptFile &f)
{
	McState &m = mc(c);
	if (!m.caches || !m.pred_sum) throw std::string("vbfm_save_state: vbfm_mcmc_init_caches first");
	uint32_t w[MC_RNG_WORDS] = {};
	w[0] = (uint32_t)m.sample; w[1] = (uint32_t)m.multilevel; w[2] = (uint32_t)m.rng; w[3] = m.seed; w[4] = m.iter;
	m.stream.chrono_state(w + 8);
	f.write(w, sizeof(w));
	dev_to_file(c, f, c->ms_w, (size_t)c->D * sizeof(double2));
	dev_to_file(c, f, c->ms_v, (size_t)c->k * c->D * sizeof(double2));
	f.write(m.w_mu.data(), G_(c) * 8);
	f.write(m.w_lambda.data(), G_(c) * 8);
	f.write(m.v_mu.data(), GK(c) * 8);
	f.write(m.v_lambda.data(), GK(c) * 8);
	const double sc[3] = {m.w0, m.alpha, m.reg0};
	f.write(sc, sizeof(sc));
	dev_to_file(c, f, m.pred_this, (size_t)c->te.n * 8);
	dev_to_file(c, f, m.pred_sum, (size_t)c->te.n * 8);
	dev_to_file(c, f, c->rows, (size_t)c->tr.n * sizeof(RowRec));
}

void mc_state_read(vbfm_ctx *c, CkptFile &f)
{
	McState &m = mc(c);
	uint32_t w[MC_RNG_WORDS];
	f.read(w, sizeof(w));
	if (w[0] != (uint32_t)m.sample || w[1] != (uint32_t)m.multilevel)
		throw std::string("checkpoint of another method (mcmc vs als): resume with the same -method");
	if (w[2] != (uint32_t)m.rng) throw std::string("checkpoint of another RNG mode (VBFM_RNG_REFERENCE / _DEVICE)");
	if (c->te.n && !c->e_test) throw std::string("no test data set (vbfm_set_test)");
	if (!m.pred_sum) require_test(c);
	if (m.col_nonempty.empty()) scan_columns(c);
	m.seed = w[3];
	m.iter = w[4];
	m.stream.set_chrono_state(w + 8);
	file_to_dev(c, f, c->ms_w, (size_t)c->D * sizeof(double2));
	file_to_dev(c, f, c->ms_v, (size_t)c->k * c->D * sizeof(double2));
	f.read(m.w_mu.data(), G_(c) * 8);
	f.read(m.w_lambda.data(), G_(c) * 8);
	f.read(m.v_mu.data(), GK(c) * 8);
	f.read(m.v_lambda.data(), GK(c) * 8);
	upload_hyper(c);
	double sc[3];
	f.read(sc, sizeof(sc));
	m.w0 = sc[0]; m.alpha = sc[1]; m.reg0 = sc[2];
	file_to_dev(c, f, m.pred_this, (size_t)c->te.n * 8);
	file_to_dev(c, f, m.pred_sum, (size_t)c->te.n * 8);
	file_to_dev(c, f, c->rows, (size_t)c->tr.n * sizeof(RowRec));
	m.caches = true;
}

}  // namespace vbi
