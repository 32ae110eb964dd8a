// vbfm_mc_math.h -- device arithmetic of the MCMC / ALS draws shared by the column-gather
// kernels (vbfm_mcmc.hip) and the level-ordered store (vbfm_lorder.hip): the counter-based
// normals of device-RNG mode and the conditional draw of one parameter (fm_learn_mcmc.h).
#pragma once
#include "vbfm_device.h"

#ifndef DEVI
#define DEVI __device__ __forceinline__
#endif

namespace {

DEVI bool bad(double v) { return __builtin_isnan(v) || __builtin_isinf(v); }

DEVI uint64_t splitmix64(uint64_t z)
{
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

// counter-based standard normal (Box-Muller on two 53-bit uniforms)
DEVI double device_normal(uint64_t seed, uint64_t stream, uint64_t j)
{
	const uint64_t base = seed * 0x9E3779B97F4A7C15ull + stream * 0xD1B54A32D192ED03ull + 2 * j;
	const double u1 = ((double)(splitmix64(base) >> 11) + 1.0) * 0x1p-53;
	const double u2 = (double)(splitmix64(base + 1) >> 11) * 0x1p-53;
	return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

// the feature's prior (group of attribute j); by value when there is one group
DEVI uint32_t mc_group(const McArgs &a, uint32_t j) { return a.hyp_uniform ? 0u : a.attr_group[j]; }
DEVI double mc_lambda(const McArgs &a, uint32_t g) { return a.hyp_uniform ? a.lambda0 : a.lambda[(size_t)g * a.hstride]; }
DEVI double mc_mu(const McArgs &a, uint32_t g) { return a.hyp_uniform ? a.mu0 : a.mu[(size_t)g * a.hstride]; }

DEVI double mc_z(const McArgs &a, uint32_t j)
{
	if (!a.sample) return 0.0;
	if (a.z) return a.z[j];
	return device_normal(a.rng_seed, a.rng_stream, j);
}

// draw of one parameter from its conditional (fm_learn_mcmc.h:680-709 for w, :793-824 for
// v, identical in form): returns false when the reference restores the old value and
// skips the correction
DEVI bool mc_draw(double mean_sum, double ss, double cur, double lambda, double mu, double alpha, double z,
                  bool zref, bool sample, bool is_v, double &out, uint32_t *counters, bool leader)
{
	double m = mean_sum;
	if (is_v) m -= cur * ss;                                   // :793 (draw_v only)
	const double s2 = (double)1.0 / (lambda + alpha * ss);     // :680 / :794
	m = -s2 * (alpha * m - mu * lambda);                       // :681 / :795
	bool skipped = sample;
	if (bad(s2)) out = 0.0;                                    // :686-687
	else if (sample) {
		const double sd = sqrt(s2);
		skipped = sd == 0.0 || __builtin_isnan(sd);
		out = skipped ? m : m + sd * z;                        // ran_gaussian(m, sd)
	} else out = m;
	// reference RNG: the host took a normal for this attribute unless z is NaN; count the
	// attributes where the data disagree (the stream then parts from the reference's)
	const bool off = zref ? (skipped != (bool)__builtin_isnan(z)) : skipped;
	if (off && leader) atomicAdd(&counters[CNT_RNG_SKIP], 1u);
	if (bad(out)) {
		if (leader)
			atomicAdd(&counters[__builtin_isnan(out) ? (is_v ? CNT_NAN_MU_V : CNT_NAN_MU_W)
			                                         : (is_v ? CNT_INF_MU_V : CNT_INF_MU_W)], 1u);
		out = cur;
		return false;
	}
	return true;
}

// One entry's terms of the train re-prediction (predict_data_and_write_to_eterms,
// fm_learn_mcmc.h:117-348) for the factor f-1 whose values are final while factor f is swept,
// with the reference's operations in the row's ascending feature order: s1 = that factor's
// q (step 1: q = 0.0, q += v*x), ev = the e accumulator (e = 0.0, e += 0.5*q*q per factor),
// q2 = the q accumulator of step 2 (q = 0.0, q -= 0.5*v*v*x*x over every factor and entry).
// At a row's first entry of a sweep the previous factor's complete s1 is folded into ev
// (pk 2), or the accumulators start (pk 1, the sweep of factor 1).
DEVI void mc_pred_acc(double &s1, double &ev, double &q2, float x, bool first, double vp, int pk)
{
	const double xd = x;
	const double a = vp * xd;
	const double b = 0.5 * vp * vp * xd * xd;
	if (first) {
		if (pk == 1) {
			ev = 0.0;
			q2 = 0.0 - b;
		} else {
			ev = ev + 0.5 * s1 * s1;
			q2 = q2 - b;
		}
		s1 = 0.0 + a;
	} else {
		s1 = s1 + a;
		q2 = q2 - b;
	}
}

}  // namespace
