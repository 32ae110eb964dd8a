// vbfm_rng.h -- the reference's random stream, restated for the host side of libvbfm.
//
// The reference draws every random number through glibc rand() after srand(seed)
// (src/util/random.h:174-176, src/libfm/libfm.cpp:123-124): uniforms rand()/(RAND_MAX+1),
// Leva's normal generator (random.h:150-164) and Marsaglia-Tsang gamma variates
// (random.h:118-148). glibc's rand() is the TYPE_3 additive feedback generator (degree 31,
// separation 3) seeded by the Park-Miller LCG and warmed up by 310 discarded outputs; it is
// restated here with a private state so a run's stream cannot be disturbed by other users
// of the process-global rand() (tests/test_capi_cpu.py checks it against libc's rand()).
#pragma once
#include <cmath>
#include <cstdint>

namespace vbrng {

class Glibc {
public:
	explicit Glibc(uint32_t seed = 1) { seed_with(seed); }
	void seed_with(uint32_t seed)
	{
		if (seed == 0) seed = 1;
		int32_t word = (int32_t)seed;
		r_[0] = word;
		for (int i = 1; i < 31; i++) {
			const long hi = word / 127773, lo = word % 127773;
			word = (int32_t)(16807 * lo - 2836 * hi);
			if (word < 0) word += 2147483647;
			r_[i] = word;
		}
		f_ = 3;
		b_ = 0;
		for (int i = 0; i < 310; i++) (void)next();
	}
	int32_t next()
	{
		const uint32_t v = (uint32_t)r_[f_] + (uint32_t)r_[b_];
		r_[f_] = (int32_t)v;
		f_ = f_ == 30 ? 0 : f_ + 1;
		b_ = b_ == 30 ? 0 : b_ + 1;
		return (int32_t)(v >> 1);
	}
	double uniform() { return next() / ((double)2147483647 + 1); }   // random.h:174-176
	// Leva (1992) ratio-of-uniforms normal with quadratic bounds (random.h:150-164)
	double gaussian()
	{
		double u, v, x, y, Q;
		for (;;) {
			do { u = uniform(); } while (u == 0.0);
			v = 1.7156 * (uniform() - 0.5);
			x = u - 0.449871;
			y = std::fabs(v) + 0.386595;
			Q = x * x + y * (0.19600 * y - 0.25472 * x);
			if (Q < 0.27597) return v / u;
			if (Q > 0.27846) continue;
			if ((v * v) > (-4.0 * u * u * std::log(u))) continue;
			return v / u;
		}
	}
	double gaussian(double mean, double stdev)   // random.h:166-172
	{
		if (stdev == 0.0 || std::isnan(stdev)) return mean;
		return mean + stdev * gaussian();
	}
	// standard gamma variate of shape a (random.h:118-148): Marsaglia & Tsang (2000) for
	// a >= 1, the U^(1/a) boost for a < 1
	double gamma(double a)
	{
		if (a < 1.0) {
			double u;
			do { u = uniform(); } while (u == 0.0);
			return gamma(a + 1.0) * std::pow(u, 1.0 / a);
		}
		const double d = a - 1.0 / 3.0, c = 1.0 / std::sqrt(9.0 * d);
		double x, v, u;
		for (;;) {
			do {
				x = gaussian();
				v = 1.0 + c * x;
			} while (v <= 0.0);
			v = v * v * v;
			u = uniform();
			if (!((u >= (1.0 - 0.0331 * (x * x) * (x * x))) &&
			      (std::log(u) >= (0.5 * x * x + d * (1.0 - v + std::log(v))))))
				return d * v;
		}
	}
	double gamma(double a, double b) { return gamma(a) / b; }   // random.h:150-152 form
	// the generator as the recurrence y_n = y_{n-31} + y_{n-3} (mod 2^32), output y_n >> 1:
	// st[i] = y_{n-31+i}, the 31 sums preceding the next output
	void chrono_state(uint32_t st[31]) const
	{
		for (int i = 0; i < 31; i++) st[i] = (uint32_t)r_[(f_ + i) % 31];
	}
	// the inverse: continue from the window st (the front pointer on st[0], the rear 3 ahead of
	// it wrapped: r[f] + r[b] = y_{n-31} + y_{n-3})
	void set_chrono_state(const uint32_t st[31])
	{
		for (int i = 0; i < 31; i++) r_[i] = (int32_t)st[i];
		f_ = 0;
		b_ = 28;
	}

private:
	int32_t r_[31];
	int f_ = 3, b_ = 0;
};

// the state right after srand(seed) and glibc's 310 discarded outputs (vbfm_replay.hip)
inline void glibc_warm_state(uint32_t seed, uint32_t st[31])
{
	Glibc g(seed);
	g.chrono_state(st);
}

}  // namespace vbrng
