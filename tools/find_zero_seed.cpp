// Host scan for seeds whose glibc stream draws a zero as Leva's u early (g++ -O2 tools/find_zero_seed.cpp)
#include "../scalable-variational-bayesian-factorization-machine_amd/csrc/vbfm_rng.h"
#include <cstdio>
// seeds whose first ~NU outputs hold a zero drawn as Leva's u (the attempt shift case)
int main() {
  const long NU = 12000000;
  int found = 0;
  for (uint32_t seed = 1; seed < 5000 && found < 3; seed++) {
    vbrng::Glibc g(seed);
    long pos = 0;
    while (pos < NU) {
      // one Leva normal, tracking positions
      for (;;) {
        int32_t a = g.next(); pos++;
        if (a == 0) { printf("seed %u zero-u at output %ld\n", seed, pos - 1); found++; continue; }
        double u = a / 2147483648.0;
        double v = 1.7156 * (g.next() / 2147483648.0 - 0.5); pos++;
        double x = u - 0.449871, y = std::fabs(v) + 0.386595, Q = x*x + y*(0.19600*y - 0.25472*x);
        if (Q < 0.27597) break;
        if (Q > 0.27846) continue;
        if ((v*v) > (-4.0*u*u*std::log(u))) continue;
        break;
      }
    }
  }
  return 0;
}
