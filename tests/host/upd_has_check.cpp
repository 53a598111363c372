// Host check: upd_has (the collect passes' Upd-only flag) equals update_view's
// RBE_UF_HAS_UPDATE over random records (tests/test_host_checks.py).
#include "rbe_host.h"
#include <cstdio>
#include <random>
using namespace rbe;
int main() {
  std::mt19937_64 rng(1);
  long bad = 0, has = 0;
  for (int it = 0; it < 2000000; it++) {
    Upd d{};
    Core c{};
    Hot h{};
    d.round = rng() % 4;
    d.flags = rng() & 0x1FF;
    d.n_msgs = rng() % 3 == 0 ? rng() % 4 : 0;
    d.n_rtr = rng() % 3 == 0 ? rng() % 3 : 0;
    d.n_drop_ent = rng() % 5 == 0;
    d.n_drop_ri = rng() % 5 == 0;
    d.save_lo = rng() % 5; d.save_hi = rng() % 5;
    d.apply_lo = rng() % 5; d.apply_hi = rng() % 5;
    const u32 round = rng() % 5;
    rbe_update u;
    update_view(d, c, h, round, u);
    const bool a = (u.flags & RBE_UF_HAS_UPDATE) != 0, b = upd_has(d, round);
    has += a;
    if (a != b) bad++;
  }
  printf("bad %ld has %ld\n", bad, has);
  return bad != 0;
}
