// Microbenchmark (diagnostic, not product): the host side of the c4h round's
// inputs (HostInputs, rbe_host.h) at C4 size — 90k ReadIndexes and 10k 16-B
// proposals staged at the leaders of 100k of 1M groups x 3 — and the copy of
// the staged records that flush_inputs makes into the pinned upload buffer.
// Build: g++ -O2 -std=c++17 -o host_push host_push.cpp
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "../../dragonboat_amd/csrc/rbe_host.h"

using namespace rbe;

int main() {
  const u64 G = 1000000, N = 3, R = G * N;
  HostInputs h;
  h.init(R, (u32)N, 200000);
  std::mt19937_64 rng(7);
  std::vector<u64> reads, props;
  for (u64 g = 0; g < G; g += 10) ((rng() % 10) ? reads : props).push_back(g * N + rng() % N);
  std::vector<u64> lo(reads.size()), hi(reads.size());
  for (size_t i = 0; i < reads.size(); i++) lo[i] = (1ull << 32) | (reads[i] + 1), hi[i] = reads[i];
  std::vector<u32> one(props.size(), 1), zero(props.size(), 0), len(props.size(), 16);
  std::vector<u8> cmd(16 * props.size(), 7);
  std::vector<u8> pinned(64 << 20);
  double tr = 0, tp = 0, tc = 0, tx = 0;
  const int K = 50;
  for (int it = 0; it < K + 5; it++) {
    auto t0 = std::chrono::steady_clock::now();
    if (h.push_read_index(reads.size(), reads.data(), lo.data(), hi.data())) return 1;
    auto t1 = std::chrono::steady_clock::now();
    if (h.push_proposals(props.size(), props.data(), one.data(), zero.data(), len.data(), cmd.data()))
      return 2;
    auto t2 = std::chrono::steady_clock::now();
    // flush_inputs' host part: records and replicas into the pinned buffer
    memcpy(pinned.data(), h.reps.data(), h.reps.size() * sizeof(u64));
    memcpy(pinned.data() + (8 << 20), h.recs.data(), h.recs.size() * sizeof(ExtIn));
    memcpy(pinned.data() + (40 << 20), h.ents.data(), h.ents.size() * sizeof(Ent));
    auto t3 = std::chrono::steady_clock::now();
    h.clear();
    auto t4 = std::chrono::steady_clock::now();
    if (it >= 5) {
      tr += std::chrono::duration<double, std::milli>(t1 - t0).count();
      tp += std::chrono::duration<double, std::milli>(t2 - t1).count();
      tc += std::chrono::duration<double, std::milli>(t3 - t2).count();
      tx += std::chrono::duration<double, std::milli>(t4 - t3).count();
    }
  }
  printf("reads %zu props %zu: push_read_index %.3f ms, push_proposals %.3f ms, copy %.3f ms, clear %.3f ms\n",
         reads.size(), props.size(), tr / K, tp / K, tc / K, tx / K);
  return 0;
}
