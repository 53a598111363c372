// Microbenchmark (diagnostic, not product): the memory shape of a C4 round of
// the fast steps (100k active groups of 1M x 3: each leader takes a ReadIndex,
// answers two HeartbeatResps, sends two Heartbeats; each follower answers one
// Heartbeat), under different work orders and plane layouts:
//   A  role lists (leaders, then followers), one lane per replica: today's shape
//   B  group order: the N replicas of a group in adjacent lanes (21 groups per
//      wave), each lane its own role's code (divergent branches)
//   C  B + messages in a per-round mailbox laid out [slot][group][dest][sender]
//   F  C + Hot/Core/Upd/count row stored chunk-major ([chunk][replica] planes of
//      16 B), so the adjacent lanes of a group write adjacent 16 B
//   D  one lane per group, its N replicas' steps in sequence
// each for the C4 workload's random 10% of the groups and for the first 100k
// groups (an awake set compacted into adjacent rows: the bound of a dense slab)
// Build: make -C scripts/microbench group_shape
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

typedef unsigned long long u64;
struct alignas(16) Msg { uint4 c[4]; };

__device__ __forceinline__ unsigned mixu(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint4 work(uint4 a, uint4 b, unsigned n) {
  // a little dependent integer work per step (the handlers' compares and selects)
  uint4 x = a;
  for (unsigned i = 0; i < n; i++) {
    x.x = mixu(x.x ^ b.y) + x.w;
    x.y ^= x.x + b.z;
    x.z += x.y ^ b.w;
    x.w = mixu(x.z + b.x);
  }
  return x;
}

struct Planes {
  uint4 *hot, *core, *upd, *cnt, *rem, *rq, *rtr;  // record-major (hot 2, core 4, upd 4 chunks per replica)
  unsigned* rem_st;
  unsigned char* idle;
  Msg *mi, *mo;
  unsigned G, maxm;
};

// message position of (group, sender, dest, slot): record-major per (sender,
// dest) list as the engine has it, or the mailbox [slot][group][dest][sender]
template <bool MBOX>
__device__ __forceinline__ size_t msg_at(const Planes& P, unsigned g, unsigned s, unsigned d,
                                         unsigned slot) {
  if (MBOX) return (((size_t)slot * P.G + g) * 3 + d) * 3 + s;
  return ((size_t)(g * 3 + s) * 3 + d) * P.maxm + slot;
}
// chunk q of replica r's row (CH chunks per row): record-major or chunk-major
template <bool CM, unsigned CH>
__device__ __forceinline__ size_t ch_at(const Planes& P, unsigned r, unsigned q) {
  if (CM) return (size_t)q * (3u * P.G) + r;
  return (size_t)r * CH + q;
}

__device__ __forceinline__ unsigned leader_of(unsigned g) { return mixu(g * 2654435761u) % 3; }

// one replica step of the C4 shape; `lead` selects the role's accesses
__device__ unsigned g_dep;  // 0: the knob below adds a dependent load level when set
template <bool MBOX, bool CM>
__device__ __forceinline__ void step(const Planes& P, unsigned g, unsigned k, unsigned ls, unsigned wk) {
  const unsigned r = g * 3 + k;
  const unsigned slot = P.maxm - 1;
  extern __shared__ uint4 occ_lds[];  // dynamic LDS caps the resident blocks per CU
  if (k == ls) {
    // gather: Hot, Core, remotes, count rows of both followers, two inbound
    // HeartbeatResps, the readIndex queue head
    uint4 h0 = P.hot[ch_at<CM, 2>(P, r, 0)], h1 = P.hot[ch_at<CM, 2>(P, r, 1)];
    uint4 c0 = P.core[ch_at<CM, 4>(P, r, 0)], c1 = P.core[ch_at<CM, 4>(P, r, 1)];
    uint4 c2 = P.core[ch_at<CM, 4>(P, r, 2)], c3 = P.core[ch_at<CM, 4>(P, r, 3)];
    uint4 m0 = P.rem[(size_t)r * 3], m1 = P.rem[(size_t)r * 3 + 1], m2 = P.rem[(size_t)r * 3 + 2];
    const unsigned st = P.rem_st[r];
    const unsigned f1 = (k + 1) % 3, f2 = (k + 2) % 3;
    uint4 w1 = P.cnt[ch_at<CM, 1>(P, g * 3 + f1, 0)], w2 = P.cnt[ch_at<CM, 1>(P, g * 3 + f2, 0)];
    const unsigned dsl = wk & 1u ? slot - ((w1.x & g_dep) != 0) : slot;  // wk odd: level 2
    Msg a = P.mi[msg_at<MBOX>(P, g, f1, k, dsl)], b = P.mi[msg_at<MBOX>(P, g, f2, k, dsl)];
    uint4 q0 = P.rq[(size_t)r * 16], q1 = P.rq[(size_t)r * 16 + 1];
    __builtin_amdgcn_s_waitcnt(0);
    uint4 x = work(h0, c0, wk);
    x.x += h1.y + c1.x + c2.y + c3.z + m0.x + m1.y + m2.z + st + w1.x + w2.y + a.c[1].x +
           b.c[2].y + q0.x + q1.y;
    Msg o = a;
    o.c[0] = x;
    // scatter: two Heartbeats, readIndex entry, ReadyToRead, Hot, a Core chunk,
    // the Update chunk, the outbox header, the idle byte
    P.mo[msg_at<MBOX>(P, g, k, f1, slot)] = o;
    o.c[0].y ^= 1;
    P.mo[msg_at<MBOX>(P, g, k, f2, slot)] = o;
    P.rq[(size_t)r * 16] = x;
    P.rq[(size_t)r * 16 + 1] = q1;
    P.rtr[(size_t)r * 4] = x;
    P.rtr[(size_t)r * 4 + 1] = q0;
    P.hot[ch_at<CM, 2>(P, r, 0)] = x;
    P.hot[ch_at<CM, 2>(P, r, 1)] = h1;
    P.core[ch_at<CM, 4>(P, r, 2)] = x;
    P.upd[ch_at<CM, 4>(P, r, 3)] = x;
    P.cnt[ch_at<CM, 1>(P, r, 0)] = x;
    P.idle[r] = (unsigned char)x.x;
    if (x.y == 0x12345u) occ_lds[threadIdx.x] = x;
  } else {
    uint4 h0 = P.hot[ch_at<CM, 2>(P, r, 0)], h1 = P.hot[ch_at<CM, 2>(P, r, 1)];
    uint4 c0 = P.core[ch_at<CM, 4>(P, r, 0)], c1 = P.core[ch_at<CM, 4>(P, r, 1)];
    uint4 c2 = P.core[ch_at<CM, 4>(P, r, 2)], c3 = P.core[ch_at<CM, 4>(P, r, 3)];
    uint4 w = P.cnt[ch_at<CM, 1>(P, g * 3 + ls, 0)];
    const unsigned dsl = wk & 1u ? slot - ((w.x & g_dep) != 0) : slot;
    Msg a = P.mi[msg_at<MBOX>(P, g, ls, k, dsl)];
    __builtin_amdgcn_s_waitcnt(0);
    uint4 x = work(h0, c0, wk);
    x.x += h1.y + c1.x + c2.y + c3.z + w.x + a.c[1].x;
    Msg o = a;
    o.c[0] = x;
    P.mo[msg_at<MBOX>(P, g, k, ls, slot)] = o;
    P.hot[ch_at<CM, 2>(P, r, 0)] = x;
    P.hot[ch_at<CM, 2>(P, r, 1)] = h1;
    P.upd[ch_at<CM, 4>(P, r, 3)] = x;
    P.cnt[ch_at<CM, 1>(P, r, 0)] = x;
    P.idle[r] = (unsigned char)x.x;
  }
}

// A: role lists.  list[i] = replica (leaders first, then followers)
__global__ __launch_bounds__(256, 2) void k_A(Planes P, const unsigned* list, unsigned n, unsigned wk) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned r = list[i], g = r / 3, k = r % 3;
  step<false, false>(P, g, k, leader_of(g), wk);
}

// B/C/F: group order, 3 adjacent lanes per group, 21 groups per wave
template <bool MBOX, bool CM>
__global__ __launch_bounds__(256, 2) void k_B(Planes P, const unsigned* groups, unsigned ng, unsigned wk) {
  const unsigned lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const unsigned j = wave * 21 + lane / 3;
  if (lane >= 63 || j >= ng) return;
  const unsigned g = groups[j], k = lane % 3;
  step<MBOX, CM>(P, g, k, leader_of(g), wk);
}

// D: one lane per group, the three steps in sequence
__global__ __launch_bounds__(256, 2) void k_D(Planes P, const unsigned* groups, unsigned ng, unsigned wk) {
  const unsigned j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ng) return;
  const unsigned g = groups[j], ls = leader_of(g);
  for (unsigned k = 0; k < 3; k++) step<false, false>(P, g, k, ls, wk);
}

int main(int argc, char** argv) {
  const unsigned G = 1u << 20, R = 3 * G, NG = 100000, MAXM = 12;
  Planes P;
  P.G = G;
  P.maxm = MAXM;
  hipMalloc(&P.hot, 32 * (size_t)R);
  hipMalloc(&P.core, 64 * (size_t)R);
  hipMalloc(&P.upd, 64 * (size_t)R);
  hipMalloc(&P.cnt, 16 * (size_t)R);
  hipMalloc(&P.rem, 48 * (size_t)R);
  hipMalloc(&P.rq, 256 * (size_t)R);
  hipMalloc(&P.rtr, 64 * (size_t)R);
  hipMalloc(&P.rem_st, 4 * (size_t)R);
  hipMalloc(&P.idle, (size_t)R);
  hipMalloc(&P.mi, sizeof(Msg) * (size_t)G * 9 * MAXM);
  hipMalloc(&P.mo, sizeof(Msg) * (size_t)G * 9 * MAXM);
  hipMemset(P.mi, 0, sizeof(Msg) * (size_t)G * 9 * MAXM);
  unsigned *dl, *dg;
  hipMalloc(&dl, 3 * NG * 4);
  hipMalloc(&dg, NG * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto t = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    hipEventRecord(e0);
    for (int w = 0; w < 20; w++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-40s %8.2f us/launch\n", name, ms * 1000 / 20);
  };
  auto lead = [](unsigned g) {
    unsigned x = g * 2654435761u;
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x % 3;
  };
  // the active groups: a random 10% of the 1M (the C4 workload's hash), or
  // the first 100k (an awake set compacted into adjacent rows)
  for (int dense = 0; dense < 2; dense++) {
    std::vector<unsigned> gs(NG);
    if (dense) {
      for (unsigned i = 0; i < NG; i++) gs[i] = i;
    } else {
      std::vector<unsigned> perm(G);
      std::mt19937 rng(1);
      for (unsigned i = 0; i < G; i++) perm[i] = i;
      std::shuffle(perm.begin(), perm.end(), rng);
      std::copy(perm.begin(), perm.begin() + NG, gs.begin());
      std::sort(gs.begin(), gs.end());
    }
    std::vector<unsigned> list;
    for (unsigned g : gs) list.push_back(g * 3 + lead(g));
    for (unsigned g : gs)
      for (unsigned k = 0; k < 3; k++)
        if (k != lead(g)) list.push_back(g * 3 + k);
    hipMemcpy(dl, list.data(), list.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dg, gs.data(), NG * 4, hipMemcpyHostToDevice);
    const unsigned nl = (unsigned)list.size();
    const unsigned gA = (nl + 255) / 256, gB = ((NG + 20) / 21 + 3) / 4, gD = (NG + 255) / 256;
    const char* set = dense ? "dense " : "random";
    for (unsigned wk : {0u, 1u}) {
      char nm[80];
      snprintf(nm, sizeof nm, "%s A role lists      work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL(k_A, dim3(gA), dim3(256), 0, 0, P, dl, nl, wk); });
      snprintf(nm, sizeof nm, "%s B group lanes     work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL((k_B<false, false>), dim3(gB), dim3(256), 0, 0, P, dg, NG, wk); });
      snprintf(nm, sizeof nm, "%s C B + mailbox     work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL((k_B<true, false>), dim3(gB), dim3(256), 0, 0, P, dg, NG, wk); });
      snprintf(nm, sizeof nm, "%s E B + chunk-major work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL((k_B<false, true>), dim3(gB), dim3(256), 0, 0, P, dg, NG, wk); });
      snprintf(nm, sizeof nm, "%s F C + chunk-major work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL((k_B<true, true>), dim3(gB), dim3(256), 0, 0, P, dg, NG, wk); });
      snprintf(nm, sizeof nm, "%s D lane per group  work %u", set, wk);
      t(nm, [&] { hipLaunchKernelGGL(k_D, dim3(gD), dim3(256), 0, 0, P, dg, NG, wk); });
    }
  }
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
