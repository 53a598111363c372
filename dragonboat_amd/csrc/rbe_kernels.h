// rbe_kernels.h — the device side of the MI355X batched Raft step engine:
// the round-pipeline kernels and their launch sequence.
//
// Included by rbe_engine.hip (the engine and its C ABI) and by rbe_round.hip,
// which is compiled once per group size N (1, 3, 5) and holds the explicit
// instantiations of launch_round<N, TRACE>, so the heavy per-N kernel code
// builds in parallel translation units.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/rbe.h"
#include "rbe_fast.h"
#include "rbe_xchg.h"

namespace rbe {


#define HIP_IGNORE(x) ((void)(x))
#define HIP_OK(x)                                                      \
  do {                                                                 \
    hipError_t err__ = (x);                                            \
    if (err__ != hipSuccess) {                                         \
      fprintf(stderr, "rbe: %s failed: %s\n", #x, hipGetErrorString(err__)); \
      return RBE_E_HIP;                                                \
    }                                                                  \
  } while (0)

static constexpr int kBlock = 256;
// minimum waves per SIMD requested for the fast-step kernels (caps their VGPRs:
// 2 -> 256, 3 -> 168, 4 -> 128; beyond the cap the compiler spills to scratch)

#ifndef RBE_FAST_LDS_CTR
#define RBE_FAST_LDS_CTR 1  // k_fast_both's event counters in LDS (LdsCounters)
#endif
#ifndef RBE_TRI_CHUNK
#define RBE_TRI_CHUNK 2048
#endif
// work-list entries carry the inbound summary word (kListAux); 0 = A/B baseline
#ifndef RBE_LIST_AUX
#define RBE_LIST_AUX 1
#endif
// k_full_list keeps the replica's remote slots in LDS for the step (MODE_FULL_LREM)
static constexpr int kFullMode = MODE_FULL_LREM;
static constexpr u32 kTriChunk = RBE_TRI_CHUNK;   // replicas per k_triage block (8 per lane)
#ifndef RBE_SMALL_TRI_MAX
#define RBE_SMALL_TRI_MAX (1u << 22)
#endif
static constexpr u64 kSmallTriMax = RBE_SMALL_TRI_MAX;  // replicas up to which scan-only engines triage 256 per block
#ifndef RBE_FAST_HALF_MAX
#define RBE_FAST_HALF_MAX (1u << 17)  // below ~512 blocks of 256: C2 fast step 48.5 -> 45.6 us; C3 (500k) must not (352 -> 483 us)
#endif
// items per k_fast_both block chunk (its blocks: 0.7 x the chunks, up to the grid; L.vgrid)
RBE_HD u32 fast_items_per_block(const Params& C) {
  return C.n_rep <= RBE_FAST_HALF_MAX ? 128u : 256u;
}
static constexpr int kCtrStripes = 64;   // counter stripes per kernel slot (flush_counters)
// counter sections, one per pipeline kernel (rbe_get_kernel_counters)
enum : int { KS_TRIAGE = 0, KS_FAST_LEAD = 1, KS_FAST_FOLL = 2, KS_FULL = 3, KS_NUM = 4 };
static constexpr u64 kCtrWords = (u64)KS_NUM * kCtrStripes * C_NUM;

// Where a kernel finds its round: the device clock {round, tclk} at `ptr`
// (graph replay, advanced on device by k_advance) or 0, plus offsets; `tick`
// says whether the round ticks (rbe_step_ex with RBE_STEP_NO_TICK: no).
struct RoundArg {
  const u32* ptr;
  u32 round_add, tclk_add, tick;
};
__device__ __forceinline__ Clk clk_of(const RoundArg& a) {
  Clk c;
  c.round = (a.ptr ? a.ptr[0] : 0u) + a.round_add;
  c.tclk = (a.ptr ? a.ptr[1] : 0u) + a.tclk_add;
  c.tick = a.tick;
  return c;
}

// ------------------------------------------------------------------ kernels
__device__ __forceinline__ u32 wave_sum(u32 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Event counters live in kCtrStripes stripes of C_NUM u64 (192 B apart, so
// each stripe is its own L2 line).  A block reduces its lanes' counters through
// shuffles and LDS and adds each non-zero total with ONE atomic into stripe
// blockIdx % kCtrStripes: same-address atomics serialise in one L2 channel, so
// one-atomic-per-wave into a single line was the round's bottleneck (r01 profile).
// Every thread of the block must call this (it synchronises the block).
template <int KS, int BS = kBlock>
__device__ __forceinline__ void flush_counters(const Planes& P, const StepCounters& c) {
#if defined(RBE_ABLATE_COUNTERS)  // diagnostic A/B builds only: the flush's cost
  if (KS >= 0) return;
#endif
  __shared__ u32 s_ctr[BS / 64][C_NUM];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) {
    u32 s = 0;
    if (__ballot(c.v[i] != 0) != 0ull) s = wave_sum(c.v[i]);
    if (lane == 0) s_ctr[w][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < C_NUM) {
    u32 t = 0;
#pragma unroll
    for (int j = 0; j < BS / 64; j++) t += s_ctr[j][threadIdx.x];
    if (t)
      atomicAdd((unsigned long long*)&P.counters[((u64)KS * kCtrStripes + blockIdx.x % kCtrStripes) *
                                                     C_NUM + threadIdx.x],
                (unsigned long long)t);
  }
}

// Event counters of the fast steps kept in LDS, one u32 slot per (counter,
// lane) (RBE_FAST_LDS_CTR): `ctr.v[i] += k` is a no-return LDS add, so the
// C_NUM running counts do not hold VGPRs across the persistent loop — at the
// 256-register cap those registers are what the compiler spills, and a scratch
// reload after the lane's first store waits for every store before it (vmcnt
// is in order).
struct LdsCounters {
  struct Ref {
    u32* a;
    __device__ __forceinline__ void operator+=(u32 k) const {
      __hip_atomic_fetch_add(a, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void operator++(int) const { *this += 1u; }
  };
  struct Arr {
    u32* base;  // &slots[0][threadIdx.x]
    __device__ __forceinline__ Ref operator[](int i) const { return Ref{base + i * kBlock}; }
  } v;
};
template <int KS>
__device__ __forceinline__ void lds_counters_init(u32 (*slots)[kBlock]) {
#pragma unroll
  for (int i = 0; i < C_NUM; i++) slots[i][threadIdx.x] = 0;
}
// Every thread of the block must call this (it synchronises the block).
template <int KS>
__device__ __forceinline__ void flush_lds_counters(const Planes& P, u32 (*slots)[kBlock]) {
#if defined(RBE_ABLATE_COUNTERS)
  if (KS >= 0) return;
#endif
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // wave w sums counters w, w + 4, ...: lane l adds slots l, l + 64, ...
  for (int i = w; i < C_NUM; i += kBlock / 64) {
    u32 s = 0;
#pragma unroll
    for (int j = 0; j < kBlock / 64; j++) s += slots[i][lane + 64 * j];
    s = wave_sum(s);
    if (lane == 0 && s)
      atomicAdd((unsigned long long*)&P.counters[((u64)KS * kCtrStripes + blockIdx.x % kCtrStripes) *
                                                     C_NUM + i],
                (unsigned long long)s);
  }
}

// The whole handler table over every replica (reference mode, RBE_MODE=full).
template <int N, bool TRACE>
__global__ __launch_bounds__(kBlock) void k_step(Planes P, Params C, RoundArg ra) {
  const Clk ck = clk_of(ra);
  const u64 r = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (r == 0) spill_clear_next(P, ck.round & 1u);
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
  if (r < C.n_rep && owned<N>(C, r)) step_replica<N, TRACE>(P, C, r, ck, c);
  flush_counters<KS_FULL>(P, c);
}

// Work lists of a round: 0 = steady-state leaders, 1 = steady-state followers,
// 2 = full handler table.  Each list is kShards regions, one per shard: a
// writing block appends to the region of shard blockIdx % kShards, so the
// returning atomics that reserve list space are spread over kShards counters
// per list, each on its own 256-B line (one counter word saturates at ~90
// returning atomics per µs, and k_triage's ~1.5k blocks made five such words
// the round's critical path).  Lists 0 and 1 fill each region from both ends:
// the front holds the common case (a leader without a proposal this round, a
// follower without a Replicate), the back the rest, so the waves of the fast
// launch are mostly homogeneous and skip the code paths none of their lanes
// take.  A consumer reads the regions as one sequence of segments (seg_build /
// seg_find) in the slot order it names (k_fast_list: fronts of every shard,
// then backs; k_fast_both: each role's backs first).
static constexpr u32 kShards = 8;
static constexpr u32 kSlots = 5;   // count slots: fronts of lists 0..2, backs of lists 0..1
static constexpr u32 kCntPad = 64;  // u32 words from one count to the next (256 B)
static constexpr u32 kListCounts = 2 * kSlots * kShards * kCntPad;  // by parity, slot, shard
struct Lists {
  u32* idx;     // list li, shard s: [off[li] + s * scap[li], + scap[li]) replica indices
  u32* aux;     // lists 0 and 1, same layout: inbound summary words (inbound_aux)
  u32* counts;  // list_cnt
  u64 scap[3];  // entries per shard region
  u64 off[3];   // first entry of each list
  // awake-group lists of group sleep in list mode (k_triage)
  u32* al[2];            // groups the round of each parity steps: k_triage block b's own
                         // region [b * al_gb, + al_gb) (its groups, a fixed group range)
  u32* al_cnt;           // their counts, [parity * al_nblk + block]
  u32 al_nblk, al_gb;    // k_triage blocks and groups per block
  u64* slp;              // sleeping totals: [0] owned replicas, [1] leaders (this round);
                         // [2 + 2p], [3 + 2p]: changes made in a round of parity p
  const u32* scan_round; // a round that must scan every group (launch, import)
  u32 al_on;             // list mode on (Quiesce, untraced, rep_world 1, a k_triage pipeline)
  u32 vgrid;             // k_fast_both's blocks per 1000 chunks (700; RBE_FAST_VGRID for A/B)
};
// work-list entries carry their inbound summary word for N = 3 (14 bits; the
// LDS compaction packs it with the 11-bit block position in one u32)
template <int N>
constexpr bool kListAux = N == 3 && RBE_TRI_CHUNK <= 2048 && RBE_LIST_AUX;
__device__ __forceinline__ u32* list_cnt(const Lists& L, u32 slot, u32 par, u32 sh) {
  return &L.counts[((par * kSlots + slot) * kShards + sh) * kCntPad];
}
// position of the j-th front (or back) entry of list li, shard sh
__device__ __forceinline__ u64 list_pos(const Lists& L, u32 li, u32 sh, bool back, u64 j) {
  const u64 base = L.off[li] + (u64)sh * L.scap[li];
  return back ? base + L.scap[li] - 1 - j : base + j;
}
// Every thread of a block calls seg_build: the first wave loads the counts of
// the NQ slots `slots` (all kShards shards of each, segment q * kShards + sh)
// and leaves their exclusive prefix in s_pre[0 .. NQ * kShards].
template <u32 NQ>
__device__ __forceinline__ void seg_build(const Lists& L, u32 par, const u32 (&slots)[NQ],
                                          u32* s_pre) {
  static_assert(NQ * kShards < 64, "one wave scans the segment counts");
  if (threadIdx.x < 64) {
    const u32 lane = threadIdx.x;
    u32 v = 0;
#pragma unroll
    for (u32 q = 0; q < NQ; q++)
      if (lane / kShards == q) v = *list_cnt(L, slots[q], par, lane % kShards);
#pragma unroll
    for (u32 o = 1; o < 64; o <<= 1) {
      const u32 t = __shfl_up(v, o, 64);
      if (lane >= o) v += t;
    }
    if (lane < NQ * kShards) s_pre[lane + 1] = v;
    if (lane == 0) s_pre[0] = 0;
  }
  __syncthreads();
}
// the segment holding sequence item i (< s_pre[NSEG]): the last one starting at or before i
template <u32 NSEG>
__device__ __forceinline__ u32 seg_find(const u32* s_pre, u32 i) {
  u32 lo = 0;
#pragma unroll
  for (u32 step = 32; step; step >>= 1)
    if (lo + step < NSEG && s_pre[lo + step] <= i) lo += step;
  return lo;
}

// wave-aggregated append to the front of list `list`: one atomic per wave
__device__ __forceinline__ void list_push(const Lists& L, u32 list, u32 par, bool want, u32 r) {
  const u64 mask = __ballot(want);
  if (!mask) return;
  const int lane = threadIdx.x & 63;
  const int first = __ffsll((unsigned long long)mask) - 1;
  const u32 sh = blockIdx.x % kShards;
  u32 base = 0;
  if (lane == first) base = atomicAdd(list_cnt(L, list, par, sh), (u32)__popcll(mask));
  base = __shfl(base, first, 64);
  if (want) L.idx[list_pos(L, list, sh, false, base + __popcll(mask & ((1ull << lane) - 1ull)))] = r;
}
// the next round's counts (other parity) start at zero: block 0 of the
// round's first kernel clears count slots [0, nslots)
__device__ __forceinline__ void list_clear_next(const Lists& L, u32 par, u32 nslots) {
  if (blockIdx.x == 0 && threadIdx.x < nslots * kShards)
    *list_cnt(L, threadIdx.x / kShards, par ^ 1u, threadIdx.x % kShards) = 0;
}

// Pass 1 over the round's groups: sleeping groups and idle rounds complete
// here; the rest is listed.
//
// Which groups a block takes.  With group sleep in list mode (Quiesce on,
// untraced, one replica set per GPU: Lists::al_on) the round steps only the
// groups of the awake list AL[round parity] (block b: the awake ones among its
// fixed group range, so a block's rows stay within a few MB and its waves
// share address translations), and
// the sleeping groups' quiesced ticks are counted from running totals
// (Lists::slp) by one thread: a round never touches a sleeping group at all.
// A scan round (launch, import, the workload's first round and the transfer
// rounds, when sleeping groups may be forced to step) instead gives each block
// kTriGroups<N> consecutive groups, reads every wake byte, finishes a sleeping
// group's round from it, and rebuilds the list and the totals.  Without group
// sleep every round is a scan of awake groups.
//
// The replicas of the groups taken are triaged one lane each.  Each listed
// replica takes a position in one of five slots (fronts of lists 0..2, backs
// of lists 0..1) from a wave-aggregated LDS atomic; the block then reserves
// space in each global list with ONE atomic per slot, lays the slots out back
// to back in one LDS array and copies them out coalesced.  A group whose
// replicas all completed lazily falls asleep; the others go to the next
// round's awake list.
template <int N>
constexpr u32 kTriGroups = kTriChunk / N;
template <int N, bool TRACE, u32 CHUNK = kTriChunk>
__global__ __launch_bounds__(kBlock) void k_triage(Planes P, Params C, RoundArg ra, Lists L) {
  constexpr u32 GB = CHUNK / N;
  constexpr u32 kNone = 7u;  // slot code of a replica that is not listed
  __shared__ u32 s_idx[CHUNK];
  __shared__ u32 s_gid[GB];  // triaged groups
  __shared__ u32 s_gst[GB];  // per triaged group: awake << 31 | busy replicas << 8 | leaders
  __shared__ u32 s_alg[GB];  // groups for the next round's awake list
  __shared__ u32 s_n[kSlots], s_base[kSlots], s_off[kSlots];
  __shared__ u32 s_ng, s_nal, s_slp[2];
  const Clk ck = clk_of(ra);
  RBE_STAMP(tt0);
  const u32 round = ck.round;
  const u32 par = round & 1u;
  list_clear_next(L, par, kSlots);
  if (blockIdx.x == 0 && threadIdx.x == 0) spill_clear_next(P, par);
  if (threadIdx.x < kSlots) s_n[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_ng = s_nal = s_slp[0] = s_slp[1] = 0;
  __syncthreads();
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
  const int lane = threadIdx.x & 63;
  const bool shortcut = !TRACE && C.quiesce;
  const bool use_list = shortcut && L.al_on;
  const bool scan = !use_list || round == *L.scan_round || forced_round(C, round);
  const u32 t1 = ck.tick ? 1u : 0u;
  if (use_list && blockIdx.x == 0 && threadIdx.x == 0) {
    // the sleeping totals: last round's changes folded in (a scan recounts)
    u64* d = &L.slp[2 + 2 * (par ^ 1u)];
    if (scan) {
      L.slp[0] = L.slp[1] = 0;
    } else {
      const u64 own = L.slp[0] + d[0], lead = L.slp[1] + d[1];
      L.slp[0] = own;
      L.slp[1] = lead;
      c.v[C_STEPS] += t1 * (u32)own;
      c.v[C_QUIESCED_TICKS] += t1 * (u32)own;
      c.v[C_LEADER_STEPS] += t1 * (u32)lead;
    }
    d[0] = d[1] = 0;
  }
  // phase 1: one lane per group, every wake byte loaded before any is used
  u64 g0 = 0;
  u32 gn = 0;
  const u32* al = L.al[par];
  if (scan) {
    g0 = (u64)blockIdx.x * GB;
    gn = g0 < C.n_groups ? (u32)(C.n_groups - g0 < GB ? C.n_groups - g0 : GB) : 0u;
  } else {  // the block's region of the awake list
    g0 = (u64)blockIdx.x * GB;
    gn = L.al_cnt[par * L.al_nblk + blockIdx.x];
  }
  constexpr u32 kP1 = (GB + kBlock - 1) / kBlock;
  u8 gws[kP1];
  u32 gids[kP1];
#pragma unroll
  for (u32 i = 0; i < kP1; i++) {
    const u32 j = threadIdx.x + i * kBlock;
    const u32 jc = j < gn ? j : 0u;
    if (scan) {
      gids[i] = (u32)(g0 + jc);
      gws[i] = shortcut && gn ? P.gwake[g0 + jc] : (u8)GW_AWAKE;
    } else {
      gids[i] = gn ? al[g0 + jc] : 0u;
      gws[i] = (u8)GW_AWAKE;  // the list holds awake groups only
    }
  }
  u32 sl_own = 0, sl_lead = 0;
#pragma unroll
  for (u32 i = 0; i < kP1; i++) {
    const u32 j = threadIdx.x + i * kBlock;
    const u32 g = gids[i];
    const bool awake = (gws[i] & GW_AWAKE) != 0;
    bool work = j < gn;
    if (work && !awake && !group_forced(C, cid_of_n<N>(C, (u64)g), round)) {
      work = false;
      u32 own = 0;
      for (u32 k = 0; k < (u32)N; k++) own += owned<N>(C, (u64)g * N + k) ? 1u : 0u;
      group_sleep_round(gws[i], own, ck, c);
      sl_own += own;  // still asleep: part of the recounted totals
      sl_lead += (gws[i] >> 1) & 7u;
    }
    const u64 mask = __ballot(work);
    if (mask) {
      const int first = __ffsll((unsigned long long)mask) - 1;
      u32 base = 0;
      if (lane == first) base = atomicAdd(&s_ng, (u32)__popcll(mask));
      base = __shfl(base, first, 64);
      if (work) {
        const u32 pos = base + __popcll(mask & ((1ull << lane) - 1ull));
        s_gid[pos] = g;
        s_gst[pos] = awake ? 0x80000000u : 0u;
      }
    }
  }
  if (use_list && sl_own) {
    atomicAdd(&s_slp[0], sl_own);
    atomicAdd(&s_slp[1], sl_lead);
  }
  __syncthreads();
  RBE_STAMP(tt1);
  // phase 2: one lane per replica of a triaged group (item t: group slot t / N,
  // replica t % N).  The idle bytes and inbound count words of all the items
  // a lane owns (strided by the block size, so each load is coalesced across
  // the wave) are loaded before any of them is processed; most rounds are then
  // decided without reading Hot: a lazy quiesced tick completes here, a
  // replica with inbound messages is listed by the role its idle byte carries.
  constexpr u32 kPer = CHUNK / kBlock;
  const u32 nr = s_ng * (u32)N;
  const u32 iters = (nr + kBlock - 1) / kBlock;  // uniform over the block
  // global replica index of item t (items past the end map to item 0)
  auto item_rep = [&](u32 t, u32* slot_out) -> u32 {
    const u32 tc = t < nr ? t : 0u;
    const u32 slot = tc / (u32)N;
    *slot_out = slot;
    return s_gid[slot] * (u32)N + (tc - slot * (u32)N);
  };
  // Loads of items past the end read the block's first replica and are masked
  // afterwards, and index math is u32: no load waits behind a branch or a
  // 64-bit division, so all the loads of a lane are in flight before the
  // first wait.
  u8 ibs[kPer];
  u16 wv[kPer][N];
#pragma unroll
  for (u32 i = 0; i < kPer; i++) {
    if (i < iters) {
      u32 slot;
      const u32 r = item_rep(threadIdx.x + i * kBlock, &slot);
      const u32 k = r % (u32)N;
      ibs[i] = P.idle[r];
      inbound_load<N>(P, r / (u32)N, k, round, wv[i]);
    }
  }
  // the per-replica bytes packed into registers, so the classification loop
  // below runs rolled (one copy of triage_lazy / triage_replica in the
  // instruction stream instead of kPer) without indexing a register array
  u64 ibp = 0;
  u32 inbp = 0;
  u64 aux_lo = 0, aux_hi = 0;  // kListAux: 14-bit summary words, items 0-3 and 4-7
#pragma unroll
  for (u32 i = 0; i < kPer; i++) {
    if (i < iters) {
      const u32 t = threadIdx.x + i * kBlock;
      const u32 k = (t < nr ? t : 0u) % (u32)N;
      ibp |= (u64)ibs[i] << (8 * i);
      inbp |= inbound_fold<N>(wv[i], k, round) << (3 * i);
      if constexpr (kListAux<N>)
        (i < 4 ? aux_lo : aux_hi) |= (u64)(inbound_aux<N>(wv[i], k, round) & 0x3FFFu)
                                     << (14 * (i % 4));
    }
  }
  RBE_STAMP(tt2);
  // per item: slot code (3 bits) | position in the slot (11 bits), items 0-3 and 4-7
  u64 sp_lo = 0, sp_hi = 0;
#pragma unroll 1
  for (u32 i = 0; i < iters; i++) {
    const u32 t = threadIdx.x + i * kBlock;
    u32 slot;
    const u64 r = item_rep(t, &slot);
    const u8 ib = (u8)(ibp >> (8 * i));
    const u32 inb = (inbp >> (3 * i)) & 7u;
    u32 cls = T_DONE;
    if (t < nr && owned<N>(C, r)) {
      bool done = false;
      if (shortcut && triage_lazy<N>(P, C, r, ck, ib, inb & 1u, c))
        done = true;
      else if (inb & 2u)
        cls = C.rl_max ? T_FULL : class_of_role(idle_role(ib));
      else
        cls = triage_replica<N, TRACE>(P, C, r, ck, c);
      if (!kFastN<N> && (cls == T_LEAD || cls == T_FOLL)) cls = T_FULL;  // no fast step for N
      if (shortcut) atomicAdd(&s_gst[slot], ((ib & IB_LEAD) ? 1u : 0u) + (done ? 0u : 256u));
    }
    // the back of the list: a leader proposing this round, a follower
    // receiving a Replicate
    bool back = false;
    if (cls == T_LEAD)
      back = wl_input(C, cid_of_n<N>(C, (u64)((u32)r / (u32)N)), round) == 1u;
    else if (cls == T_FOLL)
      back = (inb & 4u) != 0;
    const u32 code = cls == T_DONE ? kNone : (back ? cls + 2u : cls - 1u);
    u32 pos = 0;
#pragma unroll
    for (u32 sl = 0; sl < kSlots; sl++) {
      const bool want = code == sl;
      const u64 mask = __ballot(want);
      if (!mask) continue;
      const int first = __ffsll((unsigned long long)mask) - 1;
      u32 base = 0;
      if (lane == first) base = atomicAdd(&s_n[sl], (u32)__popcll(mask));
      base = __shfl(base, first, 64);
      if (want) pos = base + __popcll(mask & ((1ull << lane) - 1ull));
    }
    // (values selected, never a reference to one of the two words: a selected
    // reference in this rolled loop puts both in scratch memory)
    const u64 spv = (u64)(code | (pos << 3)) << (14 * (i % 4));
    sp_lo |= i < 4 ? spv : 0ull;
    sp_hi |= i < 4 ? 0ull : spv;
  }
  __syncthreads();
  const u32 sh = blockIdx.x % kShards;
  if (threadIdx.x < kSlots) {
    const u32 n = s_n[threadIdx.x];
    s_base[threadIdx.x] = n ? atomicAdd(list_cnt(L, threadIdx.x, par, sh), n) : 0u;
    u32 off = 0;
    for (u32 q = 0; q < threadIdx.x; q++) off += s_n[q];
    s_off[threadIdx.x] = off;
  }
  // wake-byte transitions; in list mode the groups that stay awake (or wake)
  // make the next round's list, in the order of s_gid (an ordered block
  // compaction, so list neighbours stay memory neighbours for the fast steps),
  // and the ones falling asleep join the totals
  if (shortcut) {
    __shared__ u32 s_wc[kBlock / 64];
    u32 own = 0, lead = 0, nal = 0;
    const u32 w = threadIdx.x >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    for (u32 j0 = 0; j0 < s_ng; j0 += kBlock) {  // uniform over the block
      const u32 j = j0 + threadIdx.x;
      bool keep = false;
      u32 g = 0;
      if (j < s_ng) {
        const u32 st = s_gst[j];
        g = s_gid[j];
        const bool awake = (st >> 31) != 0;
        const u32 tr = group_transition(C, cid_of_n<N>(C, (u64)g), round, awake,
                                        (st >> 8) & 0xFFu);
        if (tr == GS_SLEEP) P.gwake[g] = group_sleep_byte(st & 0xFFu);
        if (tr == GS_WAKE) P.gwake[g] = GW_AWAKE;
        keep = tr == GS_WAKE || (awake && tr == GS_KEEP);
        if (use_list && !keep) {  // asleep after this round
          own += (u32)N;
          lead += st & 0xFFu;
        }
      }
      if (!use_list) continue;
      const u64 m = __ballot(keep);
      if (lane == 0) s_wc[w] = (u32)__popcll(m);
      __syncthreads();
      u32 before = 0, total = 0;
#pragma unroll
      for (u32 q = 0; q < kBlock / 64; q++) {
        before += q < w ? s_wc[q] : 0u;
        total += s_wc[q];
      }
      if (keep) s_alg[nal + before + (u32)__popcll(m & lt)] = g;
      nal += total;
      __syncthreads();
    }
    if (threadIdx.x == 0) s_nal = nal;
    if (own) {
      atomicAdd(&s_slp[0], own);
      atomicAdd(&s_slp[1], lead);
    }
  }
  __syncthreads();
  if (use_list) {
    if (threadIdx.x == 0) L.al_cnt[(par ^ 1u) * L.al_nblk + blockIdx.x] = s_nal;
    if (threadIdx.x == 1 && s_slp[0])
      atomicAdd((unsigned long long*)&L.slp[2 + 2 * par], (unsigned long long)s_slp[0]);
    if (threadIdx.x == 2 && s_slp[1])
      atomicAdd((unsigned long long*)&L.slp[3 + 2 * par], (unsigned long long)s_slp[1]);
  }
  RBE_STAMP(tt3);
  // the slots back to back in s_idx; fast-list entries with kListAux carry
  // item index | summary word << 11
#pragma unroll 1
  for (u32 i = 0; i < iters; i++) {
    const u32 t = threadIdx.x + i * kBlock;
    const u32 e = (u32)(((i < 4 ? sp_lo : sp_hi) >> (14 * (i % 4))) & 0x3FFFu);
    const u32 code = e & 7u;
    if (code == kNone) continue;
    u32 slot;
    u32 ent = item_rep(t, &slot);
    if (kListAux<N> && code != 2u)
      ent = t | ((u32)(((i < 4 ? aux_lo : aux_hi) >> (14 * (i % 4))) & 0x3FFFu) << 11);
    s_idx[s_off[code] + (e >> 3)] = ent;
  }
  __syncthreads();
  RBE_STAMP(tt4);
#pragma unroll
  for (u32 sl = 0; sl < kSlots; sl++) {
    const u32 li = sl < 3 ? sl : sl - 3;
    for (u32 j = threadIdx.x; j < s_n[sl]; j += kBlock) {
      const u32 ent = s_idx[s_off[sl] + j];
      const u64 at = list_pos(L, li, sh, sl >= 3, s_base[sl] + j);
      if (kListAux<N> && li < 2) {
        u32 slot;
        L.idx[at] = item_rep(ent & 0x7FFu, &slot);
        L.aux[at] = ent >> 11;
      } else {
        L.idx[at] = ent;
      }
    }
  }
  if (use_list)
    for (u32 j = threadIdx.x; j < s_nal; j += kBlock)
      L.al[par ^ 1u][(u64)blockIdx.x * GB + j] = s_alg[j];
  RBE_STAMP(tt5);
  flush_counters<KS_TRIAGE>(P, c);
  RBE_STAMP(tt6);
  RBE_PHASE_ADD(2, 0, tt0, tt1);
  RBE_PHASE_ADD(2, 1, tt1, tt2);
  RBE_PHASE_ADD(2, 2, tt2, tt3);
  RBE_PHASE_ADD(2, 3, tt3, tt4);
  RBE_PHASE_ADD(2, 4, tt4, tt5);
  RBE_PHASE_ADD(2, 5, tt5, tt6);
  RBE_PHASE_ADD(2, 7, 0ull, 1ull);
}

// The fused round (default pipeline): a block triages kTriChunk consecutive
// replicas exactly like k_triage, but keeps its steady-state leaders (from the
// front) and followers (from the back) in one LDS list and steps them itself
// right away; only rounds that need the whole handler table go to the global
// full list.  One launch replaces triage + two fast-list launches, the work
// lists never touch HBM, and the latency-bound protocol work of some blocks
// overlaps the streaming triage of others.
template <int N, bool TRACE>
__global__ __launch_bounds__(kBlock, RBE_FAST_WAVES) void k_round(Planes P, Params C, RoundArg ra, Lists L) {
  __shared__ u32 s_idx[kTriChunk];
  __shared__ u32 s_nl, s_nf;
  const Clk ck = clk_of(ra);
  const u32 round = ck.round;
  const u32 par = round & 1u;
  list_clear_next(L, par, 3);  // slot 2: the full list
  if (blockIdx.x == 0 && threadIdx.x == 0) spill_clear_next(P, par);
  if (threadIdx.x == 0) s_nl = s_nf = 0;
  __syncthreads();
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
  const int lane = threadIdx.x & 63;
  const u64 lo = (u64)blockIdx.x * kTriChunk;
  for (u32 j = threadIdx.x; j < kTriChunk; j += kBlock) {
    const u64 r = lo + j;
    u32 cls = T_DONE;
    if (r < C.n_rep && owned<N>(C, r)) cls = triage_replica<N, TRACE>(P, C, r, ck, c);
#pragma unroll
    for (u32 li = 0; li < 2; li++) {
      const bool want = cls == li + 1;
      const u64 mask = __ballot(want);
      if (!mask) continue;
      const int first = __ffsll((unsigned long long)mask) - 1;
      u32 base = 0;
      if (lane == first) base = atomicAdd(li == 0 ? &s_nl : &s_nf, (u32)__popcll(mask));
      base = __shfl(base, first, 64);
      const u32 pos = base + __popcll(mask & ((1ull << lane) - 1ull));
      if (want) s_idx[li == 0 ? pos : kTriChunk - 1u - pos] = (u32)r;
    }
    list_push(L, 2, par, cls == T_FULL, (u32)r);
  }
  __syncthreads();
  const u32 nl = s_nl, nt = s_nl + s_nf;
  for (u32 i0 = 0; i0 < nt; i0 += kBlock) {
    const u32 i = i0 + threadIdx.x;
    bool slow = false;
    u32 r = 0;
    if (i < nl) {
      r = s_idx[i];
      slow = !step_fast<N, TRACE, MODE_LEAD>(P, C, r, ck, c);
    } else if (i < nt) {
      r = s_idx[kTriChunk - 1u - (i - nl)];
      slow = !step_fast<N, TRACE, MODE_FOLL>(P, C, r, ck, c);
    }
    list_push(L, 2, par, slow, r);
  }
  flush_counters<KS_TRIAGE>(P, c);
}

// Pass 2: the steady-state subset for one role over its list (persistent,
// grid-stride); rounds outside the subset are moved to the full list.
template <int N, bool TRACE, int MODE>
__global__ __launch_bounds__(kBlock, RBE_FAST_WAVES) void k_fast_list(Planes P, Params C, RoundArg ra, Lists L) {
  const Clk ck = clk_of(ra);
  const u32 round = ck.round;
  const u32 par = round & 1u;
  const u32 li = MODE == MODE_LEAD ? 0u : 1u;
  __shared__ u32 s_pre[2 * kShards + 1];
  const u32 slots[2] = {li, 3 + li};
  seg_build<2>(L, par, slots, s_pre);
  const u32 n = s_pre[2 * kShards];
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
  const u64 stride = (u64)gridDim.x * kBlock;
  for (u64 i0 = (u64)blockIdx.x * kBlock; i0 < n; i0 += stride) {
    const u64 i = i0 + threadIdx.x;
    bool slow = false;
    u32 r = 0;
    if (i < n) {
      const u32 sg = seg_find<2 * kShards>(s_pre, (u32)i);
      r = L.idx[list_pos(L, li, sg % kShards, sg >= kShards, (u32)i - s_pre[sg])];
      slow = !step_fast<N, TRACE, MODE>(P, C, r, ck, c);
    }
    list_push(L, 2, par, slow, r);
  }
  flush_counters<MODE == MODE_LEAD ? KS_FAST_LEAD : KS_FAST_FOLL>(P, c);
}

// Orders a wave's LDS accesses around a cross-lane hand-off: the wave's DS
// instructions execute in issue order, so a compiler barrier is all it takes.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Pass 2, merged (RBE_MODE=both, the default): the round's steady-state
// leaders and followers in one launch, so the two roles' waves share the SIMDs
// instead of running back to back; item i < n_lead is a leader, the rest
// followers.  Block b takes chunks b, b + g_eff, ... of the item sequence
// (per role the backs of every shard, then the fronts: seg_build / seg_find),
// one item a lane.
// Measured and not kept: rows staged through LDS for wave-wide
// stores, messages staged likewise, an XCD-aware chunk mapping, chunks that
// alternate leaders and followers.
template <int N, bool TRACE>
__global__ __launch_bounds__(kBlock, kFastWaves<N>) void k_fast_both(Planes P, Params C,
                                                                     RoundArg ra, Lists L) {
  const Clk ck = clk_of(ra);
  const u32 round = ck.round;
  const u32 par = round & 1u;
  // segments: leader backs, leader fronts, follower backs, follower fronts
  __shared__ u32 s_pre[4 * kShards + 1];
  // each role's back segments first: a leader's proposal rounds and a
  // follower's Replicate rounds are its longer steps, so they start first
  // (C4 k_fast_both 99.7 → 97.7 µs, two runs each; C3 / C2 unchanged)
  const u32 slots[4] = {3, 0, 4, 1};
  seg_build<4>(L, par, slots, s_pre);
  const u32 nl = s_pre[2 * kShards], n = s_pre[4 * kShards];
  // a small engine spreads its items over twice the blocks (half of each
  // block's lanes take an item), so more CUs share the step's memory traffic
  // (a power of two: shifts, no 64-bit division in this kernel's registers)
  const u32 per = fast_items_per_block(C);
  const u32 per_log = per == 128u ? 7u : 8u;
  const u64 nchunks = ((u64)n + per - 1) >> per_log;
  // The grid is sized at capture for the worst case; the round's chunks are
  // spread over g_eff = vgrid/1000 of their number (at least 256) blocks, the
  // rest leaving at once (the whole block: no barrier follows for it), so ~30%
  // of the blocks take a second chunk instead of waiting for a slot as a new
  // block.  0.7 measured best on C4 (k_fast_both 111.7 → 102.4 µs; 500k / 2M
  // groups 68.4 → 66.5 / 195 → 184 µs) and no worse on C3 / C2 (DESIGN.md §9,
  // round 5); C2m's 11.7k chunks stay over the 2,048-block grid.
  u64 g_eff = (nchunks * L.vgrid + 999) / 1000;
  if (g_eff < 256) g_eff = nchunks < 256 ? nchunks : 256;
  if (g_eff > gridDim.x) g_eff = gridDim.x;
  if (blockIdx.x >= g_eff) return;
#if RBE_FAST_LDS_CTR
  __shared__ u32 s_ctr_slots[C_NUM][kBlock];
  lds_counters_init<KS_FAST_LEAD>(s_ctr_slots);
  LdsCounters c{{&s_ctr_slots[0][threadIdx.x]}};
#else
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
#endif
  for (u64 ch = blockIdx.x; ch < nchunks; ch += g_eff) {
    const u64 i = (ch << per_log) + threadIdx.x;
    const bool any = threadIdx.x < per && i < n;
    const bool lead = any && i < nl;
    u32 r = 0, aux = 0;
    if (any) {
      const u32 sg = seg_find<4 * kShards>(s_pre, (u32)i);
      const u64 at = list_pos(L, sg / (2 * kShards), sg % kShards, ((sg / kShards) & 1u) == 0u,
                              (u32)i - s_pre[sg]);
      r = L.idx[at];
      if constexpr (kListAux<N>) aux = L.aux[at];
    }
    bool ok = false;
    if (lead)
      ok = step_fast<N, TRACE, MODE_LEAD, kListAux<N>>(P, C, r, ck, c, aux);
    else if (any)
      ok = step_fast<N, TRACE, MODE_FOLL, kListAux<N>>(P, C, r, ck, c, aux);
    list_push(L, 2, par, any && !ok, r);
  }
#if RBE_FAST_LDS_CTR
  flush_lds_counters<KS_FAST_LEAD>(P, s_ctr_slots);
#else
  flush_counters<KS_FAST_LEAD>(P, c);
#endif
}


// Pass 3: the whole handler table over the full list (persistent, grid-stride),
// in blocks of kFullBlock threads: one wave per block, so C3's ~8,000 general
// steps spread over ~125 CUs instead of four waves on each of ~32 (C3
// k_full_list 201 → 193 µs, C3s 121 → 113 µs against 256-thread blocks)
#ifndef RBE_FULL_BLOCK
#define RBE_FULL_BLOCK 64
#endif
static constexpr int kFullBlock = RBE_FULL_BLOCK;
static_assert(kFullBlock <= (int)kLaneCols, "k_full_list's LDS columns (rbe_step.h) hold one thread each");
template <int N, bool TRACE>
__global__ __launch_bounds__(kFullBlock) void k_full_list(Planes P, Params C, RoundArg ra, Lists L) {
  const Clk ck = clk_of(ra);
  const u32 round = ck.round;
  __shared__ u32 s_pre[kShards + 1];
  const u32 slots[1] = {2};
  seg_build<1>(L, round & 1u, slots, s_pre);
  const u32 n = s_pre[kShards];
  StepCounters c;
#pragma unroll
  for (int i = 0; i < C_NUM; i++) c.v[i] = 0;
#if defined(RBE_FULL_PROF)
  // Diagnostic build: every wave iteration's s_memrealtime span, its active
  // lanes, the classes of its lanes (role before, role after, any inbound
  // message) and the most inbound / outbound messages of a lane, for
  // scripts/full_prof.py: what the slowest waves of the general step hold.
  for (u64 b0 = (u64)blockIdx.x * kFullBlock; b0 < n; b0 += (u64)gridDim.x * kFullBlock) {
    const u64 i = b0 + threadIdx.x;
    u32 r = 0, cls_b = 0, nin = 0;
    const bool on = i < n;
    if (on) {
      const u32 sg = seg_find<kShards>(s_pre, (u32)i);
      r = L.idx[list_pos(L, 2, sg, false, (u32)i - s_pre[sg])];
      const u64 g = r / N;
      const u32 k = (u32)(r % N);
      for (u32 s = 0; s < N; s++)
        if (s != k) {
          const u32 w = in_word<N>(P, g, s, k, round);
          nin += (w & 0x7Fu) + ((w >> 7) & 0x7Fu);
        }
      cls_b = ((u32)P.hot[r].role << 4) | (nin ? 1u : 0u);
    }
    const u64 m_on = __ballot(on);
    if (m_on == 0ull) continue;
    const unsigned long long t0 = wall_clock64();
    if (on) step_replica<N, TRACE, kFullMode>(P, C, r, ck, c);
    u32 cls = 0, nout = 0;
    if (on) {
      cls = cls_b | ((u32)P.hot[r].role << 1);
      nout = P.upd[r].n_msgs;
    }
    const unsigned long long t1 = wall_clock64();
    u64 mlo = 0, mhi = 0;
    for (u32 q = 0; q < 128; q++) {  // OR of the lanes' class bits (uniform loop)
      const u64 b = __ballot(on && cls == q);
      if (b) {
        if (q < 64) mlo |= 1ull << q;
        else mhi |= 1ull << (q - 64);
      }
    }
    u32 mx_in = nin, mx_out = nout;
    for (int o = 32; o > 0; o >>= 1) {
      mx_in = max(mx_in, (u32)__shfl_xor((int)mx_in, o, 64));
      mx_out = max(mx_out, (u32)__shfl_xor((int)mx_out, o, 64));
    }
    if ((threadIdx.x & 63u) == 0 && P.prof) {
      const u64 at = atomicAdd((unsigned long long*)&P.prof[0], 1ull);
      if (at < kFullProfCap) {
        u64* rec = &P.prof[kProfHdr + at * 4];
        rec[0] = t1 - t0;
        rec[1] = mlo;
        rec[2] = mhi;
        rec[3] = (u64)__popcll(m_on) | ((u64)mx_in << 8) | ((u64)mx_out << 24);
      }
    }
  }
#else
  if ((u64)blockIdx.x * kFullBlock >= n) return;  // the whole block: no item this round
  for (u64 i = (u64)blockIdx.x * kFullBlock + threadIdx.x; i < n;
       i += (u64)gridDim.x * kFullBlock) {
    const u32 sg = seg_find<kShards>(s_pre, (u32)i);
    step_replica<N, TRACE, kFullMode>(P, C, L.idx[list_pos(L, 2, sg, false, (u32)i - s_pre[sg])],
                                      ck, c);
  }
#endif
  flush_counters<KS_FULL, kFullBlock>(P, c);
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_launch(Planes P, Params C) {
  const u64 r = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (r < C.n_rep) launch_replica<N>(P, C, r);
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_iso_bits(Planes P, Params C, u8* out) {
  const u64 g = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (g >= C.n_groups) return;
  const u64 gg = group_global(C, g);  // bits are exchanged by global group
  if (gg < C.n_groups_glob) out[gg] = (u8)iso_leader_bits<N>(P, C, g);
}
template <int N>
__global__ __launch_bounds__(kBlock) void k_iso_set(Planes P, Params C, u32 round, const u8* bits) {
  const u64 g = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (g >= C.n_groups) return;
  const u64 gg = group_global(C, g);
  if (gg < C.n_groups_glob) iso_apply(P, C, g, round, bits[gg]);
}

template <int N>
__global__ __launch_bounds__(kBlock) void k_isolate(Planes P, Params C, u32 round) {
  const u64 g = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (g < C.n_groups) iso_group<N>(P, C, g, round);
}

// Host input staged by rbe_push_* / rbe_notify_applied (rbe_host.h), one
// launch per step that has any: records to their replicas' ExtIn slots,
// applied indexes to the applied plane.

static constexpr unsigned kFastGrid = 2048;  // persistent grid of k_fast_list
// the fast launches' grid cap (kFastGrid; RBE_FAST_GRID overrides it for A/B
// runs, read once at engine creation; defined in rbe_engine.hip)
extern unsigned g_fast_grid;
#ifndef RBE_FULL_GRID
#define RBE_FULL_GRID 256
#endif
static constexpr unsigned kFullGrid = RBE_FULL_GRID;  // k_full_list's grid in 256-thread units: its ~490 registers allow one wave per SIMD, so 256 x 4 one-wave blocks fill the chip once
static inline unsigned grid_for(u64 n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// One round's launches.  With `ev` (2 * KS_NUM events) every pipeline kernel
// is launched with hipExtLaunchKernel, which stamps ev[2i] / ev[2i + 1] with
// kernel section i's own start and end (the dispatch packet's timestamps, as
// rocprofv3 reads them), so rbe_profile_rounds times the kernels without the
// launch gaps between them; a section with no kernel in the mode gets both
// events at one point (elapsed 0).
#define RBE_LAUNCH(i, K, G, B, ...)                                                         \
  do {                                                                                      \
    if (ev)                                                                                 \
      hipExtLaunchKernelGGL(K, G, B, 0, stream, ev[2 * (i)], ev[2 * (i) + 1], 0, __VA_ARGS__); \
    else                                                                                    \
      hipLaunchKernelGGL(K, G, B, 0, stream, __VA_ARGS__);                                  \
  } while (0)
template <int N, bool TRACE>
int launch_round(const Planes& P, const Params& C, const Lists& L, hipStream_t stream, int mode,
                 RoundArg ra, hipEvent_t* ev) {
  const unsigned g = grid_for(C.n_rep);
  auto none = [&](int i) {  // an empty section
    if (ev) {
      HIP_IGNORE(hipEventRecord(ev[2 * i], stream));
      HIP_IGNORE(hipEventRecord(ev[2 * i + 1], stream));
    }
  };
  const unsigned gt = (unsigned)((C.n_rep + kTriChunk - 1) / kTriChunk);
  const unsigned gtg = (unsigned)((C.n_groups + kTriGroups<N> - 1) / kTriGroups<N>);
  const unsigned gs = (g < kFullGrid ? g : kFullGrid) * (unsigned)(kBlock / kFullBlock);
  // Without group sleep (list mode needs Quiesce and no trace) the block to
  // group mapping is free: 256 replicas per block instead of 2,048, so a
  // small engine (C2: 10k groups) is triaged by 118 blocks, not 15
  const bool small_tri = !(C.quiesce && !TRACE) && C.n_rep <= kSmallTriMax;
  const unsigned gsm = (unsigned)((C.n_groups + kBlock / N - 1) / (kBlock / N));
  const unsigned gfn = (unsigned)((C.n_rep + fast_items_per_block(C) - 1) / fast_items_per_block(C));
  const unsigned gf = gfn < g_fast_grid ? gfn : g_fast_grid;
  if (mode == 2) {
    none(0);
    none(1);
    none(2);
    RBE_LAUNCH(3, (k_step<N, TRACE>), dim3(g), dim3(kBlock), P, C, ra);
  } else if (mode == 0) {
    RBE_LAUNCH(0, (k_round<N, TRACE>), dim3(gt), dim3(kBlock), P, C, ra, L);
    none(1);
    none(2);
    RBE_LAUNCH(3, (k_full_list<N, TRACE>), dim3(gs), dim3(kFullBlock), P, C, ra, L);
  } else {
    if (small_tri)
      RBE_LAUNCH(0, (k_triage<N, TRACE, kBlock>), dim3(gsm), dim3(kBlock), P, C, ra, L);
    else
      RBE_LAUNCH(0, (k_triage<N, TRACE>), dim3(gtg), dim3(kBlock), P, C, ra, L);
    if (mode == 3) {
      RBE_LAUNCH(1, (k_fast_both<N, TRACE>), dim3(gf), dim3(kBlock), P, C, ra, L);
      none(2);
    } else {
      RBE_LAUNCH(1, (k_fast_list<N, TRACE, MODE_LEAD>), dim3(gf), dim3(kBlock), P, C, ra, L);
      RBE_LAUNCH(2, (k_fast_list<N, TRACE, MODE_FOLL>), dim3(gf), dim3(kBlock), P, C, ra, L);
    }
    RBE_LAUNCH(3, (k_full_list<N, TRACE>), dim3(gs), dim3(kFullBlock), P, C, ra, L);
  }
  return hipGetLastError() == hipSuccess ? RBE_OK : RBE_E_HIP;
}
#undef RBE_LAUNCH


}  // namespace rbe
