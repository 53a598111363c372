// MI355X batched Raft step engine: kernels, device memory, C ABI (include/rbe.h).
//
// Round pipeline on one HIP stream:
//   [k_isolate  — only on fault-schedule epoch rounds, one lane per group]
//   k_step<N>   — one lane per replica: inbox → protocol → outbox + Update
// Per-lane event counters are reduced across the 64-lane wavefront with
// cross-lane shuffles and added to 64-bit device counters by one lane.
// rbe_run replays a captured HIP graph of K step launches plus a round
// advance when no per-round host work is needed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rbe.h"
#include "rbe_host.h"
#include "rbe_kernels.h"
#include "rbe_snap.h"
#include "rbe_wire_kernels.h"

namespace rbe {
int dev_sort_pairs(void* tmp, size_t* tmp_bytes, const uint64_t* kin, uint64_t* kout,
                   const uint32_t* vin, uint32_t* vout, uint64_t n, int end_bit,
                   hipStream_t stream);  // rbe_sort.hip
}

using namespace rbe;

#ifndef RBE_SINGLE_TU
// the round pipeline per group size is instantiated in rbe_round.hip (one
// translation unit per N, built in parallel)
namespace rbe {
#define RBE_EXTERN_ROUND(N, T)                                                            \
  extern template int launch_round<N, T>(const Planes&, const Params&, const Lists&,      \
                                         hipStream_t, int, RoundArg, hipEvent_t*);
RBE_EXTERN_ROUND(1, true)
RBE_EXTERN_ROUND(1, false)
RBE_EXTERN_ROUND(2, true)
RBE_EXTERN_ROUND(2, false)
RBE_EXTERN_ROUND(3, true)
RBE_EXTERN_ROUND(3, false)
RBE_EXTERN_ROUND(4, true)
RBE_EXTERN_ROUND(4, false)
RBE_EXTERN_ROUND(5, true)
RBE_EXTERN_ROUND(5, false)
RBE_EXTERN_ROUND(6, true)
RBE_EXTERN_ROUND(6, false)
RBE_EXTERN_ROUND(7, true)
RBE_EXTERN_ROUND(7, false)
#undef RBE_EXTERN_ROUND
}  // namespace rbe
#endif

// Input wakes a sleeping group.  In list mode (Lists::al_on) the group joins
// the awake list of the round about to run (parity par) and leaves the
// sleeping totals; the wake byte's word is updated atomically, so the replicas
// of one group wake it once.
__global__ __launch_bounds__(kBlock) void k_ext_scatter(Planes P, u32 nrep, const u64* reps,
                                                        const ExtIn* recs, u64 n,
                                                        const u64* app_rep, const u64* app_val,
                                                        u64 na, const CommitRec* cr, u64 nc,
                                                        const SnapRec* sr, u64 ns,
                                                        Params C, Lists L, u32 par) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) {
    P.ext[reps[i]] = recs[i];
    const u64 g = reps[i] / nrep;
    if (L.al_on) {
      const u32 sh = 8u * (u32)(g & 3u);
      const u32 old = atomicOr((u32*)(P.gwake + (g & ~3ull)), (u32)GW_AWAKE << sh);
      if (!((old >> sh) & GW_AWAKE)) {
        const u32 lead = (old >> (sh + 1u)) & 7u;
        atomicAdd((unsigned long long*)&L.slp[2 + 2 * (par ^ 1u)], (unsigned long long)(-(u64)nrep));
        if (lead)
          atomicAdd((unsigned long long*)&L.slp[3 + 2 * (par ^ 1u)], (unsigned long long)(-(u64)lead));
        const u32 b = (u32)(g / L.al_gb);
        L.al[par][(u64)b * L.al_gb + atomicAdd(&L.al_cnt[par * L.al_nblk + b], 1u)] = (u32)g;
      }
    } else {
      P.gwake[g] = GW_AWAKE;
    }
  }
  if (i < na) apply_pair(P, app_rep[i], app_val[i]);
  // rbe_commit records (one per replica, so lanes never share a row)
  if (i < nc)
    commit_update(P, C, cr[i].r, cr[i].stable_log_to, cr[i].stable_log_term, cr[i].processed,
                  cr[i].last_applied, cr[i].stable_snapshot_to);
  // rbe_snapshot_saved / rbe_compact records (one per replica)
  if (i < ns) snap_rec_apply(P, sr[i]);
}

// ---- batched Updates (rbe_collect_updates): flag → scan → write
__device__ __forceinline__ bool upd_of(const Planes& P, u64 r, u32 round, rbe_update* u) {
  update_view(P.upd[r], P.core[r], P.hot[r], round, *u);
  update_ids(*u, P.node_ids, P.ids_n, P.node_ids ? r / P.ids_n : 0);
  return (u->flags & RBE_UF_HAS_UPDATE) != 0;
}
__global__ __launch_bounds__(kBlock) void k_upd_count(Planes P, u32 n, u64 first, u64 count,
                                                      u32 round, u32* bsum);
__global__ __launch_bounds__(kBlock) void k_upd_write(Planes P, u32 n, u64 first, u64 count,
                                                      u32 round, const u64* pre, u64* rep,
                                                      rbe_update* ou);

// ---- batched outputs (rbe_collect_outputs): count → scan → write
// Exclusive prefix of v over the 256 lanes of a block; *total = the sum.
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* total) {
  __shared__ u32 s_w[kBlock / 64];
  const u32 lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  u32 x = v;
#pragma unroll
  for (u32 o = 1; o < 64; o <<= 1) {
    const u32 t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  __syncthreads();  // s_w may still be read by a previous call
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  u32 off = 0, tot = 0;
#pragma unroll
  for (u32 q = 0; q < kBlock / 64; q++) {
    off += q < w ? s_w[q] : 0u;
    tot += s_w[q];
  }
  *total = tot;
  return off + x - v;
}
// the message and ReadyToRead counts of replica r's last round (rbe_get_messages /
// rbe_get_ready_to_reads restated per lane)
__device__ __forceinline__ void out_counts(const Planes& P, const Params& C, u64 r, u32 round,
                                           u32* nm, u32* nr) {
  const u32 par = (round - 1u) & 1u;
  const CntRow row = P.cnt[par][r];
  const u32 k = (u32)(r % C.n);
  u32 m = 0;
  for (u32 d = 0; d < C.n; d++) {
    const u32 pc = row_word(row, d, k, round);
    m += list_len(P, C, par, r * C.n + d, pc);
  }
  *nm = m;
  const Upd& u = P.upd[r];
  *nr = u.round == round - 1u ? u.n_rtr : 0u;
}
__global__ __launch_bounds__(kBlock) void k_out_count(Planes P, Params C, u64 first, u64 count,
                                                      u32 round, u32* bsum) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  u32 nm = 0, nr = 0;
  if (i < count) out_counts(P, C, first + i, round, &nm, &nr);
  u32 tm, tr;
  block_excl_scan(nm, &tm);
  block_excl_scan(nr, &tr);
  if (threadIdx.x == 0) {
    bsum[2 * blockIdx.x] = tm;
    bsum[2 * blockIdx.x + 1] = tr;
  }
}
// Exclusive prefixes of the Q-tuples of block sums bsum[Q * nb] into
// pre[Q * nb], totals in pre[Q * nb ..], in three launches (launch_scan): each
// 1024-block tile scans itself (k_scan_up), one block scans the tile totals
// (k_scan_top), the tiles add their offsets (k_scan_add).  pre holds
// scan_words(Q, nb) words: the tile totals follow the grand totals.  (One
// block walking all 11.7k block sums of a C4 engine took 54-77 us.)
constexpr u32 kScanThreads = 1024;
__host__ __device__ constexpr u64 scan_tiles(u64 nb) { return (nb + kScanThreads - 1) / kScanThreads; }
__host__ __device__ constexpr u64 scan_words(u64 q, u64 nb) { return q * nb + q + q * scan_tiles(nb); }
__device__ __forceinline__ u32 block_excl_scan_1k(u32 v, u32* total) {
  __shared__ u32 s_w[kScanThreads / 64];
  const u32 lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  u32 x = v;
#pragma unroll
  for (u32 o = 1; o < 64; o <<= 1) {
    const u32 t = __shfl_up(x, o, 64);
    if (lane >= o) x += t;
  }
  __syncthreads();
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  u32 off = 0, tot = 0;
#pragma unroll
  for (u32 q = 0; q < kScanThreads / 64; q++) {
    off += q < w ? s_w[q] : 0u;
    tot += s_w[q];
  }
  *total = tot;
  return off + x - v;
}
template <int Q>
__global__ __launch_bounds__(kScanThreads) void k_scan_up(const u32* bsum, u32 nb, u64* pre) {
  const u32 b = blockIdx.x * kScanThreads + threadIdx.x;
  u64* tops = pre + (u64)Q * nb + Q;
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const u32 v = b < nb ? bsum[(u64)Q * b + q] : 0u;
    u32 tot;
    const u32 ex = block_excl_scan_1k(v, &tot);
    if (b < nb) pre[(u64)Q * b + q] = ex;
    if (threadIdx.x == 0) tops[(u64)Q * blockIdx.x + q] = tot;
  }
}
template <int Q>
__global__ __launch_bounds__(kScanThreads) void k_scan_top(u32 nb, u64* pre) {
  const u32 nt = (u32)scan_tiles(nb), t = threadIdx.x;  // nt <= 1024 (launch_scan checks)
  u64* tops = pre + (u64)Q * nb + Q;
#pragma unroll
  for (int q = 0; q < Q; q++) {
    const u32 v = t < nt ? (u32)tops[(u64)Q * t + q] : 0u;
    u32 tot;
    const u32 ex = block_excl_scan_1k(v, &tot);
    if (t < nt) tops[(u64)Q * t + q] = ex;
    if (t == 0) pre[(u64)Q * nb + q] = tot;
  }
}
template <int Q>
__global__ __launch_bounds__(kScanThreads) void k_scan_add(u32 nb, u64* pre) {
  const u32 b = blockIdx.x * kScanThreads + threadIdx.x;
  if (b >= nb || blockIdx.x == 0) return;
  const u64* tops = pre + (u64)Q * nb + Q;
#pragma unroll
  for (int q = 0; q < Q; q++) pre[(u64)Q * b + q] += tops[(u64)Q * blockIdx.x + q];
}
template <int Q>
static int launch_scan(hipStream_t st, const u32* bsum, u32 nb, u64* pre) {
  const u32 nt = (u32)scan_tiles(nb);
  if (nt > kScanThreads) return RBE_E_NOMEM;  // > 268M replicas in one call
  hipLaunchKernelGGL(k_scan_up<Q>, dim3(nt), dim3(kScanThreads), 0, st, bsum, nb, pre);
  hipLaunchKernelGGL(k_scan_top<Q>, dim3(1), dim3(kScanThreads), 0, st, nb, pre);
  if (nt > 1) hipLaunchKernelGGL(k_scan_add<Q>, dim3(nt), dim3(kScanThreads), 0, st, nb, pre);
  return hipGetLastError() == hipSuccess ? RBE_OK : RBE_E_HIP;
}
__global__ __launch_bounds__(kBlock) void k_out_write(Planes P, Params C, u64 first, u64 count,
                                                      u32 round, const u64* pre, u64* moff,
                                                      rbe_message* om, u64* roff,
                                                      rbe_ready_to_read* orr) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  u32 nm = 0, nr = 0;
  if (i < count) out_counts(P, C, first + i, round, &nm, &nr);
  u32 tm, tr;
  const u64 bm = pre[2 * blockIdx.x] + block_excl_scan(nm, &tm);
  const u64 br = pre[2 * blockIdx.x + 1] + block_excl_scan(nr, &tr);
  if (i >= count) return;
  moff[i] = bm;
  roff[i] = br;
  if (i + 1 == count) {
    moff[count] = bm + nm;
    roff[count] = br + nr;
  }
  const u64 r = first + i;
  const u32 N = C.n, par = (round - 1u) & 1u;
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  const CntRow row = P.cnt[par][r];
  u64 at = bm;
  for (u32 d = 0; d < N; d++) {
    const ListView lv = list_view(P, C, par, r * N + d, row_word(row, d, k, round));
    for (u32 j = 0; j < lv.n(); j++, at++) {
      const Msg m = lv.at(j);
      rbe_message o;
      msg_out(m, cid_of(C, g), P.node_ids, N, g, o);
      om[at] = o;
    }
  }
  const RTR* rl = rtr_list(P, C, r, nr, par);
  for (u32 j = 0; j < nr; j++) {
    const RTR x = rl[j];
    rbe_ready_to_read o;
    o.index = x.index;
    o.ctx_low = x.low;
    o.ctx_high = x.high;
    orr[br + j] = o;
  }
}

// upd_has on the device: the record's last 16-B chunk (fault, flags, events,
// round, message and ReadyToRead counts) decides for a stale record — the
// common case, a quiesced replica — and for a step without ranges; only a
// step with ranges reads the rest (the collect passes test every replica)
static_assert(offsetof(Upd, fault) == 48 && offsetof(Upd, flags) == 52 &&
                  offsetof(Upd, round) == 56 && offsetof(Upd, n_msgs) == 60 &&
                  offsetof(Upd, n_rtr) == 62,
              "Upd chunk 3 layout (upd_has_dev)");
__device__ __forceinline__ bool upd_has_dev(const Planes& P, u64 r, u32 n, u32 round) {
  // a group asleep after the round slept through it or finished it lazily
  // (group sleep, rbe_step.h group_transition): no replica of it has an Update
  if (!(P.gwake[r / n] & GW_AWAKE)) return false;
  const Upd* u = P.upd + r;
  const uint4 c3 = reinterpret_cast<const uint4*>(u)[3];
  const u32 flags = c3.y & 0xFFFFu, rnd = c3.z;
  if (!(round > 0 && rnd == round - 1)) return false;
  const u32 f = flags & ~(u32)UF_RANGES;
  if ((f & (RBE_UF_STATE_CHANGED | RBE_UF_SENT_QUIESCE | RBE_UF_SNAPSHOT | RBE_UF_APPLIED |
            RBE_UF_HAS_UPDATE)) ||
      c3.w != 0u)  // n_msgs | n_rtr << 16
    return true;
  if (!(flags & UF_RANGES)) return false;
  return upd_has(*u, round);
}

// ---- rbe_collect_step: Updates, their messages and ReadyToReads, one pass
// whether replica r's message to slot d is returned (RBE_COLLECT_REMOTE_MSGS:
// only to replicas another rank steps)
__device__ __forceinline__ bool out_msg_wanted(const Params& C, u64 g, u32 d, bool remote) {
  if (!remote) return true;
  if (C.rep_world <= 1) return false;
  const u64 gg = group_global(C, g);
  return gg < C.n_groups_glob && (u32)((gg + d) % C.rep_world) != C.rep_rank;
}
// An Update with something for the node besides the messages it carries: a
// State change, entries to save or apply, ReadyToReads, dropped requests, a
// Snapshot, an applied index to confirm, listener events, a fault
// (RBE_COLLECT_SKIP_LOCAL: a faulted replica's Update always reaches the host)
__device__ __forceinline__ bool upd_actionable_dev(const Planes& P, u64 r, u32 round) {
  const Upd* u = P.upd + r;
  const uint4 c3 = reinterpret_cast<const uint4*>(u)[3];
  const u32 flags = c3.y & 0xFFFFu, events = c3.y >> 16;
  if ((flags & (RBE_UF_STATE_CHANGED | RBE_UF_SENT_QUIESCE | RBE_UF_SNAPSHOT | RBE_UF_APPLIED |
                RBE_UF_HAS_UPDATE)) ||
      events || c3.x != 0u || (c3.w >> 16) != 0u)  // fault, n_rtr
    return true;
  if (!(flags & UF_RANGES)) return false;
  const Upd d = *u;  // ranges and drops
  return d.n_drop_ent || d.n_drop_ri || d.save_lo <= d.save_hi || d.apply_lo <= d.apply_hi;
}
__device__ __forceinline__ void step_out_counts(const Planes& P, const Params& C, u64 r, u32 round,
                                                u32 cflags, u32* f, u32* nm, u32* nr) {
  const bool remote = (cflags & RBE_COLLECT_REMOTE_MSGS) != 0;
  *f = upd_has_dev(P, r, C.n, round) ? 1u : 0u;
  *nm = *nr = 0;
  if (!*f) return;
  const u32 par = (round - 1u) & 1u, N = C.n;
  const CntRow row = P.cnt[par][r];
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  u32 m = 0;
  for (u32 d = 0; d < N; d++) {
    const u32 pc = row_word(row, d, k, round);
    if (out_msg_wanted(C, g, d, remote)) m += list_len(P, C, par, r * N + d, pc);
  }
  *nm = m;
  // RBE_COLLECT_SKIP_LOCAL: an Update whose only content is messages the
  // engine delivers itself is left out (nothing to persist, apply or send)
  if ((cflags & RBE_COLLECT_SKIP_LOCAL) && m == 0 && !upd_actionable_dev(P, r, round)) {
    *f = 0;
    return;
  }
  const Upd& x = P.upd[r];
  *nr = x.round == round - 1u ? x.n_rtr : 0u;
}
__global__ __launch_bounds__(kBlock) void k_cs_count(Planes P, Params C, u64 first, u64 count,
                                                     u32 round, u32 cflags, u32* bsum) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  u32 f = 0, nm = 0, nr = 0;
  if (i < count) step_out_counts(P, C, first + i, round, cflags, &f, &nm, &nr);
  u32 tf, tm, tr;
  block_excl_scan(f, &tf);
  block_excl_scan(nm, &tm);
  block_excl_scan(nr, &tr);
  if (threadIdx.x == 0) {
    bsum[3 * blockIdx.x] = tf;
    bsum[3 * blockIdx.x + 1] = tm;
    bsum[3 * blockIdx.x + 2] = tr;
  }
}
// the capacities of the regions k_cs_write fills (rbe_collect_step_begin:
// engine-owned mapped host memory); hdr (when non-null) receives the three
// totals and an overflow word, and nothing is written past a capacity
struct CsCaps {
  u64 n, m, r;
  u64* hdr;
};
__global__ __launch_bounds__(kBlock) void k_cs_write(Planes P, Params C, u64 first, u64 count,
                                                     u32 round, u32 cflags, const u64* pre,
                                                     u64* rep, rbe_update* ou, u64* moff,
                                                     rbe_message* om, u64* roff,
                                                     rbe_ready_to_read* orr, CsCaps caps) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const bool remote = (cflags & RBE_COLLECT_REMOTE_MSGS) != 0;
  const u64 n_tot = pre[3 * gridDim.x], m_tot = pre[3 * gridDim.x + 1],
            r_tot = pre[3 * gridDim.x + 2];
  const bool over = n_tot > caps.n || m_tot > caps.m || r_tot > caps.r;
  if (caps.hdr && blockIdx.x == 0 && threadIdx.x == 0) {
    caps.hdr[0] = n_tot;
    caps.hdr[1] = m_tot;
    caps.hdr[2] = r_tot;
    caps.hdr[3] = over ? 1u : 0u;
  }
  if (over) return;
  u32 f = 0, nm = 0, nr = 0;
  if (i < count) step_out_counts(P, C, first + i, round, cflags, &f, &nm, &nr);
  u32 t;
  const u64 at = pre[3 * blockIdx.x] + block_excl_scan(f, &t);
  const u64 bm = pre[3 * blockIdx.x + 1] + block_excl_scan(nm, &t);
  const u64 br = pre[3 * blockIdx.x + 2] + block_excl_scan(nr, &t);
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the closing offsets
    moff[n_tot] = pre[3 * gridDim.x + 1];
    roff[n_tot] = pre[3 * gridDim.x + 2];
  }
  if (!f) return;
  const u64 r = first + i;
  rbe_update u;
  upd_of(P, r, round, &u);
  rep[at] = r;
  ou[at] = u;
  moff[at] = bm;
  roff[at] = br;
  const u32 N = C.n, par = (round - 1u) & 1u;
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  const CntRow row = P.cnt[par][r];
  u64 w = bm;
  for (u32 d = 0; d < N; d++) {
    if (!out_msg_wanted(C, g, d, remote)) continue;
    const ListView lv = list_view(P, C, par, r * N + d, row_word(row, d, k, round));
    for (u32 j = 0; j < lv.n(); j++, w++) {
      const Msg m = lv.at(j);
      rbe_message o;
      msg_out(m, cid_of(C, g), P.node_ids, N, g, o);
      om[w] = o;
    }
  }
  const RTR* rl = rtr_list(P, C, r, nr, par);
  for (u32 j = 0; j < nr; j++) {
    const RTR x = rl[j];
    rbe_ready_to_read o;
    o.index = x.index;
    o.ctx_low = x.low;
    o.ctx_high = x.high;
    orr[br + j] = o;
  }
}

__global__ __launch_bounds__(kBlock) void k_upd_count(Planes P, u32 n, u64 first, u64 count,
                                                      u32 round, u32* bsum) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u32 f = i < count && upd_has_dev(P, first + i, n, round) ? 1u : 0u;
  u32 t;
  block_excl_scan(f, &t);
  if (threadIdx.x == 0) {
    bsum[2 * blockIdx.x] = t;
    bsum[2 * blockIdx.x + 1] = 0;
  }
}
__global__ __launch_bounds__(kBlock) void k_upd_write(Planes P, u32 n, u64 first, u64 count,
                                                      u32 round, const u64* pre, u64* rep,
                                                      rbe_update* ou) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u32 f = i < count && upd_has_dev(P, first + i, n, round) ? 1u : 0u;
  u32 t;
  const u64 at = pre[2 * blockIdx.x] + block_excl_scan(f, &t);
  if (!f) return;
  rbe_update u;
  upd_of(P, first + i, round, &u);
  rep[at] = first + i;
  ou[at] = u;
}

// rbe_launch: one lane per relaunched replica (rbe_step.h relaunch_replica)
struct LaunchRec {
  u64 replica, term, vote, commit, last, off;  // off: first row in the terms/bodies arrays
  u32 n, removed;                              // removed: rbe_launch_state::removed
  u64 marker, marker_term, ss_index, ss_term;  // compacted LogDB (rbe_launch_state)
};
template <int N>
__global__ __launch_bounds__(kBlock) void k_relaunch(Planes P, Params C, const LaunchRec* rec,
                                                     u64 n, const u64* terms, const Body* bodies,
                                                     u32 ppar, u32 tclk) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const LaunchRec x = rec[i];
  relaunch_replica<N>(P, C, x.replica, x.term, x.vote, x.commit, x.last, x.n, terms + x.off,
                      bodies + x.off, ppar, tclk, x.marker, x.marker_term, x.ss_index, x.ss_term,
                      x.removed);
  P.gwake[x.replica / N] = GW_AWAKE;
}

// rbe_replace_node: whether slot (replica % N) is still referenced in its
// group (rbe_step.h slot_referenced), then the new node in the slot
template <int N>
__global__ __launch_bounds__(kBlock) void k_replace_check(Planes P, Params C, const u64* reps,
                                                          u64 n, u32 round, u32* out) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  out[i] = slot_referenced<N>(P, C, reps[i] / N, (u32)(reps[i] % N), round) ? 1u : 0u;
}
template <int N>
__global__ __launch_bounds__(kBlock) void k_join(Planes P, Params C, const u64* reps, u64 n,
                                                 u32 ppar, u32 tclk) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  join_replica<N>(P, C, reps[i], ppar, tclk);
  P.gwake[reps[i] / N] = GW_AWAKE;
}

// the lowest live payload-heap position (rbe_host.h heap_low_group): one lane
// per group, a wave minimum, one 64-bit atomicMin per wave
template <int N>
__global__ __launch_bounds__(kBlock) void k_heap_low(Planes P, Params C, u32 round, u64* out) {
  const u64 g = (u64)blockIdx.x * kBlock + threadIdx.x;
  u64 lo = g < C.n_groups ? heap_low_group<N>(P, C, g, round) : ~0ull;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const u64 y = __shfl_xor(lo, o, 64);
    lo = y < lo ? y : lo;
  }
  if ((threadIdx.x & 63u) == 0 && lo != ~0ull) atomicMin((unsigned long long*)out, lo);
}

// entries [lo, hi] of replica r's log (ring window and cold log, rbe_spill.h
// log_ent_at) for the host getters; *miss counts the ones the replica does
// not hold (compacted, or below what a launch handed over)
__global__ __launch_bounds__(kBlock) void k_log_gather(Planes P, Params C, u64 r, u64 lo, u64 hi,
                                                       Ent* out, u32* miss) {
  const u64 last = P.core[r].last_index;
  for (u64 i = lo + threadIdx.x; i <= hi; i += kBlock) {
    Ent e;
    if (!log_ent_at(P, C, r, last, i, &e)) {
      atomicAdd(miss, 1u);
      e.term = e.lo = e.hi = 0;
      e.type = e.len = 0;
    }
    out[i - lo] = e;
  }
}

// rbe_import_groups: replicas [r0, r0 + n) give back their cold log and
// readIndex pages before the planes are overwritten, then rebuild them from
// the snapshot's log section (rbe_snap.h; rec_off = each record's offset)
__global__ __launch_bounds__(kBlock) void k_spill_release(Planes P, Params C, u64 r0, u64 n,
                                                          u32 par) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) spill_replica_release(P, C, r0 + i, par);
}
__global__ __launch_bounds__(kBlock) void k_snap_log_rebuild(Planes P, Params C, u64 r0, u64 n,
                                                             const u8* sec, const u64* rec_off,
                                                             u32 par, u32* fault) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  u32 f = 0;
  snap_log_rebuild(P, C, r0 + i, sec + rec_off[i], par, &f);
  if (f) atomicOr(fault, f);
}

// rbe_apply_config_change: raft's membership of each listed replica now
// (Planes::roles is valid with MB_ROLES)
__global__ __launch_bounds__(kBlock) void k_ms_gather(Planes P, const u64* replica, u64 n,
                                                      u32* ms) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Core& c = P.core[replica[i]];
  const u32 x = (c.mflags & MB_ROLES) ? P.roles[replica[i]] : 0u;
  ms[i] = pack_ms(c.members & MB_REMOVED, x & 0xFFu, x >> 8);
}

__global__ void k_advance(u32* clk, u32 k) {
  clk[0] += k;
  clk[1] += k;
}

// ---- replica-per-GPU exchange (rbe_xchg.h)
struct XchgCaps {
  u64 cap[XS_NUM];
};
// Pack: one lane per replica; each block reserves its records' slots with one
// global atomic per (peer, stream) after an LDS reduction of its lanes' counts.
template <int N>
__global__ __launch_bounds__(kBlock) void k_xchg_pack(Planes P, Params C, u32 par, u32 round,
                                                      u8* buf, XchgCaps caps, u32* gcount,
                                                      u64 hdr) {
  __shared__ u32 s_cnt[kXchgMaxWorld * XS_NUM];
  __shared__ u32 s_base[kXchgMaxWorld * XS_NUM];
  const u32 nc = C.rep_world * XS_NUM;
  for (u32 i = threadIdx.x; i < nc; i += kBlock) s_cnt[i] = 0;
  __syncthreads();
  const u64 r = (u64)blockIdx.x * kBlock + threadIdx.x;
  const bool mine = r < C.n_rep && owned<N>(C, r);
  u32 cnt[kXchgMaxWorld * XS_NUM];
  u32 base[kXchgMaxWorld * XS_NUM];
  for (u32 i = 0; i < nc; i++) cnt[i] = 0;
  if (mine) xchg_sender<N, false>(P, C, r, par, round, cnt, nullptr, nullptr, caps.cap, hdr);
  for (u32 i = 0; i < nc; i++) base[i] = cnt[i] ? atomicAdd(&s_cnt[i], cnt[i]) : 0u;
  __syncthreads();
  for (u32 i = threadIdx.x; i < nc; i += kBlock)
    s_base[i] = s_cnt[i] ? atomicAdd(&gcount[i], s_cnt[i]) : 0u;
  __syncthreads();
  if (mine) {
    for (u32 i = 0; i < nc; i++) {
      base[i] += s_base[i];
      cnt[i] = 0;
    }
    xchg_sender<N, true>(P, C, r, par, round, cnt, base, buf, caps.cap, hdr);
  }
}
// fixed layout: each peer's chunk header from the pack counts (one thread per
// peer); an overflow also marks the engine's sticky flag
__global__ void k_xchg_hdr(u8* buf, XchgCaps caps, const u32* gcount, u32 world, u32 self,
                           u32* flag) {
  const u32 p = threadIdx.x;
  if (p >= world) return;
  XHdr h;
  for (u32 i = 0; i < 12; i++) h.pad[i] = 0;
  h.overflow = 0;
  for (u32 t = 0; t < XS_NUM; t++) {
    const u32 n = gcount[p * XS_NUM + t];
    h.cnt[t] = n < caps.cap[t] ? n : (u32)caps.cap[t];
    if (n > caps.cap[t]) h.overflow = 1;
  }
  if (h.overflow) atomicOr(flag, 1u);
  *(XHdr*)(buf + xchg_fixed_off(caps.cap, p, self)) = h;
}
// fixed layout, receive side: one lane per record slot of stream t of every
// source chunk; slots past a chunk's count do nothing
__global__ __launch_bounds__(kBlock) void k_xchg_put_fixed(Planes P, Params C, u32 par,
                                                           const u8* recv, XchgCaps caps,
                                                           u32 world, u32 t, u32* flag) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  const u64 cap = caps.cap[t];
  if (i >= cap * world) return;
  u32 ovf = 0;
  xchg_put_fixed(P, C, par, recv, caps.cap, (u32)(i / cap), t, i % cap, &ovf);
  if (ovf && i % cap == 0 && t == XS_CNT) atomicOr(flag, 1u);
}
__global__ __launch_bounds__(kBlock) void k_xchg_put_cnt(Planes P, Params C, u32 par,
                                                         const XCnt* x, u64 n) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) xchg_put_cnt(P, C, par, x[i]);
}
__global__ __launch_bounds__(kBlock) void k_xchg_put_msg(Planes P, Params C, u32 par,
                                                         const XMsg* x, u64 n) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) xchg_put_msg(P, C, par, x[i]);
}
__global__ __launch_bounds__(kBlock) void k_xchg_put_ent(Planes P, Params C, u32 par,
                                                         const XEnt* x, u64 n) {
  const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) xchg_put_ent(P, C, par, x[i]);
}

// ------------------------------------------------------------------ engine
// Pinned host memory for the input staging vectors (HostInputsT): an upload
// from them is a DMA with no host copy.  A failed allocation throws, as
// std::allocator's does.
template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U>&) {}
  T* allocate(size_t n) {
    // RBE_PINNED_LIMIT_BYTES: refuse larger allocations, as a host short of
    // pinnable memory would (fault injection for the RBE_E_NOMEM path)
    static const u64 limit = [] {
      const char* v = getenv("RBE_PINNED_LIMIT_BYTES");
      return v ? strtoull(v, nullptr, 10) : 0ull;
    }();
    void* p = nullptr;
    if ((limit && n * sizeof(T) > limit) ||
        hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault) != hipSuccess || !p)
      throw std::bad_alloc();
    return (T*)p;
  }
  void deallocate(T* p, size_t) { HIP_IGNORE(hipHostFree(p)); }
  template <class U>
  bool operator==(const PinnedAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const PinnedAlloc<U>&) const { return false; }
};

// The C ABI never lets an exception out: a failed host allocation while
// staging input (a pinned PinnedAlloc growth, or std::allocator's) is
// RBE_E_NOMEM, and the staged input of the call is left as it was checked.
template <class F>
static int abi_nomem(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return RBE_E_NOMEM;
  }
}

struct rbe_engine {
  rbe_config cfg;
  Params C;
  Planes P;
  int device = 0;
  hipStream_t stream = nullptr;
  u32 round = 0;
  u32 tclk = 0;              // ticks before the next round (Clk::tclk)
  u32* d_clk = nullptr;      // device copy {round, tclk} read by graph replays
  std::vector<void*> allocs;
  // captured K-round graphs, one per round count K (rbe_run; rbe_prepare_run
  // captures ahead of a timed region), replaced round-robin
  static constexpr int kGraphs = 4;
  hipGraphExec_t graph[kGraphs] = {};
  u32 graph_rounds[kGraphs] = {};
  u32 graph_next = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int mode = 3;              // RBE_MODE: 0 fused, 1 split (triage + 2 fast lists), 2 full,
                             // 3 both (default: triage + one merged fast launch)
  Lists L;                   // per-round work lists (triage → fast → full)
  u32* xcount = nullptr;     // replica-per-GPU pack counters [rep_world * XS_NUM]
  // rbe_push_* staged for the next step (rbe_host.h); its replica, record and
  // entry vectors live in pinned memory and go to the device as they are,
  // alternating with the `up_*` spares (flush_inputs)
  HostInputsT<PinnedAlloc> hin;
  HostInputsT<PinnedAlloc>::UpVec<u64> up_reps;
  HostInputsT<PinnedAlloc>::UpVec<ExtIn> up_recs;
  HostInputsT<PinnedAlloc>::UpVec<Ent> up_ents;
  u64 in_used = 0;
  u8* in_pinned[2] = {nullptr, nullptr};  // pinned staging of the small input parts, by
  u64 in_pbytes[2] = {0, 0};              // flush parity, and their capacities
  u8* in_dev = nullptr;      // the device copy (replicas, records, applied pairs, ...)
  u64 in_bytes = 0;
  hipEvent_t in_ev[2] = {nullptr, nullptr};  // the uploads of flush parity 0 / 1 have finished
  u32 in_slot = 0;
  u8* heap = nullptr;        // payload heap (cfg.heap_bytes; positions in hin.heap)
  u64* heap_dev = nullptr;   // [0] heap head after the last upload (Planes::heap_head),
                             // [1] k_heap_low result
  u64 heap_head_host = 0;    // source of [0]
  u32 scan_at = 0;           // host copy of Lists::scan_round (the source of its upload)
  // rbe_collect_outputs: device scratch and the pinned host copy it returns
  u8* out_dev = nullptr;
  u64 out_dev_bytes = 0;
  u8* gat_dev = nullptr;  // rbe_get_entries' gather buffer (k_log_gather)
  u64 gat_dev_bytes = 0;
  u8* out_host = nullptr;
  u64 out_host_bytes = 0;
  // replica mode with the isolation schedule: every rank's leader bits, ORed
  // by the host, for the epoch round iso_round (rbe_set_iso_leaders)
  u8* iso_dev = nullptr;
  u32 iso_round = ~0u;
  // rbe_wire_ingest scratch (keys, indexes, heap offsets, sort temporary)
  u8* ing_dev = nullptr;
  u64 ing_dev_bytes = 0;
  // capacities the no-read-back ingest launches for (messages, entries, Cmd
  // bytes): the last call's counts + 25%; 0 until a call has measured them
  u64 ing_cap[3] = {0, 0, 0};
  // rbe_collect_updates: the same for the compacted Updates
  u8* upd_dev = nullptr;
  u64 upd_dev_bytes = 0;
  u8* upd_host = nullptr;
  u64 upd_host_bytes = 0;
  // rbe_collect_step: the same for Updates + their outputs
  u8* cs_dev = nullptr;
  u64 cs_dev_bytes = 0;
  u8* cs_host = nullptr;
  u64 cs_host_bytes = 0;
  // rbe_collect_step_begin / _end: mapped host memory the write kernel fills
  // directly (header | replicas | updates | offsets | messages | ReadyToReads),
  // its capacities, the pending call and its completion event
  u8* csa_buf[2] = {nullptr, nullptr};  // two, used in turn: a round's records
  u64 csa_bytes[2] = {0, 0};              // outlive the next round's _begin
  u32 csa_slot = 0;
  u8* csa_host = nullptr;                 // the slot of the pending / last call
  u64 csa_cap[3] = {0, 0, 0};
  bool csa_pending = false;
  u64 csa_first = 0, csa_count = 0;
  u32 csa_flags = 0, csa_round = 0;
  hipEvent_t csa_ev = nullptr;
  // rbe_wire_encode / rbe_wire_decode scratch
  u8* wire_dev = nullptr;    // the last rbe_wire_encode's frames (rbe_wire_fetch)
  u64 wire_dev_bytes = 0;
  u8* wire_meta = nullptr;   // cells, batches, frame index
  u64 wire_meta_bytes = 0;
  u8* wire_rec = nullptr;    // decoded records
  u64 wire_rec_bytes = 0;
  u8* wire_in = nullptr;     // rbe_wire_decode: inbound bytes and per-frame scratch
  u64 wire_in_bytes = 0;
  u8* wire_big_buf = nullptr;  // the chunked walk of big frames: exits, counts, chunk lists
  u64 wire_big_bytes = 0;
  // frames longer than this are walked by chunks (k_wire_chunk_exit / hop /
  // emit), shorter ones by one block each (k_wire_bounds); RBE_WIRE_BIG sets it
  u64 wire_big = 256u << 10;
  u64 wire_totals[4] = {0, 0, 0, 0};
  u64 wire_frames_off = 0;   // frame index inside wire_meta
};

unsigned rbe::g_fast_grid = rbe::kFastGrid;

static void drop_graphs(rbe_engine* e) {
  for (int i = 0; i < rbe_engine::kGraphs; i++)
    if (e->graph[i]) {
      HIP_IGNORE(hipGraphExecDestroy(e->graph[i]));
      e->graph[i] = nullptr;
      e->graph_rounds[i] = 0;
    }
}

// Copy `len` bytes at offset `off` of the heap record at absolute position
// `pos`: still staged, from the host copy; else from the device after every
// queued round (RBE_E_STATE once a later lap of the ring has overwritten them).
static int read_heap(rbe_engine* e, u64 pos, u64 off, u64 len, u8* dst) {
  const HostHeap& h = e->hin.heap;
  if (!h.valid(pos, off + len)) return RBE_E_STATE;
  if (h.read_staged(pos, off, len, dst)) return RBE_OK;
  HIP_OK(hipMemcpyAsync(dst, e->heap + (pos + off) % h.cap, len, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}


static int read_window(rbe_engine* e, u64 replica, u64 lo, u64 hi, std::vector<u64>& t,
                       std::vector<Body>& b);
static int grow(u8** p, u64* have, u64 need, bool pinned);
static int host_list(rbe_engine* e, u32 par, u64 li, u32 w, const Msg* pl, std::vector<Msg>& out);

static constexpr int kPlaneAllocs = 30;
static u64 bytes_of(const Params& C, u64* parts) {
  const u64 N = C.n, G = C.n_groups, R = C.n_rep;
  u64 p[kPlaneAllocs] = {
      R * sizeof(Hot),
      R * sizeof(Core),
      R * N * sizeof(RemoteMN),
      R * N,
      R * C.rq_cap * sizeof(ReadReq),
      (u64)C.ring * R * sizeof(u64),
      (u64)C.ring * R * sizeof(Body),
      2 * R * sizeof(CntRow),
      2 * G * N * N * C.maxm * sizeof(Msg),
      2 * R * C.ecap * sizeof(Ent),
      G * sizeof(u8),
      G * sizeof(u32),
      R * sizeof(Upd),
      R * C.rtr_cap * sizeof(RTR),
      R * C.dri_cap * sizeof(DropRI),
      R * sizeof(ExtIn),
      R * sizeof(u8),
      (u64)C.in_cap * sizeof(Ent),
      R * sizeof(u64),
      G * sizeof(u8),
      C.snapshot_entries ? R * sizeof(SnapSt) : 0,
      C.snapshot_entries ? R * N * sizeof(u64) : 0,
      (C.ext_commit || C.rl_max) ? R * sizeof(u64) : 0,
      C.rl_max ? R * sizeof(RlSt) : 0,
      C.membership ? R * sizeof(u16) : 0,
      // spill tiers (rbe_spill.h): pool records, pool page links, cold-log refs,
      // the round spill heap (both parities), the allocation words
      (u64)C.pool_pages * kPageEnts * sizeof(Ent),
      (u64)C.pool_pages * sizeof(PoolMeta),
      R * sizeof(ColdRef),
      2 * C.spill_units * 16,
      sizeof(SpillCtl),
  };
  u64 t = 0;
  for (int i = 0; i < kPlaneAllocs; i++) {
    if (parts) parts[i] = p[i];
    t += (p[i] + 255) & ~255ull;
  }
  return t + 256;
}

static int make_params(const rbe_config* cfg, Params* out) {
  if (!cfg || cfg->abi_version != RBE_ABI_VERSION) return RBE_E_INVALID;
  Params C;
  memset(&C, 0, sizeof(C));
  C.n = cfg->n_replicas;
  if (!valid_n(C.n)) return RBE_E_INVALID;
  C.n_voters = cfg->n_voters ? cfg->n_voters : C.n;
  if (cfg->n_groups == 0) return RBE_E_INVALID;
  C.n_groups = cfg->n_groups;
  C.n_rep = cfg->n_groups * C.n;
  C.cid_base = cfg->cid_base ? cfg->cid_base : 1;
  C.cid_stride = cfg->cid_stride ? cfg->cid_stride : 1;
  C.seed = cfg->seed;
  C.max_entry_size = cfg->max_entry_size ? cfg->max_entry_size : (64ull << 20);
  C.ring = cfg->ring ? cfg->ring : 64;
  if (C.ring & (C.ring - 1)) return RBE_E_INVALID;
  if (C.ring < 8) return RBE_E_INVALID;
  C.rq_cap = cfg->rq_cap ? cfg->rq_cap : 8;
  if (C.rq_cap >= kRqExt) return RBE_E_INVALID;  // (kRqExt marks a queue in pool pages)
  C.maxm = cfg->maxm ? cfg->maxm : 12;
  if (C.maxm > 127) return RBE_E_INVALID;
  C.ecap = cfg->ecap ? cfg->ecap : 32;
  C.rtr_cap = cfg->rtr_cap ? cfg->rtr_cap : 8;
  C.dri_cap = cfg->dri_cap ? cfg->dri_cap : 8;
  C.election_rtt = cfg->election_rtt;
  C.heartbeat_rtt = cfg->heartbeat_rtt;
  // config.Validate (config/config.go:173-208)
  if (C.heartbeat_rtt == 0 || C.election_rtt == 0 || C.election_rtt <= 2 * C.heartbeat_rtt)
    return RBE_E_INVALID;
  if (C.election_rtt > 30000) return RBE_E_INVALID;  // randomized timeout kept in u16
  C.check_quorum = cfg->check_quorum;
  C.quiesce = cfg->quiesce;
  C.trace = cfg->trace;
  C.wl_enabled = cfg->wl_enabled;
  C.wl_start_round = cfg->wl_start_round;
  C.wl_stop_round = cfg->wl_stop_round;
  C.wl_active_mod = cfg->wl_active_mod;
  C.wl_read_permille = cfg->wl_read_permille;
  C.ext_inputs = cfg->ext_inputs;
  C.iso_period = cfg->iso_period;
  C.iso_len = cfg->iso_len;
  C.iso_mod = cfg->iso_mod;
  C.rep_world = cfg->rep_world > 1 ? cfg->rep_world : 1;
  C.rep_rank = cfg->rep_rank;
  if (C.rep_world > kXchgMaxWorld || C.rep_rank >= C.rep_world) return RBE_E_INVALID;
  rep_compact_setup(C, cfg->rep_compact != 0);
  C.ext_apply = cfg->ext_apply;
  if (C.ext_apply && !C.ext_inputs) return RBE_E_INVALID;  // applied comes from rbe_notify_applied
  // the host that persists an Update (rbe_commit) applies it too: raft.applied
  // is then the host's (rbe_notify_applied), never the step's own
  C.ext_commit = cfg->ext_commit;
  if (C.ext_commit && !C.ext_apply) return RBE_E_INVALID;
  C.rl_max = cfg->max_inmem_log_size;
  C.membership = cfg->membership;
  C.cc_period = cfg->cc_period;
  C.cc_mod = cfg->cc_mod ? cfg->cc_mod : 1;
  if (C.cc_period && !C.membership) return RBE_E_INVALID;
  // spare slots (nodes that join later) need membership change; observer and
  // witness slots are disjoint spare slots
  if (C.n_voters > C.n || (C.n_voters < C.n && !C.membership)) return RBE_E_INVALID;
  C.obs_slots = cfg->observer_slots;
  C.wit_slots = cfg->witness_slots;
  {
    const u32 spare = ((1u << C.n) - 1u) & ~((1u << C.n_voters) - 1u);
    if (((C.obs_slots | C.wit_slots) & ~spare) || (C.obs_slots & C.wit_slots) ||
        ((C.obs_slots | C.wit_slots) && !C.membership))
      return RBE_E_INVALID;
  }
  C.in_cap = cfg->in_cap ? cfg->in_cap : (u32)(cfg->n_groups > 1024 ? cfg->n_groups : 1024);
  if (cfg->n_groups > 0xFFFFFFFFull && !cfg->in_cap) C.in_cap = 0xFFFFFFFFu;
  C.xfer_period = cfg->xfer_period;
  C.xfer_mod = cfg->xfer_mod;
  // node snapshots + LogDB compaction (SnapSt; rbe_step.h node_snapshot): the
  // snapshot is taken at the state machine's applied index, which is the
  // engine's own (processed) only without ext_apply
  // With ext_apply the host's state machine is snapshotted by the host's
  // snapshot worker, which tells the engine (rbe_snapshot_saved, rbe_compact);
  // the engine then never snapshots by itself.  With ext_commit a restored
  // snapshot stays in every Update until the host's UpdateCommit names it
  // (StableSnapshotTo; SnapSt::upd_ss).
  C.snapshot_entries = cfg->snapshot_entries;
  C.compaction_overhead = cfg->compaction_overhead;
  // the compaction of a snapshot at index i reads Term(i - CompactionOverhead),
  // which must still be in the in-memory window
  if (C.snapshot_entries && C.compaction_overhead >= C.ring) return RBE_E_INVALID;
  // the payload heap holds host-pushed Cmds longer than 16 bytes
  C.heap_bytes = (cfg->heap_bytes + 255) & ~255ull;
  if (C.heap_bytes && !C.ext_inputs) return RBE_E_INVALID;
  if (spill_sizes(cfg, &C)) return RBE_E_INVALID;
  *out = C;
  return RBE_OK;
}

template <typename F>
static int dispatch_n(u32 n, F&& f) {
  if (!valid_n(n)) return RBE_E_INVALID;
  return with_n(n, f);
}

template <typename T>
static int d2h(rbe_engine* e, T* dst, const T* src, u64 n) {
  HIP_OK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, e->stream));
  return RBE_OK;
}


static int launch_step(rbe_engine* e, RoundArg ra,
                       hipEvent_t* ev = nullptr) {
  return dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    return e->C.trace ? launch_round<N, true>(e->P, e->C, e->L, e->stream, e->mode, ra, ev)
                      : launch_round<N, false>(e->P, e->C, e->L, e->stream, e->mode, ra, ev);
  });
}

// Sum the counter stripes of one kernel section (ks >= 0) or of all (ks < 0).
static int read_counters(rbe_engine* e, int ks, u64* out) {
  std::vector<u64> st(kCtrWords);
  HIP_OK(hipMemcpyAsync(st.data(), e->P.counters, st.size() * sizeof(u64), hipMemcpyDeviceToHost,
                        e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  for (int i = 0; i < C_NUM; i++) out[i] = 0;
  for (int k = 0; k < KS_NUM; k++) {
    if (ks >= 0 && k != ks) continue;
    for (int j = 0; j < kCtrStripes; j++)
      for (int i = 0; i < C_NUM; i++) out[i] += st[((size_t)k * kCtrStripes + j) * C_NUM + i];
  }
  return RBE_OK;
}

extern "C" {

int rbe_abi_version(void) { return RBE_ABI_VERSION; }

int rbe_abi_sizes(uint64_t* out, uint32_t cap) {
  const uint64_t sz[6] = {sizeof(rbe_config), sizeof(rbe_replica_view), sizeof(rbe_update),
                          sizeof(rbe_message), sizeof(rbe_entry), sizeof(rbe_ready_to_read)};
  if (!out) return RBE_E_INVALID;
  uint32_t n = cap < 6 ? cap : 6;
  for (uint32_t i = 0; i < n; i++) out[i] = sz[i];
  return (int)n;
}

// Group-range snapshots (rbe_snap.h): one 2-D copy per plane on the engine
// stream, ordered after every round already queued.
int rbe_snapshot_bytes(rbe_engine* e, uint64_t count, uint64_t* bytes) {
  if (!e || !bytes || count == 0 || count > e->C.n_groups) return RBE_E_INVALID;
  *bytes = sizeof(SnapHeader) + snap_body_bytes(e->P, e->C, count);
  return RBE_OK;
}

}  // extern "C"

// The source side of a snapshot's log section (rbe_snap.h snap_log_write):
// the range's cold log refs and Core rows copied once, pages and their meta
// read as the chains are walked
struct SnapLogDev {
  rbe_engine* e;
  u64 r0;
  std::vector<ColdRef> cr;
  std::vector<Core> co;
  int rc = RBE_OK;
  SnapLogDev(rbe_engine* en, u64 first_rep, u64 n) : e(en), r0(first_rep), cr(n), co(n) {
    if (hipMemcpy(cr.data(), e->P.cold + r0, n * sizeof(ColdRef), hipMemcpyDeviceToHost) ||
        hipMemcpy(co.data(), e->P.core + r0, n * sizeof(Core), hipMemcpyDeviceToHost))
      rc = RBE_E_HIP;
  }
  ColdRef cold(u64 r) { return cr[r - r0]; }
  Core core(u64 r) { return co[r - r0]; }
  RqExt rq(u64 r) {
    ReadReq d = {};
    if (hipMemcpy(&d, e->P.rq + r * e->C.rq_cap, sizeof(d), hipMemcpyDeviceToHost)) rc = RBE_E_HIP;
    RqExt x;
    x.head = (u32)d.low;
    x.tail = (u32)(d.low >> 32);
    x.off = (u32)d.high;
    x.n = (u32)(d.high >> 32);
    return x;
  }
  PoolMeta meta(u32 p) {
    PoolMeta m = {};
    if (hipMemcpy(&m, e->P.pmeta + p, sizeof(m), hipMemcpyDeviceToHost)) rc = RBE_E_HIP;
    return m;
  }
  void page(u32 p, Ent* out) {
    if (hipMemcpy(out, e->P.pool + (u64)p * kPageEnts, kPageEnts * sizeof(Ent),
                  hipMemcpyDeviceToHost))
      rc = RBE_E_HIP;
  }
};

// Whether the range's last step left round spill heap state a snapshot cannot
// carry (rbe_snap.h snap_round_spilled)
static int snap_range_spilled(rbe_engine* e, u64 first, u64 count, bool* out) {
  const u32 N = e->C.n, par = (e->round - 1) & 1u;
  const u64 r0 = first * N, n = count * N;
  *out = false;
  if (e->round == 0) return RBE_OK;
  std::vector<CntRow> rows(n);
  std::vector<Upd> upd(n);
  std::vector<Msg> lst(n * N * e->C.maxm);
  if (d2h(e, rows.data(), e->P.cnt[par] + r0, n) || d2h(e, upd.data(), e->P.upd + r0, n) ||
      d2h(e, lst.data(), e->P.msgs[par] + r0 * N * e->C.maxm, lst.size()))
    return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u64 i = 0; i < n && !*out; i++) {
    u32 w[8];
    for (u32 d = 0; d < N; d++) w[d] = row_word(rows[i], d, (u32)((r0 + i) % N), e->round);
    *out = snap_round_spilled(e->C, w, &lst[i * N * e->C.maxm], upd[i]);
  }
  return RBE_OK;
}

extern "C" {

int rbe_export_bytes(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* bytes) {
  if (!e || !bytes || count == 0 || first >= e->C.n_groups || count > e->C.n_groups - first)
    return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipStreamSynchronize(e->stream));
  SnapLogDev src(e, first * e->C.n, count * e->C.n);
  const u64 lb = snap_log_write(e->C, first * e->C.n, count * e->C.n, src, nullptr);
  if (src.rc) return src.rc;
  *bytes = snap_log_at(snap_body_bytes(e->P, e->C, count)) + lb;
  return RBE_OK;
}

int rbe_export_groups(rbe_engine* e, uint64_t first, uint64_t count, void* buf, uint64_t cap) {
  if (!e || !buf || count == 0 || first >= e->C.n_groups || count > e->C.n_groups - first)
    return RBE_E_INVALID;
  const u64 body = snap_body_bytes(e->P, e->C, count);
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipStreamSynchronize(e->stream));
  bool spilled = false;
  int rc = snap_range_spilled(e, first, count, &spilled);
  if (rc) return rc;
  if (spilled) return RBE_E_STATE;
  const u64 r0 = first * e->C.n, nr = count * e->C.n;
  SnapLogDev src(e, r0, nr);
  const u64 lb = snap_log_write(e->C, r0, nr, src, nullptr);
  if (src.rc) return src.rc;
  if (cap < snap_log_at(body) + lb) return RBE_E_NOMEM;
  SnapHeader h;
  snap_fill_header(e->C, RBE_ABI_VERSION, e->round, e->tclk, first, count, body, &h);
  h.log_bytes = lb;
  memcpy(buf, &h, sizeof(h));
  memset((u8*)buf + sizeof(h) + body, 0, snap_log_at(body) - sizeof(h) - body);
  snap_log_write(e->C, r0, nr, src, (u8*)buf + snap_log_at(body));
  if (src.rc) return src.rc;
  SnapPlane pl[kSnapPlanes];
  snap_planes(e->P, e->C, pl);
  u8* dst = (u8*)buf + sizeof(SnapHeader);
  for (int i = 0; i < kSnapPlanes && pl[i].rows; i++) {
    const u64 w = count * pl[i].group_bytes;
    HIP_OK(hipMemcpy2DAsync(dst, w, pl[i].base + first * pl[i].group_bytes, pl[i].pitch, w,
                            pl[i].rows, hipMemcpyDeviceToHost, e->stream));
    dst += w * pl[i].rows;
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_import_groups(rbe_engine* e, const void* buf, uint64_t bytes, uint32_t flags) {
  if (!e || !buf) return RBE_E_INVALID;
  SnapHeader h;
  if (bytes < sizeof(h)) return RBE_E_INVALID;
  memcpy(&h, buf, sizeof(h));
  if (snap_check_header(e->C, RBE_ABI_VERSION, &h, bytes) ||
      h.body_bytes != snap_body_bytes(e->P, e->C, h.count))
    return RBE_E_INVALID;
  const bool resume = (flags & RBE_IMPORT_RESUME) != 0;
  if (resume && (h.first != 0 || h.count != e->C.n_groups)) return RBE_E_INVALID;
  if (!resume && h.round != e->round) return RBE_E_STATE;
  const u64 r0 = h.first * e->C.n, nr = h.count * e->C.n;
  std::vector<u64> rec_off(nr);
  if (snap_log_index(e->C, (const u8*)buf, nr, rec_off.data())) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  // the range's pages go back to the pool before its planes are replaced
  const u32 spar = e->round & 1u;
  hipLaunchKernelGGL(k_spill_release, dim3(grid_for(nr)), dim3(kBlock), 0, e->stream, e->P, e->C,
                     r0, nr, spar);
  HIP_OK(hipGetLastError());
  SnapPlane pl[kSnapPlanes];
  snap_planes(e->P, e->C, pl);
  const u8* src = (const u8*)buf + sizeof(SnapHeader);
  for (int i = 0; i < kSnapPlanes && pl[i].rows; i++) {
    const u64 w = h.count * pl[i].group_bytes;
    HIP_OK(hipMemcpy2DAsync(pl[i].base + h.first * pl[i].group_bytes, pl[i].pitch, src, w, w,
                            pl[i].rows, hipMemcpyHostToDevice, e->stream));
    src += w * pl[i].rows;
  }
  {  // the cold logs and pool-page readIndex queues of the log section
    // device staging: fault word | record offsets | the section (16-B aligned)
    const u64 lb = h.log_bytes, ob = (nr * sizeof(u64) + 15) & ~15ull;
    const int rc = grow(&e->gat_dev, &e->gat_dev_bytes, 16 + ob + lb, false);
    if (rc) return rc;
    u32* fault = (u32*)e->gat_dev;
    u64* d_off = (u64*)(e->gat_dev + 16);
    u8* d_sec = e->gat_dev + 16 + ob;
    HIP_OK(hipMemsetAsync(fault, 0, sizeof(u32), e->stream));
    HIP_OK(hipMemcpyAsync(d_off, rec_off.data(), ob, hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipMemcpyAsync(d_sec, (const u8*)buf + snap_log_at(h.body_bytes), lb,
                          hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_snap_log_rebuild, dim3(grid_for(nr)), dim3(kBlock), 0, e->stream, e->P,
                       e->C, r0, nr, (const u8*)d_sec, (const u64*)d_off, spar ^ 1u, fault);
    HIP_OK(hipGetLastError());
    u32 f = 0;
    HIP_OK(hipMemcpyAsync(&f, fault, sizeof(u32), hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (f) return RBE_E_NOMEM;
  }
  {  // the host mirror of the applied plane follows the imported rows
    std::vector<u64> app(h.count * e->C.n);
    HIP_OK(hipMemcpyAsync(app.data(), e->P.applied + h.first * e->C.n, app.size() * sizeof(u64),
                          hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    e->hin.resync_applied(app.data(), h.first * e->C.n, app.size());
  }
  // imported groups start awake (group sleep, rbe_step.h); the next round
  // scans every group to rebuild the awake list and the sleeping totals
  HIP_OK(hipMemsetAsync(e->P.gwake + h.first, GW_AWAKE, h.count, e->stream));
  if (resume) {
    // the whole engine moves to the snapshot's round; the work lists of the
    // coming round start empty, as after any round (k_triage clears them)
    e->round = h.round;
    HIP_OK(hipMemsetAsync(e->L.counts, 0, kListCounts * sizeof(u32), e->stream));
    e->tclk = h.tclk;
    const u32 clk[2] = {e->round, e->tclk};
    HIP_OK(hipMemcpyAsync(e->d_clk, clk, sizeof(clk), hipMemcpyHostToDevice, e->stream));
  }
  // the awake lists and the sleeping totals restart from the scan
  HIP_OK(hipMemsetAsync(e->L.al_cnt, 0, 2 * e->L.al_nblk * sizeof(u32), e->stream));
  HIP_OK(hipMemsetAsync(e->L.slp, 0, 6 * sizeof(u64), e->stream));
  e->scan_at = e->round;
  HIP_OK(hipMemcpyAsync((void*)e->L.scan_round, &e->scan_at, sizeof(u32), hipMemcpyHostToDevice,
                        e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_footprint(const rbe_config* cfg, uint64_t* bytes) {
  Params C;
  int rc = make_params(cfg, &C);
  if (rc) return rc;
  *bytes = bytes_of(C, nullptr) + C.heap_bytes;
  return RBE_OK;
}

int rbe_destroy(rbe_engine* e) {
  if (!e) return RBE_OK;
  HIP_IGNORE(hipSetDevice(e->device));
  if (e->stream) HIP_IGNORE(hipStreamSynchronize(e->stream));
  drop_graphs(e);
  for (void* p : e->allocs) HIP_IGNORE(hipFree(p));
  if (e->d_clk) HIP_IGNORE(hipFree(e->d_clk));
  if (e->ev0) HIP_IGNORE(hipEventDestroy(e->ev0));
  if (e->ev1) HIP_IGNORE(hipEventDestroy(e->ev1));
  for (int i = 0; i < 2; i++) {
    if (e->in_ev[i]) HIP_IGNORE(hipEventDestroy(e->in_ev[i]));
    if (e->in_pinned[i]) HIP_IGNORE(hipHostFree(e->in_pinned[i]));
  }
  if (e->in_dev) HIP_IGNORE(hipFree(e->in_dev));
  if (e->out_dev) HIP_IGNORE(hipFree(e->out_dev));
  if (e->gat_dev) HIP_IGNORE(hipFree(e->gat_dev));
  if (e->out_host) HIP_IGNORE(hipHostFree(e->out_host));
  if (e->upd_dev) HIP_IGNORE(hipFree(e->upd_dev));
  if (e->ing_dev) HIP_IGNORE(hipFree(e->ing_dev));
  if (e->iso_dev) HIP_IGNORE(hipFree(e->iso_dev));
  if (e->upd_host) HIP_IGNORE(hipHostFree(e->upd_host));
  if (e->cs_dev) HIP_IGNORE(hipFree(e->cs_dev));
  if (e->P.prof) HIP_IGNORE(hipFree(e->P.prof));
  if (e->cs_host) HIP_IGNORE(hipHostFree(e->cs_host));
  for (int i = 0; i < 2; i++)
    if (e->csa_buf[i]) HIP_IGNORE(hipHostFree(e->csa_buf[i]));
  if (e->csa_ev) HIP_IGNORE(hipEventDestroy(e->csa_ev));
  if (e->wire_dev) HIP_IGNORE(hipFree(e->wire_dev));
  if (e->wire_meta) HIP_IGNORE(hipFree(e->wire_meta));
  if (e->wire_rec) HIP_IGNORE(hipFree(e->wire_rec));
  if (e->wire_in) HIP_IGNORE(hipFree(e->wire_in));
  if (e->wire_big_buf) HIP_IGNORE(hipFree(e->wire_big_buf));
  if (e->stream) HIP_IGNORE(hipStreamDestroy(e->stream));
  delete e;
  return RBE_OK;
}

int rbe_create(const rbe_config* cfg, rbe_engine** out) {
  if (!out) return RBE_E_INVALID;
  *out = nullptr;
  Params C;
  int rc = make_params(cfg, &C);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RBE_E_NODEV;
  if (cfg->device < 0 || cfg->device >= ndev) return RBE_E_NODEV;
  HIP_OK(hipSetDevice(cfg->device));
  if (!cfg->pool_bytes) {
    // the default page pool grows to an eighth of the free HBM (at most 32
    // GiB): the cold logs keep every entry a LogDB without snapshots keeps, so
    // a long run without compaction needs room in proportion to its rounds
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      const u64 pages = std::min<u64>(fr / 8, 32ull << 30) / (kPageEnts * sizeof(Ent));
      if (pages > C.pool_pages) C.pool_pages = (u32)std::min<u64>(pages, 0xFFFFFFF0ull);
    }
  }
  rbe_engine* e = new (std::nothrow) rbe_engine();
  if (!e) return RBE_E_NOMEM;
  e->cfg = *cfg;
  e->C = C;
  e->device = cfg->device;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    rbe_destroy(e);
    return RBE_E_HIP;
  }
  HIP_IGNORE(hipEventCreate(&e->ev0));
  HIP_IGNORE(hipEventCreate(&e->ev1));
  for (int i = 0; i < 2; i++) {
    HIP_IGNORE(hipEventCreateWithFlags(&e->in_ev[i], hipEventDisableTiming));
    HIP_IGNORE(hipEventRecord(e->in_ev[i], e->stream));
  }
  u64 parts[kPlaneAllocs];
  bytes_of(C, parts);
  void* ptrs[kPlaneAllocs];
  for (int i = 0; i < kPlaneAllocs; i++) {
    u64 b = parts[i] ? parts[i] : 16;
    if (hipMalloc(&ptrs[i], b) != hipSuccess) {
      for (int j = 0; j < i; j++) e->allocs.push_back(ptrs[j]);
      rbe_destroy(e);
      return RBE_E_NOMEM;
    }
    e->allocs.push_back(ptrs[i]);
    if (hipMemsetAsync(ptrs[i], 0, b, e->stream) != hipSuccess) {
      rbe_destroy(e);
      return RBE_E_HIP;
    }
  }
  Planes& P = e->P;
  P.hot = (Hot*)ptrs[0];
  P.core = (Core*)ptrs[1];
  P.rem = (RemoteMN*)ptrs[2];
  P.rem_st = (u8*)ptrs[3];
  P.rq = (ReadReq*)ptrs[4];
  P.term_ring = (u64*)ptrs[5];
  P.pay_ring = (Body*)ptrs[6];
  P.cnt[0] = (CntRow*)ptrs[7];
  P.cnt[1] = P.cnt[0] + C.n_rep;
  u64 msg_half = C.n_groups * C.n * C.n * C.maxm;
  P.msgs[0] = (Msg*)ptrs[8];
  P.msgs[1] = P.msgs[0] + msg_half;
  u64 ar_half = C.n_rep * C.ecap;
  P.arena[0] = (Ent*)ptrs[9];
  P.arena[1] = P.arena[0] + ar_half;
  P.iso_mask = (u8*)ptrs[10];
  P.iso_until = (u32*)ptrs[11];
  P.upd = (Upd*)ptrs[12];
  P.rtr = (RTR*)ptrs[13];
  P.dri = (DropRI*)ptrs[14];
  P.ext = (ExtIn*)ptrs[15];
  P.idle = (u8*)ptrs[16];
  P.in_ents = (Ent*)ptrs[17];
  P.applied = (u64*)ptrs[18];
  P.gwake = (u8*)ptrs[19];
  P.snp = C.snapshot_entries ? (SnapSt*)ptrs[20] : nullptr;
  P.rem_snap = C.snapshot_entries ? (u64*)ptrs[21] : nullptr;
  P.imark = (C.ext_commit || C.rl_max) ? (u64*)ptrs[22] : nullptr;
  P.rl = C.rl_max ? (RlSt*)ptrs[23] : nullptr;
  P.roles = C.membership ? (u16*)ptrs[24] : nullptr;
  P.pool = (Ent*)ptrs[25];
  P.pmeta = (PoolMeta*)ptrs[26];
  P.cold = (ColdRef*)ptrs[27];
  P.spill[0] = (u8*)ptrs[28];
  P.spill[1] = P.spill[0] + C.spill_units * 16;
  P.sctl = (SpillCtl*)ptrs[29];
  // page 0 is the null page: the bump counter starts at 1
  HIP_IGNORE(hipMemsetD32Async((hipDeviceptr_t)&P.sctl->bump, 1, 1, e->stream));
  P.node_ids = nullptr;  // slot s is node s + 1 until rbe_set_node_ids
  P.ids_n = C.n;
  HIP_IGNORE(hipMemsetAsync(P.gwake, GW_AWAKE, C.n_groups, e->stream));  // every group starts awake
  e->hin.init(C.n_rep, C.n, C.in_cap, C.heap_bytes);
  e->hin.owner = C.rep_world > 1 ? &e->C : nullptr;
  if (C.heap_bytes) {
    if (hipMalloc(&e->heap, C.heap_bytes) != hipSuccess ||
        hipMalloc(&e->heap_dev, 2 * sizeof(u64)) != hipSuccess) {
      if (e->heap) e->allocs.push_back(e->heap);
      rbe_destroy(e);
      return RBE_E_NOMEM;
    }
    e->allocs.push_back(e->heap);
    e->allocs.push_back(e->heap_dev);
    HIP_IGNORE(hipMemsetAsync(e->heap_dev, 0, 2 * sizeof(u64), e->stream));
    P.heap_head = e->heap_dev;
    // the lowest live record, on demand (HostHeap::room)
    e->hin.heap.low_fn = [e](u64* lo) -> int {
      HIP_OK(hipSetDevice(e->device));
      const u64 init = ~0ull;
      HIP_OK(hipMemcpyAsync(e->heap_dev + 1, &init, sizeof(u64), hipMemcpyHostToDevice, e->stream));
      int rc = dispatch_n(e->C.n, [&](auto NN) {
        constexpr int N = decltype(NN)::value;
        hipLaunchKernelGGL(k_heap_low<N>, dim3(grid_for(e->C.n_groups)), dim3(kBlock), 0,
                           e->stream, e->P, e->C, e->round, e->heap_dev + 1);
        HIP_OK(hipGetLastError());
        return RBE_OK;
      });
      if (rc) return rc;
      HIP_OK(hipMemcpyAsync(lo, e->heap_dev + 1, sizeof(u64), hipMemcpyDeviceToHost, e->stream));
      HIP_OK(hipStreamSynchronize(e->stream));
      return RBE_OK;
    };
  }
  if (hipMalloc(&P.counters, kCtrWords * sizeof(u64)) != hipSuccess) {
    rbe_destroy(e);
    return RBE_E_NOMEM;
  }
  e->allocs.push_back(P.counters);
  HIP_IGNORE(hipMemsetAsync(P.counters, 0, kCtrWords * sizeof(u64), e->stream));
  if (hipMalloc(&e->d_clk, 2 * sizeof(u32)) != hipSuccess) {
    rbe_destroy(e);
    return RBE_E_NOMEM;
  }
  HIP_IGNORE(hipMemsetAsync(e->d_clk, 0, 2 * sizeof(u32), e->stream));
  if (const char* wb = getenv("RBE_WIRE_BIG")) e->wire_big = strtoull(wb, nullptr, 10);
  if (const char* fg = getenv("RBE_FAST_GRID")) g_fast_grid = (unsigned)strtoul(fg, nullptr, 10);
  const char* mode = getenv("RBE_MODE");
  // default: k_triage → k_fast_both → k_full_list; RBE_MODE=split runs the two
  // roles as separate launches, RBE_MODE=fused k_round + k_full_list,
  // RBE_MODE=full k_step alone
  e->mode = !mode ? 3
                  : (strcmp(mode, "full") == 0    ? 2
                     : strcmp(mode, "fused") == 0 ? 0
                     : strcmp(mode, "split") == 0 ? 1
                                                  : 3);
  if (C.n_rep >= (1ull << 32)) {
    rbe_destroy(e);
    return RBE_E_INVALID;  // list entries are 32-bit replica indices
  }
  {
    // lists 0 and 1 come from k_triage alone: a shard's region holds the
    // replicas of its blocks; list 2 takes pushes from every pipeline kernel,
    // so any shard may get any replica (each at most once per round)
    const u64 gpb = kTriChunk / C.n, nblk = (C.n_groups + gpb - 1) / gpb;
    const u64 per = (nblk + kShards - 1) / kShards * gpb * C.n;
    e->L.scap[0] = e->L.scap[1] = per;
    e->L.scap[2] = C.n_rep;
    e->L.off[0] = 0;
    e->L.off[1] = kShards * per;
    e->L.off[2] = 2 * kShards * per;
  }
  if (hipMalloc(&e->L.idx, (e->L.off[2] + kShards * C.n_rep) * sizeof(u32)) != hipSuccess ||
      hipMalloc(&e->L.aux, e->L.off[2] * sizeof(u32)) != hipSuccess ||
      hipMalloc(&e->L.counts, kListCounts * sizeof(u32)) != hipSuccess) {
    rbe_destroy(e);
    return RBE_E_NOMEM;
  }
  e->allocs.push_back(e->L.idx);
  e->allocs.push_back(e->L.aux);
  e->allocs.push_back(e->L.counts);
  {
    // group sleep in list mode (k_triage): two awake lists of one region per
    // k_triage block, their counts, the sleeping totals and the scan-round
    // word, which starts at round 0 (every group starts awake, round 0 scans)
    const u32 gb = kTriChunk / C.n;
    const u32 nblk = (u32)((C.n_groups + gb - 1) / gb);
    u32* w = nullptr;
    u8* al = nullptr;
    const u64 wbytes = 2 * (u64)nblk * sizeof(u32) + 6 * sizeof(u64) + 256;
    if (hipMalloc(&al, 2 * (u64)nblk * gb * sizeof(u32)) != hipSuccess ||
        hipMalloc(&w, wbytes) != hipSuccess) {
      if (al) HIP_IGNORE(hipFree(al));
      rbe_destroy(e);
      return RBE_E_NOMEM;
    }
    e->allocs.push_back(al);
    e->allocs.push_back(w);
    HIP_IGNORE(hipMemsetAsync(w, 0, wbytes, e->stream));
    e->L.al[0] = (u32*)al;
    e->L.al[1] = (u32*)al + (u64)nblk * gb;
    e->L.al_nblk = nblk;
    e->L.al_gb = gb;
    e->L.slp = (u64*)((u8*)w + ((2 * (u64)nblk * sizeof(u32) + 63) & ~63ull));
    e->L.al_cnt = w;
    e->L.scan_round = (const u32*)(e->L.slp + 6);
    const char* gl = getenv("RBE_GROUP_LIST");  // "0": scan every round (A/B)
    e->L.al_on = C.quiesce && !C.trace && C.rep_world == 1 && (e->mode == 1 || e->mode == 3) &&
                 !(gl && strcmp(gl, "0") == 0);
  }
  e->L.vgrid = 700u;
  if (const char* vg = getenv("RBE_FAST_VGRID")) e->L.vgrid = (u32)strtoul(vg, nullptr, 10);
  // pack counters, then the sticky overflow flag of the fixed-layout exchange
  if (hipMalloc(&e->xcount, (kXchgMaxWorld * XS_NUM + 1) * sizeof(u32)) != hipSuccess) {
    rbe_destroy(e);
    return RBE_E_NOMEM;
  }
  e->allocs.push_back(e->xcount);
  HIP_IGNORE(hipMemsetAsync(e->xcount, 0, (kXchgMaxWorld * XS_NUM + 1) * sizeof(u32), e->stream));
  HIP_IGNORE(hipMemsetAsync(e->L.counts, 0, kListCounts * sizeof(u32), e->stream));
  rc = dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_launch<N>, dim3(grid_for(C.n_rep)), dim3(kBlock), 0, e->stream, e->P,
                       e->C);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  if (rc || hipStreamSynchronize(e->stream) != hipSuccess) {
    rbe_destroy(e);
    return rc ? rc : RBE_E_HIP;
  }
  *out = e;
  return RBE_OK;
}

// fault-schedule epoch rounds: isolate the selected groups' leaders first
static int launch_iso(rbe_engine* e) {
  const Params& C = e->C;
  if (!(C.iso_period && e->round > 0 && e->round % C.iso_period == 0)) return RBE_OK;
  if (C.rep_world > 1) {  // the leaders of groups whose replicas other ranks step
    if (e->iso_round != e->round || !e->iso_dev) return RBE_E_STATE;
    return dispatch_n(C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      hipLaunchKernelGGL(k_iso_set<N>, dim3(grid_for(C.n_groups)), dim3(kBlock), 0, e->stream,
                         e->P, e->C, e->round, (const u8*)e->iso_dev);
      HIP_OK(hipGetLastError());
      return RBE_OK;
    });
  }
  return dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_isolate<N>, dim3(grid_for(C.n_groups)), dim3(kBlock), 0, e->stream,
                       e->P, e->C, e->round);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
}

// Upload the input staged since the last step (rbe_host.h) through the pinned
// buffer in one copy and scatter it on device, ahead of the round's kernels.
static int flush_inputs(rbe_engine* e) {
  auto& h = e->hin;
  if (h.empty()) {
    h.heap.settle();
    return RBE_OK;
  }
  const u32 sl = e->in_slot;
  HIP_OK(hipEventSynchronize(e->in_ev[sl]));  // the upload two flushes back is out of slot sl
  const u64 n = h.reps.size(), na = h.app_rep.size(), nc = h.commits.size(),
            ns = h.snaps.size(), nh = h.heap.head - h.heap.flushed;
  // device layout: replicas | records (16-B aligned) | applied replicas |
  // applied values | commits | snapshot records; the first two come straight
  // from the pinned staging vectors, the rest through in_pinned[sl], which
  // also carries the payload-heap bytes of the staged proposals
  const u64 o_rec = (n * sizeof(u64) + 15) & ~15ull;
  const u64 o_ar = o_rec + n * sizeof(ExtIn), o_av = o_ar + na * sizeof(u64);
  const u64 o_cr = o_av + na * sizeof(u64);
  const u64 o_sr = o_cr + nc * sizeof(CommitRec);
  const u64 total = o_sr + ns * sizeof(SnapRec);
  const u64 small = total - o_ar, pneed = small + nh + 64;
  if (total + 64 > e->in_bytes) {
    if (e->in_dev) HIP_OK(hipFree(e->in_dev));
    e->in_dev = nullptr;
    e->in_bytes = 0;
    const u64 cap = (total + 64) * 2;
    HIP_OK(hipMalloc((void**)&e->in_dev, cap));
    e->in_bytes = cap;
  }
  if (pneed > e->in_pbytes[sl]) {
    if (e->in_pinned[sl]) HIP_OK(hipHostFree(e->in_pinned[sl]));
    e->in_pinned[sl] = nullptr;
    e->in_pbytes[sl] = 0;
    HIP_OK(hipHostMalloc((void**)&e->in_pinned[sl], pneed * 2, hipHostMallocDefault));
    e->in_pbytes[sl] = pneed * 2;
  }
  u8* b = e->in_pinned[sl];
  // payload heap bytes of the staged proposals: positions [flushed, head),
  // split where they cross the end of the ring
  if (nh) {
    memcpy(b + small, h.heap.stage.data(), nh);
    for (u64 p = h.heap.flushed; p < h.heap.head;) {
      const u64 at = p % h.heap.cap, len = std::min(h.heap.head - p, h.heap.cap - at);
      HIP_OK(hipMemcpyAsync(e->heap + at, b + small + (p - h.heap.flushed), len,
                            hipMemcpyHostToDevice, e->stream));
      p += len;
    }
  }
  if (h.heap.head != e->heap_head_host) {  // Planes::heap_head for the lapped-record checks
    e->heap_head_host = h.heap.head;
    HIP_OK(hipMemcpyAsync(e->heap_dev, &e->heap_head_host, sizeof(u64), hipMemcpyHostToDevice,
                          e->stream));
  }
  if (n) {
    HIP_OK(hipMemcpyAsync(e->in_dev, h.reps.data(), n * sizeof(u64), hipMemcpyHostToDevice,
                          e->stream));
    HIP_OK(hipMemcpyAsync(e->in_dev + o_rec, h.recs.data(), n * sizeof(ExtIn),
                          hipMemcpyHostToDevice, e->stream));
  }
  if (na) {
    memcpy(b + (o_ar - o_ar), h.app_rep.data(), na * sizeof(u64));
    memcpy(b + (o_av - o_ar), h.app_val.data(), na * sizeof(u64));
  }
  if (nc) memcpy(b + (o_cr - o_ar), h.commits.data(), nc * sizeof(CommitRec));
  if (ns) memcpy(b + (o_sr - o_ar), h.snaps.data(), ns * sizeof(SnapRec));
  if (small) HIP_OK(hipMemcpyAsync(e->in_dev + o_ar, b, small, hipMemcpyHostToDevice, e->stream));
  if (!h.ents.empty())
    HIP_OK(hipMemcpyAsync(e->P.in_ents, h.ents.data(), h.ents.size() * sizeof(Ent),
                          hipMemcpyHostToDevice, e->stream));
  // three launches in the host build's order (input records and applied /
  // ready pairs, then commits, then snapshot records): a replica may have one
  // of each, and all three write its Hot flags, so no launch holds two lanes of
  // one replica (a launch of heap records alone, from rbe_push_messages, has none)
  const u64 m0 = std::max(n, na);
  for (int ph = 0; ph < 3; ph++) {
    const u64 pn = ph == 0 ? n : 0, pa = ph == 0 ? na : 0, pc = ph == 1 ? nc : 0,
              ps = ph == 2 ? ns : 0;
    const u64 m = ph == 0 ? m0 : (ph == 1 ? nc : ns);
    if (!m) continue;
    hipLaunchKernelGGL(k_ext_scatter, dim3(grid_for(m)), dim3(kBlock), 0, e->stream, e->P,
                       e->C.n, (const u64*)e->in_dev, (const ExtIn*)(e->in_dev + o_rec), pn,
                       (const u64*)(e->in_dev + o_ar), (const u64*)(e->in_dev + o_av), pa,
                       (const CommitRec*)(e->in_dev + o_cr), pc,
                       (const SnapRec*)(e->in_dev + o_sr), ps, e->C, e->L, e->round & 1u);
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipEventRecord(e->in_ev[sl], e->stream));
  // the staging vectors just uploaded become the spares; the spares, whose
  // upload (the last flush, slot sl ^ 1) has long finished, take the next input
  h.reps.swap(e->up_reps);
  h.recs.swap(e->up_recs);
  h.ents.swap(e->up_ents);
  HIP_OK(hipEventSynchronize(e->in_ev[sl ^ 1u]));
  e->in_slot = sl ^ 1u;
  h.clear();
  return RBE_OK;
}

static int step_one(rbe_engine* e, bool tick = true) {
  int rc = flush_inputs(e);
  if (rc) return rc;
  rc = launch_iso(e);
  if (rc) return rc;
  rc = launch_step(e, RoundArg{nullptr, e->round, e->tclk, tick ? 1u : 0u});
  if (rc) return rc;
  e->round++;
  if (tick) e->tclk++;
  return RBE_OK;
}

int rbe_step(rbe_engine* e) {
  if (!e) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  return step_one(e);
}

int rbe_step_ex(rbe_engine* e, uint32_t flags) {
  if (!e || (flags & ~RBE_STEP_NO_TICK)) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  return step_one(e, (flags & RBE_STEP_NO_TICK) == 0);
}

// K rounds as one graph: K step launches reading the round from device memory,
// then one advance of that counter.  The graph does not depend on the round, so
// one capture per K serves every later run of K rounds.
static int graph_for(rbe_engine* e, u32 rounds, hipGraphExec_t* out) {
  for (int i = 0; i < rbe_engine::kGraphs; i++)
    if (e->graph[i] && e->graph_rounds[i] == rounds) {
      *out = e->graph[i];
      return RBE_OK;
    }
  const int slot = (int)(e->graph_next++ % rbe_engine::kGraphs);
  if (e->graph[slot]) {
    HIP_IGNORE(hipGraphExecDestroy(e->graph[slot]));
    e->graph[slot] = nullptr;
  }
  // capture ends every queued round first; the clock copy before the replay
  // (run_graph) gives the launches their round
  HIP_OK(hipStreamSynchronize(e->stream));
  hipGraph_t g;
  HIP_OK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
  for (u32 i = 0; i < rounds; i++) {
    int rc = launch_step(e, RoundArg{e->d_clk, i, i, 1u});
    if (rc) {
      HIP_IGNORE(hipStreamEndCapture(e->stream, &g));
      return rc;
    }
  }
  hipLaunchKernelGGL(k_advance, dim3(1), dim3(1), 0, e->stream, e->d_clk, rounds);
  HIP_OK(hipStreamEndCapture(e->stream, &g));
  HIP_OK(hipGraphInstantiate(&e->graph[slot], g, nullptr, nullptr, 0));
  HIP_IGNORE(hipGraphDestroy(g));
  // the executable's first launch would otherwise upload it
  HIP_OK(hipGraphUpload(e->graph[slot], e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  e->graph_rounds[slot] = rounds;
  *out = e->graph[slot];
  return RBE_OK;
}

static bool graphable(const rbe_engine* e, u32 rounds) {
  return e->C.iso_period == 0 && !e->C.ext_inputs && rounds >= 2 &&
         getenv("RBE_NO_GRAPH") == nullptr;
}

static int run_graph(rbe_engine* e, u32 rounds) {
  hipGraphExec_t gx = nullptr;
  int rc = graph_for(e, rounds, &gx);
  if (rc) return rc;
  const u32 clk[2] = {e->round, e->tclk};
  HIP_OK(hipMemcpyAsync(e->d_clk, clk, sizeof(clk), hipMemcpyHostToDevice, e->stream));
  HIP_OK(hipGraphLaunch(gx, e->stream));
  e->round += rounds;
  e->tclk += rounds;
  return RBE_OK;
}

int rbe_prepare_run(rbe_engine* e, uint32_t rounds) {
  if (!e) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  if (!graphable(e, rounds)) return RBE_OK;
  hipGraphExec_t gx = nullptr;
  return graph_for(e, rounds, &gx);
}

int rbe_run(rbe_engine* e, uint32_t rounds) {
  if (!e) return RBE_E_INVALID;
  if (rounds == 0) return RBE_OK;
  HIP_OK(hipSetDevice(e->device));
  if (graphable(e, rounds)) return run_graph(e, rounds);
  for (u32 i = 0; i < rounds; i++) {
    int rc = step_one(e);
    if (rc) return rc;
  }
  return RBE_OK;
}

int rbe_run_timed(rbe_engine* e, uint32_t rounds, float* ms) {
  if (!e || !ms) return RBE_E_INVALID;
  int rc0 = rbe_prepare_run(e, rounds);  // any capture before the first event
  if (rc0) return rc0;
  HIP_OK(hipEventRecord(e->ev0, e->stream));
  int rc = rbe_run(e, rounds);
  if (rc) return rc;
  HIP_OK(hipEventRecord(e->ev1, e->stream));
  HIP_OK(hipEventSynchronize(e->ev1));
  HIP_OK(hipEventElapsedTime(ms, e->ev0, e->ev1));
  return RBE_OK;
}

int rbe_profile_rounds(rbe_engine* e, uint32_t rounds, float* ms_per_kernel) {
  if (!e || !ms_per_kernel || rounds == 0) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  // a start / stop pair per kernel section, stamped by the kernel's own
  // dispatch (hipExtLaunchKernel in launch_round): kernel time, not the gaps
  hipEvent_t ev[2 * KS_NUM];
  for (int i = 0; i < 2 * KS_NUM; i++) HIP_OK(hipEventCreate(&ev[i]));
  for (int i = 0; i < KS_NUM; i++) ms_per_kernel[i] = 0.f;
  int rc = RBE_OK;
  for (u32 k = 0; k < rounds && rc == RBE_OK; k++) {
    rc = launch_iso(e);
    if (rc) break;
    rc = launch_step(e, RoundArg{nullptr, e->round, e->tclk, 1u}, ev);
    if (rc) break;
    e->round++;
    e->tclk++;
    if (hipStreamSynchronize(e->stream) != hipSuccess) {
      rc = RBE_E_HIP;
      break;
    }
    for (int i = 0; i < KS_NUM; i++) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) == hipSuccess) ms_per_kernel[i] += ms;
    }
  }
  for (int i = 0; i < 2 * KS_NUM; i++) HIP_IGNORE(hipEventDestroy(ev[i]));
  return rc;
}

int rbe_sync(rbe_engine* e) {
  if (!e) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_round(const rbe_engine* e, uint32_t* round) {
  if (!e || !round) return RBE_E_INVALID;
  *round = e->round;
  return RBE_OK;
}

// Node-layer input for the next step (rbe.h; staged host-side, rbe_host.h)
int rbe_push_proposals(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint32_t* n_ents,
                       const uint32_t* type, const uint32_t* cmd_len, const uint8_t* cmd) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.push_proposals(n, replica, n_ents, type, cmd_len, cmd); });
}

int rbe_propose_entries(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint32_t* n_ents,
                        const rbe_entry* ents, const uint8_t* cmd) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.push_entries(n, replica, n_ents, ents, cmd); });
}

int rbe_push_read_index(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* lo,
                        const uint64_t* hi) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.push_read_index(n, replica, lo, hi); });
}

int rbe_request_leader_transfer(rbe_engine* e, uint64_t n, const uint64_t* replica,
                                const uint64_t* target) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.request_leader_transfer(n, replica, target); });
}

int rbe_report_unreachable(rbe_engine* e, uint64_t n, const uint64_t* replica,
                           const uint64_t* node_id) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.report_unreachable(n, replica, node_id); });
}

int rbe_report_snapshot_status(rbe_engine* e, uint64_t n, const uint64_t* replica,
                               const uint64_t* node_id, const uint8_t* reject) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.report_snapshot_status(n, replica, node_id, reject); });
}

int rbe_launch(rbe_engine* e, uint64_t n, const uint64_t* replica, const rbe_launch_state* st_ids,
               const rbe_entry* ents, const uint8_t* cmd) {
  if (!e) return RBE_E_INVALID;
  std::vector<rbe_launch_state> stv;  // votes as internal ids
  if (!e->hin.map_votes(n, replica, st_ids, stv)) return RBE_E_INVALID;
  const rbe_launch_state* st = stv.data();
  if (n && replica) {  // one replica at most once
    std::vector<u64> v(replica, replica + n);
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end()) return RBE_E_INVALID;
  }
  std::vector<u64> terms;
  std::vector<Body> bodies;
  int rc = launch_rows(e->C, e->hin.heap, n, replica, st, ents, cmd, terms, bodies);
  if (rc || n == 0) return rc;
  HIP_OK(hipSetDevice(e->device));
  std::vector<LaunchRec> rec(n);
  u64 off = 0;
  for (u64 i = 0; i < n; i++) {
    rec[i] = LaunchRec{replica[i], st[i].term,           st[i].vote,
                       st[i].commit,     st[i].last_index,     off,
                       st[i].n_entries,  st[i].removed,        st[i].marker,
                       st[i].marker_term, st[i].snapshot_index, st[i].snapshot_term};
    off += st[i].n_entries;
  }
  const u64 b_rec = n * sizeof(LaunchRec), b_t = terms.size() * sizeof(u64);
  const u64 bytes = b_rec + b_t + bodies.size() * sizeof(Body) + 64;
  rc = grow(&e->gat_dev, &e->gat_dev_bytes, bytes, false);  // (engine scratch, as rbe_replace_node)
  if (rc) return rc;
  u8* d = e->gat_dev;
  HIP_OK(hipMemcpyAsync(d, rec.data(), b_rec, hipMemcpyHostToDevice, e->stream));
  if (b_t) {
    HIP_OK(hipMemcpyAsync(d + b_rec, terms.data(), b_t, hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipMemcpyAsync(d + b_rec + b_t, bodies.data(), bodies.size() * sizeof(Body),
                          hipMemcpyHostToDevice, e->stream));
  }
  const u32 ppar = (e->round & 1u) ^ 1u;
  rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_relaunch<N>, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->P, e->C,
                       (const LaunchRec*)d, (u64)n, (const u64*)(d + b_rec),
                       (const Body*)(d + b_rec + b_t), ppar, e->tclk);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  // the next round scans every group (group sleep: the relaunched groups are awake)
  e->scan_at = e->round;
  HIP_OK(hipMemcpyAsync((void*)e->L.scan_round, &e->scan_at, sizeof(u32), hipMemcpyHostToDevice,
                        e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return rc;
}

int rbe_set_apply_ready(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint8_t* ready) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.set_apply_ready(n, replica, ready); });
}

int rbe_propose_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica,
                              const uint32_t* type, const uint64_t* node_id) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.propose_config_change(n, replica, type, node_id); });
}

int rbe_apply_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica,
                            const uint64_t* node_id, const uint32_t* type) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.membership || !e->C.ext_apply) return RBE_E_STATE;
  // raft's membership of each replica now, for the check that no node lands
  // in two of raft's maps (HostInputs::apply_config_change)
  std::vector<u32> ms(n);
  if (n && replica) {
    for (u64 i = 0; i < n; i++)
      if (replica[i] >= e->C.n_rep) return RBE_E_INVALID;
    HIP_OK(hipSetDevice(e->device));
    // one gather kernel in the engine's scratch buffer: replicas in, packed
    // memberships out, one copy each way
    const u64 ob = (n * sizeof(u64) + 15) & ~15ull;
    const int rc = grow(&e->gat_dev, &e->gat_dev_bytes, ob + n * sizeof(u32), false);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(e->gat_dev, replica, n * sizeof(u64), hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_ms_gather, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->P,
                       (const u64*)e->gat_dev, (u64)n, (u32*)(e->gat_dev + ob));
    HIP_OK(hipGetLastError());
    HIP_OK(hipMemcpyAsync(ms.data(), e->gat_dev + ob, n * sizeof(u32), hipMemcpyDeviceToHost,
                          e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
  }
  return abi_nomem([&] { return e->hin.apply_config_change(n, replica, node_id, type, false, ms.data()); });
}

int rbe_reject_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.apply_config_change(n, replica, nullptr, nullptr, true); });
}

int rbe_snapshot_saved(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* index,
                       const uint64_t* term, const uint32_t* removed) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.snapshot_entries || !e->C.ext_apply) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.snapshot_op(n, replica, SR_SAVE, index, term, removed, e->C.membership != 0); });
}

int rbe_compact(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* to) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.snapshot_entries || !e->C.ext_apply) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.snapshot_op(n, replica, SR_COMPACT, to, nullptr, nullptr, false); });
}

int rbe_set_node_ids(rbe_engine* e, uint64_t first_group, uint64_t count, const uint64_t* ids) {
  if (!e) return RBE_E_INVALID;
  if (e->round != 0) return RBE_E_STATE;  // messages in flight name slots by node id
  int rc = e->hin.set_node_ids(e->C.n_groups, first_group, count, ids);
  if (rc || count == 0) return rc;
  HIP_OK(hipSetDevice(e->device));
  const u64 bytes = e->hin.ids.size() * sizeof(u64);
  if (!e->P.node_ids) {
    u64* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return RBE_E_NOMEM;
    e->allocs.push_back(d);
    e->P.node_ids = d;
  }
  HIP_OK(hipMemcpyAsync((void*)e->P.node_ids, e->hin.ids.data(), bytes, hipMemcpyHostToDevice,
                        e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  drop_graphs(e);  // kernels take the planes by value: a captured graph holds the old ones
  return RBE_OK;
}

int rbe_replace_node(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* node_id) {
  if (!e) return RBE_E_INVALID;
  int rc = e->hin.replace_args(n, replica, node_id);
  if (rc) return rc;
  // the check reads every replica of the group: group-per-GPU only; and the
  // seeded schedules name slots, not nodes
  if (!e->C.membership || e->C.rep_world > 1 || e->C.cc_period || e->C.xfer_period)
    return RBE_E_STATE;
  if (n == 0) return RBE_OK;
  HIP_OK(hipSetDevice(e->device));
  // (the engine's scratch buffer: no allocation per call, nothing to free on
  // an error path; every user synchronizes before it returns)
  rc = grow(&e->gat_dev, &e->gat_dev_bytes, n * sizeof(u64) + n * sizeof(u32), false);
  if (rc) return rc;
  u64* d = (u64*)e->gat_dev;
  u32* dref = (u32*)(d + n);
  std::vector<u32> refd(n);
  HIP_OK(hipMemcpyAsync(d, replica, n * sizeof(u64), hipMemcpyHostToDevice, e->stream));
  rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_replace_check<N>, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->P,
                       e->C, (const u64*)d, (u64)n, e->round, dref);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  if (!rc) {
    HIP_OK(hipMemcpyAsync(refd.data(), dref, n * sizeof(u32), hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    for (u64 i = 0; i < n && !rc; i++)
      if (refd[i]) rc = RBE_E_STATE;
  }
  if (rc) return rc;
  for (u64 i = 0; i < n; i++) e->hin.assign_node(e->C.n_groups, replica[i], node_id[i]);
  const u64 bytes = e->hin.ids.size() * sizeof(u64);
  if (!e->P.node_ids) {
    u64* t = nullptr;
    if (hipMalloc(&t, bytes) != hipSuccess) return RBE_E_NOMEM;
    e->allocs.push_back(t);
    e->P.node_ids = t;
    drop_graphs(e);  // kernels take the planes by value
    HIP_OK(hipMemcpyAsync((void*)e->P.node_ids, e->hin.ids.data(), bytes, hipMemcpyHostToDevice,
                          e->stream));
  } else {
    for (u64 i = 0; i < n; i++)
      HIP_OK(hipMemcpyAsync((void*)(e->P.node_ids + replica[i]), &e->hin.ids[replica[i]],
                            sizeof(u64), hipMemcpyHostToDevice, e->stream));
  }
  const u32 ppar = (e->round & 1u) ^ 1u;
  rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_join<N>, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->P, e->C,
                       (const u64*)d, (u64)n, ppar, e->tclk);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  // the next round scans every group (group sleep: the new node's group is awake)
  e->scan_at = e->round;
  HIP_OK(hipMemcpyAsync((void*)e->L.scan_round, &e->scan_at, sizeof(u32), hipMemcpyHostToDevice,
                        e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return rc;
}

int rbe_restore_remotes(rbe_engine* e, uint64_t n, const uint64_t* replica,
                        const uint32_t* n_voters, const uint64_t* voter_ids) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.restore_remotes(n, replica, n_voters, voter_ids); });
}

int rbe_notify_applied(rbe_engine* e, uint64_t n, const uint64_t* replica,
                       const uint64_t* applied) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_apply) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.notify_applied(n, replica, applied); });
}

// Diagnostic: the k_full_list wave records of an RBE_FULL_PROF build since
// the last call (4 words each: wall-clock span, two lane-class masks, lanes |
// max inbound << 8 | max outbound << 24), at most cap of them, and clear.  The
// first call allocates the record buffer (and drops a captured graph, whose
// kernels hold the planes by value); without RBE_FULL_PROF nothing is recorded.
extern "C" int rbe_debug_full_prof(rbe_engine* e, uint64_t* out, uint64_t cap, uint64_t* n) {
  if (!e || !n) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  if (!e->P.prof) {
    HIP_OK(hipMalloc((void**)&e->P.prof, (kProfHdr + 4 * kFullProfCap) * sizeof(u64)));
    HIP_OK(hipMemset(e->P.prof, 0, kProfHdr * sizeof(u64)));  // counter | phase sums (rbe_debug_phases)
    drop_graphs(e);
    *n = 0;
    return RBE_OK;
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  u64 cnt = 0;
  HIP_OK(hipMemcpy(&cnt, e->P.prof, sizeof(u64), hipMemcpyDeviceToHost));
  const u64 m = std::min<u64>(std::min<u64>(cnt, kFullProfCap), cap);
  if (m && out) HIP_OK(hipMemcpy(out, e->P.prof + kProfHdr, m * 4 * sizeof(u64), hipMemcpyDeviceToHost));
  *n = cnt;
  HIP_OK(hipMemset(e->P.prof, 0, sizeof(u64)));
  return RBE_OK;
}

// Diagnostic: the general steps longer than 20 us of an RBE_FULL_ITEM_PROF
// build since the last call (8 words each, rbe_step.h step_replica), at most
// cap of them, and clear (the buffer comes from rbe_debug_full_prof).
extern "C" int rbe_debug_full_items(rbe_engine* e, uint64_t* out, uint64_t cap, uint64_t* n) {
  if (!e || !n) return RBE_E_INVALID;
  if (!e->P.prof) return rbe_debug_full_prof(e, nullptr, 0, n);
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipStreamSynchronize(e->stream));
  u64 cnt = 0;
  HIP_OK(hipMemcpy(&cnt, e->P.prof + 1, sizeof(u64), hipMemcpyDeviceToHost));
  const u64 m = std::min<u64>(std::min<u64>(cnt, kFullItemCap), cap);
  if (m && out) HIP_OK(hipMemcpy(out, e->P.prof + kProfHdr, m * 8 * sizeof(u64), hipMemcpyDeviceToHost));
  *n = cnt;
  HIP_OK(hipMemset(e->P.prof + 1, 0, sizeof(u64)));
  return RBE_OK;
}

// Diagnostic: the per-phase stamp sums of an RBE_PHASE_TIMING build (24
// words: leader, follower, k_triage x 8 phases; rbe_fast.h) since the last
// call, and clear.  The first call allocates the buffer (Planes::prof).
extern "C" int rbe_debug_phases(rbe_engine* e, uint64_t* out24) {
  uint64_t n = 0;
  if (!e || !out24) return RBE_E_INVALID;
  if (!e->P.prof) return rbe_debug_full_prof(e, nullptr, 0, &n);
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipStreamSynchronize(e->stream));
  HIP_OK(hipMemcpy(out24, e->P.prof + 8, 24 * sizeof(u64), hipMemcpyDeviceToHost));
  HIP_OK(hipMemset(e->P.prof + 8, 0, 24 * sizeof(u64)));
  return RBE_OK;
}

int rbe_xchg_record_bytes(uint64_t* out3) {
  if (!out3) return RBE_E_INVALID;
  for (u32 t = 0; t < XS_NUM; t++) out3[t] = kXRecBytes[t];
  return RBE_OK;
}

int rbe_xchg_pack(rbe_engine* e, void* buf, const uint64_t* cap3, uint32_t* counts) {
  if (!e || !buf || !cap3 || !counts || e->round == 0) return RBE_E_INVALID;
  // heap positions are this engine's: entries cross engines through
  // rbe_get_outbox / rbe_push_messages, which carry their bytes
  if (e->C.rep_world <= 1 || e->C.heap_bytes) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  XchgCaps caps;
  for (u32 t = 0; t < XS_NUM; t++) caps.cap[t] = cap3[t];
  const u32 par = (e->round - 1) & 1u, nc = e->C.rep_world * XS_NUM;
  HIP_OK(hipMemsetAsync(e->xcount, 0, nc * sizeof(u32), e->stream));
  int rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_xchg_pack<N>, dim3(grid_for(e->C.n_rep)), dim3(kBlock), 0, e->stream,
                       e->P, e->C, par, e->round, (u8*)buf, caps, e->xcount, (u64)0);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(counts, e->xcount, nc * sizeof(u32), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u32 i = 0; i < nc; i++)
    if (counts[i] > cap3[i % XS_NUM]) return RBE_E_NOMEM;  // a region overflowed
  return RBE_OK;
}

int rbe_xchg_chunk_bytes(const uint64_t* cap3, uint64_t* bytes) {
  if (!cap3 || !bytes) return RBE_E_INVALID;
  *bytes = xchg_chunk_bytes(cap3, kXHdrBytes);
  return RBE_OK;
}

int rbe_xchg_pack_fixed(rbe_engine* e, void* buf, const uint64_t* cap3) {
  if (!e || !buf || !cap3 || e->round == 0) return RBE_E_INVALID;
  if (e->C.rep_world <= 1 || e->C.heap_bytes) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  XchgCaps caps;
  for (u32 t = 0; t < XS_NUM; t++) caps.cap[t] = cap3[t];
  const u32 par = (e->round - 1) & 1u, nc = e->C.rep_world * XS_NUM;
  HIP_OK(hipMemsetAsync(e->xcount, 0, nc * sizeof(u32), e->stream));
  int rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_xchg_pack<N>, dim3(grid_for(e->C.n_rep)), dim3(kBlock), 0, e->stream,
                       e->P, e->C, par, e->round, (u8*)buf, caps, e->xcount, kXHdrBytes);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  if (rc) return rc;
  hipLaunchKernelGGL(k_xchg_hdr, dim3(1), dim3(64), 0, e->stream, (u8*)buf, caps,
                     (const u32*)e->xcount, e->C.rep_world, e->C.rep_rank,
                     e->xcount + kXchgMaxWorld * XS_NUM);
  HIP_OK(hipGetLastError());
  return RBE_OK;  // no host synchronisation: the counts travel in the chunk headers
}

int rbe_xchg_unpack_fixed(rbe_engine* e, const void* recv, const uint64_t* cap3) {
  if (!e || !recv || !cap3 || e->round == 0) return RBE_E_INVALID;
  if (e->C.rep_world <= 1) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  XchgCaps caps;
  for (u32 t = 0; t < XS_NUM; t++) caps.cap[t] = cap3[t];
  const u32 par = (e->round - 1) & 1u;
  // count words first (they wake the destination groups), then messages, entries
  for (u32 t = 0; t < XS_NUM; t++) {
    const u64 n = caps.cap[t] * e->C.rep_world;
    if (n)
      hipLaunchKernelGGL(k_xchg_put_fixed, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->P,
                         e->C, par, (const u8*)recv, caps, e->C.rep_world, t,
                         e->xcount + kXchgMaxWorld * XS_NUM);
  }
  HIP_OK(hipGetLastError());
  return RBE_OK;
}

int rbe_xchg_status(rbe_engine* e, uint32_t* overflow) {
  if (!e || !overflow) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipMemcpyAsync(overflow, e->xcount + kXchgMaxWorld * XS_NUM, sizeof(u32),
                        hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemsetAsync(e->xcount + kXchgMaxWorld * XS_NUM, 0, sizeof(u32), e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_stream(rbe_engine* e, void** stream) {
  if (!e || !stream) return RBE_E_INVALID;
  *stream = (void*)e->stream;
  return RBE_OK;
}

// scatter exchange records (device pointers) into the planes of the last
// round's parity (stale outbox headers of silent senders read as empty)
static int xchg_scatter(rbe_engine* e, const void* cnt, uint64_t n_cnt, const void* msg,
                        uint64_t n_msg, const void* ent, uint64_t n_ent) {
  const u32 par = (e->round - 1) & 1u;
  if (n_cnt)
    hipLaunchKernelGGL(k_xchg_put_cnt, dim3(grid_for(n_cnt)), dim3(kBlock), 0, e->stream, e->P,
                       e->C, par, (const XCnt*)cnt, n_cnt);
  if (n_msg)
    hipLaunchKernelGGL(k_xchg_put_msg, dim3(grid_for(n_msg)), dim3(kBlock), 0, e->stream, e->P,
                       e->C, par, (const XMsg*)msg, n_msg);
  if (n_ent)
    hipLaunchKernelGGL(k_xchg_put_ent, dim3(grid_for(n_ent)), dim3(kBlock), 0, e->stream, e->P,
                       e->C, par, (const XEnt*)ent, n_ent);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_xchg_unpack(rbe_engine* e, const void* cnt, uint64_t n_cnt, const void* msg, uint64_t n_msg,
                    const void* ent, uint64_t n_ent) {
  if (!e || e->round == 0) return RBE_E_INVALID;
  if (e->C.rep_world <= 1) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  return xchg_scatter(e, cnt, n_cnt, msg, n_msg, ent, n_ent);
}

int rbe_get_outbox(rbe_engine* e, uint64_t replica, rbe_message* out, uint32_t cap,
                   uint32_t* n_out, rbe_entry* ents, uint32_t ent_cap, uint32_t* n_ents,
                   uint8_t* cmd, uint64_t cmd_cap, uint64_t* cmd_bytes) {
  if (!e || !n_out || !n_ents || replica >= e->C.n_rep || e->round == 0) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  const u32 N = e->C.n, par = (e->round - 1) & 1u;
  const u64 g = replica / N;
  const u32 k = (u32)(replica % N);
  CntRow row;
  std::vector<Msg> lst((size_t)N * e->C.maxm);
  std::vector<Ent> arena(e->C.ecap);
  HIP_OK(hipMemcpyAsync(&row, e->P.cnt[par] + replica, sizeof(row), hipMemcpyDeviceToHost,
                        e->stream));
  HIP_OK(hipMemcpyAsync(lst.data(), e->P.msgs[par] + (g * N + k) * N * (u64)e->C.maxm,
                        lst.size() * sizeof(Msg), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(arena.data(), e->P.arena[par] + replica * e->C.ecap,
                        arena.size() * sizeof(Ent), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  // the lists in reading order (spilled ones from the spill heap), and the
  // entries of messages that carry theirs in the spill heap (rbe_spill.h)
  std::vector<std::vector<Msg>> lists(N);
  std::unordered_map<u64, std::vector<Ent>> xents;  // granule → entries
  for (u32 d = 0; d < N; d++) {
    int rc = host_list(e, par, replica * N + d, row_word(row, d, k, e->round), &lst[d * e->C.maxm],
                       lists[d]);
    if (rc) return rc;
    for (const Msg& m : lists[d]) {
      if (!(m.pad0 & kMsgXEnt) || xents.count(m.ent_off)) continue;
      std::vector<Ent>& v = xents[m.ent_off];
      v.resize(msg_nent(m));
      HIP_OK(hipMemcpyAsync(v.data(), e->P.spill[par] + (u64)m.ent_off * 16, v.size() * sizeof(Ent),
                            hipMemcpyDeviceToHost, e->stream));
    }
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  auto list = [&](u32 d) -> const std::vector<Msg>& { return lists[d]; };
  auto ent = [&](const Msg& m, u32 j) -> Ent {
    return (m.pad0 & kMsgXEnt) ? xents[m.ent_off][j] : arena[m.ent_off + j];
  };
  auto rd = [e](u64 pos, u64 off, u64 len, u8* dst) { return read_heap(e, pos, off, len, dst); };
  const int rc = dispatch_n(N, [&](auto NN) {
    constexpr int NC = decltype(NN)::value;
    return outbox_messages<NC>(e->C, g, k, row, e->round, list, ent, out, cap, ents, ent_cap, n_out,
                               n_ents, cmd, cmd_cap, cmd_bytes, e->hin.id_table(), rd);
  });
  HIP_OK(hipStreamSynchronize(e->stream));  // heap reads
  return rc;
}

int rbe_push_messages(rbe_engine* e, uint64_t n, const uint64_t* group, const rbe_message* msgs,
                      const rbe_entry* ents, const uint8_t* cmd) {
  if (!e || e->round == 0 || (n && (!group || !msgs))) return RBE_E_INVALID;
  if (e->C.rep_world <= 1) return RBE_E_STATE;  // every sender is stepped here
  HIP_OK(hipSetDevice(e->device));
  std::vector<XCnt> c;
  std::vector<XMsg> m;
  std::vector<XEnt> x;
  int rc = dispatch_n(e->C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    return messages_to_records<N>(e->C, e->hin.heap, e->round, n, group, msgs, ents, cmd, c, m,
                                  x, e->hin.id_table());
  });
  if (rc) return rc;
  const size_t bytes = c.size() * sizeof(XCnt) + m.size() * sizeof(XMsg) + x.size() * sizeof(XEnt);
  u8* d = nullptr;
  if (bytes) HIP_OK(hipMalloc(&d, bytes));
  const size_t om = c.size() * sizeof(XCnt), ox = om + m.size() * sizeof(XMsg);
  if (!c.empty()) HIP_OK(hipMemcpyAsync(d, c.data(), om, hipMemcpyHostToDevice, e->stream));
  if (!m.empty())
    HIP_OK(hipMemcpyAsync(d + om, m.data(), ox - om, hipMemcpyHostToDevice, e->stream));
  if (!x.empty())
    HIP_OK(hipMemcpyAsync(d + ox, x.data(), bytes - ox, hipMemcpyHostToDevice, e->stream));
  rc = xchg_scatter(e, d, c.size(), d + om, m.size(), d + ox, x.size());
  if (d) HIP_IGNORE(hipFree(d));
  return rc;
}

int rbe_kernel_name(const rbe_engine* e, int32_t kernel, char* buf, uint32_t cap) {
  if (!e || !buf || cap == 0 || kernel < 0 || kernel >= KS_NUM) return RBE_E_INVALID;
  static const char* names[4][KS_NUM] = {
      {"k_round", "", "", "k_full_list"},
      {"k_triage", "k_fast_list<LEAD>", "k_fast_list<FOLL>", "k_full_list"},
      {"", "", "", "k_step"},
      {"k_triage", "k_fast_both", "", "k_full_list"}};
  const char* n = names[e->mode][kernel];
  strncpy(buf, n, cap - 1);
  buf[cap - 1] = 0;
  return RBE_OK;
}

int rbe_get_kernel_counters(rbe_engine* e, int32_t kernel, uint64_t* out) {
  if (!e || !out || kernel < 0 || kernel >= KS_NUM) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  return read_counters(e, kernel, out);
}

int rbe_get_counters(rbe_engine* e, uint64_t* out) {
  if (!e || !out) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  return read_counters(e, -1, out);
}

int rbe_reset_counters(rbe_engine* e) {
  if (!e) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipMemsetAsync(e->P.counters, 0, kCtrWords * sizeof(u64), e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_rate_limited(rbe_engine* e, uint64_t first, uint64_t count, uint8_t* limited,
                     uint64_t* in_mem_log_size) {
  if (!e || count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first) return RBE_E_INVALID;
  if (!e->P.rl) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  std::vector<RlSt> rl(count);
  if (d2h(e, rl.data(), e->P.rl + first, count)) return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u64 i = 0; i < count; i++) {
    if (limited) limited[i] = rl_limited(rl[i], e->C.rl_max) ? 1 : 0;
    if (in_mem_log_size) in_mem_log_size[i] = rl[i].size;
  }
  return RBE_OK;
}

int rbe_get_views(rbe_engine* e, uint64_t first, uint64_t count, rbe_replica_view* out) {
  if (!e || !out || first + count > e->C.n_rep) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  const u32 N = e->C.n;
  std::vector<Hot> hot(count);
  std::vector<Core> core(count);
  std::vector<RemoteMN> rem(count * N);
  std::vector<u8> rst(count * N);
  std::vector<Upd> upd(count);
  std::vector<u16> roles(count, 0);
  if (d2h(e, hot.data(), e->P.hot + first, count) || d2h(e, core.data(), e->P.core + first, count) ||
      d2h(e, rem.data(), e->P.rem + first * N, count * N) ||
      d2h(e, rst.data(), e->P.rem_st + first * N, count * N) ||
      d2h(e, upd.data(), e->P.upd + first, count) ||
      (e->C.membership && d2h(e, roles.data(), e->P.roles + first, count)))
    return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  // the length of a readIndex queue in pool pages (its descriptor in ring slot 0)
  std::vector<u32> rqx_len(count, 0);
  for (u64 i = 0; i < count; i++) {
    if (core[i].rq_count != kRqExt) continue;
    ReadReq d;
    HIP_OK(hipMemcpy(&d, e->P.rq + (first + i) * e->C.rq_cap, sizeof(d), hipMemcpyDeviceToHost));
    rqx_len[i] = (u32)(d.high >> 32);
  }
  for (u64 i = 0; i < count; i++) {
    rbe_replica_view& v = out[i];
    memset(&v, 0, sizeof(v));
    const Hot h = materialize_hot(hot[i], e->C, e->tclk);
    const Core& c = core[i];
    v.term = c.term;
    v.vote = ext_id(e->hin.id_table(), N, (first + i) / N, c.vote);
    v.leader_id = ext_id(e->hin.id_table(), N, (first + i) / N, c.leader);
    v.committed = c.committed;
    v.last_index = c.last_index;
    v.processed = c.processed;
    v.saved_to = c.saved_to;
    v.digest = upd[i].digest;
    v.role = h.role;
    v.election_tick = h.election_tick;
    v.heartbeat_tick = h.heartbeat_tick;
    v.rand_election_timeout = h.rand_et;
    v.q_tick = h.q_tick;
    v.q_quiesced_since = h.q_quiesced_since;
    v.q_no_activity_since = h.q_no_activity_since;
    v.q_exit_quiesce_tick = h.q_exit_quiesce_tick;
    v.raft_quiesce = (h.flags & HF_RAFT_QUIESCE) ? 1 : 0;
    v.rq_count = c.rq_count == kRqExt ? rqx_len[i] : c.rq_count;
    v.votes_resp = h.votes_resp;
    v.votes_granted = h.votes_granted;
    v.events = (e->round > 0 && upd[i].round == e->round - 1) ? upd[i].events : 0u;
    v.removed = c.members & MB_REMOVED;
    if (c.mflags & MB_ROLES) {  // Planes::roles is only current while MB_ROLES is set
      v.observers = roles[i] & 0xFFu;
      v.witnesses = roles[i] >> 8;
    }
    if (h.role == R_Leader) {
      for (u32 s = 0; s < N && s < 8; s++) {
        // remotes, observers and witnesses
        if ((v.removed >> s) & ~((v.observers | v.witnesses) >> s) & 1u) continue;
        v.match[s] = rem[i * N + s].match;
        v.next[s] = rem[i * N + s].next;
        v.rstate[s] = rst[i * N + s] & 3;
        v.ractive[s] = (rst[i * N + s] >> 2) & 1;
      }
    }
  }
  return RBE_OK;
}

int rbe_get_updates(rbe_engine* e, uint64_t first, uint64_t count, rbe_update* out) {
  if (!e || !out || first + count > e->C.n_rep) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  std::vector<Upd> upd(count);
  std::vector<Core> core(count);
  std::vector<Hot> hot(count);
  if (d2h(e, upd.data(), e->P.upd + first, count) || d2h(e, core.data(), e->P.core + first, count) ||
      d2h(e, hot.data(), e->P.hot + first, count))
    return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u64 i = 0; i < count; i++) {
    update_view(upd[i], core[i], hot[i], e->round, out[i]);
    update_ids(out[i], e->hin.id_table(), e->C.n, (first + i) / e->C.n);
  }
  return RBE_OK;
}

int rbe_get_update_commits(rbe_engine* e, uint64_t first, uint64_t count, rbe_update_commit* out) {
  if (!e || !out || first + count > e->C.n_rep) return RBE_E_INVALID;
  if (!e->C.ext_commit) return RBE_E_STATE;
  std::vector<rbe_update> u(count);
  int rc = rbe_get_updates(e, first, count, u.data());
  if (rc) return rc;
  std::vector<Core> core(count);
  std::vector<u64> app(count);
  std::vector<SnapSt> snp(e->C.snapshot_entries ? count : 0);
  if (d2h(e, core.data(), e->P.core + first, count) || d2h(e, app.data(), e->P.applied + first, count))
    return RBE_E_HIP;
  if (!snp.empty() && d2h(e, snp.data(), e->P.snp + first, count)) return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u64 i = 0; i < count; i++) {
    const u64 r = first + i;
    int trc = RBE_OK;
    auto term_of = [&](u64 idx) -> u64 {
      if (idx == core[i].last_index) return core[i].t_last;
      // the log moved since the step (a relaunch): read the log
      std::vector<u64> t;
      std::vector<Body> b;
      const int x = read_window(e, r, idx, idx, t, b);
      if (x) {
        trc = x;
        return 0;
      }
      return t[0];
    };
    update_commit_view(u[i], app[i], snp.empty() ? 0 : snp[i].marker, term_of, out[i]);
    if (trc) return trc;
  }
  return RBE_OK;
}

int rbe_commit(rbe_engine* e, uint64_t n, const uint64_t* replica, const rbe_update_commit* uc) {
  if (!e) return RBE_E_INVALID;
  if (!e->C.ext_commit) return RBE_E_STATE;
  return abi_nomem([&] { return e->hin.commit(n, replica, uc); });
}

int rbe_get_update_snapshots(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* out4) {
  if (!e || !out4 || first + count > e->C.n_rep || count == 0) return RBE_E_INVALID;
  std::vector<rbe_update> u(count);
  int rc = rbe_get_updates(e, first, count, u.data());
  if (rc) return rc;
  std::vector<SnapSt> snp(e->C.snapshot_entries ? count : 0);
  if (!snp.empty()) {
    if (d2h(e, snp.data(), e->P.snp + first, count)) return RBE_E_HIP;
    HIP_OK(hipStreamSynchronize(e->stream));
  }
  for (u64 i = 0; i < count; i++)
    update_snapshot_row(u[i], snp.empty() ? nullptr : &snp[i], out4 + 4 * i);
  return RBE_OK;
}

int rbe_get_snapshot_state(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* out8) {
  if (!e || !out8 || first + count > e->C.n_rep || count == 0) return RBE_E_INVALID;
  if (!e->C.snapshot_entries) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  std::vector<SnapSt> v(count);
  if (d2h(e, v.data(), e->P.snp + first, count)) return RBE_E_HIP;
  HIP_OK(hipStreamSynchronize(e->stream));
  for (u64 i = 0; i < count; i++) snap_state_row(v[i], out8 + 8 * i);
  return RBE_OK;
}

// One message list in reading order, from its count word and the host copy of
// its plane slots (`pl`); a spilled list is read from the round spill heap
// (rbe_spill.h list_view)
static int host_list(rbe_engine* e, u32 par, u64 li, u32 w, const Msg* pl, std::vector<Msg>& out) {
  out.clear();
  const Msg* base = pl;
  u32 cap = e->C.maxm, na = w & 0x7Fu, nb = (w >> 7) & 0x7Fu;
  std::vector<Msg> blk;
  if (w & kCntSpill) {
    const Msg h = pl[0];
    cap = h.pad1;
    na = (u32)h.log_index;
    nb = (u32)h.commit;
    blk.resize(cap);
    HIP_OK(hipMemcpyAsync(blk.data(), e->P.spill[par] + h.hint * 16, (u64)cap * sizeof(Msg),
                          hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    base = blk.data();
  }
  (void)li;
  for (u32 i = 0; i < na + nb; i++) out.push_back(base[i < na ? i : cap - 1u - (i - na)]);
  return RBE_OK;
}

int rbe_get_messages(rbe_engine* e, uint64_t replica, rbe_message* out, uint32_t cap,
                     uint32_t* n_out) {
  if (!e || !n_out || replica >= e->C.n_rep || e->round == 0) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  const u32 N = e->C.n, par = (e->round - 1) & 1u;
  const u64 g = replica / N;
  const u32 k = (u32)(replica % N);
  CntRow row;
  HIP_OK(hipMemcpyAsync(&row, e->P.cnt[par] + replica, sizeof(row), hipMemcpyDeviceToHost,
                        e->stream));
  std::vector<Msg> lst((size_t)N * e->C.maxm);
  HIP_OK(hipMemcpyAsync(lst.data(), e->P.msgs[par] + (g * N + k) * N * (u64)e->C.maxm,
                        lst.size() * sizeof(Msg), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u32 n = 0;
  for (u32 d = 0; d < N; d++) {
    std::vector<Msg> ms;
    const int rc = host_list(e, par, replica * N + d, row_word(row, d, k, e->round),
                             &lst[d * e->C.maxm], ms);
    if (rc) return rc;
    for (const Msg& m : ms) {
      if (n < cap && out) msg_out(m, cid_of(e->C, g), e->hin.id_table(), N, g, out[n]);
      n++;
    }
  }
  *n_out = n;
  return RBE_OK;
}

// grow a device (pinned = false) or pinned host buffer to at least `need` bytes
static int grow(u8** p, u64* have, u64 need, bool pinned) {
  if (need <= *have) return RBE_OK;
  if (*p) HIP_OK(pinned ? hipHostFree(*p) : hipFree(*p));
  *p = nullptr;
  *have = 0;
  const u64 cap = need + need / 2 + 4096;
  if (pinned) HIP_OK(hipHostMalloc((void**)p, cap, hipHostMallocDefault));
  else HIP_OK(hipMalloc((void**)p, cap));
  *have = cap;
  return RBE_OK;
}

int rbe_collect_outputs(rbe_engine* e, uint64_t first, uint64_t count, rbe_outputs* out) {
  if (!e || !out || count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first)
    return RBE_E_INVALID;
  memset(out, 0, sizeof(*out));
  out->first = first;
  out->count = count;
  if (e->round == 0) return RBE_E_STATE;  // no round has run yet
  HIP_OK(hipSetDevice(e->device));
  const u32 nb = grid_for(count);
  const u64 a8 = 256;
  auto al = [&](u64 x) { return (x + a8 - 1) & ~(a8 - 1); };
  // device scratch: block sums | block prefixes (+ totals) | offsets | records
  const u64 o_pre = al(2ull * nb * sizeof(u32)), o_moff = o_pre + al(scan_words(2, nb) * sizeof(u64));
  const u64 o_roff = o_moff + al((count + 1) * sizeof(u64));
  const u64 o_rec = o_roff + al((count + 1) * sizeof(u64));
  int rc = grow(&e->out_dev, &e->out_dev_bytes, o_rec, false);
  if (rc) return rc;
  u32* bsum = (u32*)e->out_dev;
  u64* pre = (u64*)(e->out_dev + o_pre);
  hipLaunchKernelGGL(k_out_count, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, bsum);
  if ((rc = launch_scan<2>(e->stream, bsum, nb, pre))) return rc;
  u64 tot[2];
  HIP_OK(hipMemcpyAsync(tot, pre + 2ull * nb, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  const u64 o_rtr = o_rec + al(tot[0] * sizeof(rbe_message));
  const u64 need = o_rtr + al(tot[1] * sizeof(rbe_ready_to_read));
  if (need > e->out_dev_bytes) {  // keep the block prefixes across the regrow
    std::vector<u64> keep(2ull * nb + 2);
    HIP_OK(hipMemcpy(keep.data(), pre, keep.size() * sizeof(u64), hipMemcpyDeviceToHost));
    if ((rc = grow(&e->out_dev, &e->out_dev_bytes, need, false))) return rc;
    pre = (u64*)(e->out_dev + o_pre);
    HIP_OK(hipMemcpy(pre, keep.data(), keep.size() * sizeof(u64), hipMemcpyHostToDevice));
  }
  u8* d = e->out_dev;
  hipLaunchKernelGGL(k_out_write, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, (const u64*)(d + o_pre), (u64*)(d + o_moff),
                     (rbe_message*)(d + o_rec), (u64*)(d + o_roff),
                     (rbe_ready_to_read*)(d + o_rtr));
  HIP_OK(hipGetLastError());
  // one copy of offsets and records into the pinned host buffer
  if ((rc = grow(&e->out_host, &e->out_host_bytes, need - o_moff, true))) return rc;
  HIP_OK(hipMemcpyAsync(e->out_host, d + o_moff, need - o_moff, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u8* h = e->out_host;
  out->n_messages = tot[0];
  out->n_ready_to_reads = tot[1];
  out->msg_off = (const uint64_t*)(h + (o_moff - o_moff));
  out->rtr_off = (const uint64_t*)(h + (o_roff - o_moff));
  out->messages = (const rbe_message*)(h + (o_rec - o_moff));
  out->ready_to_reads = (const rbe_ready_to_read*)(h + (o_rtr - o_moff));
  return RBE_OK;
}

int rbe_collect_step(rbe_engine* e, uint64_t first, uint64_t count, uint32_t flags,
                     rbe_step_outputs* out) {
  if (!e || !out || count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first ||
      (flags & ~(RBE_COLLECT_REMOTE_MSGS | RBE_COLLECT_SKIP_LOCAL)))
    return RBE_E_INVALID;
  memset(out, 0, sizeof(*out));
  out->first = first;
  out->count = count;
  if (e->round == 0) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  const u32 nb = grid_for(count);
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  // device scratch: block sums (triples) | block prefixes (+ totals) | then the
  // records, laid out as the host copy: replicas | updates | msg offsets |
  // rtr offsets | messages | ReadyToReads
  const u64 o_pre = al(3ull * nb * sizeof(u32)), o_rep = o_pre + al(scan_words(3, nb) * sizeof(u64));
  int rc = grow(&e->cs_dev, &e->cs_dev_bytes, o_rep, false);
  if (rc) return rc;
  u64* pre = (u64*)(e->cs_dev + o_pre);
  hipLaunchKernelGGL(k_cs_count, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, flags, (u32*)e->cs_dev);
  if ((rc = launch_scan<3>(e->stream, (const u32*)e->cs_dev, nb, pre))) return rc;
  u64 tot[3];
  HIP_OK(hipMemcpyAsync(tot, pre + 3ull * nb, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  const u64 n = tot[0];
  const u64 o_upd = o_rep + al(n * sizeof(u64));
  const u64 o_moff = o_upd + al(n * sizeof(rbe_update));
  const u64 o_roff = o_moff + al((n + 1) * sizeof(u64));
  const u64 o_msg = o_roff + al((n + 1) * sizeof(u64));
  const u64 o_rtr = o_msg + al(tot[1] * sizeof(rbe_message));
  const u64 need = o_rtr + al(tot[2] * sizeof(rbe_ready_to_read));
  if (need > e->cs_dev_bytes) {  // keep the block prefixes across the regrow
    std::vector<u64> keep(3ull * nb + 3);
    HIP_OK(hipMemcpy(keep.data(), pre, keep.size() * sizeof(u64), hipMemcpyDeviceToHost));
    if ((rc = grow(&e->cs_dev, &e->cs_dev_bytes, need, false))) return rc;
    pre = (u64*)(e->cs_dev + o_pre);
    HIP_OK(hipMemcpy(pre, keep.data(), keep.size() * sizeof(u64), hipMemcpyHostToDevice));
  }
  u8* d = e->cs_dev;
  hipLaunchKernelGGL(k_cs_write, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, flags, (const u64*)(d + o_pre), (u64*)(d + o_rep),
                     (rbe_update*)(d + o_upd), (u64*)(d + o_moff), (rbe_message*)(d + o_msg),
                     (u64*)(d + o_roff), (rbe_ready_to_read*)(d + o_rtr),
                     CsCaps{n, tot[1], tot[2], nullptr});
  HIP_OK(hipGetLastError());
  if ((rc = grow(&e->cs_host, &e->cs_host_bytes, need - o_rep, true))) return rc;
  HIP_OK(hipMemcpyAsync(e->cs_host, d + o_rep, need - o_rep, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u8* h = e->cs_host - o_rep;
  out->n = n;
  out->n_messages = tot[1];
  out->n_ready_to_reads = tot[2];
  out->replica = (const uint64_t*)(h + o_rep);
  out->updates = (const rbe_update*)(h + o_upd);
  out->msg_off = (const uint64_t*)(h + o_moff);
  out->rtr_off = (const uint64_t*)(h + o_roff);
  out->messages = (const rbe_message*)(h + o_msg);
  out->ready_to_reads = (const rbe_ready_to_read*)(h + o_rtr);
  return RBE_OK;
}

// rbe_collect_step in two halves (rbe.h): _begin enqueues the count, scan
// and write kernels, the write kernel filling engine-owned mapped host memory
// directly, and returns at once; _end waits for them and hands out the
// records.  The host's own work of the next round (rbe_push_*) fits between.
static u64 csa_layout(const u64* cap, u64* o) {  // region offsets in the mapped buffer
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  o[0] = 256;                                             // replicas (after the header)
  o[1] = o[0] + al(cap[0] * sizeof(u64));                 // updates
  o[2] = o[1] + al(cap[0] * sizeof(rbe_update));          // msg offsets
  o[3] = o[2] + al((cap[0] + 1) * sizeof(u64));           // rtr offsets
  o[4] = o[3] + al((cap[0] + 1) * sizeof(u64));           // messages
  o[5] = o[4] + al(cap[1] * sizeof(rbe_message));         // ReadyToReads
  return o[5] + al(cap[2] * sizeof(rbe_ready_to_read));  // total
}
int rbe_collect_step_begin(rbe_engine* e, uint64_t first, uint64_t count, uint32_t flags) {
  if (!e || count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first ||
      (flags & ~(RBE_COLLECT_REMOTE_MSGS | RBE_COLLECT_SKIP_LOCAL)))
    return RBE_E_INVALID;
  if (e->round == 0 || e->csa_pending) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  // capacities: at least a quarter of the range's Updates and the last
  // call's totals with room; a round past them is collected again by _end
  const u64 floor_n = std::min<u64>(count, std::max<u64>(count / 4, 4096));
  if (e->csa_cap[0] < floor_n) e->csa_cap[0] = floor_n;
  if (e->csa_cap[2] < 4096) e->csa_cap[2] = 4096;
  u64 o[6];
  const u64 need = csa_layout(e->csa_cap, o);
  const u32 sl = e->csa_slot;
  e->csa_slot ^= 1u;
  if (need > e->csa_bytes[sl]) {
    if (e->csa_buf[sl]) HIP_OK(hipHostFree(e->csa_buf[sl]));
    e->csa_buf[sl] = nullptr;
    e->csa_bytes[sl] = 0;
    HIP_OK(hipHostMalloc((void**)&e->csa_buf[sl], need, hipHostMallocMapped));
    e->csa_bytes[sl] = need;
  }
  e->csa_host = e->csa_buf[sl];
  if (!e->csa_ev) HIP_OK(hipEventCreateWithFlags(&e->csa_ev, hipEventDisableTiming));
  u8* d = nullptr;
  HIP_OK(hipHostGetDevicePointer((void**)&d, e->csa_host, 0));
  const u32 nb = grid_for(count);
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  const u64 o_pre = al(3ull * nb * sizeof(u32)), o_end = o_pre + al(scan_words(3, nb) * sizeof(u64));
  int rc = grow(&e->cs_dev, &e->cs_dev_bytes, o_end, false);
  if (rc) return rc;
  const u64* pre = (const u64*)(e->cs_dev + o_pre);
  hipLaunchKernelGGL(k_cs_count, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, flags, (u32*)e->cs_dev);
  if ((rc = launch_scan<3>(e->stream, (const u32*)e->cs_dev, nb, (u64*)pre))) return rc;
  hipLaunchKernelGGL(k_cs_write, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C, (u64)first,
                     (u64)count, e->round, flags, pre, (u64*)(d + o[0]), (rbe_update*)(d + o[1]),
                     (u64*)(d + o[2]), (rbe_message*)(d + o[4]), (u64*)(d + o[3]),
                     (rbe_ready_to_read*)(d + o[5]),
                     CsCaps{e->csa_cap[0], e->csa_cap[1], e->csa_cap[2], (u64*)d});
  HIP_OK(hipGetLastError());
  HIP_OK(hipEventRecord(e->csa_ev, e->stream));
  e->csa_pending = true;
  e->csa_first = first;
  e->csa_count = count;
  e->csa_flags = flags;
  e->csa_round = e->round;
  return RBE_OK;
}

int rbe_collect_step_end(rbe_engine* e, rbe_step_outputs* out) {
  if (!e || !out) return RBE_E_INVALID;
  if (!e->csa_pending) return RBE_E_STATE;
  e->csa_pending = false;
  if (e->round != e->csa_round) return RBE_E_STATE;  // a step ran in between: outputs gone
  HIP_OK(hipSetDevice(e->device));
  HIP_OK(hipEventSynchronize(e->csa_ev));
  const volatile u64* hdr = (const volatile u64*)e->csa_host;
  const u64 n = hdr[0], nm = hdr[1], nr = hdr[2];
  if (hdr[3]) {  // past the capacities: grow them, collect synchronously this once
    e->csa_cap[0] = std::max(e->csa_cap[0], n + n / 4);
    e->csa_cap[1] = std::max(e->csa_cap[1], nm + nm / 4);
    e->csa_cap[2] = std::max(e->csa_cap[2], nr + nr / 4);
    return rbe_collect_step(e, e->csa_first, e->csa_count, e->csa_flags, out);
  }
  u64 o[6];
  csa_layout(e->csa_cap, o);
  memset(out, 0, sizeof(*out));
  out->first = e->csa_first;
  out->count = e->csa_count;
  out->n = n;
  out->n_messages = nm;
  out->n_ready_to_reads = nr;
  u8* h = e->csa_host;
  out->replica = (const uint64_t*)(h + o[0]);
  out->updates = (const rbe_update*)(h + o[1]);
  out->msg_off = (const uint64_t*)(h + o[2]);
  out->rtr_off = (const uint64_t*)(h + o[3]);
  out->messages = (const rbe_message*)(h + o[4]);
  out->ready_to_reads = (const rbe_ready_to_read*)(h + o[5]);
  return RBE_OK;
}

int rbe_collect_updates(rbe_engine* e, uint64_t first, uint64_t count, rbe_update_list* out) {
  if (!e || !out || count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first)
    return RBE_E_INVALID;
  memset(out, 0, sizeof(*out));
  out->first = first;
  out->count = count;
  if (e->round == 0) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  const u32 nb = grid_for(count);
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  // device scratch: block sums (pairs) | block prefixes (+ totals) | replicas | records
  const u64 o_pre = al(2ull * nb * sizeof(u32)), o_rep = o_pre + al(scan_words(2, nb) * sizeof(u64));
  int rc = grow(&e->upd_dev, &e->upd_dev_bytes, o_rep, false);
  if (rc) return rc;
  u64* pre = (u64*)(e->upd_dev + o_pre);
  hipLaunchKernelGGL(k_upd_count, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C.n, (u64)first,
                     (u64)count, e->round, (u32*)e->upd_dev);
  if ((rc = launch_scan<2>(e->stream, (const u32*)e->upd_dev, nb, pre))) return rc;
  u64 tot[2];
  HIP_OK(hipMemcpyAsync(tot, pre + 2ull * nb, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  const u64 o_rec = o_rep + al(tot[0] * sizeof(u64)), need = o_rec + al(tot[0] * sizeof(rbe_update));
  if (need > e->upd_dev_bytes) {  // keep the block prefixes across the regrow
    std::vector<u64> keep(2ull * nb + 2);
    HIP_OK(hipMemcpy(keep.data(), pre, keep.size() * sizeof(u64), hipMemcpyDeviceToHost));
    if ((rc = grow(&e->upd_dev, &e->upd_dev_bytes, need, false))) return rc;
    pre = (u64*)(e->upd_dev + o_pre);
    HIP_OK(hipMemcpy(pre, keep.data(), keep.size() * sizeof(u64), hipMemcpyHostToDevice));
  }
  u8* d = e->upd_dev;
  hipLaunchKernelGGL(k_upd_write, dim3(nb), dim3(kBlock), 0, e->stream, e->P, e->C.n, (u64)first,
                     (u64)count, e->round, (const u64*)(d + o_pre), (u64*)(d + o_rep),
                     (rbe_update*)(d + o_rec));
  HIP_OK(hipGetLastError());
  if ((rc = grow(&e->upd_host, &e->upd_host_bytes, need - o_rep, true))) return rc;
  if (need > o_rep)
    HIP_OK(hipMemcpyAsync(e->upd_host, d + o_rep, need - o_rep, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  out->n = tot[0];
  out->replica = (const uint64_t*)e->upd_host;
  out->updates = (const rbe_update*)(e->upd_host + (o_rec - o_rep));
  return RBE_OK;
}

int rbe_get_ready_to_reads(rbe_engine* e, uint64_t replica, rbe_ready_to_read* out, uint32_t cap,
                           uint32_t* n_out) {
  if (!e || !n_out || replica >= e->C.n_rep) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  Upd u;
  HIP_OK(hipMemcpyAsync(&u, e->P.upd + replica, sizeof(u), hipMemcpyDeviceToHost, e->stream));
  std::vector<RTR> v(e->C.rtr_cap);
  HIP_OK(hipMemcpyAsync(v.data(), e->P.rtr + replica * e->C.rtr_cap, v.size() * sizeof(RTR),
                        hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u32 n = u.n_rtr;
  if (e->round == 0 || u.round != e->round - 1) n = 0;
  if (n > e->C.rtr_cap) {  // the list moved to the round spill heap (rbe_spill.h rtr_list)
    const u64 gr = v[0].index;
    v.resize(n);
    HIP_OK(hipMemcpyAsync(v.data(), e->P.spill[u.round & 1u] + gr * 16, n * sizeof(RTR),
                          hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
  }
  for (u32 i = 0; i < n && i < cap && out; i++) {
    out[i].index = v[i].index;
    out[i].ctx_low = v[i].low;
    out[i].ctx_high = v[i].high;
  }
  *n_out = n;
  return RBE_OK;
}

// Terms and bodies of entries [lo, hi] of one replica's log window, read on
// the engine stream after every queued round.
static int read_window(rbe_engine* e, u64 replica, u64 lo, u64 hi, std::vector<u64>& t,
                       std::vector<Body>& b) {
  if (replica >= e->C.n_rep || lo == 0 || hi < lo) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  Core c;
  HIP_OK(hipMemcpyAsync(&c, e->P.core + replica, sizeof(c), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  if (hi > c.last_index) return RBE_E_INVALID;
  // the ring window and the cold log below it (the LogDB's entries above its
  // marker): one gather kernel, one copy
  const u64 n = hi - lo + 1;
  int rc = grow(&e->gat_dev, &e->gat_dev_bytes, n * sizeof(Ent) + 256, false);
  if (rc) return rc;
  u32* miss = (u32*)(e->gat_dev + n * sizeof(Ent));
  HIP_OK(hipMemsetAsync(miss, 0, sizeof(u32), e->stream));
  hipLaunchKernelGGL(k_log_gather, dim3(1), dim3(kBlock), 0, e->stream, e->P, e->C, replica, lo, hi,
                     (Ent*)e->gat_dev, miss);
  std::vector<Ent> en(n);
  u32 nmiss = 0;
  HIP_OK(hipMemcpyAsync(en.data(), e->gat_dev, n * sizeof(Ent), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(&nmiss, miss, sizeof(u32), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  if (nmiss) return RBE_E_STATE;  // compacted (ErrCompacted), or never handed over
  t.resize(n);
  b.resize(n);
  for (u64 i = 0; i < n; i++) {
    t[i] = en[i].term;
    b[i].type = en[i].type;
    b[i].len = en[i].len;
    b[i].lo = en[i].lo;
    b[i].hi = en[i].hi;
  }
  return RBE_OK;
}



int rbe_get_entries(rbe_engine* e, uint64_t replica, uint64_t lo, uint64_t hi, rbe_entry* out) {
  if (!e || !out) return RBE_E_INVALID;
  std::vector<u64> t;
  std::vector<Body> b;
  int rc = read_window(e, replica, lo, hi, t, b);
  if (rc) return rc;
  auto rd = [e](u64 pos, u64 off, u64 len, u8* dst) { return read_heap(e, pos, off, len, dst); };
  for (u64 i = lo; i <= hi; i++) {
    const Body& x = b[i - lo];
    rbe_entry& o = out[i - lo];
    memset(&o, 0, sizeof(o));
    Ent en;
    en.term = t[i - lo];
    en.type = x.type;
    en.len = x.len;
    en.lo = x.lo;
    en.hi = x.hi;
    if ((rc = entry_out(en, &o, nullptr, rd))) {
      HIP_IGNORE(hipStreamSynchronize(e->stream));
      return rc;
    }
    o.index = i;
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_get_entry_cmds(rbe_engine* e, uint64_t replica, uint64_t lo, uint64_t hi, uint8_t* buf,
                       uint64_t cap, uint64_t* offsets) {
  if (!e || !offsets) return RBE_E_INVALID;
  std::vector<u64> t;
  std::vector<Body> b;
  int rc = read_window(e, replica, lo, hi, t, b);
  if (rc) return rc;
  u64 off = 0;
  for (u64 i = 0; i < b.size(); i++) {
    offsets[i] = off;
    off += b[i].len;
  }
  offsets[b.size()] = off;
  if (off > cap || (off && !buf)) return RBE_E_NOMEM;
  for (u64 i = 0; i < b.size(); i++) {
    const Body& x = b[i];
    u8* d = buf + offsets[i];
    if (!ent_heap(x.type)) {
      u8 w[16];
      memcpy(w, &x.lo, 8);
      memcpy(w + 8, &x.hi, 8);
      memcpy(d, w, x.len);
    } else if (x.len && (rc = read_heap(e, x.hi, kHeapHdr, x.len, d))) {
      HIP_IGNORE(hipStreamSynchronize(e->stream));
      return rc;
    }
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_spill_stats(rbe_engine* e, uint64_t* out) {
  if (!e || !out) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  SpillCtl s;
  HIP_OK(hipMemcpyAsync(&s, e->P.sctl, sizeof(s), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  out[0] = s.live;
  out[1] = e->C.pool_pages - 1;
  out[2] = std::max(s.peak[0], s.peak[1]) * 16;
  out[3] = e->C.spill_units * 16;
  out[4] = s.oom;
  return RBE_OK;
}

int rbe_fault_summary(rbe_engine* e, uint64_t* n_faulty, uint32_t* fault_or) {
  if (!e || !n_faulty || !fault_or) return RBE_E_INVALID;
  HIP_OK(hipSetDevice(e->device));
  const u64 R = e->C.n_rep;
  std::vector<Upd> upd(R);
  HIP_OK(hipMemcpyAsync(upd.data(), e->P.upd, R * sizeof(Upd), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u64 n = 0;
  u32 o = 0;
  for (u64 i = 0; i < R; i++) {
    if (upd[i].fault) n++;
    o |= upd[i].fault;
  }
  *n_faulty = n;
  *fault_or = o;
  return RBE_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- wire format
int rbe_wire_encode(rbe_engine* e, const rbe_wire_config* wc, uint64_t totals[4]) {
  if (!e || !wc || !totals) return RBE_E_INVALID;
  if (e->round == 0) return RBE_E_STATE;
  const Params& C = e->C;
  if (C.n < 2) return RBE_E_INVALID;  // no peer to send to
  HIP_OK(hipSetDevice(e->device));
  WireArgs A;
  memset(&A, 0, sizeof(A));
  A.deployment_id = wc->deployment_id;
  A.bin_ver = wc->bin_ver;
  if (wc->dst_rank >= (int32_t)C.rep_world || (wc->dst_rank >= 0 && C.rep_world <= 1))
    return RBE_E_INVALID;
  A.dst_rank = wc->dst_rank;
  const u64 gpb = wc->groups_per_batch ? wc->groups_per_batch : C.n_groups;
  if (gpb > 0xFFFFFFFFull) return RBE_E_INVALID;
  A.gpb = (u32)gpb;
  A.nchunks = (u32)((C.n_groups + gpb - 1) / gpb);
  A.npairs = C.n * (C.n - 1);
  A.round = e->round;
  // the device heap holds the positions below `flushed` (records staged since
  // the last step are never in the last round's outbox)
  A.heap_head = e->hin.heap.flushed;
  for (u32 k = 0; k < C.n; k++) {
    const char* s = wc->source_address[k];
    const size_t l = s ? strlen(s) : 0;
    if (l >= sizeof(A.addr[k])) return RBE_E_INVALID;
    A.alen[k] = (u32)l;
    if (l) memcpy(A.addr[k], s, l);
  }
  const u64 ncell = (u64)A.npairs * C.n_groups, nbatch = (u64)A.npairs * A.nchunks;
  if (nbatch > 0xFFFFFFFFull) return RBE_E_INVALID;
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  const u64 o_msgs = al(ncell * 4), o_off = o_msgs + al(ncell * 4), o_pay = o_off + al(ncell * 4);
  const u64 o_bm = o_pay + al(nbatch * 8), o_bi = o_bm + al(nbatch * 4), o_fo = o_bi + al(nbatch * 4);
  const u64 o_fr = o_fo + al(nbatch * 8), o_tot = o_fr + al(nbatch * sizeof(WireFrame));
  int rc = grow(&e->wire_meta, &e->wire_meta_bytes, o_tot + 64, false);
  if (rc) return rc;
  u8* m = e->wire_meta;
  HIP_OK(hipMemsetAsync(m + o_tot, 0, 64, e->stream));
  WireBufs B{(u32*)m, (u32*)(m + o_msgs), (u32*)(m + o_off), (u64*)(m + o_pay), (u32*)(m + o_bm),
             (u32*)(m + o_bi), (u64*)(m + o_fo), (WireFrame*)(m + o_fr), (u64*)(m + o_tot)};
  e->wire_frames_off = o_fr;
  const unsigned gc = (unsigned)((ncell + 255) / 256);
  rc = dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL((k_wire_size<N>), dim3(gc), dim3(256), 0, e->stream, e->P, C, A, B,
                       (const u8*)e->heap);
    return RBE_OK;
  });
  if (rc) return rc;
  const u32 nseg = (u32)((gpb + kWireBatchSeg - 1) / kWireBatchSeg);  // segments per batch
  if (nseg <= 1) {
    hipLaunchKernelGGL(k_wire_batch, dim3((unsigned)nbatch), dim3(256), 0, e->stream, C, A, B);
  } else {
    if ((rc = grow(&e->wire_big_buf, &e->wire_big_bytes, nbatch * nseg * 16, false))) return rc;
    u64* seg_tot = (u64*)e->wire_big_buf;
    hipLaunchKernelGGL(k_wire_batch_part, dim3((unsigned)nbatch, nseg), dim3(256), 0, e->stream,
                       C, A, B, seg_tot);
    hipLaunchKernelGGL(k_wire_batch_fix, dim3((unsigned)nbatch), dim3(256), 0, e->stream, C, A,
                       B, seg_tot, nseg);
    hipLaunchKernelGGL(k_wire_batch_add, dim3((unsigned)nbatch, nseg), dim3(256), 0, e->stream,
                       C, A, B, (const u64*)seg_tot);
  }
  hipLaunchKernelGGL(k_wire_frames, dim3(1), dim3(256), 0, e->stream, C, A, B, (u32)nbatch);
  HIP_OK(hipGetLastError());
  u64 tot[5];
  HIP_OK(hipMemcpyAsync(tot, B.totals, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  memset(e->wire_totals, 0, sizeof(e->wire_totals));
  if (tot[4]) return RBE_E_STATE;  // an entry's heap record was overwritten: no frames
  rc = grow(&e->wire_dev, &e->wire_dev_bytes, tot[0] + 64, false);
  if (rc) return rc;
  if (tot[1]) {
    rc = dispatch_n(C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      hipLaunchKernelGGL((k_wire_write<N>), dim3(gc), dim3(256), 0, e->stream, e->P, C, A, B,
                         (const u8*)e->heap, e->wire_dev);
      return RBE_OK;
    });
    if (rc) return rc;
    hipLaunchKernelGGL(k_wire_trailers, dim3((unsigned)((nbatch + 255) / 256)), dim3(256), 0,
                       e->stream, C, A, B, (u32)nbatch, e->wire_dev);
    // frames over 256 KiB of payload (wire_big, as the decode's chunked walk)
    // take their crc by 64 KiB segments over many blocks: their sizes come
    // from the frame index (read only when the stream could hold one)
    const u64 big = e->wire_big;
    std::vector<WireEncSeg> segs;
    std::vector<u32> bigf;
    if (tot[0] > big + kWireHeader) {
      std::vector<WireFrame> fr(tot[1]);
      HIP_OK(hipMemcpy(fr.data(), B.frames, tot[1] * sizeof(WireFrame), hipMemcpyDeviceToHost));
      for (u64 i = 0; i < tot[1]; i++) {
        const u64 n = fr[i].bytes - kWireHeader;
        if (n <= big) continue;
        bigf.push_back((u32)i);
        for (u64 o = 0; o < n; o += kWireEncSeg) segs.push_back(WireEncSeg{(u32)i, 0u, o});
      }
    }
    hipLaunchKernelGGL(k_wire_crc, dim3((unsigned)tot[1]), dim3(256), 0, e->stream, B,
                       e->wire_dev, big);
    if (!bigf.empty()) {
      const u64 nb = bigf.size(), ns = segs.size();
      const u64 o_acc = al(ns * sizeof(WireEncSeg)), o_bf = o_acc + al(tot[1] * 4);
      if ((rc = grow(&e->wire_big_buf, &e->wire_big_bytes, o_bf + al(nb * 4), false))) return rc;
      u8* b = e->wire_big_buf;
      WireEncSeg* dseg = (WireEncSeg*)b;
      u32 *acc = (u32*)(b + o_acc), *dbf = (u32*)(b + o_bf);
      HIP_OK(hipMemcpyAsync(dseg, segs.data(), ns * sizeof(WireEncSeg), hipMemcpyHostToDevice,
                            e->stream));
      HIP_OK(hipMemcpyAsync(dbf, bigf.data(), nb * 4, hipMemcpyHostToDevice, e->stream));
      HIP_OK(hipMemsetAsync(acc, 0, tot[1] * 4, e->stream));
      hipLaunchKernelGGL(k_wire_crc_seg, dim3((unsigned)ns), dim3(256), 0, e->stream, B,
                         (const WireEncSeg*)dseg, acc, (const u8*)e->wire_dev);
      hipLaunchKernelGGL(k_wire_crc_fin, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0,
                         e->stream, B, (const u32*)dbf, (u32)nb, (const u32*)acc, e->wire_dev);
    }
    HIP_OK(hipGetLastError());
  }
  HIP_OK(hipStreamSynchronize(e->stream));
  for (int i = 0; i < 4; i++) totals[i] = e->wire_totals[i] = tot[i];
  return RBE_OK;
}

int rbe_wire_fetch(rbe_engine* e, void* out, uint64_t cap, rbe_wire_frame* frames,
                   uint32_t frames_cap) {
  if (!e) return RBE_E_INVALID;
  if (!e->wire_meta) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  const u64 bytes = e->wire_totals[0], nf = e->wire_totals[1];
  if ((out && cap < bytes) || (frames && frames_cap < nf)) return RBE_E_NOMEM;
  static_assert(sizeof(WireFrame) == sizeof(rbe_wire_frame), "frame index layout");
  if (out && bytes)
    HIP_OK(hipMemcpyAsync(out, e->wire_dev, bytes, hipMemcpyDeviceToHost, e->stream));
  if (frames && nf)
    HIP_OK(hipMemcpyAsync(frames, e->wire_meta + e->wire_frames_off, nf * sizeof(WireFrame),
                          hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

// Decoded records of a byte stream, left in device memory (e->wire_rec):
// messages in frame order, their entries (message j's from ent0[j]) and Cmd
// bytes (message j's from cmd0[j]).
struct WireDecoded {
  u64 frames = 0, tm = 0, te = 0, tc = 0;
  rbe_message* msgs = nullptr;
  rbe_entry* ents = nullptr;
  u8* cmd = nullptr;
  u64 *ent0 = nullptr, *cmd0 = nullptr;
};

// The front of a decode: the frame boundaries (magic + size of each header,
// the receiver's reads, on the host), the stream and the frame table
// uploaded, both crc32s verified, and every frame's requests found into its
// single-pass slots (one block per frame; big frames by chunks).  Nothing is
// read back.
struct WireFront {
  std::vector<WireIn> fr;
  WireIn* dfr = nullptr;
  WireMsgPos* spos = nullptr;
  u64 big = 0, nch = 0;
  u32 *ent = nullptr, *cbase = nullptr;
  WireChunk* dch = nullptr;
  u32 compact_y = 1;  // blocks per frame of k_wire_compact
};
static int wire_front(rbe_engine* e, const void* data, uint64_t bytes, WireFront* wf) {
  std::vector<WireIn>& fr = wf->fr;
  // the frame boundaries: magic + size of each header (the receiver's reads)
  const u8* d = (const u8*)data;
  for (u64 i = 0; i < bytes;) {
    if (bytes - i < kWireHeader || d[i] != 0xAE || d[i + 1] != 0x7D) return RBE_E_CORRUPT;
    u64 size = 0;
    for (int b = 0; b < 8; b++) size = (size << 8) | d[i + 4 + b];
    if (size == 0 || size > bytes - i - kWireHeader) return RBE_E_CORRUPT;
    WireIn w;
    memset(&w, 0, sizeof(w));
    w.offset = i + kWireHeader;
    w.size = size;
    fr.push_back(w);
    i += kWireHeader + size;
  }
  if (fr.empty()) return RBE_OK;
  HIP_OK(hipSetDevice(e->device));
  const u64 nf = fr.size();
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  // single-pass position slots: one per 16 payload bytes (a marshaled request
  // is far longer; a frame that has more falls back to two walks)
  u64 slots = 0;
  for (auto& w : fr) {
    w.pos0 = slots;
    w.pos_cap = (u32)(w.size / 16 + 1);
    slots += w.pos_cap;
  }
  const u64 o_fr = al(bytes), o_sp = o_fr + al(nf * sizeof(WireIn));
  int rc = grow(&e->wire_in, &e->wire_in_bytes, o_sp + al(slots * sizeof(WireMsgPos)), false);
  if (rc) return rc;
  WireIn* dfr = (WireIn*)(e->wire_in + o_fr);
  WireMsgPos* spos = (WireMsgPos*)(e->wire_in + o_sp);
  // big frames: their chunks and crc segments, in frame order (host lists,
  // uploaded with the frames)
  const u64 big = std::min<u64>(e->wire_big, 0xFFFFFF00ull);  // positions are u32
  std::vector<WireChunk> chunks;
  std::vector<WireSeg> segs;
  std::vector<u32> bigf, chunk0;
  for (u64 i = 0; i < nf; i++)
    if (fr[i].size > big) {
      bigf.push_back((u32)i);
      chunk0.push_back((u32)chunks.size());
      for (u64 c = 0; c < fr[i].size; c += kWireChunk) chunks.push_back(WireChunk{(u32)i, (u32)c});
      for (u64 c = 0; c < fr[i].size; c += kWireCrcSeg) segs.push_back(WireSeg{(u32)i, (u32)c});
    }
  const u64 nch = chunks.size(), nbig = bigf.size(), nseg = segs.size();
  u32 *exitv = nullptr, *ent = nullptr, *cbase = nullptr, *dbig = nullptr, *dch0 = nullptr;
  u16* cntv = nullptr;
  WireChunk* dch = nullptr;
  WireSeg* dseg = nullptr;
  if (nbig) {
    const u64 o_c = al(bytes * 4), o_ent = o_c + al(bytes * 2), o_base = o_ent + al(nch * 4);
    const u64 o_ch = o_base + al(nch * 4), o_bf = o_ch + al(nch * sizeof(WireChunk));
    const u64 o_c0 = o_bf + al(nbig * 4), o_sg = o_c0 + al(nbig * 4);
    const u64 need = o_sg + al(nseg * sizeof(WireSeg));
    if ((rc = grow(&e->wire_big_buf, &e->wire_big_bytes, need, false))) return rc;
    u8* b = e->wire_big_buf;
    exitv = (u32*)b;
    cntv = (u16*)(b + o_c);
    ent = (u32*)(b + o_ent);
    cbase = (u32*)(b + o_base);
    dch = (WireChunk*)(b + o_ch);
    dbig = (u32*)(b + o_bf);
    dch0 = (u32*)(b + o_c0);
    dseg = (WireSeg*)(b + o_sg);
    HIP_OK(hipMemcpyAsync(dch, chunks.data(), nch * sizeof(WireChunk), hipMemcpyHostToDevice,
                          e->stream));
    HIP_OK(hipMemcpyAsync(dbig, bigf.data(), nbig * 4, hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipMemcpyAsync(dch0, chunk0.data(), nbig * 4, hipMemcpyHostToDevice, e->stream));
    HIP_OK(hipMemcpyAsync(dseg, segs.data(), nseg * sizeof(WireSeg), hipMemcpyHostToDevice,
                          e->stream));
    HIP_OK(hipMemsetAsync(ent, 0xFF, nch * 4, e->stream));
  }
  HIP_OK(hipMemcpyAsync(dfr, fr.data(), nf * sizeof(WireIn), hipMemcpyHostToDevice, e->stream));
  // one copy of the stream (a piecewise upload on a second stream, each piece
  // verified as it landed, measured slower on the 512-group ingest workload:
  // 3.57 against 3.26 ms per round; the walk cannot start before the last piece)
  HIP_OK(hipMemcpyAsync(e->wire_in, data, bytes, hipMemcpyHostToDevice, e->stream));
  hipLaunchKernelGGL(k_wire_verify, dim3((unsigned)nf), dim3(256), 0, e->stream, e->wire_in, dfr,
                     0u, big);
  // one block per frame: its walk is a chain of LDS reads (~0.2 ms for an
  // 18 KB frame) whatever the grid
  hipLaunchKernelGGL(k_wire_bounds, dim3((unsigned)nf), dim3(kWireWalkBlock), 0, e->stream,
                     e->wire_in, dfr, 2, spos, big, 0u);
  if (nbig) {
    hipLaunchKernelGGL(k_wire_chunk_crc, dim3((unsigned)nseg), dim3(256), 0, e->stream, e->wire_in,
                       dfr, dseg);
    hipLaunchKernelGGL(k_wire_crc_check, dim3((unsigned)((nbig + 63) / 64)), dim3(64), 0,
                       e->stream, dfr, dbig, (u32)nbig);
    hipLaunchKernelGGL(k_wire_chunk_exit, dim3((unsigned)nch), dim3(256), 0, e->stream,
                       e->wire_in, dfr, dch, exitv, cntv);
    hipLaunchKernelGGL(k_wire_hop, dim3((unsigned)nbig), dim3(64), 0, e->stream, dfr, dbig, dch0,
                       exitv, cntv, ent, cbase);
    hipLaunchKernelGGL(k_wire_chunk_emit, dim3((unsigned)nch), dim3(64), 0, e->stream, e->wire_in,
                       dfr, dch, ent, cbase, 2, spos);
  }
  HIP_OK(hipGetLastError());
  u32 ymax = 1;  // blocks per frame of k_wire_compact
  for (const auto& w : fr) ymax = std::max<u32>(ymax, std::min<u32>(64, w.pos_cap / 4096 + 1));
  wf->compact_y = ymax;
  wf->dfr = dfr;
  wf->spos = spos;
  wf->big = big;
  wf->nch = nch;
  wf->ent = ent;
  wf->cbase = cbase;
  wf->dch = dch;
  return RBE_OK;
}

// rbe_wire_decode's device part: verify, find, count, scan and parse.  With
// `caps` non-null (the caller's capacities: messages, entries, Cmd bytes) the
// records are not parsed when one is short (RBE_E_NOMEM, counts reported).
static int wire_decode_dev(rbe_engine* e, const void* data, uint64_t bytes, WireDecoded* o,
                           const u64* caps) {
  WireFront wf;
  int rc = wire_front(e, data, bytes, &wf);
  if (rc || wf.fr.empty()) return rc;
  std::vector<WireIn>& fr = wf.fr;
  const u64 nf = fr.size(), nch = wf.nch, big = wf.big;
  WireIn* dfr = wf.dfr;
  WireMsgPos* spos = wf.spos;
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  HIP_OK(hipMemcpyAsync(fr.data(), dfr, nf * sizeof(WireIn), hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  u64 tm = 0;
  bool refill = false;
  for (auto& w : fr) {
    if (w.status == 4) {  // more requests than slots: positions from a second walk
      refill = true;
      w.status = 0;
    }
    if (w.status) return RBE_E_CORRUPT;
    w.msg0 = tm;
    tm += w.n_msgs;
  }
  o->frames = nf;
  o->tm = tm;
  if (tm > 0xFFFFFFFFull) return RBE_E_NOMEM;
  // per message: position, entry and Cmd counts (scanned), error flag, scan tops
  const u64 nbk = (tm + 255) / 256;
  const u64 o_ec = al(tm * sizeof(WireMsgPos)), o_cc = o_ec + al(tm * 8), o_t1 = o_cc + al(tm * 8);
  const u64 o_t2 = o_t1 + al((nbk + 1) * 8), o_err = o_t2 + al((nbk + 1) * 8);
  const u64 o_rec = o_err + 256;
  rc = grow(&e->wire_rec, &e->wire_rec_bytes, o_rec, false);
  if (rc) return rc;
  u8* w = e->wire_rec;
  WireMsgPos* pos = (WireMsgPos*)w;
  u64 *ec = (u64*)(w + o_ec), *cc = (u64*)(w + o_cc), *t1 = (u64*)(w + o_t1), *t2 = (u64*)(w + o_t2);
  u32* err = (u32*)(w + o_err);
  HIP_OK(hipMemcpyAsync(dfr, fr.data(), nf * sizeof(WireIn), hipMemcpyHostToDevice, e->stream));
  HIP_OK(hipMemsetAsync(err, 0, 4, e->stream));
  if (refill) {
    hipLaunchKernelGGL(k_wire_bounds, dim3((unsigned)nf), dim3(kWireWalkBlock), 0, e->stream,
                       e->wire_in, dfr, 1, pos, big, 0u);
    if (nch)
      hipLaunchKernelGGL(k_wire_chunk_emit, dim3((unsigned)nch), dim3(64), 0, e->stream,
                         e->wire_in, dfr, wf.dch, wf.ent, wf.cbase, 1, pos);
  } else
    hipLaunchKernelGGL(k_wire_compact, dim3((unsigned)nf, wf.compact_y), dim3(256), 0, e->stream,
                       dfr, spos, pos, ~0ull);
  const unsigned gm = (unsigned)nbk;
  if (tm) {
    hipLaunchKernelGGL(k_wire_parse, dim3(gm), dim3(256), 0, e->stream, e->wire_in, pos, tm, 0,
                       ec, cc, nullptr, nullptr, nullptr, err);
    hipLaunchKernelGGL(k_scan_blocks, dim3(gm), dim3(256), 0, e->stream, ec, tm, t1);
    hipLaunchKernelGGL(k_scan_blocks, dim3(gm), dim3(256), 0, e->stream, cc, tm, t2);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, t1, (u32)nbk);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, t2, (u32)nbk);
    hipLaunchKernelGGL(k_scan_add, dim3(gm), dim3(256), 0, e->stream, ec, tm, t1);
    hipLaunchKernelGGL(k_scan_add, dim3(gm), dim3(256), 0, e->stream, cc, tm, t2);
  }
  HIP_OK(hipGetLastError());
  u64 te = 0, tc = 0;
  u32 herr = 0;
  if (tm) {
    HIP_OK(hipMemcpyAsync(&te, t1 + nbk, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipMemcpyAsync(&tc, t2 + nbk, 8, hipMemcpyDeviceToHost, e->stream));
  }
  HIP_OK(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  if (herr) return RBE_E_CORRUPT;
  o->te = te;
  o->tc = tc;
  if (te > 0xFFFFFFFFull) return RBE_E_NOMEM;
  if (caps && (tm > caps[0] || te > caps[1] || tc > caps[2])) return RBE_E_NOMEM;
  const u64 o_m = o_rec, o_e = o_m + al(tm * sizeof(rbe_message)),
            o_c = o_e + al(te * sizeof(rbe_entry));
  {
    // keep the scratch above while growing (a fresh buffer only when short)
    const u64 need = o_c + al(tc) + 256;
    if (need > e->wire_rec_bytes) {
      u8* nb = nullptr;
      HIP_OK(hipMalloc((void**)&nb, need + need / 2));
      HIP_OK(hipMemcpyAsync(nb, e->wire_rec, o_rec, hipMemcpyDeviceToDevice, e->stream));
      HIP_OK(hipStreamSynchronize(e->stream));
      HIP_OK(hipFree(e->wire_rec));
      e->wire_rec = nb;
      e->wire_rec_bytes = need + need / 2;
    }
  }
  w = e->wire_rec;
  pos = (WireMsgPos*)w;
  ec = (u64*)(w + o_ec);
  cc = (u64*)(w + o_cc);
  err = (u32*)(w + o_err);
  rbe_message* dm = (rbe_message*)(w + o_m);
  rbe_entry* de = (rbe_entry*)(w + o_e);
  u8* dc = w + o_c;
  if (tm)
    hipLaunchKernelGGL(k_wire_parse, dim3(gm), dim3(256), 0, e->stream, e->wire_in, pos, tm, 1,
                       ec, cc, dm, de, dc, err);
  HIP_OK(hipGetLastError());
  o->msgs = dm;
  o->ents = de;
  o->cmd = dc;
  o->ent0 = ec;
  o->cmd0 = cc;
  return RBE_OK;
}

int rbe_wire_decode(rbe_engine* e, const void* data, uint64_t bytes, rbe_message* msgs,
                    uint32_t cap, uint32_t* n_msgs, rbe_entry* ents, uint32_t ent_cap,
                    uint32_t* n_ents, uint8_t* cmd, uint64_t cmd_cap, uint64_t* cmd_bytes) {
  if (!e || (bytes && !data) || !n_msgs || !n_ents || !cmd_bytes) return RBE_E_INVALID;
  *n_msgs = *n_ents = 0;
  *cmd_bytes = 0;
  WireDecoded o;
  const u64 caps[3] = {msgs ? cap : 0u, ents ? ent_cap : 0u, cmd ? cmd_cap : 0u};
  const int rc = wire_decode_dev(e, data, bytes, &o, caps);
  *n_msgs = (u32)(o.tm < 0xFFFFFFFFull ? o.tm : 0xFFFFFFFFull);
  *n_ents = (u32)(o.te < 0xFFFFFFFFull ? o.te : 0xFFFFFFFFull);
  *cmd_bytes = o.tc;
  if (rc) return rc;
  if (o.tm) HIP_OK(hipMemcpyAsync(msgs, o.msgs, o.tm * sizeof(rbe_message), hipMemcpyDeviceToHost, e->stream));
  if (o.te) HIP_OK(hipMemcpyAsync(ents, o.ents, o.te * sizeof(rbe_entry), hipMemcpyDeviceToHost, e->stream));
  if (o.tc) HIP_OK(hipMemcpyAsync(cmd, o.cmd, o.tc, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

static void note_ingest_caps(rbe_engine* e, u64 tm, u64 te, u64 tc) {
  e->ing_cap[0] = tm + tm / 4 + 1024;
  e->ing_cap[1] = te + te / 4 + 1024;
  e->ing_cap[2] = tc + tc / 4 + 4096;
}

// The ingest with ONE read-back (no payload heap): decode and ingest kernels
// launched back to back for the capacities of e->ing_cap, every count read on
// the device, the writing walk gated on the device by every check before it.
// *retry: a capacity was short, a frame needs the second walk or was refused —
// nothing was written and the caller runs the exact path (rbe_wire_ingest),
// which reports the same statuses as always.
static int wire_ingest_fast(rbe_engine* e, const void* data, uint64_t bytes,
                            rbe_wire_ingest_stats* st, bool* retry) {
  *retry = false;
  const Params& C = e->C;
  WireFront wf;
  int rc = wire_front(e, data, bytes, &wf);
  if (rc || wf.fr.empty()) return rc;
  const u64 nf = wf.fr.size();
  const u64 cm = e->ing_cap[0], ce = e->ing_cap[1], cc = e->ing_cap[2];
  const u64 nbk = (cm + 255) / 256;
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  // decode records: positions | entry counts | Cmd counts | their scan tops |
  // message total | messages | entries | Cmd bytes
  const u64 o_ec = al(cm * sizeof(WireMsgPos)), o_cc = o_ec + al(cm * 8), o_t1 = o_cc + al(cm * 8);
  const u64 o_t2 = o_t1 + al((nbk + 1) * 8), o_tot = o_t2 + al((nbk + 1) * 8);
  const u64 o_m = o_tot + 256, o_e = o_m + al(cm * sizeof(rbe_message));
  const u64 o_c = o_e + al(ce * sizeof(rbe_entry)), need_rec = o_c + al(cc) + 256;
  if ((rc = grow(&e->wire_rec, &e->wire_rec_bytes, need_rec, false))) return rc;
  u8* w = e->wire_rec;
  WireMsgPos* pos = (WireMsgPos*)w;
  u64 *ec = (u64*)(w + o_ec), *ccn = (u64*)(w + o_cc), *t1 = (u64*)(w + o_t1), *t2 = (u64*)(w + o_t2);
  u64* tot = (u64*)(w + o_tot);
  rbe_message* dm = (rbe_message*)(w + o_m);
  rbe_entry* de = (rbe_entry*)(w + o_e);
  u8* dc = w + o_c;
  // ingest scratch, as the exact path's, for cm messages
  const u64 drop = (u64)C.n_rep * C.n;
  int bits = 1;
  while (bits < 64 && (drop >> bits)) bits++;
  size_t tb = 0;
  if (dev_sort_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, cm, bits, e->stream))
    return RBE_E_HIP;
  const u64 o_sk = al(cm * 8), o_hb = o_sk + al(cm * 8), o_hs = o_hb + al(cm * 8);
  const u64 o_ix = o_hs + al(cm * 8), o_si = o_ix + al(cm * 4), o_top = o_si + al(cm * 4);
  const u64 o_err = o_top + al((nbk + 1) * 8), o_tmp = o_err + 256;
  if ((rc = grow(&e->ing_dev, &e->ing_dev_bytes, o_tmp + al(tb), false))) return rc;
  u8* b = e->ing_dev;
  u64 *key = (u64*)b, *skey = (u64*)(b + o_sk), *hb = (u64*)(b + o_hb), *hs = (u64*)(b + o_hs);
  u32 *idx = (u32*)(b + o_ix), *sidx = (u32*)(b + o_si);
  u64* top = (u64*)(b + o_top);
  u32* err = (u32*)(b + o_err);     // [0] ingest checks (ING_*), [1] decode flags (WD_*)
  u32* dfl = err + 1;
  unsigned long long* ndrop = (unsigned long long*)(b + o_err + 8);
  HIP_OK(hipMemsetAsync(b + o_err, 0, 16, e->stream));
  const unsigned g = (unsigned)nbk;
  hipLaunchKernelGGL(k_wire_frames_scan, dim3(1), dim3(256), 0, e->stream, wf.dfr, (u32)nf, cm,
                     tot, dfl);
  hipLaunchKernelGGL(k_wire_compact, dim3((unsigned)nf, wf.compact_y), dim3(256), 0, e->stream,
                     wf.dfr, wf.spos, pos, cm);
  hipLaunchKernelGGL(k_wire_parse, dim3(g), dim3(256), 0, e->stream, e->wire_in, pos, cm, 0, ec,
                     ccn, nullptr, nullptr, nullptr, dfl, tot, nullptr, nullptr, 0ull, 0ull, dfl);
  hipLaunchKernelGGL(k_scan_blocks, dim3(g), dim3(256), 0, e->stream, ec, cm, t1);
  hipLaunchKernelGGL(k_scan_blocks, dim3(g), dim3(256), 0, e->stream, ccn, cm, t2);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, t1, (u32)nbk);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, t2, (u32)nbk);
  hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(256), 0, e->stream, ec, cm, t1);
  hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(256), 0, e->stream, ccn, cm, t2);
  hipLaunchKernelGGL(k_wire_parse, dim3(g), dim3(256), 0, e->stream, e->wire_in, pos, cm, 1, ec,
                     ccn, dm, de, dc, dfl, tot, t1 + nbk, t2 + nbk, ce, cc, dfl);
  const u32 par = (e->round - 1) & 1u;
  rc = dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_ing_key<N>, dim3(g), dim3(256), 0, e->stream, C, (u64)C.heap_bytes, dm,
                       (const rbe_entry*)de, (const u64*)ec, cm, key, idx, hb, err, ndrop,
                       e->P.node_ids, (const u64*)tot, (const u32*)dfl);
    return RBE_OK;
  });
  if (rc) return rc;
  HIP_OK(hipGetLastError());
  if (dev_sort_pairs(b + o_tmp, &tb, key, skey, idx, sidx, cm, bits, e->stream)) return RBE_E_HIP;
  hipLaunchKernelGGL(k_ing_gather, dim3(g), dim3(256), 0, e->stream, (const u32*)sidx,
                     (const u64*)hb, hs, cm);
  hipLaunchKernelGGL(k_scan_blocks, dim3(g), dim3(256), 0, e->stream, hs, cm, top);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, top, (u32)nbk);
  hipLaunchKernelGGL(k_scan_add, dim3(g), dim3(256), 0, e->stream, hs, cm, (const u64*)top);
  for (int wr = 0; wr < 2; wr++) {
    rc = dispatch_n(C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      if (wr)
        hipLaunchKernelGGL((k_ing_walk<N, true>), dim3(g), dim3(256), 0, e->stream, e->P, C, par,
                           e->round, (const u64*)skey, (const u32*)sidx, cm, (const rbe_message*)dm,
                           (const rbe_entry*)de, (const u64*)ec, (const u64*)ccn, (const u8*)dc,
                           e->heap, (u64)C.heap_bytes, 0ull, (const u64*)hs, err, (const u32*)err);
      else
        hipLaunchKernelGGL((k_ing_walk<N, false>), dim3(g), dim3(256), 0, e->stream, e->P, C, par,
                           e->round, (const u64*)skey, (const u32*)sidx, cm, (const rbe_message*)dm,
                           (const rbe_entry*)de, (const u64*)ec, (const u64*)ccn, (const u8*)dc,
                           e->heap, (u64)C.heap_bytes, 0ull, (const u64*)hs, err, nullptr);
      HIP_OK(hipGetLastError());
      return RBE_OK;
    });
    if (rc) return rc;
  }
  u64 back[6];  // err | flags, drops, messages, entries, Cmd bytes, heap bytes
  HIP_OK(hipMemcpyAsync(back, err, 16, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(back + 2, tot, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(back + 3, t1 + nbk, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(back + 4, t2 + nbk, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(back + 5, top + nbk, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  const u32 ferr = (u32)back[0], flags = (u32)(back[0] >> 32);
  if (flags || back[5]) {  // nothing written: the exact path decides (and reports)
    *retry = true;
    return RBE_OK;
  }
  st->frames = nf;
  st->messages = back[2];
  st->entries = back[3];
  st->cmd_bytes = back[4];
  note_ingest_caps(e, back[2], back[3], back[4]);
  if (ferr & ING_INVALID) return RBE_E_INVALID;
  if (ferr & ING_NOMEM) return RBE_E_NOMEM;
  st->dropped = back[1];
  return RBE_OK;
}

// Device ingest of inbound frames (rbe_ingest.h): decode, check, sort by inbox
// list, check capacities, one read-back, reserve heap room, write the lists.
// Without a payload heap, and once a call has measured the traffic, the whole
// pipeline runs with one read-back at its end (wire_ingest_fast); the exact
// path below reads counts back between its stages.
int rbe_wire_ingest(rbe_engine* e, const void* data, uint64_t bytes, rbe_wire_ingest_stats* st) {
  if (!e || (bytes && !data) || !st || e->round == 0) return RBE_E_INVALID;
  memset(st, 0, sizeof(*st));
  const Params& C = e->C;
  if (C.rep_world <= 1) return RBE_E_STATE;  // every sender is stepped here
  HIP_OK(hipSetDevice(e->device));
  if (!C.heap_bytes && e->ing_cap[0] && !getenv("RBE_INGEST_EXACT")) {
    bool retry = false;
    const int rc = wire_ingest_fast(e, data, bytes, st, &retry);
    if (!retry) return rc;
    memset(st, 0, sizeof(*st));
  }
  WireDecoded o;
  int rc = wire_decode_dev(e, data, bytes, &o, nullptr);
  st->frames = o.frames;
  st->messages = o.tm;
  st->entries = o.te;
  st->cmd_bytes = o.tc;
  if (rc) return rc;
  note_ingest_caps(e, o.tm, o.te, o.tc);
  const u64 tm = o.tm;
  if (tm == 0) return RBE_OK;
  if (tm > 0x7FFFFFFFull) return RBE_E_NOMEM;
  const u64 nbk = (tm + 255) / 256;
  const u64 drop = (u64)C.n_rep * C.n;
  int bits = 1;
  while (bits < 64 && (drop >> bits)) bits++;
  size_t tb = 0;
  if (dev_sort_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, tm, bits, e->stream))
    return RBE_E_HIP;
  auto al = [](u64 x) { return (x + 255) & ~255ull; };
  // keys | sorted keys | heap bytes | sorted heap offsets | idx | sorted idx | tops | err | sort tmp
  const u64 o_sk = al(tm * 8), o_hb = o_sk + al(tm * 8), o_hs = o_hb + al(tm * 8);
  const u64 o_ix = o_hs + al(tm * 8), o_si = o_ix + al(tm * 4), o_top = o_si + al(tm * 4);
  const u64 o_err = o_top + al((nbk + 1) * 8), o_tmp = o_err + 256;
  if ((rc = grow(&e->ing_dev, &e->ing_dev_bytes, o_tmp + al(tb), false))) return rc;
  u8* b = e->ing_dev;
  u64 *key = (u64*)b, *skey = (u64*)(b + o_sk), *hb = (u64*)(b + o_hb), *hs = (u64*)(b + o_hs);
  u32 *idx = (u32*)(b + o_ix), *sidx = (u32*)(b + o_si);
  u64* top = (u64*)(b + o_top);
  u32* err = (u32*)(b + o_err);
  unsigned long long* ndrop = (unsigned long long*)(b + o_err + 8);
  HIP_OK(hipMemsetAsync(b + o_err, 0, 16, e->stream));
  const u32 par = (e->round - 1) & 1u;
  rc = dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_ing_key<N>, dim3((unsigned)nbk), dim3(256), 0, e->stream, C,
                       (u64)C.heap_bytes, (rbe_message*)o.msgs, (const rbe_entry*)o.ents,
                       (const u64*)o.ent0, tm, key, idx, hb, err, ndrop, e->P.node_ids);
    return RBE_OK;
  });
  if (rc) return rc;
  HIP_OK(hipGetLastError());
  if (dev_sort_pairs(b + o_tmp, &tb, key, skey, idx, sidx, tm, bits, e->stream)) return RBE_E_HIP;
  hipLaunchKernelGGL(k_ing_gather, dim3((unsigned)nbk), dim3(256), 0, e->stream, (const u32*)sidx,
                     (const u64*)hb, hs, tm);
  hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nbk), dim3(256), 0, e->stream, hs, tm, top);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, e->stream, top, (u32)nbk);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nbk), dim3(256), 0, e->stream, hs, tm,
                     (const u64*)top);
  auto walk = [&](bool write, u64 base) {
    return dispatch_n(C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      if (write)
        hipLaunchKernelGGL((k_ing_walk<N, true>), dim3((unsigned)nbk), dim3(256), 0, e->stream,
                           e->P, C, par, e->round, (const u64*)skey, (const u32*)sidx, tm,
                           (const rbe_message*)o.msgs, (const rbe_entry*)o.ents,
                           (const u64*)o.ent0, (const u64*)o.cmd0, (const u8*)o.cmd, e->heap,
                           (u64)C.heap_bytes, base, (const u64*)hs, err);
      else
        hipLaunchKernelGGL((k_ing_walk<N, false>), dim3((unsigned)nbk), dim3(256), 0, e->stream,
                           e->P, C, par, e->round, (const u64*)skey, (const u32*)sidx, tm,
                           (const rbe_message*)o.msgs, (const rbe_entry*)o.ents,
                           (const u64*)o.ent0, (const u64*)o.cmd0, (const u8*)o.cmd, e->heap,
                           (u64)C.heap_bytes, base, (const u64*)hs, err);
      HIP_OK(hipGetLastError());
      return RBE_OK;
    });
  };
  if ((rc = walk(false, 0))) return rc;
  u64 back[3];  // err | drops, heap bytes
  HIP_OK(hipMemcpyAsync(back, b + o_err, 16, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipMemcpyAsync(back + 2, top + nbk, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  const u32 ferr = (u32)back[0];
  if (ferr & ING_INVALID) return RBE_E_INVALID;
  if (ferr & ING_NOMEM) return RBE_E_NOMEM;
  st->dropped = back[1];
  const u64 need = back[2];
  st->heap_bytes = need;
  HostHeap& H = e->hin.heap;
  u64 base = 0;
  if (need) {
    // records staged by earlier pushes of this round go up first, so the
    // device region follows them and the stage stays [flushed, head)
    for (u64 p = H.flushed; p < H.head;) {
      const u64 at = p % H.cap, len = std::min(H.head - p, H.cap - at);
      HIP_OK(hipMemcpyAsync(e->heap + at, H.stage.data() + (p - H.flushed), len,
                            hipMemcpyHostToDevice, e->stream));
      p += len;
    }
    HIP_OK(hipStreamSynchronize(e->stream));  // the stage is pageable
    // one region that does not cross the end of the ring
    const u64 skip = H.head % H.cap + need > H.cap ? H.cap - H.head % H.cap : 0;
    if ((rc = H.room(need + skip))) return rc;
    if (H.flushed < H.round_lo) H.round_lo = H.flushed;
    H.stage.clear();
    base = H.head + skip;
    H.head = base + need;
    H.flushed = H.head;
    e->heap_head_host = H.head;  // Planes::heap_head for the lapped-record checks
    HIP_OK(hipMemcpyAsync(e->heap_dev, &e->heap_head_host, sizeof(u64), hipMemcpyHostToDevice,
                          e->stream));
  }
  if ((rc = walk(true, base))) return rc;
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

// Replica mode with the isolation schedule: the epoch's leader
// bits of this engine's replicas, and the OR over ranks back in.
int rbe_iso_leaders(rbe_engine* e, uint8_t* out, uint32_t* epoch) {
  if (!e || !epoch) return RBE_E_INVALID;
  const Params& C = e->C;
  *epoch = C.iso_period && e->round > 0 && e->round % C.iso_period == 0 ? 1u : 0u;
  if (!*epoch || !out) return RBE_OK;
  HIP_OK(hipSetDevice(e->device));
  if (!e->iso_dev) HIP_OK(hipMalloc((void**)&e->iso_dev, C.n_groups_glob));
  HIP_OK(hipMemsetAsync(e->iso_dev, 0, C.n_groups_glob, e->stream));
  const int rc = dispatch_n(C.n, [&](auto NN) {
    constexpr int N = decltype(NN)::value;
    hipLaunchKernelGGL(k_iso_bits<N>, dim3(grid_for(C.n_groups)), dim3(kBlock), 0, e->stream,
                       e->P, e->C, e->iso_dev);
    HIP_OK(hipGetLastError());
    return RBE_OK;
  });
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(out, e->iso_dev, C.n_groups_glob, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  return RBE_OK;
}

int rbe_set_iso_leaders(rbe_engine* e, const uint8_t* bits) {
  if (!e || !bits) return RBE_E_INVALID;
  const Params& C = e->C;
  if (!(C.iso_period && e->round > 0 && e->round % C.iso_period == 0)) return RBE_E_STATE;
  HIP_OK(hipSetDevice(e->device));
  if (!e->iso_dev) HIP_OK(hipMalloc((void**)&e->iso_dev, C.n_groups_glob));
  HIP_OK(hipMemcpyAsync(e->iso_dev, bits, C.n_groups_glob, hipMemcpyHostToDevice, e->stream));
  HIP_OK(hipStreamSynchronize(e->stream));
  e->iso_round = e->round;
  return RBE_OK;
}

int rbe_local_groups(rbe_engine* e, uint64_t* n_local, uint64_t* global_of) {
  if (!e || !n_local) return RBE_E_INVALID;
  *n_local = e->C.n_groups;
  if (global_of)
    for (u64 g = 0; g < e->C.n_groups; g++) {
      const u64 gg = group_global(e->C, g);
      global_of[g] = gg < e->C.n_groups_glob ? gg : ~0ull;
    }
  return RBE_OK;
}
