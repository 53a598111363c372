// MI355X batched Raft step engine — the per-replica step.
//
// One lane steps one replica through one lockstep round: the dragonboat node
// step (node.go:1016-1067 stepNode/handleEvents, 1171-1205
// handleReceivedMessages, 1384-1399 tick, quiesce.go) driving the raft
// protocol (internal/raft/raft.go) on struct-of-arrays state in HBM.
// Inbound messages are read from the senders' previous-round outbox lists,
// outbound messages are written to this round's lists; nothing a lane writes
// is read by another lane in the same launch (DESIGN.md §Round semantics).
//
// Kernel groups of the north star map onto this file as:
//   (1) ReplicateResp → tryCommit: on_replicate_resp / try_commit / kth_match
//   (2) log matching: on_replicate / match_term / try_append
//   (3) vote tally: campaign / on_vote_resp / on_request_vote
//   (4) ReadIndex quorum: on_leader_read_index / rq_confirm / on_heartbeat_resp
//   (5) tick / quiesce: node_tick / raft_tick / quiesce manager
#pragma once
#include "rbe_types.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define RBE_HD __host__ __device__ __forceinline__
#else
#define RBE_HD inline
#endif

namespace rbe {

// Global group of local group g (rep_compact), and its cluster id
RBE_HD u64 group_global(const Params& C, u64 g) {
  return C.rep_compact ? (g / C.n) * C.rep_world + C.res[g % C.n] : g;
}
RBE_HD u64 cid_of(const Params& C, u64 g) { return C.cid_base + group_global(C, g) * C.cid_stride; }
// the same with the group size a compile-time constant (the step kernels:
// no 64-bit division by a runtime value in their register budget)
template <int N>
RBE_HD u64 cid_of_n(const Params& C, u64 g) {
  const u64 gg = C.rep_compact ? (g / N) * C.rep_world + C.res[g % N] : g;
  return C.cid_base + gg * C.cid_stride;
}
// rate limiter (server/rate.go): Enabled and RateLimited with its gc (rate.go:
// 109-149): the largest fresh follower report or the replica's own in-memory
// log size above the limit
RBE_HD bool rl_enabled(u64 max) { return max > 0 && max != ~0ull; }  // rate.go:59-61
// rl.RateLimited() (rate.go:109-137) with its gc: the largest fresh follower
// report or the replica's own size above the limit
RBE_HD bool rl_limited(RlSt& s, u64 max) {
  if (!rl_enabled(max)) return false;
  u64 m = 0;
  for (u32 i = 0; i < 8; i++) {
    if (!((s.fmask >> i) & 1u)) continue;
    if (s.tick - s.f_tick[i] > kRlGcTick) {
      s.fmask &= ~(1u << i);  // gc()
      continue;
    }
    if (s.f_size[i] > m) m = s.f_size[i];
  }
  if (s.size > m) m = s.size;
  return m > max;
}
// the in-memory marker (Planes::imark) is kept for rbe_commit and for the limiter
RBE_HD bool imark_on(const Params& C) { return C.ext_commit || C.rl_max; }
// Is replica k of local group g stepped by this engine?  (replica mode:
// replica k of global group G is stepped on rank (G + k) % rep_world; the
// padding groups of a compacted engine by none)
RBE_HD bool owns_replica(const Params& C, u64 g, u32 k) {
  if (C.rep_world <= 1) return true;
  const u64 gg = group_global(C, g);
  return gg < C.n_groups_glob && (u32)((gg + k) % C.rep_world) == C.rep_rank;
}
// cfg.rep_compact: keep only the groups this rank steps a replica of.  The
// rank touches global group G iff G % W is one of the N residues (rank - k)
// mod W; local group l is G = (l / N) * W + res[l % N] (the last block may
// hold padding groups past the global count, which no rank steps).
RBE_HD void rep_compact_setup(Params& C, bool on) {
  C.n_groups_glob = C.n_groups;
  C.rep_compact = 0;
  for (int i = 0; i < 8; i++) C.res[i] = 0;
  if (on && C.rep_world > 1 && C.n < C.rep_world) {
    u32 m = 0;
    for (u32 rho = 0; rho < C.rep_world; rho++)
      for (u32 k = 0; k < C.n; k++)
        if ((rho + k) % C.rep_world == C.rep_rank) {
          C.res[m++] = (u8)rho;
          break;
        }
    C.rep_compact = 1;
    C.n_groups = (C.n_groups_glob + C.rep_world - 1) / C.rep_world * C.n;
  }
  C.n_rep = C.n_groups * C.n;
}
// Local group of global group gg, if this engine holds it
RBE_HD bool group_local(const Params& C, u64 gg, u64* g) {
  if (!C.rep_compact) {
    *g = gg;
    return gg < C.n_groups;
  }
  const u32 rho = (u32)(gg % C.rep_world);
  for (u32 j = 0; j < C.n; j++)
    if (C.res[j] == rho) {
      *g = (gg / C.rep_world) * C.n + j;
      return gg < C.n_groups_glob;
    }
  return false;
}

RBE_HD u64 mix64(u64 x) {  // splitmix64 finalizer (same constants as the oracle)
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
RBE_HD u64 hfold(u64 h, u64 x) { return mix64(h ^ x); }
// Entry type and payload-heap bit of a Body/Ent `type` word (rbe_types.h ET_HEAP)
RBE_HD u32 ent_type(u32 t) { return t & ET_TYPE_MASK; }
RBE_HD bool ent_heap(u32 t) { return (t & ET_HEAP) != 0; }
// The second Cmd word a trace digest folds: the inline bytes 8-15, or 0 for a
// payload-heap record, whose `hi` is a heap position (rbe_host.h) and whose
// `lo` fingerprint already stands for the bytes and session fields
RBE_HD u64 cmd_hi(u32 type, u64 hi) { return ent_heap(type) ? 0 : hi; }
// The (type, Cmd length) word a trace digest folds for an entry
RBE_HD u64 ent_word(u32 type, u32 len) { return (u64)ent_type(type) | ((u64)len << 32); }
// A heap record at `pos` was overwritten by a later lap of the heap (the entry
// is older than the in-memory window the heap keeps: F_WINDOW, as a ring miss)
RBE_HD bool heap_lapped(const Planes& P, const Params& C, u32 type, u64 pos) {
  return ent_heap(type) && C.heap_bytes && P.heap_head && pos + C.heap_bytes < *P.heap_head;
}
RBE_HD u64 umin64(u64 a, u64 b) { return a < b ? a : b; }
RBE_HD u64 umax64(u64 a, u64 b) { return a > b ? a : b; }
RBE_HD u32 popc8(u32 x) {
  x = x - ((x >> 1) & 0x55u);
  x = (x & 0x33u) + ((x >> 2) & 0x33u);
  return (x + (x >> 4)) & 0x0Fu;
}

}  // namespace rbe
#include "rbe_spill.h"
namespace rbe {

// ----------------------------------------------------------------- workload
// DESIGN.md §Workload; restated independently in oracle/harness.cpp.
RBE_HD u64 wl_payload_lo(u64 seed, u64 cid, u64 round) {
  return mix64(seed ^ (cid * 0xD1B54A32D192ED03ULL) ^ (round << 1));
}
// uniform draw in [0, m) from the high 32 bits of x (multiply-shift, no division)
RBE_HD u32 below(u64 x, u32 m) { return (u32)(((x >> 32) * (u64)m) >> 32); }
RBE_HD bool wl_group_active(const Params& C, u64 cid) {
  if (C.wl_active_mod <= 1) return true;
  return below(mix64(C.seed ^ 0xA5A5A5A5A5A5A5A5ULL ^ (cid * 0x9E3779B97F4A7C15ULL)),
               C.wl_active_mod) == 0;
}
RBE_HD u32 wl_input(const Params& C, u64 cid, u32 round) {
  if (!C.wl_enabled) return 0;
  if (round < C.wl_start_round) return 0;
  if (C.wl_stop_round != 0 && round >= C.wl_stop_round) return 0;
  if (!wl_group_active(C, cid)) return 0;
  if (C.wl_read_permille == 0) return 1;
  u32 u = below(mix64(C.seed ^ (cid * 0xC2B2AE3D27D4EB4FULL) ^ ((u64)round << 20)), 1000);
  return u < C.wl_read_permille ? 2u : 1u;
}
// leader-transfer schedule: at every xfer_period-th
// round, in groups selected by hash, one seeded replica (any role) gets a
// Peer.RequestLeaderTransfer(target) (node.go:1069-1075 → peer.go:106-113)
// with a seeded target node id; returns the target, 0 for none.  Restated
// independently in oracle/harness.cpp.
RBE_HD u32 xfer_input(const Params& C, u64 cid, u32 round, u32 k) {
  if (!C.xfer_period || round == 0 || round % C.xfer_period != 0) return 0;
  const u64 epoch = round / C.xfer_period;
  if (C.xfer_mod > 1 &&
      below(mix64(C.seed ^ (cid * 0xA24BAED4963EE407ULL) ^ (epoch << 36)), C.xfer_mod) != 0)
    return 0;
  const u64 h = mix64(C.seed ^ (cid * 0x9FB21C651E98DF25ULL) ^ (epoch << 12) ^ 0x5851F42DULL);
  if (below(h, C.n) != k) return 0;
  return below(mix64(h), C.n) + 1;
}
// config-change schedule (restated in oracle/harness.cpp
// cc_selected / cc_target): every cc_period-th round, in groups selected 1 in
// cc_mod, the replica leading at round start proposes removing a seeded voter
// (while more than two vote) or adding it back
RBE_HD bool cc_selected(const Params& C, u64 cid, u32 round) {
  if (!C.cc_period || round == 0 || round % C.cc_period != 0) return false;
  const u64 epoch = round / C.cc_period;
  return C.cc_mod <= 1 ||
         below(mix64(C.seed ^ (cid * 0xE7037ED1A0B428DBULL) ^ (epoch << 28)), C.cc_mod) == 0;
}
RBE_HD u32 cc_target(const Params& C, u64 cid, u32 round) {
  const u64 epoch = round / C.cc_period;
  return below(mix64(C.seed ^ (cid * 0x8EBC6AF09C88C6E3ULL) ^ (epoch << 20) ^ 0xCC), C.n) + 1;
}
// A group's membership packed as slot masks (bit s = slot s): bits 0-7 the
// slots not in Addresses (raft.remotes), 8-15 Observers, 16-23 Witnesses
// (pb.Membership, raft.pb.go:733-739; rbe_launch_state::removed, the snapshot
// state, rbe_restore_remotes)
RBE_HD u32 pack_ms(u32 rem, u32 obs, u32 wit) {
  return (rem & 0xFFu) | ((obs & 0xFFu) << 8) | ((wit & 0xFFu) << 16);
}
// a packed membership over n slots: each node in at most one of observers /
// witnesses, and those not in Addresses
RBE_HD bool ms_valid(u32 ms, u32 n) {
  const u32 rem = ms & 0xFFu, obs = (ms >> 8) & 0xFFu, wit = (ms >> 16) & 0xFFu;
  return !(ms >> 24) && !(rem >> n) && !(obs >> n) && !(wit >> n) && !(obs & wit) &&
         !((obs | wit) & ~rem);
}
// Whether the state machine accepts a committed ConfigChange (rsm
// membership.go:299-321 handleConfigChange), judged on the membership `ms`
// (packed) raft holds when the entry is applied: an add of a node that already
// is a voter, observer or witness is rejected — alreadyMember,
// nodeBecomingObserver / Witness, witnessBecomingNode, observerBecomingWitness
// — except AddNode of an observer (isPromotingObserver); removing the only
// voter is rejected (isDeletingOnlyNode).  A rejected one goes back to raft as
// RejectConfigChange.  (The stand-in keeps no Removed set, so re-adding a
// removed node is accepted: the membership schedule relies on it.)
RBE_HD bool cc_accepted(u32 ms, u32 t, u64 nid, u32 n) {
  if (nid < 1 || nid > n) return true;
  const u32 b = 1u << (nid - 1), rem = ms & 0xFFu, obs = (ms >> 8) & 0xFFu, wit = (ms >> 16) & 0xFFu;
  const u32 voters = ((1u << n) - 1u) & ~rem;
  if (t == CC_RemoveNode) return voters != b;
  if (t == CC_AddNode && (obs & b)) return true;
  return !((voters | obs | wit) & b);
}
// the state machine's membership after applying a ConfigChange (rsm
// membership.go: AddNode also promotes an observer; RemoveNode drops the node
// from every set)
RBE_HD void ms_apply(u32& ms, u32 t, u64 nid, u32 n) {
  if (nid < 1 || nid > n) return;
  const u32 b = 1u << (nid - 1);
  u32 rem = ms & 0xFFu, obs = (ms >> 8) & 0xFFu, wit = (ms >> 16) & 0xFFu;
  if (t == CC_AddNode) {
    rem &= ~b;
    obs &= ~b;
  } else if (t == CC_RemoveNode) {
    rem |= b;
    obs &= ~b;
    wit &= ~b;
  } else if (t == CC_AddObserver) {
    obs |= b;
  } else if (t == CC_AddWitness) {
    wit |= b;
  }
  ms = pack_ms(rem, obs, wit);
}

// The stand-in ConfigChange Cmd the engine shares with the oracle harness (8
// bytes, LE of 0xCC << 56 | type << 48 | node id; bootstrap's entries are its
// AddNode form): what the engine's own state machine decodes when it applies
// a committed ConfigChange entry (cfg.membership without ext_apply).
RBE_HD u64 cc_word(u32 type, u64 node) {
  return 0xCC00000000000000ULL | ((u64)(type & 0xFFu) << 48) | (node & 0xFFFFFFFFFFFFULL);
}

RBE_HD bool iso_selected(const Params& C, u64 cid, u32 epoch) {
  if (C.iso_mod <= 1) return true;
  return below(mix64(C.seed ^ (cid * 0x94D049BB133111EBULL) ^ ((u64)epoch << 40)), C.iso_mod) ==
         0;
}
// injected replacement for random.LockGuardedRand (raft.go:632)
RBE_HD u64 rto_rand(u64 seed, u64 cid, u64 nid, u64 count) {
  return mix64(seed ^ (cid * 0x9E3779B97F4A7C15ULL) ^ (nid << 32) ^ count);
}

// Lazy quiesced ticks.  With Quiesce on, every round advances the quiesce
// tick of every replica by exactly one, so at the start of round `round` a
// replica's q_tick equals `round`.  k_triage skips the Hot write of a round
// that is nothing but a QuiescedTick (electionTick++ and tick++, raft.go:
// 623-629, quiesce.go:43-55), so a stored record may lag; every reader
// applies the missed ticks here.  Without Quiesce nothing is skipped.
RBE_HD Hot materialize_hot(Hot h, const Params& C, u32 round) {
  if (C.quiesce) {
    const u32 lag = round - h.q_tick;
    h.election_tick += lag;
    h.q_tick = round;
  }
  return h;
}
RBE_HD Hot load_hot(const Planes& P, const Params& C, u64 r, u32 round) {
  return materialize_hot(P.hot[r], C, round);
}

// The idle byte of a replica (Planes::idle), rewritten with every Hot write:
//   IB_LAZY  the next round is a pure QuiescedTick unless an input arrives
//            (Quiesce on, quiesced, RAFT_QUIESCE already set, nothing to apply);
//   IB_LEAD  the replica leads (only a leader takes client input);
//   bits 4-6 the role, so a replica with inbound messages is classified
//            without reading Hot.
enum : u8 { IB_LAZY = 1, IB_LEAD = 2, IB_ROLE_SHIFT = 4 };
RBE_HD u8 idle_byte(const Params& C, u8 role, u8 flags, u32 qs) {
  // with ext_commit a quiesced step may still owe an Update (entries the host
  // has not acknowledged as saved are returned again), so no round is lazy
  const bool lazy = C.quiesce && qs > 0 && (flags & HF_RAFT_QUIESCE) && !C.ext_commit &&
                    !(flags & (HF_APPLY_PENDING | HF_APPLIED_NEW | HF_SNAP_WORK));
  return (u8)((lazy ? IB_LAZY : 0) | (role == R_Leader ? IB_LEAD : 0) | ((role & 7u) << IB_ROLE_SHIFT));
}
RBE_HD u32 idle_role(u8 ib) { return (ib >> IB_ROLE_SHIFT) & 7u; }

// The count word of list (sender slot s → destination slot d) that a step of
// round `round` reads: the sender's outbox header of the previous round's
// parity, valid only if that round wrote it (CntRow::stamp == round).
// the index in CntRow::w of destination slot d's word in sender slot k's row
RBE_HD u32 cnt_widx(u32 d, u32 k) { return d < 6u ? d : k; }
// the count word of destination slot d in sender slot k's row, read in `round`
// (none to itself: in a group of 7 that index holds slot 6's word)
// (the word is shifted out of the row's two 64-bit halves: indexing CntRow::w
// with a run-time index puts the row in scratch memory, a store and two loads)
RBE_HD u32 row_word(const CntRow& row, u32 d, u32 k, u32 round) {
  u64 lo, hi;
  __builtin_memcpy(&lo, &row, 8);
  __builtin_memcpy(&hi, (const char*)&row + 8, 8);
  const u32 i = cnt_widx(d, k);  // w[i] at byte 4 + 2i
  const u64 x = i < 2u ? lo >> (32u + 16u * i) : hi >> (16u * (i - 2u));
  return (u32)lo == round && d != k ? (u32)(x & 0xFFFFu) : 0u;
}
template <int N>
RBE_HD u32 in_word(const Planes& P, u64 g, u32 s, u32 d, u32 round) {
  if (round == 0) return 0u;
  return row_word(P.cnt[(round & 1u) ^ 1u][g * N + s], d, s, round);
}
// This sender's outbox header of round `round` (one 16-B store).
RBE_HD void put_row(const Planes& P, u64 r, u32 round, u32 n, const u32* w) {
  CntRow row;
  row.stamp = round + 1u;
  const u32 k = (u32)(r % n);
  for (u32 d = 0; d < 6; d++) row.w[d] = (u16)(d < n && d != k ? w[d] : 0u);
  if (n > 6 && k < 6) row.w[k] = (u16)w[6];  // slot 6's word in the sender's own place
  P.cnt[round & 1u][r] = row;
}

// The Update helpers of peer.go on the engine's range form of an Update
// (EntriesToSave = [save_lo, save_hi], CommittedEntries = [apply_lo,
// apply_hi], empty when lo > hi).
// setFastApply (peer.go:209-226)
RBE_HD bool update_fast_apply(bool has_snapshot, u64 save_lo, u64 save_hi, u64 apply_lo,
                              u64 apply_hi) {
  if (has_snapshot) return false;
  if (apply_lo <= apply_hi && save_lo <= save_hi && apply_hi >= save_lo && apply_hi <= save_hi)
    return false;
  return true;
}
// validateUpdate (peer.go:228-245): false where the reference panics
RBE_HD bool update_valid(u64 commit, u64 save_lo, u64 save_hi, u64 apply_lo, u64 apply_hi) {
  if (commit > 0 && apply_lo <= apply_hi && apply_hi > commit) return false;
  if (apply_lo <= apply_hi && save_lo <= save_hi && apply_hi > save_hi) return false;
  return true;
}
// getUpdateCommit (peer.go:410-427): {processed, stable_log_to,
// stable_snapshot_to}; StableLogTerm is the term of entry save_hi
RBE_HD void update_commit(u64 save_lo, u64 save_hi, u64 apply_lo, u64 apply_hi, u64 snap_index,
                          u64* processed, u64* stable_log_to, u64* stable_snapshot_to) {
  *processed = apply_lo <= apply_hi ? apply_hi : 0;
  *stable_log_to = save_lo <= save_hi ? save_hi : 0;
  *stable_snapshot_to = snap_index;
  if (snap_index != 0 && snap_index > *processed) *processed = snap_index;
}

// Peer.Commit's log part with a host-supplied UpdateCommit (rbe_commit,
// ext_commit mode): entryLog.commitUpdate (logentry.go:335-355) =
// inMemory.commitUpdate → savedLogTo (inmemory.go:108-137), then processed,
// then inMemory.appliedLogTo (139-167).  `imark` is inMemory.markerIndex; the
// in-memory log holds [imark, last_index] (empty when imark > last_index).
// A reference panic sets F_PANIC in the sticky fault word and changes nothing
// further.  stable_snapshot_to clears the snapshot the Updates carry
// (savedSnapshotTo, inmemory.go:168-176) when it names that snapshot; another
// index only logs a warning in the reference and changes nothing here.
// Returns the fault bits raised.
RBE_HD u32 commit_update(const Planes& P, const Params& C, u64 r, u64 stable_log_to,
                         u64 stable_log_term, u64 processed, u64 last_applied,
                         u64 stable_snapshot_to) {
  Core c = P.core[r];
  u64 mark = P.imark[r];
  u32 fault = 0;
  const bool held = mark <= c.last_index;  // len(im.entries) > 0
  if (stable_log_to > 0 && held && stable_log_to >= mark && stable_log_to <= c.last_index) {
    u64 t = c.t_last;
    if (stable_log_to != c.last_index) {
      if (c.last_index - stable_log_to >= C.ring) fault |= F_WINDOW;
      else t = P.term_ring[(stable_log_to & (u64)(C.ring - 1)) * C.n_rep + r];
    }
    if (!fault && t == stable_log_term) c.saved_to = stable_log_to;
  }
  if (!fault && stable_snapshot_to > 0 && C.snapshot_entries) {
    SnapSt& sp = P.snp[r];
    if (sp.upd_ss && sp.marker == stable_snapshot_to) sp.upd_ss = 0;
  }
  if (!fault && processed > 0) {
    if (processed < c.processed || processed > c.committed) fault |= F_PANIC;
    else c.processed = processed;
  }
  if (!fault && last_applied > 0) {
    if (last_applied > c.committed || last_applied > c.processed) {
      fault |= F_PANIC;
    } else if (held && last_applied >= mark && last_applied <= c.last_index) {
      if (rl_enabled(C.rl_max)) {  // the limiter's part of appliedLogTo (Lane::rl_applied_to)
        RlSt& s = P.rl[r];
        u64 sum = 0;
        for (u64 i = s.new_ent ? mark : mark + 1; i <= last_applied; i++) {
          if (c.last_index - i >= C.ring) {
            fault |= F_WINDOW;
            break;
          }
          sum += kEntryInMem + P.pay_ring[(i & (u64)(C.ring - 1)) * C.n_rep + r].len;
        }
        if (!fault) {  // a fault exit changes nothing further (size, marker)
          s.size -= sum;
          s.new_ent = 0;
        }
      }
      if (!fault) mark = last_applied;
    }
  }
  P.core[r] = c;
  P.imark[r] = mark;
  Hot* h = &P.hot[r];
  u8 f = h->flags;
  if (c.processed < c.committed) f |= HF_APPLY_PENDING;
  else f &= (u8)~HF_APPLY_PENDING;
  if (fault) {
    f |= HF_FAULTED;
    P.upd[r].fault |= fault;
  }
  h->flags = f;
  return fault;
}

// Host-driven node snapshots (snapshot_entries with ext_apply; rbe_snapshot_saved
// / rbe_compact): the node's snapshot worker saved a snapshot of the host's
// state machine and the LogDB took it (doSaveSnapshot → LogReader.CreateSnapshot,
// node.go:619-692; ErrSnapshotOutOfDate at or below the LogDB's: ignored), or
// the node asks for a compaction (compactSnapshot's compactLogTo, run by the
// replica's next step as compactLog, node.go:849-866).  One record per
// replica between two steps, applied in place (the step re-reads SnapSt).
struct SnapRec {
  u64 r, index, term, compact_to;
  u32 rem;   // the snapshot's membership (removed mask)
  u32 kind;  // SR_SAVE | SR_COMPACT
};
enum : u32 { SR_SAVE = 1, SR_COMPACT = 2 };
RBE_HD void snap_rec_apply(const Planes& P, const SnapRec& x) {
  SnapSt& sp = P.snp[x.r];
  if ((x.kind & SR_SAVE) && x.index > sp.ss_index) {
    sp.ss_index = x.index;
    sp.ss_term = x.term;
    sp.ss_rem = (u8)(x.rem & 0xFFu);  // packed membership (pack_ms)
    sp.ss_obs = (u8)((x.rem >> 8) & 0xFFu);
    sp.ss_wit = (u8)((x.rem >> 16) & 0xFFu);
  }
  if (x.kind & SR_COMPACT) {
    sp.compact_to = x.compact_to;
    // the next step takes the full table and compacts after its Update
    P.hot[x.r].flags |= HF_SNAP_WORK;
    P.idle[x.r] &= (u8)~IB_LAZY;
  }
}

// entryutils.go:97-104 / 106-114: message types only a node makes for its own
// raft (Peer.Handle panics on them), and response types (dropped when the
// sender is not a member)
RBE_HD bool is_local_message(u32 t) {
  return t == M_Election || t == M_LeaderHeartbeat || t == M_Unreachable || t == M_SnapshotStatus ||
         t == M_CheckQuorum || t == M_LocalTick || t == M_BatchedReadIndex;
}
RBE_HD bool is_response_message(u32 t) {
  return t == M_ReplicateResp || t == M_RequestVoteResp || t == M_HeartbeatResp ||
         t == M_ReadIndexResp || t == M_Unreachable || t == M_SnapshotStatus ||
         t == M_LeaderTransfer;
}
// The node id of internal id x (slot + 1; 0 = NoNode) of local group g: the
// group's node-id table (Planes::node_ids on the device, the host copy in host
// code; rbe_set_node_ids) or, without one, x itself
RBE_HD u64 ext_id(const u64* ids, u32 n, u64 g, u64 x) {
  return (ids && x >= 1 && x <= n) ? ids[g * n + x - 1] : x;
}
// message fields that hold a node id besides From/To: a RequestVote's Hint
// (the leader-transfer candidate, raft.go:1098-1102) and a LeaderTransfer's
// (its target, raft.go:1712-1734)
RBE_HD bool hint_is_node(u32 type) { return type == M_RequestVote || type == M_LeaderTransfer; }
// The internal id (slot + 1) of node id `id` in local group g, 0 when none of
// the group's slots has it (0 = NoNode stays 0); without a table the id itself
template <int N>
RBE_HD u64 int_id(const u64* ids, u64 g, u64 id) {
  if (!ids) return id;
  if (id == 0) return 0;
  for (u32 s = 0; s < (u32)N; s++)
    if (ids[g * N + s] == id) return s + 1;
  return 0;
}

// rbe_message.reserved of an engine message: an InstallSnapshot's snapshot
// membership (Snapshot.Membership as the removed mask, Msg::pad0), else 0
RBE_HD u32 msg_reserved(const Msg& m) {
  return m.type == M_InstallSnapshot ? ((u32)m.pad0 | ((m.pad1 & 0xFFFFu) << 8)) : 0u;
}
RBE_HD bool is_leader_message(u32 t) {  // raft.go:1382-1385
  return t == M_Replicate || t == M_InstallSnapshot || t == M_Heartbeat || t == M_TimeoutNow ||
         t == M_ReadIndexResp;
}

// per-lane step result handed back to the kernel wrapper for wave reduction
struct StepCounters {
  u32 v[C_NUM];
};

// ----------------------------------------------------------------- the lane
enum : int {
  MODE_FULL = 0, MODE_LEAD = 1, MODE_FOLL = 2,
  MODE_FULL_LREM = 4,  // the whole table, the replica's remote slots in LDS (k_full_list)
};
// entries per batch of the general step's entry loops (Lane::copy_ring_to_arena,
// on_replicate): loads of a batch are issued together, then its stores
constexpr u32 kEntBatch = 8;
// The replica's remote slots during a step of the general table in LDS
// (MODE_FULL_LREM, k_full_list): loaded once before the step's first store,
// written back at its end.  The handlers read and update them message by
// message; in global memory each such read after the step's first store
// waited for every store before it (vmcnt is in order), a round trip per
// handler: C3's general step spent ~10 us per inbound message.
// threads per k_full_list block (rbe_kernels.h): the LDS arrays below hold
// one column per thread of the block
#ifndef RBE_FULL_BLOCK
#define RBE_FULL_BLOCK 64
#endif
constexpr u32 kLaneCols = RBE_FULL_BLOCK;
#if defined(__HIPCC__) || defined(__HIP__)
__device__ __forceinline__ RemoteMN (&lane_rem())[kMaxN][kLaneCols] {
  __shared__ RemoteMN s_rem[kMaxN][kLaneCols];
  return s_rem;
}
__device__ __forceinline__ u8 (&lane_rst())[kMaxN][kLaneCols] {
  __shared__ u8 s_rst[kMaxN][kLaneCols];
  return s_rst;
}
#endif
// The spill-tier state of one step (rbe_spill.h): the cold log's ref (loaded
// on first use), the outbox stash, the ReadyToRead / dropped-ReadIndex lists
// moved to the spill heap (granule, capacity; capacity 0 = still in the
// plane), the readIndex queue in pool pages (rqx, rqd)
struct LaneX {
  ColdRef cref;
  OutStash ost;
  u64 rtr_x, dri_x;
  RqExt rqd;
  u32 rtr_xcap, dri_xcap;
  bool cref_ld, cref_dirty, rqx;
};
#if defined(__HIPCC__) || defined(__HIP__)
__device__ __forceinline__ LaneX (&lane_x())[kLaneCols] {
  __shared__ LaneX s_x[kLaneCols];
  return s_x;
}
#endif

template <int N, bool TRACE, int MODE>
struct Lane {
  static constexpr bool FULL = MODE == MODE_FULL || MODE == MODE_FULL_LREM;  // the whole handler table
#if defined(__HIP_DEVICE_COMPILE__)
  static constexpr bool LREM = MODE == MODE_FULL_LREM;  // remote slots in LDS
#else
  static constexpr bool LREM = false;  // host builds keep them in the planes
#endif
  static constexpr bool LEAD = MODE == MODE_LEAD;  // steady-state leader subset
  static constexpr bool FOLL = MODE == MODE_FOLL;  // steady-state follower subset
  const Planes& P;
  const Params& C;
  const u64 r;      // global replica index
  const u64 g;      // group
  const u32 k;      // slot; node id = k + 1
  const u32 round;
  const u32 par;    // round & 1: outbox buffer written this round
  const Clk clk;    // round, ticks before it, whether it ticks
  const u64 cid;
  const u8 self;    // node id

  // registers: hot + core
  u8 role, flags, vresp, vgrant;
  u32 etick, htick, ret;
  u32 q_tick, q_qs, q_nas, q_eqt, rngc;
  bool q_new;
  u64 term, committed, last, processed, saved_to;
  u64 t_last;  // term of entry `last` (log-tail cache, kept in Core)
  u64 lead_start;  // leader: index of its no-op (Core::lead_start)
  u8 vote, leader, ltt, rq_head, rq_count;
  u8 members, cc_apply;  // Core::members / cc_apply (membership)
  u32 cc_acc;            // ConfigChanges the state machine accepted this step (Upd::cc_acc)
  u64 cc_i, cc_e;        // CCA_MULTI: the last step's apply range being handed to raft
  u32 cc_bits, cc_n;     //   its accepted bits, ConfigChanges passed so far
  bool cc_scan;
  u8 mfl;                // Core::mflags (MB_ROLES | MB_CC_IN_LOG)
  u8 obs, wit;           // raft.observers / raft.witnesses (Planes::roles; membership)
  u8 roles0;             // MB_ROLES at load: Planes::roles holds something to rewrite
  u64 c_match[N], c_next[N];  // LEAD: remote slots held in registers
  u32 c_st[N];
  u8 iso;  // isolation mask of this group for this round
  // spill-tier state of the step (LaneX): in LDS for k_full_list, whose
  // lanes are at the register limit, else a member
  mutable LaneX xm;
  RBE_HD LaneX& X() const {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (LREM) return lane_x()[threadIdx.x];
#endif
    return xm;
  }
  // snapshot_entries > 0: the LogDB compaction marker (SnapSt), the
  // InstallSnapshots sent this step (SnapshotStatus for the next one) and a
  // snapshot restored from one received
  u64 marker, marker_term;
  u8 snp_pend, snp_rej;
  bool snap_restored;
  u32 sm_ms;  // SnapSt::sm_*: the state machine's membership, packed (snapshot_entries)
  u64 applied0;  // raft.applied of this step (NotifyRaftLastApplied at its start)

  // per-step outputs
  u64 pc_lo, pc_hi;  // per destination 16-bit A | B << 7 | quiesce << 15 (registers)
  u32 arena_used;
  u64 seg_lo;
  u32 seg_off, seg_len;
  u64 mseg_lo;  // the last metadata copy for a witness (arena_meta_range)
  u32 mseg_off, mseg_len;
  bool seg_x, mseg_x;  // the segment is in the round spill heap (offsets are granules)
  u64 msg_hash, rtr_hash, drop_hash;
  u32 n_msgs, n_rtr, n_drop_ent, n_drop_ri;
  u32 fault;
  u32 events;        // EV_* of this step (Upd::events)
  // deferred fan-out actions, executed in this order after each event
  u32 rep_mask;      // slots to sendReplicateMessage to
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
  // diagnostic builds only: where a general step's wall time goes
  // (s_memrealtime ticks): before the event loop, inbox messages, local
  // events and ticks, the deferred fan-out after each event; the longest
  // inbox message; inbox messages handled
  u64 ip_t0 = 0, ip_pre = 0, ip_in = 0, ip_loc = 0, ip_fan = 0, ip_max = 0;
  u32 ip_nin = 0, ip_maxtype = 0;
#endif
  u8 tn_to;          // TimeoutNow target
  bool hb_pending;   // broadcastHeartbeatMessageWithHint(hb_lo, hb_hi)
  bool rq_pending;   // handleReadIndexLeaderConfirmation(rq_m)
  u64 hb_lo, hb_hi;
  u64 rq_lo, rq_hi;
  u8 rq_from;
  StepCounters& ctr;

  RBE_HD Lane(const Planes& P_, const Params& C_, u64 r_, Clk clk_, StepCounters& c_)
      : P(P_), C(C_), r(r_), g(r_ / N), k((u32)(r_ % N)), round(clk_.round),
        par(clk_.round & 1u), clk(clk_), cid(cid_of(C_, r_ / N)),
        self((u8)(r_ % N + 1)), ctr(c_) {}

  // ------------------------------------------------------------- faults
  RBE_HD void set_fault(u32 f) {
    if (!(fault & f)) ctr.v[C_FAULTS]++;
    fault |= f;
  }

  // ------------------------------------------------------------- log (term ring)
  // The in-memory window is the term / payload ring: entries [max(marker + 1,
  // last - ring + 1), last] (the invariant every append and merge below keeps).
  // Older entries above the LogDB marker are in the replica's cold log
  // (rbe_spill.h), the ILogDB read path of logentry.go:144-161 / 186-246.
  RBE_HD u64 ring_slot(u64 idx) const { return (idx & (u64)(C.ring - 1)) * C.n_rep + r; }
  RBE_HD ColdRef& cold() {
    if (!X().cref_ld) {
      X().cref = P.cold[r];
      X().cref_ld = true;
    }
    return X().cref;
  }
  // entry idx (marker < idx <= last) from the ring or the cold log
  RBE_HD Ent log_ent(u64 idx) {
    Ent e;
    if (last - idx < C.ring) {
      const u64 s = ring_slot(idx);
      const Body b = P.pay_ring[s];
      e.term = P.term_ring[s];
      e.type = b.type;
      e.len = b.len;
      e.lo = b.lo;
      e.hi = b.hi;
    } else if (!cold_get_ol(P, C, cold(), idx, &e)) {
      set_fault(F_WINDOW);  // the launch gave only the LogDB's tail
      e.term = e.lo = e.hi = 0;
      e.type = e.len = 0;
    }
    return e;
  }
  RBE_HD Body log_body(u64 idx) {
    if (last - idx < C.ring) return P.pay_ring[ring_slot(idx)];
    const Ent e = log_ent(idx);
    Body b;
    b.type = e.type;
    b.len = e.len;
    b.lo = e.lo;
    b.hi = e.hi;
    return b;
  }
  // entryLog.term (logentry.go:142-161): 0 with no error outside
  // [firstIndex-1, lastIndex]; firstIndex - 1 is the LogDB's compaction marker
  // (0 without snapshot_entries), whose term the LogDB keeps (Term(marker)).
  RBE_HD u64 log_term(u64 idx) {
    if (idx > last || idx == 0) return 0;
    if (idx == last) return t_last;
    if (C.snapshot_entries && idx <= marker) return idx == marker ? marker_term : 0;
    ctr.v[C_RING_ACCESS]++;
    if (last - idx < C.ring) return P.term_ring[ring_slot(idx)];
    return log_ent(idx).term;
  }
  RBE_HD bool match_term(u64 idx, u64 t) { return log_term(idx) == t; }  // logentry.go:357-363
  // log_term split for batched lookups: the value without side effects (a
  // prefetch that may run ahead of the loop that uses it; an index below the
  // ring peeks 0 and is looked up by log_term_account's caller), and the
  // ring-access count log_term would have raised for it
  RBE_HD u64 log_term_peek(u64 idx) const {
    if (idx > last || idx == 0) return 0;
    if (idx == last) return t_last;
    if (C.snapshot_entries && idx <= marker) return idx == marker ? marker_term : 0;
    if (last - idx >= C.ring) return 0;
    return P.term_ring[ring_slot(idx)];
  }
  RBE_HD bool log_term_cold(u64 idx) const {  // log_term(idx) reads the cold log
    return idx < last && idx != 0 && !(C.snapshot_entries && idx <= marker) && last - idx >= C.ring;
  }
  RBE_HD void log_term_account(u64 idx) {
    if (idx > last || idx == 0 || idx == last) return;
    if (C.snapshot_entries && idx <= marker) return;
    ctr.v[C_RING_ACCESS]++;
  }
  // Evict entry j (its ring slot about to be overwritten) into the cold log
  RBE_HD void evict(u64 j) {
    const u64 s = ring_slot(j);
    const Body b = P.pay_ring[s];
    Ent e;
    e.term = P.term_ring[s];
    e.type = b.type;
    e.len = b.len;
    e.lo = b.lo;
    e.hi = b.hi;
    cold_store(j, e);
  }
  RBE_HD void cold_store(u64 j, const Ent& e) {
    if (!cold_put_ol(P, C, cold(), j, e, par)) set_fault(F_NOMEM);
    X().cref_dirty = true;
  }
  // an append at idx = last + 1: the entry the ring slot held (idx - ring) goes
  // to the cold log unless it is compacted
  RBE_HD void log_append(u64 idx, u64 t, u32 type, u32 len, u64 lo, u64 hi) {
    if (idx > C.ring && idx - C.ring > marker) evict(idx - C.ring);
    ring_put(idx, t, type, len, lo, hi);
  }
  RBE_HD bool up_to_date(u64 idx, u64 t) {  // logentry.go:365-377
    u64 lt = log_term(last);
    if (t >= lt) {
      if (t > lt) return true;
      return idx >= last;
    }
    return false;
  }
  RBE_HD void commit_to(u64 idx) {  // logentry.go:324-333
    if (idx <= committed) return;
    if (idx > last) {
      set_fault(F_PANIC);
      return;
    }
    committed = idx;
  }
  RBE_HD bool log_try_commit(u64 idx, u64 t) {  // logentry.go:379-394
    if (idx <= committed) return false;
    u64 lt = log_term(idx);
    if (lt == t) {
      commit_to(idx);
      return true;
    }
    return false;
  }
  RBE_HD void ring_put(u64 idx, u64 t, u32 type, u32 len, u64 lo, u64 hi) {
    u64 s = ring_slot(idx);
    P.term_ring[s] = t;
    Body b;
    b.type = type;
    b.len = len;
    b.lo = lo;
    b.hi = hi;
    P.pay_ring[s] = b;
    ctr.v[C_RING_ACCESS]++;
  }
  // limitSize (entryutils.go:52-64) over [lo, hi] with sizes 128 + len
  RBE_HD u64 limit_count(u64 lo, u64 hi) {
    u64 n = hi - lo + 1;
    if (!C.heap_bytes && n * (128 + 16) <= C.max_entry_size) return n;  // Cmd <= 16 B
    u64 total = 128 + log_body(lo).len;
    u64 inc = 1;
    for (; inc < n; inc++) {
      total += 128 + log_body(lo + inc).len;
      if (total > C.max_entry_size) break;
    }
    return inc;
  }

  // ------------------------------------------------------------- remotes
  // Value accessors.  The leader-specialized fast mode keeps the N remote
  // slots in registers for the whole round (loaded by load(), written back by
  // store()); the selects over a compile-time N keep them out of scratch.
  // The other modes read and write the SoA planes directly.
#if defined(__HIP_DEVICE_COMPILE__)
  __device__ __forceinline__ RemoteMN& lrem(u32 s) const { return lane_rem()[s][threadIdx.x]; }
  __device__ __forceinline__ u8& lrst(u32 s) const { return lane_rst()[s][threadIdx.x]; }
#else
  RemoteMN& lrem(u32 s) const { return P.rem[r * N + s]; }  // (not instantiated on the host)
  u8& lrst(u32 s) const { return P.rem_st[r * N + s]; }
#endif
  RBE_HD u64 rmatch(u32 s) const {
    if constexpr (LEAD) {
      u64 v = 0;
      for (u32 i = 0; i < N; i++)
        if (i == s) v = c_match[i];
      return v;
    } else if constexpr (LREM) {
      return lrem(s).match;
    } else {
      return P.rem[r * N + s].match;
    }
  }
  RBE_HD u64 rnext(u32 s) const {
    if constexpr (LEAD) {
      u64 v = 0;
      for (u32 i = 0; i < N; i++)
        if (i == s) v = c_next[i];
      return v;
    } else if constexpr (LREM) {
      return lrem(s).next;
    } else {
      return P.rem[r * N + s].next;
    }
  }
  RBE_HD u32 rst(u32 s) const {
    if constexpr (LEAD) {
      u32 v = 0;
      for (u32 i = 0; i < N; i++)
        if (i == s) v = c_st[i];
      return v;
    } else if constexpr (LREM) {
      return lrst(s);
    } else {
      return P.rem_st[r * N + s];
    }
  }
  RBE_HD void set_rmatch(u32 s, u64 v) {
    if constexpr (LEAD) {
      for (u32 i = 0; i < N; i++)
        if (i == s) c_match[i] = v;
    } else if constexpr (LREM) {
      lrem(s).match = v;
    } else {
      P.rem[r * N + s].match = v;
    }
  }
  RBE_HD void set_rnext(u32 s, u64 v) {
    if constexpr (LEAD) {
      for (u32 i = 0; i < N; i++)
        if (i == s) c_next[i] = v;
    } else if constexpr (LREM) {
      lrem(s).next = v;
    } else {
      P.rem[r * N + s].next = v;
    }
  }
  RBE_HD void set_rst(u32 s, u32 v) {
    if constexpr (LEAD) {
      for (u32 i = 0; i < N; i++)
        if (i == s) c_st[i] = v;
    } else if constexpr (LREM) {
      lrst(s) = (u8)v;
    } else {
      P.rem_st[r * N + s] = (u8)v;
    }
  }
  RBE_HD u32 rstate(u32 slot) const { return rst(slot) & 3u; }
  RBE_HD void set_rstate(u32 slot, u32 s) { set_rst(slot, (rst(slot) & ~3u) | s); }
  RBE_HD bool ractive(u32 slot) const { return (rst(slot) >> 2) & 1u; }
  RBE_HD void set_active(u32 slot, bool a) { set_rst(slot, (rst(slot) & 3u) | (a ? 4u : 0u)); }
  RBE_HD bool is_paused(u32 slot) const {  // remote.go:173-186
    u32 s = rstate(slot);
    return s == RS_Wait || s == RS_Snapshot;
  }
  RBE_HD void wait_to_retry(u32 slot) {  // remote.go:94-98
    if (rstate(slot) == RS_Wait) set_rstate(slot, RS_Retry);
  }
  RBE_HD void become_retry(u32 slot) {  // remote.go:75-83
    u64 nx = rmatch(slot) + 1;
    if (rstate(slot) == RS_Snapshot) nx = umax64(nx, P.rem_snap[r * N + slot] + 1);
    set_rnext(slot, nx);
    set_rstate(slot, RS_Retry);
  }
  RBE_HD void become_snapshot(u32 slot, u64 idx) {  // remote.go:108-112
    P.rem_snap[r * N + slot] = idx;
    set_rstate(slot, RS_Snapshot);
  }
  RBE_HD void become_replicate(u32 slot) {  // remote.go:102-106
    set_rnext(slot, rmatch(slot) + 1);
    set_rstate(slot, RS_Replicate);
  }
  RBE_HD bool try_update(u32 slot, u64 idx) {  // remote.go:123-133
    ctr.v[C_REMOTE_TOUCH]++;
    if (rnext(slot) < idx + 1) set_rnext(slot, idx + 1);
    if (rmatch(slot) < idx) {
      wait_to_retry(slot);
      set_rmatch(slot, idx);
      return true;
    }
    return false;
  }
  RBE_HD void progress(u32 slot, u64 li) {  // remote.go:135-143
    u32 s = rstate(slot);
    if (s == RS_Replicate) set_rnext(slot, li + 1);
    else if (s == RS_Retry) set_rstate(slot, RS_Wait);
    else set_fault(F_PANIC);
  }
  RBE_HD void responded_to(u32 slot) {  // remote.go:145-153
    u32 s = rstate(slot);
    if (s == RS_Retry) become_replicate(slot);
    else if (s == RS_Snapshot && rmatch(slot) >= P.rem_snap[r * N + slot]) become_retry(slot);
  }
  RBE_HD bool decrease_to(u32 slot, u64 rejected, u64 lst) {  // remote.go:155-171
    if (rstate(slot) == RS_Replicate) {
      if (rejected <= rmatch(slot)) return false;
      set_rnext(slot, rmatch(slot) + 1);
      return true;
    }
    if (rnext(slot) - 1 != rejected) return false;
    wait_to_retry(slot);
    set_rnext(slot, umax64(1, umin64(rejected, lst + 1)));
    return true;
  }

  // ------------------------------------------------------------- emission
  RBE_HD u32 get_pc(u32 d) const {
    return d < 4 ? (u32)((pc_lo >> (16 * d)) & 0xFFFFu) : (u32)((pc_hi >> (16 * (d - 4))) & 0xFFFFu);
  }
  RBE_HD void add_pc(u32 d, u32 v) {
    if (d < 4) pc_lo += (u64)v << (16 * d);
    else pc_hi += (u64)v << (16 * (d - 4));
  }
  RBE_HD u64 msg_slot_base(u32 sender, u32 dest) const {
    return ((g * N + sender) * N + dest) * (u64)C.maxm;
  }
  // raft.send + finalizeMessageTerm (raft.go:640-658) + the network: the
  // message joins Update.Messages (hashed here, in emission order) and is
  // written to the (self → dest) list, Replicate messages in front (node.go
  // sends them before persistence, 897-905) and the rest behind (888-895).
  RBE_HD void send(Msg& m) {
    m.from = self;
    if (m.type != M_RequestVote) {
      if (m.type == M_Propose || m.type == M_ReadIndex) m.term = 0;
      else m.term = term;
    }
    n_msgs++;
    const u32 ne = msg_nent(m);
    if (TRACE) {
      u64 h = msg_hash;
      h = hfold(h, (u64)m.type | ((u64)m.reject << 8) | ((u64)ne << 16));
      h = hfold(h, m.to);
      h = hfold(h, m.from);
      h = hfold(h, m.term);
      h = hfold(h, m.log_term);
      h = hfold(h, m.log_index);
      h = hfold(h, m.commit);
      h = hfold(h, m.hint);
      h = hfold(h, m.hint_high);
      if (ne) {
        const Ent* a = msg_ents(P, C, par, r, m);
        for (u32 i = 0; i < ne; i++) {
          Ent e = a[i];
          u64 idx = m.type == M_Replicate ? m.log_index + 1 + i : 0;
          h = hfold(h, idx);
          h = hfold(h, e.term);
          h = hfold(h, ent_word(e.type, e.len));
          h = hfold(h, e.lo);
          h = hfold(h, cmd_hi(e.type, e.hi));
        }
      }
      msg_hash = h;
    }
    if (m.to < 1 || m.to > N) return;
    u32 d = m.to - 1u;
    if (((iso >> k) & 1u) || ((iso >> d) & 1u)) {
      ctr.v[C_MSG_DROPPED]++;
      return;
    }
    const u32 pc = get_pc(d);
    u32 a = pc & 0x7Fu, b = (pc >> 7) & 0x7Fu;
    if (a + b >= C.maxm) {
      // the plane list is full: the message joins the step's stash, and the
      // list moves whole to the spill heap at the step's end (outbox_relocate)
      if (stash_put_ol(P, C, par, X().ost, m)) {
        ctr.v[C_MSG_OUT]++;
        ctr.v[C_ENT_OUT] += ne;
      } else {
        set_fault(F_NOMEM);
      }
      return;
    }
    u32 slot;
    if (m.type == M_Replicate) {
      slot = a;
      add_pc(d, 1u);
    } else {
      slot = C.maxm - 1u - b;
      add_pc(d, 1u << 7);
    }
    const u64 at = msg_slot_base(k, d) + slot;
    ctr.v[C_MSG_OUT]++;
    ctr.v[C_ENT_OUT] += ne;
    P.msgs[par][at] = m;
  }
  RBE_HD Msg mk(u32 type, u8 to) const {
    Msg m;
    m.type = (u8)type;
    m.from = 0;
    m.to = to;
    m.reject = 0;
    m.n_ent = 0;
    m.pad0 = 0;
    m.ent_off = 0;
    m.pad1 = 0;
    m.term = m.log_term = m.log_index = m.commit = m.hint = m.hint_high = 0;
    return m;
  }
  // log entries [lo, lo + cnt) from the ring (or the cold log below it) to
  // `out`, kEntBatch at a time (every load of a batch before its stores)
  RBE_HD void copy_ring_to_arena(u64 lo, u32 cnt, Ent* out) {
    for (u32 i0 = 0; i0 < cnt; i0 += kEntBatch) {
      Ent e[kEntBatch];
#pragma unroll
      for (u32 j = 0; j < kEntBatch; j++) {
        if (i0 + j >= cnt) continue;
        const u64 idx = lo + i0 + j;
        if (last - idx >= C.ring) {
          e[j] = log_ent(idx);
          continue;
        }
        const u64 s = ring_slot(idx);
        const Body b = P.pay_ring[s];
        e[j].term = P.term_ring[s];
        e[j].type = b.type;
        e[j].len = b.len;
        e[j].lo = b.lo;
        e[j].hi = b.hi;
      }
#pragma unroll
      for (u32 j = 0; j < kEntBatch; j++) {
        if (i0 + j >= cnt) continue;
        if (heap_lapped(P, C, e[j].type, e[j].hi)) set_fault(F_WINDOW);
        out[i0 + j] = e[j];
      }
    }
  }
  // cnt entries of the round spill heap for a message whose entries do not
  // fit the sender's arena (granule in *off), ~0 when the heap is full
  RBE_HD Ent* spill_ents(u32 cnt, u32* off) {
    const u64 g = spill_alloc_ol(P, C, par, (u64)cnt * sizeof(Ent));
    if (g == ~0ull) {
      set_fault(F_NOMEM);
      return nullptr;
    }
    *off = (u32)g;
    return spill_at<Ent>(P, par, g);
  }
  // copy log entries [lo, lo+cnt) into this round's arena (reusing the last
  // copied segment when it already covers them), or into the round spill heap
  // when the arena cannot take them (*x): makeReplicateMessage's entries,
  // limited only by MaxEntrySize (raft.go:709-740)
  RBE_HD bool arena_log_range(u64 lo, u32 cnt, u32* off, bool* x) {
    if (seg_len && lo >= seg_lo && lo + cnt <= seg_lo + seg_len) {
      *off = seg_off + (u32)(lo - seg_lo) * (seg_x ? 2u : 1u);
      *x = seg_x;
      return true;
    }
    Ent* a = &P.arena[par][r * C.ecap];
    if (!seg_x && seg_len && lo >= seg_lo && lo <= seg_lo + seg_len &&
        seg_off + seg_len == arena_used) {
      u64 have_hi = seg_lo + seg_len;  // exclusive
      u32 extra = (u32)(lo + cnt - have_hi);
      if (arena_used + extra <= C.ecap) {
        copy_ring_to_arena(have_hi, extra, a + arena_used);
        ctr.v[C_RING_ACCESS] += extra;
        arena_used += extra;
        seg_len += extra;
        *off = seg_off + (u32)(lo - seg_lo);
        *x = false;
        return true;
      }
    }
    Ent* dst = nullptr;
    u32 o = arena_used;
    const bool sx = arena_used + cnt > C.ecap;
    if (sx) {
      if (!(dst = spill_ents(cnt, &o))) return false;
    } else {
      dst = a + arena_used;
      arena_used += cnt;
    }
    copy_ring_to_arena(lo, cnt, dst);
    ctr.v[C_RING_ACCESS] += cnt;
    seg_lo = lo;
    seg_off = o;
    seg_len = cnt;
    seg_x = sx;
    *off = o;
    *x = sx;
    return true;
  }
  // entries [lo, lo+cnt) for a witness (makeMetadataEntries, raft.go:742-756):
  // a copy of their own in the arena where every entry but a ConfigChange is a
  // MetadataEntry with only its index and term
  RBE_HD bool arena_meta_range(u64 lo, u32 cnt, u32* off, bool* x) {
    if (mseg_len && lo >= mseg_lo && lo + cnt <= mseg_lo + mseg_len) {
      *off = mseg_off + (u32)(lo - mseg_lo) * (mseg_x ? 2u : 1u);
      *x = mseg_x;
      return true;
    }
    Ent* a = nullptr;
    u32 o = arena_used;
    const bool sx = arena_used + cnt > C.ecap;
    if (sx) {
      if (!(a = spill_ents(cnt, &o))) return false;
    } else {
      a = &P.arena[par][r * C.ecap + arena_used];
      arena_used += cnt;
    }
    copy_ring_to_arena(lo, cnt, a);
    ctr.v[C_RING_ACCESS] += cnt;
    for (u32 i = 0; i < cnt; i++)
      if (ent_type(a[i].type) != E_ConfigChange) {
        a[i].type = E_Metadata;
        a[i].len = 0;
        a[i].lo = a[i].hi = 0;
      }
    mseg_lo = lo;
    mseg_off = o;
    mseg_len = cnt;
    mseg_x = sx;
    *off = o;
    *x = sx;
    return true;
  }
  // entries of a Propose this step sends or hands to its own handler; the
  // pointer it can read them from (null when the spill heap is exhausted)
  RBE_HD const Ent* arena_put(const Ent* src, u32 cnt, u32* off, bool* x) {
    Ent* a = nullptr;
    *x = arena_used + cnt > C.ecap;
    if (*x) {
      if (!(a = spill_ents(cnt, off))) return nullptr;
    } else {
      a = &P.arena[par][r * C.ecap + arena_used];
      *off = arena_used;
      arena_used += cnt;
    }
    for (u32 i = 0; i < cnt; i++) a[i] = src[i];
    return a;
  }
  // a message's entry reference: the arena offset, or the spill heap
  RBE_HD static void set_ents(Msg& m, u32 cnt, u32 off, bool x) {
    m.n_ent = (u16)(cnt > 0xFFFFu ? 0xFFFFu : cnt);
    m.ent_off = off;
    if (x) {
      m.pad0 |= kMsgXEnt;
      m.pad1 = cnt;
    }
  }

  // ------------------------------------------------------------- outputs
  // The step's ReadyToReads / dropped ReadIndexes: the plane list, then, past
  // its capacity, the whole list in the round spill heap (rtr_x / dri_x, its
  // granule; the plane's slot 0 names it at the step's end)
  template <class T>
  RBE_HD bool out_list_put(T* plane, u32 pcap, u32 n, u64& xg, u32& xcap, const T& v) {
    if (n < pcap) {
      plane[n] = v;
      return true;
    }
    if (n >= xcap) {  // (re)allocate at twice the size and copy what is there
      const u32 cap = n * 2u;
      const u64 g = spill_alloc_ol(P, C, par, (u64)cap * sizeof(T));
      if (g == ~0ull) return false;
      T* nb = spill_at<T>(P, par, g);
      const T* ob = xcap ? spill_at<T>(P, par, xg) : plane;
      for (u32 i = 0; i < n; i++) nb[i] = ob[i];
      xg = g;
      xcap = cap;
    }
    spill_at<T>(P, par, xg)[n] = v;
    return true;
  }
  RBE_HD void add_ready_to_read(u64 index, u64 low, u64 high) {  // raft.go:1624-1630
    RTR x;
    x.index = index;
    x.low = low;
    x.high = high;
    if (!out_list_put(&P.rtr[r * C.rtr_cap], C.rtr_cap, n_rtr, X().rtr_x, X().rtr_xcap, x)) {
      set_fault(F_NOMEM);
      return;
    }
    n_rtr++;
    if (TRACE) {
      rtr_hash = hfold(rtr_hash, index);
      rtr_hash = hfold(rtr_hash, low);
      rtr_hash = hfold(rtr_hash, high);
    }
  }
  RBE_HD void add_dropped_ri(u64 low, u64 high) {
    DropRI x;
    x.low = low;
    x.high = high;
    if (!out_list_put(&P.dri[r * C.dri_cap], C.dri_cap, n_drop_ri, X().dri_x, X().dri_xcap, x)) {
      set_fault(F_NOMEM);
      return;
    }
    n_drop_ri++;
  }
  RBE_HD void report_dropped_read_index(u64 low, u64 high) {  // raft.go:1999-2012
    add_dropped_ri(low, high);
    events |= EV_READ_INDEX_DROPPED;
  }
  RBE_HD void report_dropped_proposal(const Ent* e, u32 cnt) {  // raft.go:1987-1997
    if (cnt) events |= EV_PROPOSAL_DROPPED;
    for (u32 i = 0; i < cnt; i++) {
      n_drop_ent++;
      if (TRACE) {
        drop_hash = hfold(drop_hash, 0);
        drop_hash = hfold(drop_hash, e[i].term);
        drop_hash = hfold(drop_hash, ent_word(e[i].type, e[i].len));
        drop_hash = hfold(drop_hash, e[i].lo);
        drop_hash = hfold(drop_hash, cmd_hi(e[i].type, e[i].hi));
      }
    }
  }

  // ------------------------------------------------------------- state transitions
  RBE_HD void set_randomized_election_timeout() {  // raft.go:631-634
    u64 x = below(rto_rand(C.seed, cid, self, rngc++), C.election_rtt);
    ret = (u32)(C.election_rtt + x);
  }
  RBE_HD void reset_remotes() {  // raft.go:1023-1032
    for (u32 s = 0; s < N; s++) {
      set_rmatch(s, s == k ? last : 0);
      set_rnext(s, last + 1);
      set_rst(s, 0);
    }
    ctr.v[C_REMOTE_TOUCH] += N;
  }
  RBE_HD void reset(u64 t) {  // raft.go:989-1008
    if (term != t) {
      term = t;
      vote = 0;
    }
    vresp = vgrant = 0;
    etick = 0;
    htick = 0;
    set_randomized_election_timeout();
    rq_clear();
    flags &= (u8)~HF_PENDING_CC;
    ltt = 0;
    reset_remotes();
    seg_len = mseg_len = 0;
    if (rl_on()) P.rl[r].fmask = 0;  // rl.ResetFollowerState
  }
  RBE_HD void become_follower(u64 t, u8 lid) {  // raft.go:947-955
    if (role == R_Witness) set_fault(F_PANIC);  // "transitioning to follower from witness state"
    role = R_Follower;
    reset(t);
    leader = lid;
  }
  RBE_HD void become_nonvoting(u64 t, u8 lid) {  // becomeObserver / becomeWitness, raft.go:926-946
    reset(t);
    leader = lid;
  }
  RBE_HD void become_candidate() {  // raft.go:957-973
    role = R_Candidate;
    reset(term + 1);
    leader = 0;
    vote = self;
  }
  RBE_HD void become_leader() {  // raft.go:975-987
    role = R_Leader;
    reset(term);
    leader = self;
    // preLeaderPromotionHandleConfigChange (raft.go:1010-1018): count config
    // change entries in (committed, last]
    u32 ncc = 0;
    for (u64 i = committed + 1; i <= last; i++)
      if (ent_type(log_body(i).type) == E_ConfigChange) ncc++;
    if (ncc > 1) set_fault(F_PANIC);
    else if (ncc == 1) flags |= HF_PENDING_CC;
    // p72 of the raft thesis: an empty entry at the new term
    append_entry(E_Application, 0, 0, 0);
    lead_start = last;
  }
  // appendEntries (raft.go:909-920) for one entry
  RBE_HD void append_entry(u32 type, u32 len, u64 lo, u64 hi) {
    u64 idx = last + 1;
    rl_grow(len);
    log_append(idx, term, type, len, lo, hi);
    last = idx;
    t_last = term;
    try_update(k, last);
    if (quorum() == 1) try_commit();
  }

  // ------------------------------------------------------------- rate limiter
  // server.RateLimiter through the in-memory log's size hooks (inmemory.go:
  // 139-246) and raft.go:660-683; sizes from the payload ring's Cmd lengths
  RBE_HD bool rl_on() const { return rl_enabled(C.rl_max); }
  RBE_HD void rl_grow(u32 len) {  // merge of an appended entry: rl.Increase
    if (rl_on()) P.rl[r].size += kEntryInMem + len;
  }
  // sum over log entries [lo, hi] of `base` + Cmd length (the ring holds them
  // while last - i < ring; F_WINDOW otherwise)
  RBE_HD u64 rl_range(u64 lo, u64 hi, u64 base) {
    u64 s = 0;
    for (u64 i = lo; i <= hi && i >= lo; i++) s += base + log_body(i).len;
    return s;
  }
  // inMemory.merge (inmemory.go:201-234) of entries from `first` on, before
  // the ring takes them: append, replace or cut-and-append
  RBE_HD void rl_merge(u64 first, const Ent* ents, u32 cnt) {
    RlSt& s = P.rl[r];
    u64 add = 0;
    for (u32 i = 0; i < cnt; i++) add += kEntryInMem + ents[i].len;
    const u64 im = P.imark[r];
    if (first == last + 1) {
      s.size += add;
    } else if (first <= im) {
      s.new_ent = 1;
      s.size = add;
    } else {
      s.size = add + rl_range(im, first - 1, kEntryInMem);
      s.new_ent = 1;
    }
  }
  // inMemory.appliedLogTo (inmemory.go:139-167): the marker moves to `idx` and
  // the entries applied leave the count, the old marker only after a rebuild
  RBE_HD void rl_applied_to(u64 idx) {
    const u64 im = P.imark[r];
    if (idx < im || im > last || idx > last) return;
    RlSt& s = P.rl[r];
    const u64 lo = s.new_ent ? im : im + 1;
    if (lo <= idx) s.size -= rl_range(lo, idx, kEntryInMem);
    s.new_ent = 0;
    P.imark[r] = idx;
  }
  RBE_HD void send_rate_limit() {  // sendRateLimitMessage, raft.go:660-683 (not a leader)
    if (leader == 0) return;  // skipped, no leader
    u64 mv = 0;
    if (rl_limited(P.rl[r], C.rl_max)) {  // max(inmemSz-notCommitedSz, 0) on uint64: wraps
      // getUncommittedEntries (logentry.go:180-183) reads the in-memory log
      // only: [max(committed + 1, markerIndex), last] (getEntriesFromInMem,
      // logentry.go:205-211)
      const u64 lo = umax64(committed + 1, P.imark[r]);
      mv = P.rl[r].size - (lo <= last ? rl_range(lo, last, kEntryNonCmd) : 0);
    }
    Msg x = mk(M_RateLimit, leader);
    x.hint = mv;
    send(x);
  }

  // ------------------------------------------------------------- membership
  // raft.remotes of this replica's view: every slot not in Core::members'
  // removed bits (raft.go:366-416 numVotingMembers / quorum / votingMembers);
  // observers and witnesses in Planes::roles (obs / wit)
  RBE_HD bool voter(u32 s) const { return !((members >> s) & 1u); }  // in raft.remotes
  RBE_HD u32 voters_mask() const { return ((1u << N) - 1u) & ~(u32)members; }
  RBE_HD bool is_obs(u32 s) const { return (obs >> s) & 1u; }
  RBE_HD bool is_wit(u32 s) const { return (wit >> s) & 1u; }
  // votingMembers (raft.go:410-419): remotes and witnesses
  RBE_HD u32 vmask() const { return voters_mask() | wit; }
  RBE_HD u32 quorum() const { return popc8(vmask()) / 2 + 1; }  // raft.go:366-372
  // remotes, observers and witnesses: lw (raft.go:2013-2027), Peer.Handle
  RBE_HD bool member(u32 s) const { return voter(s) || is_obs(s) || is_wit(s); }
  RBE_HD bool from_member(u32 from) const { return from >= 1 && from <= N && member(from - 1u); }
  RBE_HD void set_remote(u32 s) {  // setRemote / setObserver / setWitness(id, 0, lastIndex + 1)
    set_rmatch(s, 0);
    set_rnext(s, last + 1);
    set_rst(s, 0);
  }
  // handleNodeConfigChange (raft.go:1537-1556) → addNode / removeNode /
  // addObserver / addWitness (raft.go:1135-1198); `m.hint` = node id,
  // `m.hint_high` = ConfigChangeType
  RBE_HD void on_config_change(const Msg& m) {
    if (!C.membership) {
      set_fault(F_UNSUPPORTED);
      return;
    }
    if (m.reject) {  // RejectConfigChange: clearPendingConfigChange
      flags &= (u8)~HF_PENDING_CC;
      return;
    }
    const u64 nid = m.hint;
    const u32 type = (u32)m.hint_high;
    if (type > CC_AddWitness) {
      set_fault(F_PANIC);  // "unexpected config change type"
      return;
    }
    if (nid < 1 || nid > N) {  // a node outside the group's slots
      set_fault(F_UNSUPPORTED);
      return;
    }
    const u32 s = (u32)nid - 1u;
    const u8 bit = (u8)(1u << s);
    flags &= (u8)~HF_PENDING_CC;  // clearPendingConfigChange
    if (type == CC_AddNode) {
      if (s == k && role == R_Witness) {  // "is a witness"
        set_fault(F_PANIC);
        return;
      }
      if (voter(s)) return;  // already a voting member
      if (is_obs(s)) {  // an observer is promoted with its progress (raft.go:1144-1151)
        obs &= (u8)~bit;
        members &= (u8)~bit;
        if (s == k) become_follower(term, leader);
        return;
      }
      if (is_wit(s)) {  // "could not promote witness to a full member"
        set_fault(F_PANIC);
        return;
      }
      members &= (u8)~bit;
      set_remote(s);
      return;
    }
    if (type == CC_AddObserver || type == CC_AddWitness) {  // raft.go:1159-1180
      const bool ob = type == CC_AddObserver;
      if (s == k && role != (ob ? R_Observer : R_Witness)) {  // "is not an observer / a witness"
        set_fault(F_PANIC);
        return;
      }
      if (ob ? is_obs(s) : is_wit(s)) return;
      if (member(s)) {  // a node in two of the maps at once: not held by a slot
        set_fault(F_UNSUPPORTED);
        return;
      }
      if (ob) obs |= bit;
      else wit |= bit;
      set_remote(s);
      return;
    }
    // RemoveNode: deleteRemote / deleteObserver / deleteWitness
    members |= bit;
    obs &= (u8)~bit;
    wit &= (u8)~bit;
    if (s == k && role == R_Leader) become_follower(term, 0);
    if (ltt != 0 && role == R_Leader && ltt == (u8)nid) ltt = 0;  // abortLeaderTransfer
    if (role == R_Leader && vmask() != 0) {
      if (try_commit()) broadcast_replicate();
    }
  }
  // restoreRemotes (raft.go:472-517) for Handle(SnapshotReceived), which
  // Peer.RestoreRemotes sends once the state machine recovered from a snapshot
  // (peer.go:159-165): raft.remotes / observers / witnesses become the
  // snapshot's (`ms`: slots not in Addresses | Observers << 8 | Witnesses << 16),
  // every remote restarts at match 0 / next lastIndex + 1 (self: match
  // lastIndex), Retry and inactive; an observer the snapshot lists as a voter
  // becomes a follower, a leader it does not list steps down.
  RBE_HD void restore_remotes(u32 ms) {
    const u32 full = (1u << N) - 1u;
    const u32 addr = full & ~(ms & 0xFFu);
    if (addr & wit) {  // "Assumed witness could not promote to full member"
      set_fault(F_PANIC);
      return;
    }
    if (((addr >> k) & 1u) && role == R_Observer) become_follower(term, leader);
    members = (u8)(~addr & MB_REMOVED & full);
    obs = (u8)((ms >> 8) & full);
    wit = (u8)((ms >> 16) & full);
    for (u32 s = 0; s < N; s++) {
      set_rmatch(s, s == k ? last : 0);
      set_rnext(s, last + 1);
      set_rst(s, 0);
    }
    ctr.v[C_REMOTE_TOUCH] += N;
    if (!voter(k) && role == R_Leader) become_follower(term, 0);  // selfRemoved() && isLeader()
  }
  // a log entry that is a ConfigChange: MB_CC_IN_LOG until it is applied
  RBE_HD void note_cc(u32 type) {
    if (ent_type(type) == E_ConfigChange) mfl |= MB_CC_IN_LOG;
  }

  // ------------------------------------------------------------- commit (kernel 1)
  // tryCommit (raft.go:886-907): q = matched[n - quorum] of the sorted match
  // values = the quorum-th largest; a register-resident selection over N.
  RBE_HD u64 kth_match() {
    u64 m[N];
    // non-voters sort below every voter (match 0), so the quorum-th largest of
    // the voters is the quorum-th largest of all N (raft.go tryCommit over
    // r.remotes and r.witnesses)
    for (u32 s = 0; s < N; s++) m[s] = (voter(s) || is_wit(s)) ? rmatch(s) : 0;
    // odd-even transposition sort (fully unrolled for a compile-time N)
    for (u32 pass = 0; pass < N; pass++) {
      for (u32 i = pass & 1u; i + 1 < N; i += 2) {
        u64 a = m[i], b = m[i + 1];
        m[i] = a < b ? a : b;
        m[i + 1] = a < b ? b : a;
      }
    }
    ctr.v[C_REMOTE_TOUCH] += N;
    return m[N - quorum()];
  }
  RBE_HD bool try_commit() { return log_try_commit(kth_match(), term); }

  // ------------------------------------------------------------- replication
  RBE_HD void send_replicate(u32 slot) {  // raft.go:758-792
    if (is_paused(slot)) return;
    u64 next = rnext(slot);
    if (C.snapshot_entries && next <= marker) {
      // entries(next) is ErrCompacted (logentry.go:163-178): the remote gets
      // the LogDB's snapshot if it is active (makeInstallSnapshotMessage,
      // raft.go:684-697); the record carries its (index, term) as LogIndex /
      // LogTerm, and the transport reports its outcome to the next step
      if (!ractive(slot)) return;
      const SnapSt& sp = P.snp[r];
      // entryLog.snapshot (logentry.go:248-253): the in-memory snapshot while
      // the host has not committed it (ext_commit; it sits at the marker), else
      // the LogDB's latest
      const bool im = C.ext_commit && sp.upd_ss;
      const u64 si = im ? marker : sp.ss_index;
      Msg m = mk(M_InstallSnapshot, (u8)(slot + 1));
      m.log_index = si;
      m.log_term = im ? marker_term : sp.ss_term;
      // Snapshot.Membership: the slots not in Addresses, its Observers and Witnesses
      m.pad0 = im ? sp.upd_rem : sp.ss_rem;
      m.pad1 = im ? ((u32)sp.upd_obs | ((u32)sp.upd_wit << 8))
                  : ((u32)sp.ss_obs | ((u32)sp.ss_wit << 8));
      become_snapshot(slot, si);
      const u32 bit = 1u << slot;
      snp_pend |= (u8)bit;
      if (((iso >> k) & 1u) || ((iso >> slot) & 1u)) snp_rej |= (u8)bit;
      else snp_rej &= (u8)~bit;
      send(m);
      return;
    }
    // makeReplicateMessage (raft.go:709-740)
    u64 lt = log_term(next - 1);
    Msg m = mk(M_Replicate, (u8)(slot + 1));
    m.log_index = next - 1;
    m.log_term = lt;
    m.commit = committed;
    if (next <= last) {
      u64 cnt = limit_count(next, last);
      u32 off = 0;
      bool x = false;
      const bool ok = ((wit >> slot) & 1u) ? arena_meta_range(next, (u32)cnt, &off, &x)
                                           : arena_log_range(next, (u32)cnt, &off, &x);
      if (ok) set_ents(m, (u32)cnt, off, x);
      progress(slot, next + cnt - 1);
    }
    send(m);
  }
  // Fan-out sends are deferred to the single post-event site in run() (same
  // emission order: every handler requests them as its last action).
  RBE_HD void broadcast_replicate() {  // raft.go:794-808 (r.nodes(): remotes, observers, witnesses)
    rep_mask |= (voters_mask() | obs | wit) & ~(1u << k);
  }
  RBE_HD void request_replicate(u32 slot) { rep_mask |= 1u << slot; }  // sendReplicateMessage
  RBE_HD void send_heartbeat(u32 slot, u64 low, u64 high) {  // raft.go:810-820
    Msg m = mk(M_Heartbeat, (u8)(slot + 1));
    m.commit = umin64(rmatch(slot), committed);
    m.hint = low;
    m.hint_high = high;
    send(m);
  }
  RBE_HD void broadcast_heartbeat_with_hint(u64 low, u64 high) {  // raft.go:834-846
    hb_pending = true;
    hb_lo = low;
    hb_hi = high;
  }
  RBE_HD void broadcast_heartbeat() {  // raft.go:824-832
    if (rq_len() > 0) {
      const ReadReq& q = *rq_at(rq_len() - 1u);
      broadcast_heartbeat_with_hint(q.low, q.high);
    } else {
      broadcast_heartbeat_with_hint(0, 0);
    }
  }

  // ------------------------------------------------------------- readIndex (kernel 4)
  // The queue (readindex.go:24-34, unbounded) is the plane ring of rq_cap
  // entries (rq_head, rq_count) until it would overflow; then it moves whole
  // into pool pages (rqx, rqd; rbe_spill.h) and returns when it drains.
  RBE_HD u32 rq_wrap(u32 x) const { return x >= C.rq_cap ? x - C.rq_cap : x; }  // x < 2*cap
  RBE_HD u32 rq_len() const { return X().rqx ? X().rqd.n : (u32)rq_count; }
  RBE_HD ReadReq* rq_at(u32 i) {
    if (X().rqx) return rq_ext_at(P, X().rqd, i);
    return &P.rq[r * C.rq_cap + rq_wrap((u32)rq_head + i)];
  }
  // the queue of a full ring into pool pages; false when the pool is exhausted
  RBE_HD bool rq_extend() {
    RqExt x;
    x.head = x.tail = pool_alloc_ol(P, C, par);
    if (!x.head) return false;
    P.pmeta[x.head].next = 0;
    x.off = 0;
    x.n = 0;
    for (u32 i = 0; i < rq_count; i++) {
      if (i > 0 && i % kPageEnts == 0) {
        const u32 p = pool_alloc_ol(P, C, par);
        if (!p) {
          rq_ext_free_ol(P, C, x, par);
          return false;
        }
        P.pmeta[p].next = 0;
        P.pmeta[x.tail].next = p;
        x.tail = p;
      }
      *(ReadReq*)pool_ent(P, x.tail, i % kPageEnts) = P.rq[r * C.rq_cap + rq_wrap((u32)rq_head + i)];
      x.n++;
    }
    X().rqd = x;
    X().rqx = true;
    rq_head = 0;
    return true;
  }
  RBE_HD bool rq_push(const ReadReq& q) {
    if (!X().rqx && rq_count < C.rq_cap) {
      *rq_at(rq_count) = q;
      rq_count++;
      return true;
    }
    if (!X().rqx && !rq_extend()) return false;
    const u32 pos = X().rqd.off + X().rqd.n;
    if (pos % kPageEnts == 0) {  // the tail page is full
      const u32 p = pool_alloc_ol(P, C, par);
      if (!p) return false;
      P.pmeta[p].next = 0;
      P.pmeta[X().rqd.tail].next = p;
      X().rqd.tail = p;
    }
    *(ReadReq*)pool_ent(P, X().rqd.tail, pos % kPageEnts) = q;
    X().rqd.n++;
    return true;
  }
  RBE_HD void rq_pop(u32 done) {
    if (!X().rqx) {
      rq_head = (u8)rq_wrap((u32)rq_head + done);
      rq_count = (u8)(rq_count - done);
      return;
    }
    X().rqd.n -= done;
    X().rqd.off += done;
    if (X().rqd.n == 0) {  // drained: back to the plane ring
      rq_ext_free_ol(P, C, X().rqd, par);
      X().rqx = false;
      rq_head = rq_count = 0;
      return;
    }
    while (X().rqd.off >= kPageEnts) {
      const u32 nx = P.pmeta[X().rqd.head].next;
      pool_free_ol(P, C, par, X().rqd.head);
      X().rqd.head = nx;
      X().rqd.off -= kPageEnts;
    }
  }
  RBE_HD void rq_clear() {
    if (X().rqx) rq_ext_free_ol(P, C, X().rqd, par);
    X().rqx = false;
    rq_head = rq_count = 0;
  }
  RBE_HD void rq_add(u64 index, u64 low, u64 high, u8 from) {  // readindex.go:43-67
    const u32 n = rq_len();
    for (u32 i = 0; i < n; i++) {
      ReadReq* q = rq_at(i);
      if (q->low == low && q->high == high) return;
    }
    if (n > 0 && index < rq_at(n - 1)->index) set_fault(F_PANIC);
    ReadReq q;
    q.low = low;
    q.high = high;
    q.index = index;
    q.from = from;
    q.confirmed = 0;
    for (int i = 0; i < 6; i++) q.pad[i] = 0;
    if (!rq_push(q)) {
      set_fault(F_NOMEM);
      return;
    }
    ctr.v[C_RQ_TOUCH]++;
  }
  // readIndex.confirm (readindex.go:77-116) + handleReadIndexLeaderConfirmation
  // (raft.go:1736-1756)
  RBE_HD void rq_confirm(u64 low, u64 high, u8 from, u64 m_hint, u64 m_hint_high) {
    int pos = -1;
    const u32 n = rq_len();
    for (u32 i = 0; i < n; i++) {
      ReadReq* q = rq_at(i);
      if (q->low == low && q->high == high) {
        pos = (int)i;
        break;
      }
    }
    if (pos < 0) return;
    ReadReq* p = rq_at((u32)pos);
    p->confirmed |= (u8)(1u << (from - 1));
    ctr.v[C_RQ_TOUCH]++;
    if ((int)popc8(p->confirmed) + 1 < (int)quorum()) return;
    u64 sindex = p->index;
    u32 done = (u32)pos + 1;
    for (u32 i = 0; i < done; i++) {
      ReadReq q = *rq_at(i);
      if (q.index > sindex) set_fault(F_PANIC);
      if (q.from == 0 || q.from == self) {
        add_ready_to_read(sindex, q.low, q.high);
      } else {
        Msg m = mk(M_ReadIndexResp, q.from);
        m.log_index = sindex;
        m.hint = m_hint;
        m.hint_high = m_hint_high;
        send(m);
      }
    }
    ctr.v[C_RQ_TOUCH] += done;
    rq_pop(done);
  }

  // ------------------------------------------------------------- leader handlers
  RBE_HD void on_leader_propose(const Ent* ents, u32 cnt) {  // raft.go:1587-1606
    if (ltt != 0) {  // leaderTransfering
      report_dropped_proposal(ents, cnt);
      return;
    }
    if (!C.membership) {
      for (u32 i = 0; i < cnt; i++) {
        if (ent_type(ents[i].type) == E_ConfigChange) {
          set_fault(F_UNSUPPORTED);  // config change proposals need cfg.membership
          return;
        }
      }
    }
    for (u32 i = 0; i < cnt; i++) {
      u64 idx = last + 1;
      Ent e = ents[i];
      if (ent_type(e.type) == E_ConfigChange) {
        if (flags & HF_PENDING_CC) {
          // reportDroppedConfigChange (raft.go:1983-1985): the entry joins
          // DroppedEntries and an empty application entry takes its place
          n_drop_ent++;
          if (TRACE) {
            drop_hash = hfold(drop_hash, 0);
            drop_hash = hfold(drop_hash, e.term);
            drop_hash = hfold(drop_hash, ent_word(e.type, e.len));
            drop_hash = hfold(drop_hash, e.lo);
            drop_hash = hfold(drop_hash, cmd_hi(e.type, e.hi));
          }
          e.type = E_Application;
          e.len = 0;
          e.lo = e.hi = 0;
        }
        flags |= HF_PENDING_CC;  // setPendingConfigChange
      }
      note_cc(e.type);
      rl_grow(e.len);
      log_append(idx, term, e.type, e.len, e.lo, e.hi);
      last = idx;
      t_last = term;
    }
    try_update(k, last);
    if (quorum() == 1) try_commit();
    broadcast_replicate();
  }
  RBE_HD void on_leader_read_index(u64 low, u64 high, u8 from) {  // raft.go:1633-1665
    if (quorum() != 1) {
      // hasCommittedEntryAtCurrentTerm (raft.go:1609-1618)
      if (log_term(committed) != term) {
        report_dropped_read_index(low, high);
        return;
      }
      rq_add(committed, low, high, from);
      broadcast_heartbeat_with_hint(low, high);
    } else {
      add_ready_to_read(committed, low, high);
    }
  }
  RBE_HD void on_replicate_resp(const Msg& m, u32 slot) {  // raft.go:1667-1696
    set_active(slot, true);
    if (!m.reject) {
      bool paused = is_paused(slot);
      if (try_update(slot, m.log_index)) {
        responded_to(slot);
        if (try_commit()) broadcast_replicate();
        else if (paused) request_replicate(slot);
        // sendReplicateMessage never changes match/lastIndex/ltt, so the
        // TimeoutNow condition is evaluated here and the send deferred after
        // the replicate fan-out, as in the reference
        if (ltt != 0 && role == R_Leader && m.from == ltt && last == rmatch(slot)) tn_to = ltt;
      }
    } else {
      if (decrease_to(slot, m.log_index, m.hint)) {
        if (rstate(slot) == RS_Replicate) become_retry(slot);  // enterRetryState
        request_replicate(slot);
      }
    }
  }
  RBE_HD void on_heartbeat_resp(const Msg& m, u32 slot) {  // raft.go:1698-1710
    set_active(slot, true);
    wait_to_retry(slot);
    ctr.v[C_REMOTE_TOUCH]++;
    if (rmatch(slot) < last) request_replicate(slot);
    if (m.hint != 0) {  // handleReadIndexLeaderConfirmation, after the replicate
      rq_pending = true;
      rq_lo = m.hint;
      rq_hi = m.hint_high;
      rq_from = m.from;
    }
  }
  RBE_HD void on_leader_transfer(const Msg& m, u32 slot) {  // raft.go:1712-1734
    u64 target = m.hint;
    if (target == 0) {
      set_fault(F_PANIC);
      return;
    }
    if (ltt != 0) return;
    if (self == target) return;
    ltt = (u8)target;
    etick = 0;
    if (rmatch(slot) == last) {
      Msg t = mk(M_TimeoutNow, (u8)target);
      send(t);
    }
  }
  RBE_HD bool leader_has_quorum() {  // raft.go:378-388 (votingMembers)
    u32 c = 0;
    for (u32 s = 0; s < N; s++) {
      if (!((vmask() >> s) & 1u)) continue;  // votingMembers
      if (s == k || ractive(s)) {
        c++;
        set_active(s, false);
      }
    }
    return c >= quorum();
  }

  // ------------------------------------------------------------- follower side (kernel 2)
  // inMemory.merge's log side (inmemory.go:201-234) for the entries src[0,
  // cnt) at indexes [c, c + cnt), c <= last + 1: they replace everything from c
  // on.  The ring invariant holds after it: the window entries the old tail
  // had overwritten come back from the cold log, the old entries the new ones
  // overwrite go to it, and new entries below the new window go straight there.
  RBE_HD void log_merge(u64 c, const Ent* src, u32 cnt) {
    const u64 L0 = last, nl = c + cnt - 1, R = C.ring;
    const u64 wlo = nl >= R ? nl - R + 1 : 1;  // the new window (before the marker)
    const u64 rs = c > wlo ? c : wlo;          // the first entry the ring takes
    // 1. the old window's live entries below c that leave the window go to
    // the cold log before the ring writes below overwrite their slots (the
    // new entries of [rs, nl] cover the slots of every one of them)
    {
      u64 j = umax64(umax64(marker + 1, L0 >= R ? L0 - R + 1 : 1), 1);
      const u64 je = umin64(umin64(L0, c - 1), wlo - 1);
      for (; j <= je; j++) evict(j);
    }
    // 2. new entries below the new window
    for (u64 i = c; i < rs; i++) {
      if (i > marker) cold_store(i, src[i - c]);
      note_cc(src[i - c].type);
      ctr.v[C_RING_ACCESS]++;
    }
    // 3. the ring's entries, batched: a batch's entries are loaded before any
    // ring store, so no load waits behind the stores of earlier entries (vmcnt
    // is in order)
    for (u64 i0 = rs; i0 <= nl; i0 += kEntBatch) {
      Ent e[kEntBatch];
#pragma unroll
      for (u32 j = 0; j < kEntBatch; j++)
        if (i0 + j <= nl) e[j] = src[i0 + j - c];
#pragma unroll
      for (u32 j = 0; j < kEntBatch; j++) {
        if (i0 + j <= nl) {
          ring_put(i0 + j, e[j].term, e[j].type, e[j].len, e[j].lo, e[j].hi);
          note_cc(e[j].type);
        }
      }
    }
    // 4. the window below c: slots the old tail overwrote come back
    if (L0 > R) {
      u64 lo = umax64(umax64(marker + 1, wlo), 1);
      const u64 hi = umin64(c - 1, L0 - R);
      for (; lo <= hi; lo++) {
        Ent e;
        if (!cold_get_ol(P, C, cold(), lo, &e)) {
          set_fault(F_WINDOW);
          continue;
        }
        const u64 s = ring_slot(lo);
        P.term_ring[s] = e.term;
        Body b;
        b.type = e.type;
        b.len = e.len;
        b.lo = e.lo;
        b.hi = e.hi;
        P.pay_ring[s] = b;
      }
    }
    last = nl;
    t_last = src[cnt - 1].term;
  }
  RBE_HD void on_replicate(const Msg& m, const Ent* ents) {  // raft.go:1339-1372
    Msg resp = mk(M_ReplicateResp, m.from);
    if (m.log_index < committed) {
      resp.log_index = committed;
      send(resp);
      return;
    }
    const u32 ne = msg_nent(m);
    if (match_term(m.log_index, m.log_term)) {
      // tryAppend (logentry.go:291-302) / getConflictIndex (315-322)
      // The lookups go in batches of kEntBatch: all loads of a batch are
      // issued before any is used, instead of one dependent round trip per entry
      u64 conflict = 0;
      u32 ci = 0;
      for (u32 i0 = 0; i0 < ne && conflict == 0; i0 += kEntBatch) {
        u64 et[kEntBatch], lt[kEntBatch];
#pragma unroll
        for (u32 j = 0; j < kEntBatch; j++) {
          et[j] = lt[j] = 0;
          if (i0 + j < ne) {
            et[j] = ents[i0 + j].term;
            lt[j] = log_term_peek(m.log_index + 1 + i0 + j);
          }
        }
#pragma unroll
        for (u32 j = 0; j < kEntBatch; j++) {
          const u32 i = i0 + j;
          if (conflict == 0 && i < ne) {
            const u64 idx = m.log_index + 1 + i;
            log_term_account(idx);
            // an entry below the ring: the cold log (the ILogDB read path)
            const u64 t = log_term_cold(idx) ? log_ent(idx).term : lt[j];
            if (t != et[j]) {
              conflict = idx;
              ci = i;
            }
          }
        }
      }
      if (conflict != 0) {
        if (conflict <= committed) {
          set_fault(F_PANIC);
        } else {
          // inMemory.merge (inmemory.go:201-234): checkEntriesToAppend then
          // truncate-and-append; savedTo = min(savedTo, first-1)
          if (conflict - 1 >= 1 && conflict - 1 <= last && log_term(conflict - 1) > ents[ci].term)
            set_fault(F_PANIC);
          if (rl_on()) rl_merge(conflict, ents + ci, ne - ci);
          log_merge(conflict, ents + ci, ne - ci);
          saved_to = umin64(saved_to, conflict - 1);
          if (imark_on(C) && conflict <= P.imark[r]) P.imark[r] = conflict;
          seg_len = mseg_len = 0;
        }
      }
      u64 last_idx = m.log_index + ne;
      commit_to(umin64(last_idx, m.commit));
      resp.log_index = last_idx;
    } else {
      resp.reject = 1;
      resp.log_index = m.log_index;
      resp.hint = last;
      events |= EV_REPLICATION_REJECTED;  // raft.go:1359-1369
    }
    send(resp);
  }
  // handleInstallSnapshotMessage + restore (raft.go:1311-1337, 439-470) with
  // entryLog.restore (logentry.go:396-401): the log becomes the snapshot
  RBE_HD void on_install_snapshot(const Msg& m) {
    Msg resp = mk(M_ReplicateResp, m.from);
    const u64 si = m.log_index, st = m.log_term;
    bool restored = false;
    if (si > committed) {
      // restore (raft.go:444-459): a snapshot listing this node as an observer
      // or a witness it is not panics
      const u32 sobs = m.pad1 & 0xFFu, swit = (m.pad1 >> 8) & 0xFFu;
      if ((role != R_Observer && ((sobs >> k) & 1u)) || (role != R_Witness && ((swit >> k) & 1u))) {
        set_fault(F_PANIC);
        return;
      }
      if (match_term(si, st)) {
        commit_to(si);
      } else if (!C.snapshot_entries) {
        set_fault(F_UNSUPPORTED);  // no SnapSt plane to take it
      } else {
        last = si;
        t_last = st;
        committed = processed = saved_to = si;
        marker = si;
        marker_term = st;
        cold_release_ol(P, C, cold(), ~0ull, par);  // the log is the snapshot now
        X().cref_dirty = true;
        P.term_ring[ring_slot(si)] = st;  // the fast steps read Term(marker) from the ring
        SnapSt& sp = P.snp[r];
        sp.ss_index = si;  // LogDB.ApplySnapshot (after the step's Update)
        sp.ss_term = st;
        sp.ss_rem = (u8)(m.pad0 & MB_REMOVED);  // and its membership
        sp.ss_obs = (u8)(m.pad1 & 0xFFu);
        sp.ss_wit = (u8)((m.pad1 >> 8) & 0xFFu);
        // inMemory.restore (inmemory.go:236-246): the in-memory log starts
        // after the snapshot, which it holds until a Commit names it
        if (imark_on(C)) P.imark[r] = si + 1;
        if (rl_on()) {
          P.rl[r].new_ent = 1;
          P.rl[r].size = 0;
        }
        sp.upd_ss = (u8)(C.ext_commit ? 1 : 0);
        sp.upd_rem = sp.ss_rem;
        sp.upd_obs = sp.ss_obs;
        sp.upd_wit = sp.ss_wit;
        seg_len = mseg_len = 0;
        snap_restored = true;
        restored = true;
      }
    }
    if (restored) {
      resp.log_index = last;
    } else {
      resp.log_index = committed;
      events |= EV_SNAPSHOT_REJECTED;
    }
    send(resp);
  }
  RBE_HD void on_heartbeat(const Msg& m) {  // raft.go:1301-1309
    commit_to(m.commit);
    Msg resp = mk(M_HeartbeatResp, m.from);
    resp.hint = m.hint;
    resp.hint_high = m.hint_high;
    send(resp);
  }

  // ------------------------------------------------------------- elections (kernel 3)
  RBE_HD void campaign() {  // raft.go:1080-1116
    become_candidate();
    ctr.v[C_CAMPAIGNS]++;
    events |= EV_CAMPAIGN_LAUNCHED;
    // handleVoteResp(self, false)
    vresp |= (u8)(1u << k);
    vgrant |= (u8)(1u << k);
    if (quorum() == 1) {  // isSingleNodeQuorum
      become_leader();
      return;
    }
    u64 hint = 0;
    if (flags & HF_IS_LTT) {
      hint = self;
      flags &= (u8)~HF_IS_LTT;
    }
    u64 lt = log_term(last);
    for (u32 s = 0; s < N; s++) {
      if (s == k || !((vmask() >> s) & 1u)) continue;  // votingMembers
      Msg m = mk(M_RequestVote, (u8)(s + 1));
      m.term = term;
      m.log_index = last;
      m.log_term = lt;
      m.hint = hint;
      send(m);
    }
  }
  // raft.applied: NotifyRaftLastApplied at the start of the step (node.go:
  // 1010-1014), the value run() captured in applied0: with ext_apply the
  // host's; else the harness's state machine, which applies every committed
  // entry the step it is returned, so `processed` at step start — or the
  // LogDB snapshot it recovered from at a restart while the re-applied
  // entries are still below it (rsm skips entries it already holds)
  RBE_HD u64 applied_index() const { return applied0; }
  RBE_HD void on_election() {  // handleNodeElection, raft.go:1482-1512
    if (role != R_Leader) {
      // hasConfigChangeToApply (raft.go:1460-1472): committed > applied
      if (committed > applied_index()) {
        events |= EV_CAMPAIGN_SKIPPED;
        return;
      }
      campaign();
    }
  }
  RBE_HD void on_request_vote(const Msg& m) {  // raft.go:1514-1535
    Msg resp = mk(M_RequestVoteResp, m.from);
    bool can_grant = vote == 0 || vote == m.from || m.term > term;
    bool utd = up_to_date(m.log_index, m.log_term);
    if (can_grant && utd) {
      etick = 0;
      vote = m.from;
    } else {
      resp.reject = 1;
    }
    send(resp);
  }
  RBE_HD void on_vote_resp(const Msg& m) {  // raft.go:1964-1981, 1060-1078
    u8 bit = (u8)(1u << (m.from - 1));
    if (!(vresp & bit)) {
      vresp |= bit;
      if (!m.reject) vgrant |= bit;
    }
    u32 count = popc8(vgrant);
    u32 q = quorum();
    if (count == q) {
      become_leader();
      broadcast_replicate();
    } else if (popc8(vresp) - count == q) {
      become_follower(term, 0);
    }
  }

  // ------------------------------------------------------------- ticks (kernel 5)
  RBE_HD void raft_tick();
  RBE_HD void non_leader_tick() {  // raft.go:566-590
    etick++;
    if (rl_on() && P.rl[r].tick_count % C.election_rtt == 0) {  // timeForRateLimitCheck
      P.rl[r].tick++;  // rl.HeartbeatTick
      send_rate_limit();
    }
    // non-voting members and witnesses never campaign (raft.go:577-581)
    if (role != R_Observer && role != R_Witness && voter(k) && etick >= ret) {  // !selfRemoved() && timeForElection()
      etick = 0;
      // Handle(Election): term 0 passes the gate; handled in any role
      if constexpr (FULL) on_election();
      else set_fault(F_UNSUPPORTED);  // excluded by fast_eligible()
    }
  }
  RBE_HD void leader_tick() {  // raft.go:592-621
    etick++;
    if (rl_on() && P.rl[r].tick_count % C.election_rtt == 0) P.rl[r].tick++;
    bool abort_lt = ltt != 0 && role == R_Leader && etick >= C.election_rtt;
    if (etick >= C.election_rtt) {
      etick = 0;
      if (C.check_quorum) {
        // Handle(CheckQuorum): dispatched by role; leader only
        if constexpr (FULL) {
          if (role == R_Leader) {
            if (!leader_has_quorum()) become_follower(term, 0);
          }
        } else {
          set_fault(F_UNSUPPORTED);  // excluded by fast_eligible()
        }
      }
    }
    if (abort_lt) ltt = 0;
    htick++;
    if (htick >= C.heartbeat_rtt) {
      htick = 0;
      if (role == R_Leader) broadcast_heartbeat();  // Handle(LeaderHeartbeat)
    }
  }
  RBE_HD void quiesced_tick() {  // raft.go:623-629
    if (!(flags & HF_RAFT_QUIESCE)) flags |= HF_RAFT_QUIESCE;
    etick++;
  }
  RBE_HD void on_timeout_now() {  // raft.go:1906-1916
    etick = ret;
    flags |= HF_IS_LTT;
    raft_tick();
    flags &= (u8)~HF_IS_LTT;
  }

  // ------------------------------------------------------------- quiesce manager
  RBE_HD u32 q_threshold() const { return C.election_rtt * 2 * 10; }
  RBE_HD bool q_quiesced() const { return C.quiesce && q_qs > 0; }
  RBE_HD bool q_new_to_quiesce() const {
    if (!q_quiesced()) return false;
    return q_tick - q_qs < C.election_rtt * 2;
  }
  RBE_HD bool q_just_exited() const {
    if (q_quiesced()) return false;
    return q_tick - q_eqt < q_threshold();
  }
  RBE_HD void q_enter() {
    q_qs = q_tick;
    q_nas = q_tick;
    q_new = true;
  }
  RBE_HD void q_exit() {
    q_qs = 0;
    q_eqt = q_tick;
  }
  RBE_HD void q_increase_tick() {  // quiesce.go:43-55
    if (!C.quiesce) return;
    q_tick++;
    if (!q_quiesced()) {
      if (q_tick - q_nas > q_threshold()) q_enter();
    }
  }
  RBE_HD void q_record_activity(u32 t) {  // quiesce.go:64-82
    if (!C.quiesce) return;
    if (t == M_Heartbeat || t == M_HeartbeatResp) {
      if (!q_quiesced()) return;
      if (q_new_to_quiesce()) return;
    }
    q_nas = q_tick;
    if (q_quiesced()) q_exit();
  }
  RBE_HD void q_try_enter() {  // quiesce.go:102-110
    if (q_just_exited()) return;
    if (!q_quiesced()) q_enter();
  }

  // ------------------------------------------------------------- Handle
  // raft.Handle (raft.go:1451-1458): term gate then the (role, type) table
  // of initializeHandlerMap (raft.go:2037-2098).
  RBE_HD void handle(const Msg& m, const Ent* ents) {
    if constexpr (!FULL) {
      handle_fast(m, ents);
      return;
    }
    // onMessageTermNotMatched (raft.go:1415-1449)
    if (m.term != 0 && m.term != term) {
      // dropRequestVoteFromHighTermNode (raft.go:1387-1409)
      if (m.type == M_RequestVote && C.check_quorum && m.term > term) {
        if (m.hint != m.from) {
          if (role == R_Leader && !(flags & HF_RAFT_QUIESCE) && etick >= C.election_rtt)
            set_fault(F_PANIC);
          if (leader != 0 && etick < C.election_rtt) return;
        }
      }
      if (m.term > term) {
        u8 lid = is_leader_message(m.type) ? m.from : (u8)0;
        // an observer / a witness keeps its state (raft.go:1430-1436)
        if (role == R_Observer || role == R_Witness) become_nonvoting(m.term, lid);
        else become_follower(m.term, lid);
      } else {
        if (is_leader_message(m.type) && C.check_quorum) {
          Msg x = mk(M_NoOP, m.from);
          send(x);
        }
        return;
      }
    }
    switch (role) {
      case R_Follower:
        switch (m.type) {
          case M_Propose:  // raft.go:1841-1853
            if (leader == 0) {
              report_dropped_proposal(ents, msg_nent(m));
            } else {
              Msg f = m;
              f.to = leader;
              u32 off = 0;
              bool x = false;
              const u32 ne = msg_nent(m);
              if (ne && arena_put(ents, ne, &off, &x)) set_ents(f, ne, off, x);
              send(f);
            }
            return;
          case M_Replicate:  // raft.go:1859-1863
            etick = 0;
            leader = m.from;
            on_replicate(m, ents);
            return;
          case M_Heartbeat:  // raft.go:1865-1869
            etick = 0;
            leader = m.from;
            on_heartbeat(m);
            return;
          case M_ReadIndex:  // raft.go:1871-1879
            if (leader == 0) {
              report_dropped_read_index(m.hint, m.hint_high);
            } else {
              Msg f = m;
              f.to = leader;
              send(f);
            }
            return;
          case M_LeaderTransfer:  // raft.go:1881-1888
            if (leader != 0) {
              Msg f = m;
              f.to = leader;
              send(f);
            }
            return;
          case M_ReadIndexResp:  // raft.go:1890-1898
            etick = 0;
            leader = m.from;
            add_ready_to_read(m.log_index, m.hint, m.hint_high);
            return;
          case M_Election: on_election(); return;
          case M_RequestVote: on_request_vote(m); return;
          case M_TimeoutNow: on_timeout_now(); return;
          case M_InstallSnapshot:  // raft.go:1900-1904
            etick = 0;
            leader = m.from;
            on_install_snapshot(m);
            return;
          case M_ConfigChangeEvent: on_config_change(m); return;
          case M_SnapshotReceived: restore_remotes((u32)m.hint); return;  // raft.go:1566
          default: return;
        }
      case R_Candidate:
        switch (m.type) {
          case M_Heartbeat:  // raft.go:1959-1962
            become_follower(term, m.from);
            on_heartbeat(m);
            return;
          case M_Propose: report_dropped_proposal(ents, msg_nent(m)); return;  // 1928-1931
          case M_ReadIndex:  // raft.go:1933-1941 (reported twice, as in the reference)
            report_dropped_read_index(m.hint, m.hint_high);
            add_dropped_ri(m.hint, m.hint_high);
            return;
          case M_Replicate:  // raft.go:1949-1952
            become_follower(term, m.from);
            on_replicate(m, ents);
            return;
          case M_RequestVoteResp: on_vote_resp(m); return;
          case M_Election: on_election(); return;
          case M_RequestVote: on_request_vote(m); return;
          case M_InstallSnapshot:  // raft.go:1954-1957
            become_follower(term, m.from);
            on_install_snapshot(m);
            return;
          case M_ConfigChangeEvent: on_config_change(m); return;
          case M_SnapshotReceived: restore_remotes((u32)m.hint); return;  // raft.go:1566
          default: return;
        }
      case R_Leader:
        switch (m.type) {
          case M_Propose: on_leader_propose(ents, msg_nent(m)); return;
          case M_ReadIndex: on_leader_read_index(m.hint, m.hint_high, m.from); return;
          // lw (raft.go:2013-2035): the remote of m.From, or nothing when
          // it is not a member of this replica's view
          case M_ReplicateResp:
            if (from_member(m.from)) on_replicate_resp(m, m.from - 1u);
            return;
          case M_HeartbeatResp:
            if (from_member(m.from)) on_heartbeat_resp(m, m.from - 1u);
            return;
          case M_LeaderTransfer:
            if (from_member(m.from)) on_leader_transfer(m, m.from - 1u);
            return;
          case M_Unreachable:  // raft.go:1773-1777
            if (from_member(m.from) && rstate(m.from - 1u) == RS_Replicate)
              become_retry(m.from - 1u);
            return;
          case M_SnapshotStatus:  // raft.go:1758-1771
            if (from_member(m.from) && rstate(m.from - 1u) == RS_Snapshot) {
              const u32 sl = m.from - 1u;
              if (m.reject) P.rem_snap[r * N + sl] = 0;  // clearPendingSnapshot
              become_retry(sl);                        // becomeWait
              if (rstate(sl) == RS_Retry) set_rstate(sl, RS_Wait);
            }
            return;
          case M_Election: return;        // leader ignores Election
          case M_RequestVote: on_request_vote(m); return;
          case M_ConfigChangeEvent: on_config_change(m); return;
          case M_SnapshotReceived: restore_remotes((u32)m.hint); return;  // raft.go:1566
          case M_RateLimit:  // handleLeaderRateLimit (raft.go:1779-1785)
            if (rl_on() && m.from >= 1 && m.from <= N) {
              RlSt& s = P.rl[r];
              s.fmask |= 1u << (m.from - 1u);
              s.f_tick[m.from - 1u] = s.tick;
              s.f_size[m.from - 1u] = m.hint;
            }
            return;  // rl disabled: dropped
          default: return;
        }
      case R_Observer:  // raft.go:2084-2092: the follower handlers for the data path
        switch (m.type) {
          case M_Heartbeat:  // handleObserverHeartbeat
            etick = 0;
            leader = m.from;
            on_heartbeat(m);
            return;
          case M_Replicate:  // handleObserverReplicate
            etick = 0;
            leader = m.from;
            on_replicate(m, ents);
            return;
          case M_InstallSnapshot:  // handleObserverSnapshot
            etick = 0;
            leader = m.from;
            on_install_snapshot(m);
            return;
          case M_Propose:  // handleObserverPropose
            if (leader == 0) {
              report_dropped_proposal(ents, msg_nent(m));
            } else {
              Msg f = m;
              f.to = leader;
              u32 off = 0;
              bool x = false;
              const u32 ne = msg_nent(m);
              if (ne && arena_put(ents, ne, &off, &x)) set_ents(f, ne, off, x);
              send(f);
            }
            return;
          case M_ReadIndex:  // handleObserverReadIndex
            if (leader == 0) {
              report_dropped_read_index(m.hint, m.hint_high);
            } else {
              Msg f = m;
              f.to = leader;
              send(f);
            }
            return;
          case M_ReadIndexResp:  // handleObserverReadIndexResp
            etick = 0;
            leader = m.from;
            add_ready_to_read(m.log_index, m.hint, m.hint_high);
            return;
          case M_ConfigChangeEvent: on_config_change(m); return;
          case M_SnapshotReceived: restore_remotes((u32)m.hint); return;
          default: return;
        }
      case R_Witness:  // raft.go:2093-2097
        switch (m.type) {
          case M_Heartbeat:  // handleWitnessHeartbeat
            etick = 0;
            leader = m.from;
            on_heartbeat(m);
            return;
          case M_Replicate:  // handleWitnessReplicate
            etick = 0;
            leader = m.from;
            on_replicate(m, ents);
            return;
          case M_InstallSnapshot:  // handleWitnessSnapshot
            etick = 0;
            leader = m.from;
            on_install_snapshot(m);
            return;
          case M_RequestVote: on_request_vote(m); return;
          case M_ConfigChangeEvent: on_config_change(m); return;
          case M_SnapshotReceived: restore_remotes((u32)m.hint); return;
          default: return;
        }
      default:
        set_fault(F_UNSUPPORTED);
        return;
    }
  }

  // ------------------------------------------------------------- fast path
  // The steady-state subset of the handler table.  fast_eligible() admits a
  // replica's round to the fast kernel only when every event of the round is
  // in this subset (same term, no role change, no election, no check-quorum
  // boundary, no leader transfer); the result is then identical to handle().
  RBE_HD void handle_fast(const Msg& m, const Ent* ents) {
    if (m.term != 0 && m.term != term) {
      set_fault(F_UNSUPPORTED);
      return;
    }
    if constexpr (FOLL) {
      switch (m.type) {
        case M_Replicate:  // raft.go:1859-1863
          etick = 0;
          leader = m.from;
          on_replicate(m, ents);
          return;
        case M_Heartbeat:  // raft.go:1865-1869
          etick = 0;
          leader = m.from;
          on_heartbeat(m);
          return;
        case M_ReadIndexResp:  // raft.go:1890-1898
          etick = 0;
          leader = m.from;
          add_ready_to_read(m.log_index, m.hint, m.hint_high);
          return;
        default: set_fault(F_UNSUPPORTED); return;
      }
    }
    if constexpr (LEAD) {
      switch (m.type) {
        case M_Propose: on_leader_propose(ents, msg_nent(m)); return;
        case M_ReadIndex: on_leader_read_index(m.hint, m.hint_high, m.from); return;
        case M_ReplicateResp: on_replicate_resp(m, m.from - 1u); return;
        case M_HeartbeatResp: on_heartbeat_resp(m, m.from - 1u); return;
        default: set_fault(F_UNSUPPORTED); return;
      }
    }
  }
  // Called after load() and before any state is written.  Reads only the
  // 24-byte message headers of the inbox.
  RBE_HD bool fast_eligible(u32 inp) const {
    if (C.rl_max) return false;  // rate limiter: full handler table
    if (flags & HF_SNAP_WORK) return false;  // compaction / SnapshotStatus: full table
    if (role != (LEAD ? R_Leader : R_Follower)) return false;
    if (flags & HF_APPLY_PENDING) return false;
    if (ltt != 0 || (flags & HF_IS_LTT)) return false;
    if (role == R_Follower && inp) return false;
    if (!clk.tick) return false;
    if (C.xfer_period && xfer_input(C, cid, round, k)) return false;
    if (C.ext_inputs && P.ext[r].flags) return false;
    bool from_leader = false;
    u32 n_in = 0;
    if (round > 0) {
      const u32 ppar = par ^ 1u;
      for (u32 s = 0; s < N; s++) {
        if (s == k) continue;
        const u32 pc = in_word<N>(P, g, s, k, round);
        if (pc & kCntSpill) return false;  // a spilled list: the full handler table
        const ListView lv = list_view(P, C, ppar, (g * N + s) * N + k, pc);
        const u32 n = lv.n();
        n_in += n;
        for (u32 i = 0; i < n; i++) {
          const Msg* mp = &lv.at(i);
          const u32 t = mp->type;
          const u64 mt = mp->term;
          if (role == R_Follower) {
            if (mt != term || mp->from != leader || leader == 0) return false;
            if (t != M_Replicate && t != M_Heartbeat && t != M_ReadIndexResp) return false;
            from_leader = true;
          } else {
            if (t == M_ReplicateResp || t == M_HeartbeatResp) {
              if (mt != term) return false;
            } else if (t == M_Propose || t == M_ReadIndex) {
              if (mt != 0) return false;
              if (t == M_Propose &&
                  ent_type(msg_ents(P, C, ppar, g * N + s, *mp)->type) == E_ConfigChange)
                return false;
            } else {
              return false;
            }
          }
        }
      }
    }
    // With no message and no client input nothing can exit quiesce before the
    // tick, so whether the tick is a QuiescedTick is known exactly.
    const bool idle = n_in == 0 && inp == 0;
    const bool q_at_tick =
        idle && C.quiesce && (q_qs > 0 || (q_tick + 1u - q_nas > q_threshold()));
    if (role == R_Follower) {
      // the tick must not reach the election timeout (non_leader_tick)
      if (!from_leader && !q_at_tick && etick + 1u >= ret) return false;
    } else {
      // the tick must not reach the check-quorum boundary (leader_tick)
      if (C.check_quorum && !q_at_tick && etick + 1u >= C.election_rtt) return false;
    }
    return true;
  }

  // ------------------------------------------------------------- membership bookkeeping
  // A ConfigChange entry of the stand-in form (cc_word) at ring body b: its
  // type and node id, false when the engine cannot decode it
  RBE_HD static bool cc_decode(const Body& b, u32* t, u64* nid) {
    const u64 w = b.lo;
    *t = (u32)((w >> 48) & 0xFFu);
    *nid = w & 0xFFFFFFFFFFFFULL;
    return !(ent_heap(b.type) || b.len != 8 || (w >> 56) != 0xCCu || *t > CC_AddWitness ||
             *nid > N);
  }
  // After the step's Update: without ext_apply the engine's state machine
  // applies the CommittedEntries, and each ConfigChange among them goes back
  // to raft at the node's next step, in log order (the state machine calls
  // node.ApplyConfigChange / ConfigChangeProcessed per entry under raftMu,
  // node.go:217-277, rsm/statemachine.go:951): one in cc_apply, or with
  // several (a node catching up, e.g. one that joins and replays the group's
  // history) CCA_MULTI and the accepted ones as bits of Upd::cc_acc (the next
  // step re-reads them from this range, which stays in the ring until then);
  // MB_CC_IN_LOG is dropped once (processed, last] holds no ConfigChange.
  RBE_HD void membership_after_update(const Upd& u) {
    if (!C.ext_apply && u.apply_hi >= u.apply_lo) {
      u32 ms = pack_ms(members & MB_REMOVED, obs, wit);  // raft's, as accepted changes go by
      u32 ncc = 0;
      for (u64 i = u.apply_lo; i <= u.apply_hi; i++) {
        const Body b = log_body(i);
        if (ent_type(b.type) != E_ConfigChange) continue;
        u32 t;
        u64 nid;
        if (!cc_decode(b, &t, &nid)) {
          set_fault(F_UNSUPPORTED);  // not a ConfigChange the engine can decode
          continue;
        }
        if (ncc == 32) {  // more than Upd::cc_acc holds
          set_fault(F_UNSUPPORTED);
          break;
        }
        if (!cc_accepted(ms, t, nid, N)) {
          cc_apply = (u8)(CCA_VALID | CCA_REJECT);
          ncc++;
          continue;
        }
        cc_apply = (u8)(CCA_VALID | (t << 3) | (u32)nid);
        cc_acc |= 1u << ncc;
        ncc++;
        ms_apply(ms, t, nid, N);
        // the state machine's own membership, which the next snapshot records
        ms_apply(sm_ms, t, nid, N);
      }
      if (ncc > 1) cc_apply = (u8)(CCA_VALID | CCA_MULTI);
    }
    if (mfl & MB_CC_IN_LOG) {
      bool any = false;
      for (u64 i = processed + 1; i <= last && !any; i++)
        if (ent_type(log_body(i).type) == E_ConfigChange) any = true;
      if (!any) mfl &= (u8)~MB_CC_IN_LOG;
    }
  }

  // ------------------------------------------------------------- node snapshots
  // After the step's Update (snapshot_entries > 0), in the node's order: a
  // snapshot restored from InstallSnapshot is the LogDB's (ApplySnapshot) and
  // the state machine's applied index; the compaction the last snapshot asked
  // for runs (compactLog, node.go:849-866; LogDB.Compact: only inside
  // (marker, lastIndex]); then saveSnapshotRequired (node.go:585-605) with the
  // applied index makes a snapshot at it and asks for a compaction to
  // index - CompactionOverhead at the next step (doSaveSnapshot /
  // compactSnapshot, node.go:619-692), done within the step.
  RBE_HD void node_snapshot() {
    SnapSt sp = P.snp[r];
    // smAppliedIndex moved to the snapshot (with ext_apply the host's state
    // machine recovers it and reports its applied index itself)
    if (snap_restored && !C.ext_apply) flags |= HF_APPLIED_NEW;
    // the state machine recovered from the snapshot: its membership is the
    // snapshot's, and the node restores raft's remotes from it at the next
    // step (RestoreRemotes, rsm/statemachine.go:236); the last step's is done
    if (snap_restored) sm_ms = pack_ms(sp.ss_rem, sp.ss_obs, sp.ss_wit);
    sp.rr_pend = (u8)(snap_restored && C.membership && !C.ext_apply ? 1 : 0);
    sp.marker = marker;
    sp.marker_term = marker_term;
    // (with ext_commit a compaction waits while the Updates carry a restored
    // snapshot the host has not committed: the node runs compactLog before
    // that Commit within one step, node.go:975-999, so the log's first index
    // never moves past a snapshot it still holds in memory)
    if (sp.compact_to && !sp.upd_ss) {
      // LogDB.Compact inside (marker, lastIndex], never past its snapshot
      const u64 c = sp.compact_to;
      if (c > marker && c <= last && c <= sp.ss_index) {
        sp.marker_term = log_term(c);
        sp.marker = c;
        cold_release_ol(P, C, cold(), c, par);  // the cold log's pages at or below it
        X().cref_dirty = true;
      }
      sp.compact_to = 0;
    }
    // saveSnapshotRequired: the engine's own state machine only; with ext_apply
    // the host's snapshot worker decides (rbe_snapshot_saved / rbe_compact)
    const u64 S = C.snapshot_entries, la = processed;
    if (!C.ext_apply && la > S + sp.ss_index && la > S + sp.ss_req) {
      sp.ss_req = la;
      const u64 t = log_term(la);
      if (t != 0) {
        sp.ss_index = la;
        sp.ss_term = t;
        sp.ss_rem = (u8)(sm_ms & 0xFFu);  // Snapshot.Membership: the state machine's at la
        sp.ss_obs = (u8)((sm_ms >> 8) & 0xFFu);
        sp.ss_wit = (u8)((sm_ms >> 16) & 0xFFu);
        sp.compact_to = la > C.compaction_overhead ? la - C.compaction_overhead : 0;
      }
    }
    sp.pend = snp_pend;
    sp.pend_rej = snp_rej;
    sp.sm_rem = (u8)(sm_ms & 0xFFu);
    sp.sm_obs = (u8)((sm_ms >> 8) & 0xFFu);
    sp.sm_wit = (u8)((sm_ms >> 16) & 0xFFu);
    P.snp[r] = sp;
    marker = sp.marker;
    marker_term = sp.marker_term;
    if (sp.compact_to || sp.pend || sp.rr_pend || sp.upd_ss) flags |= HF_SNAP_WORK;
    else flags &= (u8)~HF_SNAP_WORK;
  }

  // ------------------------------------------------------------- the step
  RBE_HD void load() {
    Hot h = load_hot(P, C, r, clk.tclk);
    role = h.role;
    flags = h.flags;
    vresp = h.votes_resp;
    vgrant = h.votes_granted;
    etick = h.election_tick;
    htick = h.heartbeat_tick;
    ret = h.rand_et;
    q_tick = h.q_tick;
    q_qs = h.q_quiesced_since;
    q_nas = h.q_no_activity_since;
    q_eqt = h.q_exit_quiesce_tick;
    rngc = h.rng_count;
    Core c = P.core[r];
    term = c.term;
    committed = c.committed;
    last = c.last_index;
    processed = c.processed;
    saved_to = c.saved_to;
    t_last = c.t_last;
    lead_start = c.lead_start;
    vote = c.vote;
    leader = c.leader;
    ltt = c.ltt;
    rq_head = c.rq_head;
    rq_count = c.rq_count;
    X().rqx = rq_count == kRqExt;  // the queue lives in pool pages (rbe_spill.h)
    if (X().rqx) X().rqd = rq_ext_load(P, C, r);
    X().cref_ld = X().cref_dirty = false;
    members = c.members;
    cc_apply = c.cc_apply;
    cc_acc = 0;
    cc_scan = false;
    mfl = c.mflags;
    roles0 = (u8)(mfl & MB_ROLES);
    obs = wit = 0;
    if (roles0) {
      const u16 x = P.roles[r];
      obs = (u8)(x & 0xFFu);
      wit = (u8)(x >> 8);
    }
  }
  RBE_HD void store() {
    Hot h;
    h.role = role;
    h.flags = flags;
    h.votes_resp = vresp;
    h.votes_granted = vgrant;
    h.election_tick = etick;
    h.heartbeat_tick = (u16)htick;
    h.rand_et = (u16)ret;
    h.q_tick = q_tick;
    h.q_quiesced_since = q_qs;
    h.q_no_activity_since = q_nas;
    h.q_exit_quiesce_tick = q_eqt;
    h.rng_count = rngc;
    P.hot[r] = h;
    P.idle[r] = idle_byte(C, role, flags, q_qs);
    Core c;
    c.term = term;
    c.committed = committed;
    c.last_index = last;
    c.processed = processed;
    c.saved_to = saved_to;
    c.vote = vote;
    c.leader = leader;
    c.ltt = ltt;
    c.rq_head = rq_head;
    c.rq_count = X().rqx ? kRqExt : rq_count;
    if (X().rqx) rq_ext_store(P, C, r, X().rqd);
    if (X().cref_dirty) P.cold[r] = X().cref;
    // MB_ROLES: the replica has observers or witnesses (Planes::roles)
    mfl = (u8)((mfl & ~MB_ROLES) | ((obs | wit) ? MB_ROLES : 0u));
    if (C.membership && (roles0 || (obs | wit))) P.roles[r] = (u16)(obs | ((u16)wit << 8));
    c.members = members;
    c.cc_apply = cc_apply;
    c.mflags = mfl;
    c.t_last = t_last;
    c.lead_start = lead_start;
    P.core[r] = c;
    if constexpr (LEAD) {
      for (u32 s = 0; s < N; s++) {
        RemoteMN x;
        x.match = c_match[s];
        x.next = c_next[s];
        P.rem[r * N + s] = x;
        P.rem_st[r * N + s] = (u8)c_st[s];
      }
    }
    if constexpr (LREM) {
      for (u32 s = 0; s < N; s++) {
        P.rem[r * N + s] = lrem(s);
        P.rem_st[r * N + s] = lrst(s);
      }
    }
  }

  // Steps the replica through one round.  The fast variant (FULL = false)
  // returns false without writing anything when the round needs the full
  // handler table; the caller then queues the replica for k_full.
  RBE_HD bool run() {
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
    ip_t0 = wall_clock64();
#endif
    load();
    if constexpr (!FULL) {
      if (!fast_eligible(role == R_Leader ? wl_input(C, cid, round) : 0u)) return false;
    }
    if constexpr (LEAD) {
      for (u32 s = 0; s < N; s++) {
        RemoteMN x = P.rem[r * N + s];
        c_match[s] = x.match;
        c_next[s] = x.next;
        c_st[s] = P.rem_st[r * N + s];
      }
    }
    if constexpr (LREM) {
      for (u32 s = 0; s < N; s++) {
        lrem(s) = P.rem[r * N + s];
        lrst(s) = P.rem_st[r * N + s];
      }
    }
    fault = (flags & HF_FAULTED) ? P.upd[r].fault : 0u;
    const u64 digest0 = TRACE ? P.upd[r].digest : 0;
    snp_pend = snp_rej = 0;
    snap_restored = false;
    u8 pend0 = 0, pend_rej0 = 0;
    marker = marker_term = 0;
    applied0 = C.ext_apply ? P.applied[r] : processed;
    // RestoreRemotes due at this step (bit 31 | the packed membership): the
    // state machine recovered from a received snapshot at the end of the last
    // step (SnapSt::rr_pend), or the host calls it (EXT_RESTORE, below)
    u32 restore = 0;
    sm_ms = 0;
    if (C.snapshot_entries) {
      const SnapSt& sp = P.snp[r];
      marker = sp.marker;
      marker_term = sp.marker_term;
      pend0 = sp.pend;
      pend_rej0 = sp.pend_rej;
      // the state machine recovered from the LogDB's snapshot (with ext_apply
      // the host reports what its state machine has applied)
      if (!C.ext_apply) applied0 = umax64(applied0, sp.ss_index);
      sm_ms = pack_ms(sp.sm_rem, sp.sm_obs, sp.sm_wit);
      if (sp.rr_pend) restore = 0x80000000u | pack_ms(sp.ss_rem, sp.ss_obs, sp.ss_wit);
    }
    pc_lo = pc_hi = 0;
    arena_used = 0;
    seg_lo = 0;
    seg_off = seg_len = 0;
    mseg_lo = 0;
    mseg_off = mseg_len = 0;
    seg_x = mseg_x = false;
    stash_init(X().ost);
    X().rtr_x = X().dri_x = 0;
    X().rtr_xcap = X().dri_xcap = 0;
    msg_hash = rtr_hash = drop_hash = 0;
    n_msgs = n_rtr = n_drop_ent = n_drop_ri = 0;
    q_new = false;
    if (C.iso_period) {
      const u32 until = P.iso_until[g];
      iso = round < until ? P.iso_mask[g] : (u8)0;
    } else {
      iso = 0;
    }
    const u64 committed0 = committed;
    const u64 term0 = term, vote0 = vote;
    const u8 leader0 = leader;
    events = 0;
    // Client input of the round.  The synthetic workload goes to replicas
    // that lead at round start; host-pushed input (ExtIn) to the replica it
    // names, any role, with the ReadIndex ctx / proposal batch it carries.
    const u32 wl = role == R_Leader ? wl_input(C, cid, round) : 0u;
    bool do_read = wl == 2, do_prop = wl == 1;
    // Peer.ProposeConfigChange of the round: the config-change schedule at the
    // replica leading at round start (its membership before this step), or host
    // input (EXT_CC_PROPOSE); the entry carries the stand-in Cmd (cc_word)
    bool do_cc = false;
    u32 cc_type = 0;
    u64 cc_node = 0;
    if (C.membership && C.cc_period && role == R_Leader && cc_selected(C, cid, round)) {
      // (oracle/harness.cpp step_replica): a voter is removed while more than
      // two are in raft.remotes, and added back; an observer slot's node is
      // added as an observer, then promoted and kept; a witness slot's node is
      // added as a witness and removed again
      cc_node = cc_target(C, cid, round);
      const u32 s = (u32)cc_node - 1u;
      const bool v = voter(s), big = popc8(voters_mask()) > 2;
      if ((C.obs_slots >> s) & 1u) {
        if (is_obs(s)) do_cc = true, cc_type = CC_AddNode;
        else if (!v) do_cc = true, cc_type = CC_AddObserver;
      } else if ((C.wit_slots >> s) & 1u) {
        if (!is_wit(s)) do_cc = true, cc_type = CC_AddWitness;
        else if (big) do_cc = true, cc_type = CC_RemoveNode;
      } else if (!v || big) {
        do_cc = true;
        cc_type = v ? CC_RemoveNode : CC_AddNode;
      }
    }
    u64 read_lo = 0, read_hi = 0;
    u32 prop_n = 0, xfer = C.xfer_period ? xfer_input(C, cid, round, k) : 0u;
    const Ent* prop_ents = nullptr;
    u8 unreach = 0, snap_nodes = 0, snap_reject = 0;
    bool ext_applied = false;
    if (C.ext_inputs) {
      const ExtIn ext = P.ext[r];
      if (ext.flags) {
        ExtIn z;
        z.flags = z.n_prop = z.prop_off = 0;
        z.xfer_target = z.unreach = z.snap_nodes = z.snap_reject = 0;
        z.ctx_low = z.ctx_high = 0;
        z.pad[0] = z.pad[1] = z.pad[2] = z.pad[3] = 0;
        P.ext[r] = z;
        if (ext.flags & EXT_READ) {
          do_read = true;
          read_lo = ext.ctx_low;
          read_hi = ext.ctx_high;
        }
        if (ext.flags & EXT_PROPOSE) {
          do_prop = true;
          prop_n = ext.n_prop;
          prop_ents = &P.in_ents[ext.prop_off];
        }
        if (ext.flags & EXT_XFER) xfer = ext.xfer_target;
        ext_applied = (ext.flags & EXT_APPLIED) != 0;
        if (ext.flags & EXT_UNREACH) unreach = ext.unreach;
        if (ext.flags & EXT_SNAPST) {
          snap_nodes = ext.snap_nodes;
          snap_reject = ext.snap_reject;
        }
        if (ext.flags & EXT_CC_PROPOSE) {
          do_cc = true;
          cc_type = (u32)(ext.pad[0] & 0xFFu);
          cc_node = ext.pad[0] >> 8;
        }
        if (ext.flags & EXT_CC_APPLY) cc_apply = (u8)ext.pad[1];
        // the host's RestoreRemotes (it comes after the device's own, which it replaces)
        if (ext.flags & EXT_RESTORE) restore = 0x80000000u | (u32)(ext.pad[2] & 0xFFFFFFu);
      }
    }
    if (pend0) {
      // the transport's outcome of last step's InstallSnapshots joins the host
      // reports (ReportSnapshotStatus, peer.go:177-184), a host report winning
      snap_reject = (u8)((snap_reject & snap_nodes) | (pend_rej0 & ~snap_nodes));
      snap_nodes = (u8)(snap_nodes | pend0);
    }
    if (!clk.tick) {
      // a round without a tick is a step only if handleEvents finds an event
      // (node.go:1030-1067): a message or notice, client input, an entry to apply
      bool ev = do_read || do_prop || xfer || unreach || snap_nodes || ext_applied || do_cc ||
                cc_apply || restore || (flags & (HF_APPLY_PENDING | HF_APPLIED_NEW));
      for (u32 s = 0; s < N; s++)
        if (s != k && in_word<N>(P, g, s, k, round) != 0) ev = true;
      if (!ev) return true;  // no step: no outbox header either
    }
    ctr.v[C_STEPS]++;
    if (do_read && !(C.ext_inputs && read_lo != 0)) {  // the workload's ctx
      read_lo = ((u64)(round + 1) << 32) | (u64)self;
      read_hi = cid + 1;
    }
    // handleReadIndexRequests (node.go:1108-1118)
    if (do_read) {
      q_record_activity(M_ReadIndex);
      ctr.v[C_READS]++;
    }
    // One event loop, one handle() site.  Events in node order (handleEvents,
    // node.go:1030-1067):
    //   host-reported Unreachable / SnapshotStatus (node-handled messages of
    //     the inbox, node.go:1207-1220: no activity recorded), delivered first
    //   handleReceivedMessages (node.go:1171-1205): inbox in (sender, stream) order
    //   batchedReadIndex (node.go:1379-1382) → Peer.ReadIndex
    //   handleLocalTickMessage → node.tick (node.go:1384-1399): one tick per
    //     ticking round
    //   handleProposals (node.go:1091-1106) → Peer.ProposeEntries
    //   handleLeaderTransferRequest (node.go:1069-1075) → Peer.RequestLeaderTransfer
    const u32 ppar = par ^ 1u;
    u32 cs = 0, ci = 0, cn = 0;  // inbox cursor: sender, index, count
    ListView cview;              // the sender's list (rbe_spill.h)
    cview.base = nullptr;
    cview.cap = cview.na = cview.nb = 0;
    bool copen = false;
    const u32 phase0 = (unreach | snap_nodes) ? 0u : (round > 0 ? 1u : 2u);
    // calls the node makes under raftMu between two steps come first:
    // Peer.RestoreRemotes (peer.go:159-165, after the state machine recovered
    // from a snapshot), then a ConfigChange the state machine applied: Peer.
    // ApplyConfigChange / RejectConfigChange (node.go applyConfigChange;
    // peer.go:138-157)
    u32 phase = restore ? 9u : (cc_apply ? 8u : phase0);
    bool cc_proposed = false;
    u32 rep_bit = 0;  // local reports: next node bit
    rep_mask = 0;
    tn_to = 0;
    hb_pending = rq_pending = false;
    hb_lo = hb_hi = rq_lo = rq_hi = 0;
    rq_from = 0;
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
    ip_pre = wall_clock64() - ip_t0;
#endif
#pragma unroll 1
    for (;;) {
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
      const u64 ip_it = wall_clock64();
#endif
      u32 kind = 0;  // 0 none, 1 inbox message, 2 local message, 3 tick
      Msg m;
      const Ent* ents = nullptr;
      if (phase == 9) {  // Handle(SnapshotReceived) with the snapshot's membership
        phase = cc_apply ? 8u : phase0;
        m = mk(M_SnapshotReceived, self);
        m.hint = restore & 0xFFFFFFu;
        kind = 2;
      } else if (phase == 8 && (cc_apply & CCA_MULTI)) {
        // the ConfigChanges of the last step's apply range, one per pass, in
        // log order: rejected, or applied (node id 0: only
        // clearPendingConfigChange); the range is still in the ring
        if (!cc_scan) {
          const Upd pu = P.upd[r];
          cc_i = pu.apply_lo;
          cc_e = pu.apply_hi;
          cc_bits = pu.cc_acc;
          cc_n = 0;
          cc_scan = true;
        }
#pragma unroll 1
        // (membership_after_update evaluated at most 32 of them: Upd::cc_acc)
        while (kind == 0 && cc_i <= cc_e && cc_i <= last && cc_n < 32) {
          const Body b = log_body(cc_i++);
          u32 t;
          u64 nid;
          if (ent_type(b.type) != E_ConfigChange || !cc_decode(b, &t, &nid)) continue;
          const bool ok = (cc_bits >> cc_n) & 1u;
          cc_n++;
          if (ok && nid == 0) {
            flags &= (u8)~HF_PENDING_CC;  // ApplyConfigChange(NoNode): clearPendingConfigChange
            continue;
          }
          m = mk(M_ConfigChangeEvent, self);
          if (ok) {
            m.hint = nid;
            m.hint_high = t;
          } else {
            m.reject = 1;
          }
          kind = 2;
        }
        if (kind == 0) {
          cc_apply = 0;
          phase = phase0;
        }
      } else if (phase == 8) {
        phase = phase0;
        const u8 a = cc_apply;
        cc_apply = 0;
        if (a & CCA_REJECT) {
          m = mk(M_ConfigChangeEvent, self);
          m.reject = 1;
          kind = 2;
        } else if ((a & 7u) == 0) {
          flags &= (u8)~HF_PENDING_CC;  // ApplyConfigChange(NoNode): clearPendingConfigChange
        } else {
          m = mk(M_ConfigChangeEvent, self);
          m.hint = a & 7u;
          m.hint_high = (a >> 3) & 3u;
          kind = 2;
        }
      }
      if (kind == 0 && phase == 0) {
        // Peer.ReportUnreachableNode / ReportSnapshotStatus (peer.go:168-183)
#pragma unroll 1
        while (rep_bit < 2 * N) {
          const u32 b = rep_bit++;
          const u32 node = b < N ? b : b - N;
          if (b < N && ((unreach >> node) & 1u)) {
            m = mk(M_Unreachable, self);
            m.from = (u8)(node + 1);
            kind = 2;
            break;
          }
          if (b >= N && ((snap_nodes >> node) & 1u)) {
            m = mk(M_SnapshotStatus, self);
            m.from = (u8)(node + 1);
            m.reject = (u8)((snap_reject >> node) & 1u);
            kind = 2;
            break;
          }
        }
        if (kind == 0) phase = round > 0 ? 1u : 2u;
      }
      if (kind == 0 && phase == 1) {
#pragma unroll 1
        while (cs < N) {
          if (!copen) {
            if (cs == k) {
              cs++;
              continue;
            }
            const u32 pc = in_word<N>(P, g, cs, k, round);
            if (pc & 0x8000u) {  // Quiesce first in the sender's stream (node.go:1207-1210)
              ctr.v[C_MSG_IN]++;
              q_try_enter();
            }
            cview = list_view(P, C, ppar, (g * N + cs) * N + k, pc);
            cn = cview.n();
            ci = 0;
            copen = true;
          }
          if (ci < cn) {
            m = cview.at(ci);
            ents = msg_ents(P, C, ppar, g * N + cs, m);
            ci++;
            kind = 1;
            break;
          }
          cs++;
          copen = false;
        }
        if (kind == 0) phase = 2;
      }
      if (kind == 0 && phase == 2) {
        phase = 3;
        if (do_read) {
          m = mk(M_ReadIndex, 0);
          m.hint = read_lo;
          m.hint_high = read_hi;
          kind = 2;
        }
      }
      if (kind == 0 && phase == 3) {
        phase = 4;
        if (clk.tick) kind = 3;
      }
      if (kind == 0 && phase == 4 && do_cc && !cc_proposed) {
        // handleConfigChangeMessage (node.go:1120-1142): recordActivity, then
        // ProposeConfigChange (peer.go:126-135), one ConfigChange entry
        cc_proposed = true;
        q_record_activity(M_ConfigChangeEvent);
        Ent e;
        e.term = 0;
        e.type = E_ConfigChange;
        e.len = 8;
        e.lo = cc_word(cc_type, cc_node);
        e.hi = 0;
        u32 off = 0;
        bool x = false;
        if (const Ent* a = arena_put(&e, 1, &off, &x)) {
          m = mk(M_Propose, 0);
          m.from = self;
          m.n_ent = 1;
          ents = a;
          kind = 2;
        }
      }
      if (kind == 0 && phase == 4) {
        phase = 5;
        if (do_prop) {
          if (prop_ents == nullptr) {
            // the workload's proposal, staged in this round's arena so every
            // handler reads entries from global memory
            Ent e;
            e.term = 0;
            e.type = E_Application;
            e.len = 16;
            e.lo = wl_payload_lo(C.seed, cid, round);
            e.hi = mix64(e.lo);
            u32 off = 0;
            bool x = false;
            if (const Ent* a = arena_put(&e, 1, &off, &x)) {
              prop_ents = a;
              prop_n = 1;
            }
          }
          if (prop_ents != nullptr) {
            m = mk(M_Propose, 0);
            m.from = self;  // Peer.ProposeEntries (peer.go:117-123)
            m.n_ent = (u16)prop_n;
            ents = prop_ents;
            kind = 2;
          }
          ctr.v[C_PROPOSALS]++;
        }
      }
      if (kind == 0 && phase == 5) {
        phase = 6;
        if (xfer) {  // Peer.RequestLeaderTransfer (peer.go:106-113)
          m = mk(M_LeaderTransfer, self);
          m.from = (u8)xfer;
          m.hint = xfer;
          kind = 2;
        }
      }
      if (kind == 0) break;
      if (kind == 3) {
        q_increase_tick();
        if (q_quiesced()) {
          quiesced_tick();
          ctr.v[C_QUIESCED_TICKS]++;
        } else {
          flags &= (u8)~HF_RAFT_QUIESCE;  // raft.tick: r.quiesce = false
          raft_tick();
          ctr.v[C_ACTIVE_TICKS]++;
        }
      } else {
        bool deliver = true;
        if (kind == 1) {
          ctr.v[C_MSG_IN]++;
          ctr.v[C_ENT_IN] += msg_nent(m);
          // tryRecordNodeActivity (node.go:1161-1169)
          if ((m.type == M_Heartbeat || m.type == M_HeartbeatResp) && m.hint > 0)
            q_record_activity(M_ReadIndex);
          else
            q_record_activity(m.type);
          // Peer.Handle (peer.go:186-198): a response from a node that is not a
          // member of this replica's view is dropped
          if (C.membership && is_response_message(m.type) && !from_member(m.from)) deliver = false;
        }
        if (deliver) handle(m, ents);
      }
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
      const u64 ip_ev = wall_clock64();
      if (kind == 1) {
        ip_in += ip_ev - ip_it;
        ip_nin++;
        if (ip_ev - ip_it > ip_max) {
          ip_max = ip_ev - ip_it;
          ip_maxtype = m.type;
        }
      } else {
        ip_loc += ip_ev - ip_it;
      }
#endif
      // deferred fan-out, in the reference's emission order
      // remotes, then observers, then witnesses, each ascending (raft.go:390-402 nodes())
#pragma unroll 1
      for (u32 cls = 0; cls < 3 && rep_mask; cls++) {
        u32 mk_ = rep_mask & (cls == 0 ? voters_mask() : (cls == 1 ? (u32)obs : (u32)wit));
        rep_mask &= ~mk_;
        while (mk_) {
          const u32 s = (u32)__builtin_ctz(mk_);
          mk_ &= mk_ - 1u;
          send_replicate(s);
        }
      }
      rep_mask = 0;
      if (tn_to) {
        Msg t = mk(M_TimeoutNow, tn_to);
        tn_to = 0;
        send(t);
      }
      if (hb_pending) {
        hb_pending = false;
#pragma unroll 1
        // votingMembers with the ctx, then observers when it is empty (raft.go:834-846)
        for (u32 s = 0; s < N; s++)
          if (s != k && ((vmask() >> s) & 1u)) send_heartbeat(s, hb_lo, hb_hi);
        if (hb_lo == 0 && hb_hi == 0)
          for (u32 s = 0; s < N; s++)
            if (is_obs(s)) send_heartbeat(s, 0, 0);
        ctr.v[C_REMOTE_TOUCH] += N - 1;
      }
      if (rq_pending) {
        rq_pending = false;
        rq_confirm(rq_lo, rq_hi, rq_from, rq_lo, rq_hi);
      }
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
      ip_fan += wall_clock64() - ip_ev;
#endif
    }
    // stepNode: newQuiesceState → sendEnterQuiesceMessages (node.go:873-886)
    const bool send_q = q_new;
    if (send_q) {
      for (u32 d = 0; d < N; d++) {
        if (d == k) continue;
        if (((iso >> k) & 1u) || ((iso >> d) & 1u)) {
          ctr.v[C_MSG_DROPPED]++;
          continue;
        }
        add_pc(d, 0x8000u);
        ctr.v[C_MSG_OUT]++;
      }
    }
    // this round's outbox header: the count word of every destination list;
    // a list with stashed messages moves whole to the spill heap (rbe_spill.h)
    if (X().ost.n) {
      const u32 f = outbox_relocate_ol(P, C, par, r, N, X().ost, pc_lo, pc_hi);
      if (f) set_fault(f);
    }
    u32 ow[N];
    for (u32 dd = 0; dd < N; dd++) ow[dd] = get_pc(dd);
    // the ReadyToReads / dropped ReadIndexes that moved to the spill heap:
    // the plane's slot 0 names their block
    if (n_rtr > C.rtr_cap) {
      RTR h;
      h.index = X().rtr_x;
      h.low = X().rtr_xcap;
      h.high = 0;
      P.rtr[r * C.rtr_cap] = h;
    }
    if (n_drop_ri > C.dri_cap) {
      DropRI h;
      h.low = X().dri_x;
      h.high = X().dri_xcap;
      P.dri[r * C.dri_cap] = h;
    }
    // getUpdate / Commit (peer.go:201-293): the harness persists and applies
    // everything at once, so savedTo := lastIndex and processed := committed.
    Upd u;
    u.save_lo = saved_to + 1;
    u.save_hi = last;
    // entriesToSave (inmemory.go:117-123) returns nothing when the in-memory
    // log no longer holds savedTo + 1: with ext_commit a host that reported an
    // entry applied (appliedLogTo) before saving it never sees it to save again
    if (C.ext_commit && saved_to + 1 < P.imark[r]) u.save_lo = last + 1;
    u.apply_lo = processed + 1;
    u.apply_hi = committed;
    if (flags & HF_APPLY_HELD) {  // moreEntriesToApply == false (node.go:908-915)
      u.apply_hi = processed;
    } else if (committed > processed) {
      u64 cnt = limit_count(processed + 1, committed);
      u.apply_hi = processed + cnt;
    }
    u64 apply_hash = 0;
    if (C.trace && u.apply_hi >= u.apply_lo) {
      for (u64 i = u.apply_lo; i <= u.apply_hi; i++) {
        const Ent e = log_ent(i);
        apply_hash = hfold(apply_hash, i);
        apply_hash = hfold(apply_hash, e.term);
        apply_hash = hfold(apply_hash, ent_word(e.type, e.len));
        apply_hash = hfold(apply_hash, e.lo);
        apply_hash = hfold(apply_hash, cmd_hi(e.type, e.hi));
      }
    }
    if (u.apply_hi >= u.apply_lo) ctr.v[C_ENT_APPLIED] += (u32)(u.apply_hi - u.apply_lo + 1);
    if (u.save_hi >= u.save_lo) ctr.v[C_ENT_SAVED] += (u32)(u.save_hi - u.save_lo + 1);
    if (n_rtr) ctr.v[C_READS_CONFIRMED] += n_rtr;
    ctr.v[C_DROPPED_PROPOSALS] += n_drop_ent;
    ctr.v[C_DROPPED_READS] += n_drop_ri;
    // Peer.Commit (peer.go:282-293): the outputs are consumed here; its log
    // part (savedTo, processed) is the harness's own unless the host sends it
    // (rbe_commit, ext_commit), as the node does after SaveRaftState
    if (!C.ext_commit) {
      if (u.apply_hi >= u.apply_lo) processed = u.apply_hi;
      saved_to = last;
    }
    // the limiter's appliedLogTo(LastApplied) (logentry.go:335-355) runs only in
    // a Peer.Commit, i.e. for a step the node takes an Update from: HasUpdate
    // (peer.go:253-280) or an applied index to confirm (node.go:907-923)
    if (C.rl_max && !C.ext_commit && applied0 > 0 && rl_on()) {
      const bool has = term != term0 || vote != vote0 || committed != committed0 || n_msgs ||
                       n_rtr || n_drop_ent || n_drop_ri || u.save_hi >= u.save_lo ||
                       u.apply_hi >= u.apply_lo || send_q || snap_restored || ext_applied ||
                       (flags & HF_APPLIED_NEW);
      if (has) rl_applied_to(applied0);
    }
    if (processed < committed) flags |= HF_APPLY_PENDING;
    else flags &= (u8)~HF_APPLY_PENDING;
    // the state machine's applied index moved (entries it held already, re-applied
    // after a restart, leave it): the node confirms it with the next Update
    if (u.apply_hi >= u.apply_lo && !C.ext_apply && u.apply_hi > applied0) flags |= HF_APPLIED_NEW;
    else flags &= (u8)~HF_APPLIED_NEW;
    if (C.membership) membership_after_update(u);
    if (C.snapshot_entries) node_snapshot();
    if (fault) flags |= HF_FAULTED;
    if (role == R_Leader) {
      ctr.v[C_COMMITTED] += (u32)(committed - committed0);
      ctr.v[C_LEADER_STEPS]++;
    }
    u64 d = digest0;
    if (TRACE) {
      u64 dh = drop_hash;
      const DropRI* dl = dri_list(P, C, r, n_drop_ri, par);
      for (u32 i = 0; i < n_drop_ri; i++) {
        DropRI x = dl[i];
        dh = hfold(dh, x.low);
        dh = hfold(dh, x.high);
      }
      d = hfold(d, round);
      d = hfold(d, (u64)role | ((u64)(q_quiesced() ? 1 : 0) << 8) | ((u64)(send_q ? 1 : 0) << 9) |
                       ((u64)((flags & HF_RAFT_QUIESCE) ? 1 : 0) << 10));
      d = hfold(d, term);
      d = hfold(d, vote);
      d = hfold(d, leader);
      d = hfold(d, committed);
      d = hfold(d, last);
      d = hfold(d, processed);
      d = hfold(d, (u64)etick | ((u64)htick << 32));
      d = hfold(d, ret);
      d = hfold(d, msg_hash);
      d = hfold(d, n_msgs);
      d = hfold(d, rtr_hash);
      d = hfold(d, apply_hash);
      d = hfold(d, dh);
    }
    u.digest = d;
    u.n_msgs = (u16)n_msgs;
    u.n_rtr = (u16)n_rtr;
    u.n_drop_ent = (u16)n_drop_ent;
    u.n_drop_ri = (u16)n_drop_ri;
    u.fault = fault;
    // Update.Snapshot (peer.go:345-347): restored in this step, or still held
    // in memory because the host has not committed it (ext_commit)
    const bool snap_carried =
        snap_restored || (C.ext_commit && C.snapshot_entries && P.snp[r].upd_ss);
    u.flags = (u16)((term != term0 || vote != vote0 || committed != committed0 ? UF_STATE_CHANGED
                                                                                : 0u) |
                    (send_q ? UF_SENT_QUIESCE : 0u) | (snap_carried ? UF_SNAPSHOT : 0u) |
                    (ext_applied ? UF_APPLIED : 0u) | UF_RANGES);
    u.events = (u16)(events | (leader != leader0 ? EV_LEADER_UPDATED : 0u));
    u.round = round;
    u.cc_acc = cc_acc;
    P.upd[r] = u;
    {
      put_row(P, r, round, N, ow);
    }
    store();
    return true;
  }
};

template <int N, bool TRACE, int MODE>
RBE_HD void Lane<N, TRACE, MODE>::raft_tick() {  // raft.go:551-564
  flags &= (u8)~HF_RAFT_QUIESCE;
  if (rl_on()) P.rl[r].tick_count++;  // tickCount
  if (role == R_Leader) leader_tick();
  else non_leader_tick();
}

// the full handler table: always completes the round
template <int N, bool TRACE, int MODE = MODE_FULL>
RBE_HD void step_replica(const Planes& P, const Params& C, u64 r, Clk ck, StepCounters& ctr) {
  Lane<N, TRACE, MODE> lane(P, C, r, ck, ctr);
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
  const u8 role0 = P.hot[r].role;
#endif
  lane.run();
#if defined(RBE_FULL_ITEM_PROF) && defined(__HIP_DEVICE_COMPILE__)
  // a step longer than 20 us leaves a record (rbe_debug_full_items): total,
  // before the loop, inbox, local, fan-out, longest message, counts, replica
  const u64 tot = wall_clock64() - lane.ip_t0;
  if (P.prof && tot > 2000) {
    const u64 at = atomicAdd((unsigned long long*)&P.prof[1], 1ull);
    if (at < kFullItemCap) {
      u64* rec = &P.prof[kProfHdr + at * 8];
      rec[0] = tot;
      rec[1] = lane.ip_pre;
      rec[2] = lane.ip_in;
      rec[3] = lane.ip_loc;
      rec[4] = lane.ip_fan;
      rec[5] = lane.ip_max | ((u64)lane.ip_maxtype << 48);
      rec[6] = (u64)lane.ip_nin | ((u64)lane.n_msgs << 16) | ((u64)role0 << 32) |
               ((u64)P.hot[r].role << 40);
      rec[7] = r;
    }
  }
#endif
}
// the steady-state subset: returns false (nothing written) when the round
// needs the full table
template <int N, bool TRACE, int MODE>
RBE_HD bool step_replica_fast(const Planes& P, const Params& C, u64 r, Clk ck,
                              StepCounters& ctr) {
  Lane<N, TRACE, MODE> lane(P, C, r, ck, ctr);
  return lane.run();
}

// ------------------------------------------------------------------ launch
// A replica restarts or a new node takes its slot: its cold log and a
// readIndex queue in pool pages go back to the pool (rbe_spill.h)
RBE_HD void spill_replica_release(const Planes& P, const Params& C, u64 r, u32 par) {
  ColdRef cr = P.cold[r];
  if (cr.head) {
    cold_release_ol(P, C, cr, ~0ull, par);
    P.cold[r] = cr;
  }
  Core& c = P.core[r];
  if (c.rq_count == kRqExt) {
    rq_ext_free_ol(P, C, rq_ext_load(P, C, r), par);
    c.rq_count = 0;
    c.rq_head = 0;
  }
}
// The voters a replica starts with, as the slots it does not count (removed
// mask): the initial members for one of them, nobody for a slot that joins
// later (Params::n_voters; the membership its LogDB reports before any snapshot)
RBE_HD u32 boot_removed(const Params& C, u32 k) {
  const u32 all = (1u << C.n) - 1u;
  return k < C.n_voters ? all & ~((1u << C.n_voters) - 1u) : all;
}
// Launch (peer.go:64-86) + bootstrap (peer.go:378-408) for one replica:
// newRaft → becomeFollower(0) draws a timeout, Launch → becomeFollower(1)
// draws another; one config-change entry per initial voter at term 1,
// committed; remotes {match 0, next V+1}.  A slot beyond the initial voters is
// a node that joins later (node.go:280-292, no peers, initial = false): term
// 1, an empty log, no remotes; one started as an observer or a witness
// (config.IsObserver / IsWitness: newRaft's becomeObserver / becomeWitness,
// raft.go:274-281, and no becomeFollower(1), peer.go:71-73) stays at term 0
// with its one randomized timeout.
// `join`: the replica is a node that joins now whatever its slot (a node
// replacing a removed one, rbe_replace_node).
template <int N>
RBE_HD void launch_replica(const Planes& P, const Params& C, u64 r, bool join = false) {
  const u32 k = (u32)(r % N);
  const u64 cid = cid_of(C, r / N);
  const u64 self = k + 1;
  const bool boot = k < C.n_voters && !join;
  const u32 V = boot ? C.n_voters : 0u;  // bootstrap entries in this replica's log
  const bool nv = ((C.obs_slots | C.wit_slots) >> k) & 1u;  // a non-voting start
  Hot h;
  h.role = ((C.obs_slots >> k) & 1u) ? R_Observer : (((C.wit_slots >> k) & 1u) ? R_Witness : R_Follower);
  h.flags = boot ? HF_APPLY_PENDING : (u8)0;  // the bootstrap entries are saved and applied in round 0
  h.votes_resp = h.votes_granted = 0;
  h.election_tick = 0;
  h.heartbeat_tick = 0;
  // the second draw wins (becomeFollower(0) then (1)); an observer / a witness draws once
  u64 rt = below(rto_rand(C.seed, cid, self, nv ? 0 : 1), C.election_rtt);
  h.rand_et = (u16)(C.election_rtt + rt);
  h.q_tick = h.q_quiesced_since = h.q_no_activity_since = h.q_exit_quiesce_tick = 0;
  h.rng_count = nv ? 1 : 2;
  P.hot[r] = h;
  P.idle[r] = idle_byte(C, h.role, h.flags, 0);
  Core c;
  c.term = nv ? 0 : 1;
  c.committed = V;
  c.last_index = V;
  c.processed = 0;
  c.saved_to = 0;
  c.vote = 0;
  c.leader = 0;
  c.ltt = 0;
  c.rq_head = c.rq_count = 0;
  c.members = c.cc_apply = c.mflags = 0;
  c.t_last = boot ? 1 : 0;  // bootstrap entries are at term 1
  c.lead_start = 0;
  // the bootstrap ConfigChanges, applied in round 0; the slots outside the
  // replica's initial membership
  const u32 rem0 = boot ? boot_removed(C, k) : (1u << N) - 1u;
  if (C.membership) {
    c.members = (u8)rem0;
    c.mflags = boot ? MB_CC_IN_LOG : 0u;
    P.roles[r] = 0;
  }
  P.core[r] = c;
  if (imark_on(C)) P.imark[r] = 1;  // inMemory.init(0), then bootstrap appends 1..V
  if (C.rl_max) {  // newRateLimiter; bootstrap's append is a merge that adds its entries
    RlSt s = {};
    s.new_ent = 1;
    s.size = rl_enabled(C.rl_max) ? V * (kEntryInMem + 8) : 0;
    P.rl[r] = s;
  }
  if (C.snapshot_entries) {  // the LogDB's membership before any snapshot: the bootstrap's
    SnapSt sp = {};
    sp.ss_rem = sp.sm_rem = (u8)rem0;
    P.snp[r] = sp;
  }
  for (u32 s = 0; s < N; s++) {
    RemoteMN x;
    x.match = 0;
    x.next = V + 1;
    P.rem[r * N + s] = x;
    P.rem_st[r * N + s] = 0;
  }
  for (u32 i = 1; i <= V; i++) {
    u64 slot = (i & (u64)(C.ring - 1)) * C.n_rep + r;
    P.term_ring[slot] = 1;
    Body b;
    b.type = E_ConfigChange;
    b.len = 8;
    b.lo = 0xCC00000000000000ULL | (u64)i;
    b.hi = 0;
    P.pay_ring[slot] = b;
  }
  Upd u;
  u.digest = 0;
  u.save_lo = 1;
  u.save_hi = 0;
  u.apply_lo = 1;
  u.apply_hi = 0;
  u.n_msgs = u.n_rtr = u.n_drop_ent = u.n_drop_ri = 0;
  u.fault = 0;
  u.flags = UF_RANGES;
  u.events = 0;
  u.round = ~0u;
  u.cc_acc = 0;
  P.upd[r] = u;
}

// Restart of replica r from persisted state (rbe_launch): Peer.Launch over an
// existing log (peer.go:64-86 with initial = newNode = false) = newRaft
// (raft.go:234-289: remotes next 1, loadState term/vote/commit) then
// becomeFollower(term, NoLeader) (one randomized timeout drawn, count 0);
// entryLog over the stored log: committed = processed = firstIndex - 1 = the
// LogDB's compaction marker, then loadState's commit; savedTo = lastIndex
// (logentry.go:86-96, inmemory.go:46-56).  `t`/`b` hold the terms and bodies of
// entries [last - n + 1, last].  With snapshots the LogDB's marker and latest
// snapshot go to SnapSt (the node's pending compaction and snapshot request
// stay, as the harness keeps them) and the state machine recovers from that
// snapshot (Lane::applied0), which the node confirms with its first Update.
// The node restarts with it: fresh quiesce state, and the messages in flight
// to and from the replica of the round about to run (parity `ppar` lists) are
// dropped.
template <int N>
RBE_HD void relaunch_replica(const Planes& P, const Params& C, u64 r, u64 term, u64 vote,
                             u64 commit, u64 last, u32 n, const u64* t, const Body* b, u32 ppar,
                             u32 tclk, u64 marker = 0, u64 marker_term = 0, u64 ss_index = 0,
                             u64 ss_term = 0, u32 removed = 0) {
  const u32 k = (u32)(r % N);
  const u64 g = r / N;
  const u64 cid = cid_of(C, g);
  const u64 self = k + 1;
  const bool faulted = P.upd[r].fault != 0;
  u8 snap_flags = 0;
  // the old incarnation's cold log and readIndex queue pages go back to the pool
  const u32 par = ppar ^ 1u;
  spill_replica_release(P, C, r, par);
  u32 sfault = 0;
  if (C.snapshot_entries) {
    SnapSt& sp = P.snp[r];
    sp.marker = marker;
    sp.marker_term = marker_term;
    sp.ss_index = ss_index;
    sp.ss_term = ss_term;
    // the snapshot's membership; the state machine recovers it
    sp.ss_rem = sp.sm_rem = (u8)(removed & 0xFFu);
    sp.ss_obs = sp.sm_obs = (u8)((removed >> 8) & 0xFFu);
    sp.ss_wit = sp.sm_wit = (u8)((removed >> 16) & 0xFFu);
    sp.rr_pend = 0;
    sp.upd_ss = 0;  // a new Peer's in-memory log holds no snapshot
    if (sp.compact_to || sp.pend) snap_flags |= HF_SNAP_WORK;
    if (ss_index && !C.ext_apply) snap_flags |= HF_APPLIED_NEW;  // recovered: confirmedIndex 0 lags it
    // Term(marker) for the steps' log lookups (the ring slot is free: the
    // entries above the marker are fewer than the ring)
    if (marker) P.term_ring[(marker & (u64)(C.ring - 1)) * C.n_rep + r] = marker_term;
  }
  Hot h;
  // newRaft in the node's configured state (raft.go:274-281): a witness slot's
  // node is a witness, an observer slot's node an observer until it has been
  // promoted into Addresses
  h.role = ((C.wit_slots >> k) & 1u) ? R_Witness
           : (((C.obs_slots >> k) & 1u) && ((removed >> k) & 1u)) ? R_Observer
                                                                 : R_Follower;
  h.flags = (u8)((commit > marker ? HF_APPLY_PENDING : 0u) | (faulted ? HF_FAULTED : 0u) |
                 snap_flags);
  h.votes_resp = h.votes_granted = 0;
  h.election_tick = 0;
  h.heartbeat_tick = 0;
  h.rand_et = (u16)(C.election_rtt + below(rto_rand(C.seed, cid, self, 0), C.election_rtt));
  // a fresh quiesce manager on the tick clock (oracle/harness.cpp
  // harness_restart): quiesce.go compares only differences of its counters
  const u32 q0 = C.quiesce ? tclk : 0u;
  h.q_tick = h.q_no_activity_since = h.q_exit_quiesce_tick = q0;
  h.q_quiesced_since = 0;
  h.rng_count = 1;
  P.hot[r] = h;
  P.idle[r] = idle_byte(C, h.role, h.flags, 0);
  Core c;
  c.term = term;
  c.committed = commit;
  c.last_index = last;
  c.processed = marker;
  c.saved_to = last;
  c.vote = (u8)vote;
  c.leader = 0;
  c.ltt = 0;
  c.rq_head = c.rq_count = 0;
  c.members = c.cc_apply = c.mflags = 0;
  c.t_last = n ? t[n - 1] : (last == marker ? marker_term : 0);
  c.lead_start = 0;
  // the restarted raft reads the group's members from the LogDB (NodeState:
  // its snapshot's membership, raft.go:260-270; every slot a voter without one,
  // as oracle/harness.cpp harness_restart)
  if (C.membership) {
    const u16 roles = (u16)(((removed >> 8) & 0xFFu) | (((removed >> 16) & 0xFFu) << 8));
    c.members = (u8)(removed & MB_REMOVED);
    c.mflags = roles ? MB_ROLES : 0u;
    P.roles[r] = roles;
    for (u32 i = 0; i < n; i++)
      if (ent_type(b[i].type) == E_ConfigChange) c.mflags |= MB_CC_IN_LOG;
  }
  P.core[r] = c;
  if (imark_on(C)) P.imark[r] = last + 1;  // inMemory.init(lastIndex), inmemory.go:46-57
  if (C.rl_max) {  // a new raft: a fresh limiter over an empty in-memory log
    RlSt s = {};
    s.new_ent = 1;
    P.rl[r] = s;
  }
  for (u32 s = 0; s < N; s++) {  // becomeFollower → reset → resetRemotes (raft.go:1023-1031)
    RemoteMN x;
    x.match = s == k ? last : 0;
    x.next = last + 1;
    P.rem[r * N + s] = x;
    P.rem_st[r * N + s] = 0;
  }
  // the LogDB's entries: the in-memory window in the ring, the older ones in
  // the cold log (rbe_spill.h)
  ColdRef cr = P.cold[r];
  for (u32 i = 0; i < n; i++) {
    const u64 idx = last - n + 1 + i;
    if (last - idx >= C.ring) {
      Ent e;
      e.term = t[i];
      e.type = b[i].type;
      e.len = b[i].len;
      e.lo = b[i].lo;
      e.hi = b[i].hi;
      if (!cold_put_ol(P, C, cr, idx, e, par)) sfault |= F_NOMEM;
      continue;
    }
    const u64 slot = (idx & (u64)(C.ring - 1)) * C.n_rep + r;
    P.term_ring[slot] = t[i];
    P.pay_ring[slot] = b[i];
  }
  P.cold[r] = cr;
  if (sfault) {
    P.upd[r].fault |= sfault;
    P.hot[r].flags |= HF_FAULTED;
  }
  // messages in flight: none from this replica, none to it
  P.cnt[ppar][r].stamp = 0;
  for (u32 s = 0; s < N; s++)
    if (s != k) P.cnt[ppar][g * N + s].w[cnt_widx(k, s)] = 0;
}

// A new node takes slot k of group g (rbe_replace_node): the node that held
// the slot was removed from the group (raft.go:1212-1237 removeNode at every
// replica) and another node id joins in its place, started as dragonboat starts
// a node that joins a running cluster (node.go:280-292: no peers, an empty
// LogDB, Launch with newNode, peer.go:64-86) in the slot's configured kind.
// Its quiesce manager is fresh on the tick clock (as relaunch_replica), the
// messages still addressed to the slot are dropped (none comes from it:
// slot_referenced), and its Update record starts over.
template <int N>
RBE_HD void join_replica(const Planes& P, const Params& C, u64 r, u32 ppar, u32 tclk) {
  spill_replica_release(P, C, r, ppar ^ 1u);  // the removed node's pages
  launch_replica<N>(P, C, r, true);
  Hot& h = P.hot[r];
  const u32 q0 = C.quiesce ? tclk : 0u;
  h.q_tick = h.q_no_activity_since = h.q_exit_quiesce_tick = q0;
  h.q_quiesced_since = 0;
  if (C.ext_apply) P.applied[r] = 0;
  const u32 k = (u32)(r % N);
  const u64 g = r / N;
  P.cnt[ppar][r].stamp = 0;
  for (u32 s = 0; s < N; s++)
    if (s != k) P.cnt[ppar][g * N + s].w[cnt_widx(k, s)] = 0;
}

// Whether anything in group g other than slot s's own replica still refers to
// the node in slot s, so a new node id there would not be a new node to the
// others: a replica that holds it in raft.remotes / observers / witnesses, as
// its vote, leader or leader-transfer target, in an ongoing vote tally, as the
// sender or a confirmer of a queued ReadIndex or in the rate limiter's
// follower reports; or a
// message it sent in the last round (read by the round about to run).  Once
// every replica applied the RemoveNode and the group moved on (a new term
// clears votes and tallies), none does.
template <int N>
RBE_HD bool slot_referenced(const Planes& P, const Params& C, u64 g, u32 s, u32 round) {
  const u8 id = (u8)(s + 1);
  for (u32 j = 0; j < N; j++) {
    if (j == s) continue;
    const u64 r = g * N + j;
    const Core c = P.core[r];
    if (!((c.members >> s) & 1u)) return true;
    if (C.membership && ((P.roles[r] >> s) & 0x101u)) return true;
    if (c.vote == id || c.leader == id || c.ltt == id) return true;
    const Hot h = P.hot[r];
    if (((h.votes_resp | h.votes_granted) >> s) & 1u) return true;
    const u32 nq = rq_length(P, C, r, c);
    for (u32 q = 0; q < nq; q++) {
      const ReadReq& x = *rq_entry(P, C, r, c, q);
      if (x.from == id || ((x.confirmed >> s) & 1u)) return true;
    }
    if (rl_enabled(C.rl_max) && ((P.rl[r].fmask >> s) & 1u)) return true;
  }
  if (round > 0) {
    const CntRow row = P.cnt[(round & 1u) ^ 1u][g * N + s];
    for (u32 d = 0; d < N; d++)
      if (d != s && row_word(row, d, s, round)) return true;
  }
  return false;
}

// ------------------------------------------------------------------ triage
// First pass of every round over every replica.  A round with no inbound
// message (Quiesce notices aside), no client input and a tick that neither
// elects nor heartbeats is executed completely here, in registers, touching
// only the hot plane and the outbox-count row: handleReceivedMessages sees
// only Quiesce (node.go:1207-1210 → quiesce.go:102-110), node.tick
// (node.go:1384-1399) runs increaseQuiesceTick + QuiescedTick, or Tick with
// electionTick++ below the randomized timeout (raft.go:566-590, 623-629).
// Everything else is routed to the leader / follower / full lists.
enum : u32 { T_DONE = 0, T_LEAD = 1, T_FOLL = 2, T_FULL = 3 };

// The lazy-idle shortcut (bench configuration: no trace, Quiesce on).  A
// replica whose idle byte says IB_LAZY, with no inbound message or Quiesce
// notice (`inbound` = any non-zero inbound count word) and no client input,
// runs a round that is one QuiescedTick: it is applied lazily
// (materialize_hot), so it writes nothing at all (its outbox header of this
// parity stays stale, which reads as empty).  The
// caller has loaded `ib` and `inbound` (k_triage prefetches them for all the
// replicas a lane owns).  Returns true when the round is complete.
template <int N>
RBE_HD bool triage_lazy(const Planes& P, const Params& C, u64 r, const Clk& ck, u8 ib,
                        bool inbound, StepCounters& ctr) {
  if (!(ib & IB_LAZY) || inbound) return false;
  const u32 round = ck.round;
  const u32 g = (u32)r / (u32)N;  // replica indices fit u32 (work lists hold u32)
  const u64 cid = cid_of(C, (u64)g);
  if ((ib & IB_LEAD) && wl_input(C, cid, round)) return false;
  if ((ib & IB_LEAD) && C.cc_period && cc_selected(C, cid, round)) return false;
  if (C.xfer_period && xfer_input(C, cid, round, (u32)r - g * (u32)N)) return false;
  if (C.ext_inputs && P.ext[r].flags) return false;
  // a round without a tick and without input is no step at all (handleEvents
  // finds no event, node.go:1030-1067)
  const u32 t = ck.tick ? 1u : 0u;
  ctr.v[C_STEPS] += t;
  ctr.v[C_QUIESCED_TICKS] += t;
  ctr.v[C_LEADER_STEPS] += (ib & IB_LEAD) ? t : 0u;
  return true;
}
// Group sleep (Planes::gwake, one byte per group; bench configuration: no
// trace, Quiesce on).  A group whose owned replicas all finished a round in
// triage_lazy falls asleep: from the next round on k_triage completes its
// rounds from this byte alone, without loading the replicas' idle bytes or
// outbox headers, until something wakes it.  Nothing inside the step can: a
// lazy replica has no timer (a quiesced replica neither campaigns nor
// heartbeats, quiesce.go / raft.go:623-629), and messages come only from the
// group's own replicas, which are lazy too.  What wakes a group is host input
// (k_ext_scatter / HostInputs::apply_host), an exchanged outbox header
// (xchg_put_cnt), an import or a launch (all groups awake), and the seeded
// workload or transfer input of a round (group_forced, checked every round).
//   bit 0     awake
//   bits 1-3  leaders among the group's owned replicas (while asleep)
RBE_HD bool group_forced(const Params& C, u64 cid, u32 round) {
  if (wl_input(C, cid, round)) return true;
  if (C.cc_period && cc_selected(C, cid, round)) return true;
  if (C.xfer_period && round % C.xfer_period == 0)
    for (u32 k = 0; k < C.n; k++)
      if (xfer_input(C, cid, round, k)) return true;
  return false;
}
// The rounds on which group_forced may hold for a group that fell asleep
// earlier (the workload's first round, leader-transfer and membership-schedule
// rounds): k_triage's list mode reads every wake byte on them, besides the
// host's scan rounds (launch, import), since the awake lists do not hold
// sleeping groups.
RBE_HD bool forced_round(const Params& C, u32 round) {
  return (C.wl_enabled && round == C.wl_start_round) ||
         (C.xfer_period && round % C.xfer_period == 0) ||
         (C.cc_period && round % C.cc_period == 0);
}
// the round of a sleeping group: one QuiescedTick per owned replica, exactly
// what triage_lazy counts for each of them
RBE_HD void group_sleep_round(u8 gw, u32 n_owned, const Clk& ck, StepCounters& ctr) {
  const u32 t = ck.tick ? 1u : 0u;
  ctr.v[C_STEPS] += t * n_owned;
  ctr.v[C_QUIESCED_TICKS] += t * n_owned;
  ctr.v[C_LEADER_STEPS] += t * ((gw >> 1) & 7u);
}
// the byte a group that fell asleep this round keeps
RBE_HD u8 group_sleep_byte(u32 leaders) { return (u8)(leaders << 1); }
// What a triaged round does to a group's wake byte (`busy` owned replicas did
// not finish lazily): an awake group whose replicas all finished lazily falls
// asleep (GS_SLEEP) unless the next round forces input on it, so a sleeping
// group is never forced outside a scan round (k_triage); a sleeping group that
// a round forced to step wakes (GS_WAKE) when any replica made a real step, as
// its messages of this round must be delivered next round.
enum : u32 { GS_KEEP = 0, GS_SLEEP = 1, GS_WAKE = 2 };
RBE_HD u32 group_transition(const Params& C, u64 cid, u32 round, bool awake, u32 busy) {
  if (awake) return busy == 0 && !group_forced(C, cid, round + 1) ? GS_SLEEP : GS_KEEP;
  return busy > 0 ? GS_WAKE : GS_KEEP;
}

// the inbound count words of replica r in this round: bit 0 = any non-zero
// word, bit 1 = any message (a Quiesce notice alone leaves it clear), bit 2 =
// any Replicate.  Split in a load phase and a fold so k_triage can issue the
// words of all its replicas before it waits for any: every word of the
// replica's column (its own slot included) is loaded unconditionally and the
// own slot is masked in the fold, so no load sits behind a branch.
template <int N>
RBE_HD void inbound_load(const Planes& P, u32 g, u32 k, u32 round, u16 (&w)[N]) {
  const CntRow* rows = &P.cnt[(round & 1u) ^ 1u][(u64)g * N];
  for (u32 s = 0; s < N; s++) {
    const CntRow row = rows[s];
    w[s] = (u16)row_word(row, k, s, round);
  }
}
template <int N>
RBE_HD u32 inbound_fold(const u16 (&w)[N], u32 k, u32 round) {
  u32 any = 0;
  for (u32 s = 0; s < N; s++) {
    const u32 pc = s == k ? 0u : (u32)w[s];
    any |= (pc != 0 ? 1u : 0u) | ((pc & 0x3FFFu) != 0 ? 2u : 0u) | ((pc & 0x7Fu) != 0 ? 4u : 0u);
  }
  return round == 0 ? 0u : any;
}
template <int N>
RBE_HD u32 inbound_bits(const Planes& P, u64 r, u32 round) {
  const u32 g = (u32)(r / N), k = (u32)(r % N);
  u16 w[N];
  inbound_load<N>(P, g, k, round, w);
  return inbound_fold<N>(w, k, round);
}
// The inbound summary word a work-list entry carries to the fast kernel
// (Lists::aux): for the j-th other sender (sender j + (j >= k)), 7 bits =
// min(A, 7) | min(B, 7) << 3 | quiesce << 6 of its count word this round.
// The fast steps rebuild their count words from it (aux_count_word) without
// loading them, so their message loads issue in the first gather level.  The
// clamp keeps every decision the fast steps take on the words: a leader
// declines A > 0 or B > MAXM (< 7), a follower more than FMAXM (< 7) inbound
// messages, and every count that is used is below 7.
template <int N>
RBE_HD u32 inbound_aux(const u16 (&w)[N], u32 k, u32 round) {
  u32 aux = 0;
  for (u32 j = 0; j + 1 < N; j++) {
    const u32 s = j + (j >= k ? 1u : 0u);
    u32 pc = 0;
    for (u32 t = 0; t < N; t++)
      if (t == s) pc = w[t];
    const u32 a = pc & 0x7Fu, b = (pc >> 7) & 0x7Fu;
    const u32 f = (a < 7u ? a : 7u) | ((b < 7u ? b : 7u) << 3) | (((pc >> 15) & 1u) << 6);
    aux |= f << (7 * j);
  }
  return round == 0 ? 0u : aux;
}
// count word of sender slot s (!= k) rebuilt from an inbound summary word
template <int N>
RBE_HD u32 aux_count_word(u32 aux, u32 k, u32 s) {
  const u32 j = s - (s > k ? 1u : 0u);
  const u32 f = (aux >> (7 * j)) & 0x7Fu;
  return (f & 7u) | (((f >> 3) & 7u) << 7) | (((f >> 6) & 1u) << 15);
}

// the group sizes with steady-state fast steps (rbe_fast.h lead_fast /
// foll_fast); other sizes step every replica-round on the full handler table
template <int N>
constexpr bool kFastN = N >= 3 && N <= 5;
RBE_HD u32 class_of_role(u32 role) {
  return role == R_Leader ? 1u /*T_LEAD*/ : (role == R_Follower ? 2u /*T_FOLL*/ : 3u /*T_FULL*/);
}

template <int N, bool TRACE>
RBE_HD u32 triage_replica(const Planes& P, const Params& C, u64 r, const Clk& ck,
                          StepCounters& ctr) {
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  const u32 round = ck.round;
  const Hot h = load_hot(P, C, r, ck.tclk);
  u32 nmsg = 0, qbits = 0;
  if (round > 0) {
    for (u32 s = 0; s < N; s++) {
      if (s == k) continue;
      const u32 pc = in_word<N>(P, g, s, k, round);
      nmsg += (pc & 0x7Fu) + ((pc >> 7) & 0x7Fu);
      if (pc & 0x8000u) qbits |= 1u << s;
    }
  }
  const u64 cid = cid_of(C, g);
  // the rate limiter's hooks live in the full handler table only
  const u32 cls = C.rl_max ? T_FULL
                           : (h.role == R_Leader ? T_LEAD : (h.role == R_Follower ? T_FOLL : T_FULL));
  if (nmsg || (h.flags & HF_APPLY_PENDING)) return cls;
  if (C.ext_commit) return cls;
  // a step after an apply may owe raft a ConfigChange (Core::cc_apply)
  if (C.membership && (h.flags & HF_APPLIED_NEW)) return cls;
  if (C.cc_period && h.role == R_Leader && cc_selected(C, cid, round)) return cls;  // the step may owe entries to save (Core is not read here)
  if (h.flags & HF_SNAP_WORK) return T_FULL;  // SnapshotStatus / compaction (node_snapshot)
  if (!ck.tick && (h.flags & HF_APPLIED_NEW)) return cls;
  if (h.role == R_Leader && wl_input(C, cid, round)) return cls;
  if (C.xfer_period && xfer_input(C, cid, round, k)) return cls;
  if (C.ext_inputs && P.ext[r].flags) return cls;
  // quiesceManager (quiesce.go) on registers
  const u32 et2 = C.election_rtt * 2, thr = et2 * 10;
  u32 qt = h.q_tick, qs = h.q_quiesced_since, qn = h.q_no_activity_since, qe = h.q_exit_quiesce_tick;
  bool qnew = false;
  for (u32 s = 0; s < N; s++) {
    if (!((qbits >> s) & 1u)) continue;
    // tryEnterQuiesce: not right after an exit, not already quiesced
    const bool quiesced = C.quiesce && qs > 0;
    const bool just_exited = !quiesced && qt - qe < thr;
    if (!just_exited && !quiesced) {
      qs = qt;
      qn = qt;
      qnew = true;
    }
  }
  if (C.quiesce && ck.tick) {  // increaseQuiesceTick
    qt++;
    if (!(qs > 0) && qt - qn > thr) {
      qs = qt;
      qn = qt;
      qnew = true;
    }
  }
  const bool quiesced = C.quiesce && qs > 0;
  u32 etick = h.election_tick;
  u8 flags = (u8)(h.flags & ~HF_APPLIED_NEW);  // this step returns no entries
  if (ck.tick) {
    if (quiesced) {
      flags |= HF_RAFT_QUIESCE;  // quiescedTick
      etick++;
    } else {
      if (h.role == R_Leader) return cls;          // leaderTick broadcasts heartbeats
      if (etick + 1u >= h.rand_et) return cls;     // nonLeaderTick would elect
      if (C.rl_max) return T_FULL;                 // tickCount and the rate-limit check
      flags &= (u8)~HF_RAFT_QUIESCE;
      etick++;
    }
  }
  // a round without a tick, input or Quiesce notice is no step at all
  // (handleEvents finds no event): nothing but a clean count row
  const bool noop = !ck.tick && qbits == 0;
  // commit the idle round
  const u32 st = noop ? 0u : 1u;
  ctr.v[C_STEPS] += st;
  ctr.v[C_MSG_IN] += popc8(qbits);
  // branch-free bumps (see FastOut in rbe_fast.h: sibling branches bumping
  // different counters become one indexed bump and the counters go to scratch)
  ctr.v[C_QUIESCED_TICKS] += ck.tick && quiesced ? 1u : 0u;
  ctr.v[C_ACTIVE_TICKS] += ck.tick && !quiesced ? 1u : 0u;
  ctr.v[C_LEADER_STEPS] += h.role == R_Leader ? st : 0u;
  u8 iso = 0;
  if (qnew && C.iso_period) {
    const u32 until = P.iso_until[g];
    iso = round < until ? P.iso_mask[g] : (u8)0;
  }
  // A round that is only a QuiescedTick of an already-flagged replica writes
  // nothing (lazy ticks, materialize_hot; its stale outbox header reads as
  // empty); any other step writes its header, Quiesce notices included.
  const bool lazy = noop || (!TRACE && quiesced && !qnew && qbits == 0 &&
                             (h.flags & HF_RAFT_QUIESCE) && !(h.flags & HF_APPLIED_NEW));
  if (!lazy) {
    u32 w[N];
    for (u32 d = 0; d < N; d++) {
      w[d] = 0;
      if (qnew && d != k) {  // sendEnterQuiesceMessages (node.go:873-886)
        const u32 drop = ((iso >> k) & 1u) | ((iso >> d) & 1u);
        ctr.v[C_MSG_DROPPED] += drop;
        ctr.v[C_MSG_OUT] += 1u - drop;
        w[d] = drop ? 0u : 0x8000u;
      }
    }
    put_row(P, r, round, N, w);
  }
  if (!lazy) {
    Hot o = h;
    o.flags = flags;
    o.election_tick = etick;
    o.q_tick = qt;
    o.q_quiesced_since = qs;
    o.q_no_activity_since = qn;
    o.q_exit_quiesce_tick = qe;
    P.hot[r] = o;
    P.idle[r] = idle_byte(C, h.role, flags, qs);
  }
  if (TRACE && !noop) {
    const Core c = P.core[r];
    Upd u = P.upd[r];
    u64 d = u.digest;
    d = hfold(d, round);
    d = hfold(d, (u64)h.role | ((u64)(quiesced ? 1 : 0) << 8) | ((u64)(qnew ? 1 : 0) << 9) |
                     ((u64)((flags & HF_RAFT_QUIESCE) ? 1 : 0) << 10));
    d = hfold(d, c.term);
    d = hfold(d, c.vote);
    d = hfold(d, c.leader);
    d = hfold(d, c.committed);
    d = hfold(d, c.last_index);
    d = hfold(d, c.processed);
    d = hfold(d, (u64)etick | ((u64)h.heartbeat_tick << 32));
    d = hfold(d, h.rand_et);
    for (int i = 0; i < 5; i++) d = hfold(d, 0);  // no messages, reads, applies, drops
    u.digest = d;
    u.save_lo = c.saved_to + 1;
    u.save_hi = c.last_index;
    u.apply_lo = c.processed + 1;
    u.apply_hi = c.committed;
    u.n_msgs = u.n_rtr = u.n_drop_ent = u.n_drop_ri = 0;
    u.flags = (u16)((qnew ? UF_SENT_QUIESCE : 0u) | UF_RANGES);
    u.events = 0;
    u.round = round;
    P.upd[r] = u;
  }
  return T_DONE;
}

// fault schedule: at epoch rounds, isolate the replicas of
// selected groups that lead at round start; one lane per group.
// The epoch's isolation of group g from its leaders' slots (`mask`)
RBE_HD void iso_apply(const Planes& P, const Params& C, u64 g, u32 round, u32 mask) {
  const u64 cid = cid_of(C, g);
  if (!iso_selected(C, cid, round / C.iso_period)) return;
  if (mask) {
    P.iso_mask[g] = (u8)mask;
    P.iso_until[g] = round + C.iso_len;
  }
}
// Slots of group g's leaders among the replicas this engine steps (all of
// them with one replica set per engine; replica mode ORs every rank's bits,
// rbe_iso_leaders / rbe_set_iso_leaders)
template <int N>
RBE_HD u32 iso_leader_bits(const Planes& P, const Params& C, u64 g) {
  u32 mask = 0;
  for (u32 k = 0; k < N; k++) {
    const u64 r = g * N + k;
    const bool own = owns_replica(C, g, k);
    if (own && P.hot[r].role == R_Leader) mask |= 1u << k;
  }
  return mask;
}
template <int N>
RBE_HD void iso_group(const Planes& P, const Params& C, u64 g, u32 round) {
  iso_apply(P, C, g, round, iso_leader_bits<N>(P, C, g));
}

}  // namespace rbe
