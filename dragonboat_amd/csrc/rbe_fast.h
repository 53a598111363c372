// MI355X batched Raft step engine: the steady-state fast paths.
//
// k_round (rbe_engine.hip) steps most replica-rounds with these two
// functions instead of the general Lane (rbe_step.h):
//   lead_fast<N, TRACE>: a leader whose inbox holds only ReplicateResp /
//     HeartbeatResp of its own term, with an optional local ReadIndex or
//     proposal and a tick that is not a check-quorum boundary;
//   foll_fast<N, TRACE>: a follower whose inbox holds only Replicate /
//     Heartbeat / ReadIndexResp from its known leader, and whose tick does not
//     start an election.
// Both produce bit-for-bit the state, messages, outputs, counters and trace
// digest that Lane<N, TRACE, MODE_FULL>::run() produces for the same round
// (tests/test_soa_cpu_parity.py and the -m gpu tests diff them against the
// oracle every round).  A round outside the subset returns false before
// anything is written, and the caller queues the replica for k_full_list.
//
// The general Lane reads memory on demand inside a long, divergent handler
// chain; its kernels need ~250 VGPRs and its critical path is dozens of
// dependent loads.  Here the round is gather → compute → scatter:
//   1. every independent load is issued up front: Hot, Core, the remote slots,
//      the Update record, the isolation word and the inbound count words;
//   2. the inbound message headers (and the leader's readIndex queue head)
//      are the second level; nothing else waits on memory unless the round
//      needs an entry older than the cached log tail (rare in steady state);
//   3. all per-slot state lives in registers (every slot loop is unrolled, so
//      every array index is a compile-time constant and nothing spills);
//   4. results are written once at the end.
#pragma once
#include "rbe_step.h"

// the fast leader step takes check-quorum ticks whose quorum holds (A/B knob)
#ifndef RBE_FAST_CQ
#define RBE_FAST_CQ 1
#endif

namespace rbe {

// Diagnostic build only (-DRBE_PHASE_TIMING, scripts/phase_timing.py): per-wave
// s_memtime stamps between the phases of the fast steps and k_triage, summed
// per phase into Planes::prof[8 + 8 * role + phase] (role: leader, follower,
// k_triage; rbe_debug_phases).
#if defined(RBE_PHASE_TIMING) && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ unsigned long long rbe_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ unsigned long long rbe_rstamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define RBE_STAMP(var) const unsigned long long var = rbe_stamp()
#define RBE_RSTAMP(var) const unsigned long long var = rbe_rstamp()
#define RBE_PHASE_ADD(role, i, a, b)                                                   \
  do {                                                                                 \
    if ((threadIdx.x & 63) == (u32)(__ffsll((unsigned long long)__ballot(1)) - 1))     \
      if (P.prof) atomicAdd((unsigned long long*)&P.prof[8 + 8 * (role) + (i)],         \
                            (unsigned long long)((b) - (a)));                           \
  } while (0)
#else
#define RBE_STAMP(var)
#define RBE_RSTAMP(var)
#define RBE_PHASE_ADD(role, i, a, b)
#endif

// Wait until every outstanding load of the lane has returned (a no-op on the
// host build).  Placed between the gather and the first store of a fast step.
RBE_HD void rbe_wait_all_loads() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_waitcnt(0);
#endif
}

#ifndef RBE_LDS_INBOX
#define RBE_LDS_INBOX 1
#endif
// waves per SIMD of the fast kernels (launch bounds), every group size: two
// (groups of 4-5 spill their wider remote state at two waves, and one wave
// measured slower still: DESIGN.md §9)
#ifndef RBE_FAST_WAVES
#define RBE_FAST_WAVES 2
#endif
template <int N>
constexpr int kFastWaves = RBE_FAST_WAVES;
#ifndef RBE_FAST_MAXM_WIDE  // leader inbound messages per follower, N >= 4
#define RBE_FAST_MAXM_WIDE 5
#endif
template <int N>
struct FastCaps {
  static constexpr u32 MAXM = N <= 3 ? 4 : RBE_FAST_MAXM_WIDE;  // leader: inbound messages per follower
  static constexpr u32 FMAXM = 6;              // follower: from its leader
  static constexpr u32 RQ = 3;                 // readIndex queue entries in registers
};

// one inbound message, the fields a steady-state handler reads
struct InMsg {
  u32 type, reject, n_ent, ent_off;
  u64 term, log_term, log_index, commit, hint, hint_high;
};

RBE_HD InMsg load_in(const Msg* p) {
  const Msg m = *p;
  InMsg x;
  x.type = m.type;
  x.reject = m.reject;
  // entries in the round spill heap (rbe_spill.h kMsgXEnt): a count no fast
  // step takes, so the round goes to the full handler table
  x.n_ent = (m.pad0 & kMsgXEnt) ? 0xFFFFu : m.n_ent;
  x.ent_off = m.ent_off;
  x.term = m.term;
  x.log_term = m.log_term;
  x.log_index = m.log_index;
  x.commit = m.commit;
  x.hint = m.hint;
  x.hint_high = m.hint_high;
  return x;
}

// the fields a steady-state leader keeps of an accepted ReplicateResp
// (a = LogIndex) or HeartbeatResp (a = Hint, b = HintHigh) after the gather
struct LeadIn {
  u32 w;  // type, from, to, reject (raw)
  u64 a, b;
};
// the fields a steady-state leader reads from a ReplicateResp / HeartbeatResp
struct LeadMsg {
  u32 w;  // type, from, to, reject (raw; decoded where used, outside the load's branch)
  u64 term, log_index, hint, hint_high;
};
RBE_HD LeadMsg load_lead(const Msg* p) {
  LeadMsg x;
  x.w = *(const u32*)p;
  x.term = p->term;
  x.log_index = p->log_index;
  x.hint = p->hint;
  x.hint_high = p->hint_high;
  return x;
}

// A/B knobs (build variants): the evicted entry's cold-log store as the
// step's first store, freeing its registers early; the outbox stash in LDS
#ifndef RBE_FAST_EV_EARLY
#define RBE_FAST_EV_EARLY 1
#endif
#ifndef RBE_FAST_PAUSED  // leaders with a paused remote behind take the fast step
#define RBE_FAST_PAUSED 1
#endif
#ifndef RBE_FAST_STASH_LDS
#define RBE_FAST_STASH_LDS 0
#endif
static constexpr u32 kFastStashLanes = 256;
#if defined(__HIP_DEVICE_COMPILE__) && RBE_FAST_STASH_LDS
__device__ __forceinline__ OutStash (&fast_stash())[kFastStashLanes] {
  __shared__ OutStash s_ost[kFastStashLanes];
  return s_ost;
}
#endif

// Output side shared by both roles: message emission (raft.send +
// finalizeMessageTerm, raft.go:640-658, then the network list), ReadyToRead,
// counters, the running trace hashes.  Mirrors Lane::send exactly.
template <int N, bool TRACE>
struct FastOut {
  u64 r, g;
  u32 k, par, self, round_;
  u8 iso;
  u64 pc;  // per destination 16 bits: A | B << 7 | quiesce << 15 (N <= 4 fits; N = 5 uses pc_hi)
  u64 pc_hi;
  u32 fault, n_msgs, n_rtr, n_drop_ri;
  u64 msg_hash, rtr_hash, drop_hash;
  u64 term;
  // event counts added to the lane's counters once, in fast_finish: every
  // increment here is unconditional (a 0/1 value), because two branches
  // that bump different counters get merged into one dynamically indexed
  // bump, which puts the counter array in scratch memory — and a scratch
  // reload after the lane's first store waits for every store before it
  u32 fault0, n_out, n_drop_msg, n_ent_out;
  u32 events;  // EV_* of the step (Upd::events)
  // messages past a full plane list (rbe_spill.h; relocated in fast_finish)
#if defined(__HIP_DEVICE_COMPILE__) && RBE_FAST_STASH_LDS
  RBE_HD OutStash& ost() const { return fast_stash()[threadIdx.x]; }
#else
  mutable OutStash ost_m;
  RBE_HD OutStash& ost() const { return ost_m; }
#endif

  RBE_HD u32 get_pc(u32 d) const {
    return d < 4 ? (u32)((pc >> (16 * d)) & 0xFFFFu) : (u32)((pc_hi >> (16 * (d - 4))) & 0xFFFFu);
  }
  RBE_HD void add_pc(u32 d, u32 v) {
    if (d < 4) pc += (u64)v << (16 * d);
    else pc_hi += (u64)v << (16 * (d - 4));
  }
  template <class CT>
  RBE_HD void set_fault(CT& ctr, u32 f) {
    (void)ctr;  // counted in fast_finish (new bits of the sticky word)
    fault |= f;
  }
  // Fault and event bits are OR-ed in unconditionally (0 when the condition
  // fails): two sibling branches that OR constants into different fields get
  // merged by the compiler into one store through a selected pointer, which
  // puts the whole FastOut in scratch memory — and a scratch reload after the
  // lane's first store waits for every store before it (vmcnt is in order).
  RBE_HD void fault_if(bool c, u32 f) { fault |= c ? f : 0u; }
  RBE_HD void event_if(bool c, u32 e) { events |= c ? e : 0u; }
  // `ent` points at the message's entries in this round's arena (may be null
  // when n_ent == 0).
  template <class CT>
  RBE_HD void send(const Planes& P, const Params& C, CT& ctr, Msg& m, const Ent* ent) {
    m.from = (u8)self;
    if (m.type != M_RequestVote) {
      if (m.type == M_Propose || m.type == M_ReadIndex) m.term = 0;
      else m.term = term;
    }
    n_msgs++;
    if (TRACE) {
      u64 h = msg_hash;
      h = hfold(h, (u64)m.type | ((u64)m.reject << 8) | ((u64)m.n_ent << 16));
      h = hfold(h, m.to);
      h = hfold(h, m.from);
      h = hfold(h, m.term);
      h = hfold(h, m.log_term);
      h = hfold(h, m.log_index);
      h = hfold(h, m.commit);
      h = hfold(h, m.hint);
      h = hfold(h, m.hint_high);
      for (u32 i = 0; i < m.n_ent; i++) {
        const Ent e = ent[i];
        h = hfold(h, m.type == M_Replicate ? m.log_index + 1 + i : 0);
        h = hfold(h, e.term);
        h = hfold(h, ent_word(e.type, e.len));
        h = hfold(h, e.lo);
        h = hfold(h, cmd_hi(e.type, e.hi));
      }
      msg_hash = h;
    }
    if (m.to < 1 || m.to > N) return;
    const u32 d = m.to - 1u;
    const u32 drop = ((iso >> k) & 1u) | ((iso >> d) & 1u);
    const u32 c = get_pc(d);
    const u32 a = c & 0x7Fu, b = (c >> 7) & 0x7Fu;
    const u32 full = drop ? 0u : (a + b >= C.maxm ? 1u : 0u);
    const u32 ok = 1u - drop;
    n_drop_msg += drop;
    n_out += ok;
    n_ent_out += ok ? (u32)m.n_ent : 0u;
    if (!ok) return;
    if (full) {  // the list moves to the spill heap at the step's end
      fault_if(!stash_put(P, C, par, ost(), m), F_NOMEM);
      RBE_AUDIT(AS_STASH, nullptr, sizeof(Msg));
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
#ifndef RBE_DIAG_NO_MSG_STORES
    P.msgs[par][((g * N + k) * N + d) * (u64)C.maxm + slot] = m;
    RBE_AUDIT(AS_MSG, &P.msgs[par][((g * N + k) * N + d) * (u64)C.maxm + slot],
              sizeof(Msg) | (u64)m.type << 32);
#endif
  }
  template <class CT>
  RBE_HD void dropped_read_index(const Planes& P, const Params& C, CT& ctr, u64 low,
                                 u64 high) {  // raft.go:1999-2012
    // (the fast leader drops at most one ReadIndex a step, and dri_cap >= 1)
    const bool full = n_drop_ri >= C.dri_cap;
    fault_if(full, F_NOMEM);
    event_if(!full, EV_READ_INDEX_DROPPED);
    if (full) return;
    DropRI x;
    x.low = low;
    x.high = high;
    P.dri[r * C.dri_cap + n_drop_ri] = x;
    RBE_AUDIT(AS_DRI, &P.dri[r * C.dri_cap + n_drop_ri], sizeof(x));
    n_drop_ri++;
    if (TRACE) {
      drop_hash = hfold(drop_hash, low);
      drop_hash = hfold(drop_hash, high);
    }
  }
  template <class CT>
  RBE_HD void ready_to_read(const Planes& P, const Params& C, CT& ctr, u64 index,
                            u64 low, u64 high) {  // raft.go:1624-1630
    // (eligibility keeps a fast step's ReadyToReads within rtr_cap)
    const bool full = n_rtr >= C.rtr_cap;
    fault_if(full, F_NOMEM);
    if (full) return;
    RTR x;
    x.index = index;
    x.low = low;
    x.high = high;
    P.rtr[r * C.rtr_cap + n_rtr] = x;
    RBE_AUDIT(AS_RTR, &P.rtr[r * C.rtr_cap + n_rtr], sizeof(x));
    n_rtr++;
    if (TRACE) {
      rtr_hash = hfold(rtr_hash, index);
      rtr_hash = hfold(rtr_hash, low);
      rtr_hash = hfold(rtr_hash, high);
    }
  }
};

RBE_HD Msg mk_msg(u32 type, u32 to) {
  Msg m;
  m.type = (u8)type;
  m.from = 0;
  m.to = (u8)to;
  m.reject = 0;
  m.n_ent = 0;
  m.pad0 = 0;
  m.ent_off = 0;
  m.pad1 = 0;
  m.term = m.log_term = m.log_index = m.commit = m.hint = m.hint_high = 0;
  return m;
}

// quiesceManager on registers (quiesce.go; Lane::q_*)
struct FastQ {
  u32 tick, qs, nas, eqt;
  bool qnew;
  RBE_HD bool quiesced(const Params& C) const { return C.quiesce && qs > 0; }
  RBE_HD bool new_to_quiesce(const Params& C) const {
    return quiesced(C) && tick - qs < C.election_rtt * 2;
  }
  RBE_HD bool just_exited(const Params& C) const {
    return !quiesced(C) && tick - eqt < C.election_rtt * 20;
  }
  RBE_HD void enter() {
    qs = tick;
    nas = tick;
    qnew = true;
  }
  RBE_HD void increase_tick(const Params& C) {  // quiesce.go:43-55
    if (!C.quiesce) return;
    tick++;
    if (!quiesced(C) && tick - nas > C.election_rtt * 20) enter();
  }
  RBE_HD void record_activity(const Params& C, u32 t) {  // quiesce.go:64-82
    if (!C.quiesce) return;
    if (t == M_Heartbeat || t == M_HeartbeatResp) {
      if (!quiesced(C)) return;
      if (new_to_quiesce(C)) return;
    }
    nas = tick;
    if (quiesced(C)) {
      qs = 0;
      eqt = tick;
    }
  }
  RBE_HD void try_enter(const Params& C) {  // quiesce.go:102-110
    if (just_exited(C)) return;
    if (!quiesced(C)) enter();
  }
};

// saveSnapshotRequired / doSaveSnapshot (node.go:585-605, 619-692) after a
// fast step that applied entries (snapshot_entries > 0): the snapshot at the
// applied index la and the compaction it asks for (run by the next step, a
// full one: HF_SNAP_WORK).  A fast step never restores or compacts, and with
// nothing applied the threshold cannot have been crossed (Lane::node_snapshot).
template <int N, bool TRACE, class CT>
RBE_HD void fast_node_snapshot(const Planes& P, const Params& C, CT& ctr,
                               FastOut<N, TRACE>& o, u64 la, u64 last, u64 t_last, u8& flags) {
  SnapSt* sp = &P.snp[o.r];
  const u64 S = C.snapshot_entries;
  if (!(la > S + sp->ss_index && la > S + sp->ss_req)) return;
  sp->ss_req = la;
  RBE_AUDIT(AS_SNAP, &sp->ss_req, 8);
  u64 t = t_last;
  if (la != last) {
    const bool miss = last - la >= C.ring;
    o.fault_if(miss, F_WINDOW);
    if (miss) return;
    t = P.term_ring[(la & (u64)(C.ring - 1)) * C.n_rep + o.r];
  }
  if (t == 0) return;
  sp->ss_index = la;
  sp->ss_term = t;
  // a fast step applies no ConfigChange: the state machine's membership
  sp->ss_rem = sp->sm_rem;
  sp->ss_obs = sp->sm_obs;
  sp->ss_wit = sp->sm_wit;
  const u64 ct = la > C.compaction_overhead ? la - C.compaction_overhead : 0;
  sp->compact_to = ct;
  RBE_AUDIT(AS_SNAP, &sp->ss_index, 8 * 3 + 3);
  if (ct) flags |= HF_SNAP_WORK;
}

// Common epilogue: stepNode's quiesce send, getUpdate/Commit, the trace digest,
// the Update record, this round's outbox counts, Hot/Core write-back.
// Mirrors the tail of Lane::run().
template <int N, bool TRACE, class CT>
RBE_HD void fast_finish(const Planes& P, const Params& C, CT& ctr, FastOut<N, TRACE>& o,
                        FastQ& q, u8 role, u8 flags, Hot h, Core c, u32 etick, u32 htick,
                        u64 committed0, u64 digest0, u32 core_dirty = 0xFu) {
  const u64 r = o.r;
  // stepNode: sendEnterQuiesceMessages (node.go:873-886)
  const bool send_q = q.qnew;
  if (send_q) {
#pragma unroll
    for (u32 d = 0; d < N; d++) {
      if (d == o.k) continue;
      const u32 drop = ((o.iso >> o.k) & 1u) | ((o.iso >> d) & 1u);
      o.n_drop_msg += drop;
      o.n_out += 1u - drop;
      if (!drop) o.add_pc(d, 0x8000u);
    }
  }
  ctr.v[C_MSG_OUT] += o.n_out;
  ctr.v[C_MSG_DROPPED] += o.n_drop_msg;
  ctr.v[C_ENT_OUT] += o.n_ent_out;
  // this sender's outbox header: stamp + the N count words; lists with
  // stashed messages move whole to the spill heap (rare: rbe_spill.h)
  if (o.ost().n) o.fault |= outbox_relocate(P, C, o.par, r, N, o.ost(), o.pc, o.pc_hi);
  u32 ow[N];
#pragma unroll
  for (u32 dd = 0; dd < N; dd++) ow[dd] = o.get_pc(dd) & 0xFFFFu;
  Upd u;
  u.save_lo = c.saved_to + 1;
  u.save_hi = c.last_index;
  u.apply_lo = c.processed + 1;
  u.apply_hi = c.committed;
  if (flags & HF_APPLY_HELD) {  // moreEntriesToApply == false (node.go:908-915)
    u.apply_hi = c.processed;
  } else if (c.committed > c.processed) {
    // limitSize (entryutils.go:52-64) with sizes 128 + len
    const u64 lo = c.processed + 1, hi = c.committed;
    u64 n = hi - lo + 1;
    // (no Cmd exceeds 16 bytes without the payload heap)
    if (C.heap_bytes || n * (128 + 16) > C.max_entry_size) {
      u64 total = 128 + P.pay_ring[(lo & (u64)(C.ring - 1)) * C.n_rep + r].len;
      u64 inc = 1;
      for (; inc < n; inc++) {
        total += 128 + P.pay_ring[((lo + inc) & (u64)(C.ring - 1)) * C.n_rep + r].len;
        if (total > C.max_entry_size) break;
      }
      n = inc;
    }
    u.apply_hi = c.processed + n;
  }
  u64 apply_hash = 0;
  if (TRACE && u.apply_hi >= u.apply_lo) {
    for (u64 i = u.apply_lo; i <= u.apply_hi; i++) {
      const bool miss = c.last_index - i >= C.ring;
      o.fault_if(miss, F_WINDOW);
      if (miss) break;
      const u64 s = (i & (u64)(C.ring - 1)) * C.n_rep + r;
      const Body b = P.pay_ring[s];
      apply_hash = hfold(apply_hash, i);
      apply_hash = hfold(apply_hash, P.term_ring[s]);
      apply_hash = hfold(apply_hash, ent_word(b.type, b.len));
      apply_hash = hfold(apply_hash, b.lo);
      apply_hash = hfold(apply_hash, cmd_hi(b.type, b.hi));
    }
  }
  if (u.apply_hi >= u.apply_lo) ctr.v[C_ENT_APPLIED] += (u32)(u.apply_hi - u.apply_lo + 1);
  if (u.save_hi >= u.save_lo) ctr.v[C_ENT_SAVED] += (u32)(u.save_hi - u.save_lo + 1);
  if (o.n_rtr) ctr.v[C_READS_CONFIRMED] += o.n_rtr;
  ctr.v[C_DROPPED_READS] += o.n_drop_ri;
  // Peer.Commit's log part: the harness's own unless the host sends it
  // (rbe_commit, ext_commit; Lane::run)
  const bool own_commit = !C.ext_commit;
  const bool applies = own_commit && u.apply_hi >= u.apply_lo;
  if (applies) c.processed = u.apply_hi;
  // Core's 16-B chunks this step changed: [term, committed] [last_index,
  // processed] [saved_to, vote..rq_count] [t_last, lead_start]; the caller
  // passes the chunks its handlers wrote
  core_dirty |= (c.committed != committed0 ? 1u : 0u) | (applies ? 2u : 0u) |
                (own_commit && c.saved_to != c.last_index ? 4u : 0u);
  if (own_commit) c.saved_to = c.last_index;
  if (c.processed < c.committed) flags |= HF_APPLY_PENDING;
  else flags &= (u8)~HF_APPLY_PENDING;
  if (u.apply_hi >= u.apply_lo && !C.ext_apply) flags |= HF_APPLIED_NEW;
  else flags &= (u8)~HF_APPLIED_NEW;
  if (C.snapshot_entries && !C.ext_apply && u.apply_hi >= u.apply_lo)  // (host's with ext_apply)
    fast_node_snapshot<N, TRACE>(P, C, ctr, o, c.processed, c.last_index, c.t_last, flags);
  if (role == R_Leader) {
    ctr.v[C_COMMITTED] += (u32)(c.committed - committed0);
    ctr.v[C_LEADER_STEPS]++;
  }
  u64 d = digest0;
  if (TRACE) {
    d = hfold(d, o.round_);
    d = hfold(d, (u64)role | ((u64)(q.quiesced(C) ? 1 : 0) << 8) | ((u64)(send_q ? 1 : 0) << 9) |
                     ((u64)((flags & HF_RAFT_QUIESCE) ? 1 : 0) << 10));
    d = hfold(d, c.term);
    d = hfold(d, c.vote);
    d = hfold(d, c.leader);
    d = hfold(d, c.committed);
    d = hfold(d, c.last_index);
    d = hfold(d, c.processed);
    d = hfold(d, (u64)etick | ((u64)htick << 32));
    d = hfold(d, h.rand_et);
    d = hfold(d, o.msg_hash);
    d = hfold(d, o.n_msgs);
    d = hfold(d, o.rtr_hash);
    d = hfold(d, apply_hash);
    d = hfold(d, o.drop_hash);  // dropped ReadIndexes (no dropped proposals here)
  }
  u.digest = d;
  u.n_msgs = (u16)o.n_msgs;
  u.n_rtr = (u16)o.n_rtr;
  u.n_drop_ent = 0;
  u.n_drop_ri = (u16)o.n_drop_ri;
  u.fault = o.fault;
  ctr.v[C_FAULTS] += popc8(o.fault & ~o.fault0 & 0xFFu) + ((o.fault & ~o.fault0) >> 8 & 1u);
  // chunks 0-2 only when they carry something (Upd, rbe_types.h)
  const bool ranges = TRACE || u.save_lo <= u.save_hi || u.apply_lo <= u.apply_hi ||
                      o.n_drop_ri != 0;
  u.flags = (u16)((c.committed != committed0 ? UF_STATE_CHANGED : 0u) |
                  (send_q ? UF_SENT_QUIESCE : 0u) | (ranges ? UF_RANGES : 0u));
  u.events = (u16)o.events;
  u.round = o.round_;
  u.cc_acc = 0;
#ifndef RBE_DIAG_NO_STATE_STORES
  if (ranges) P.upd[r] = u;
  else __builtin_memcpy((char*)&P.upd[r] + 48, (const char*)&u + 48, 16);
  RBE_AUDIT(ranges ? AS_UPD : AS_UPD3, (char*)&P.upd[r] + (ranges ? 0 : 48),
            ranges ? sizeof(Upd) : 16);
  put_row(P, r, o.round_, N, ow);  // one 16-B store
  RBE_AUDIT(AS_CNT, &P.cnt[o.round_ & 1u][r], sizeof(CntRow));
  h.flags = o.fault ? (u8)(flags | HF_FAULTED) : flags;
  h.election_tick = etick;
  h.heartbeat_tick = (u16)htick;
  h.q_tick = q.tick;
  h.q_quiesced_since = q.qs;
  h.q_no_activity_since = q.nas;
  h.q_exit_quiesce_tick = q.eqt;
  P.hot[r] = h;
  RBE_AUDIT(AS_HOT, &P.hot[r], sizeof(Hot));
#pragma unroll
  for (u32 i = 0; i < 4; i++)
    if (core_dirty & (1u << i)) {
      __builtin_memcpy((char*)&P.core[r] + 16 * i, (const char*)&c + 16 * i, 16);
      RBE_AUDIT(AS_CORE, (char*)&P.core[r] + 16 * i, 16);
    }
  P.idle[r] = idle_byte(C, role, flags, q.qs);
  RBE_AUDIT(AS_IDLE, &P.idle[r], 1);
#endif
}

// ---------------------------------------------------------------- leader
// One steady-state leader round (see the file comment for the subset).
// Mirrors Lane<N, TRACE, MODE_FULL>::run() event by event:
//   inbox (ascending sender; Quiesce marker, then the sender's messages) →
//   local ReadIndex → tick → proposal, each followed by the deferred fan-out
//   (Replicate sends in ascending slot order, heartbeats, readIndex confirm).
template <int N, bool TRACE, bool AUX = false, class CT>
RBE_HD bool lead_fast(const Planes& P, const Params& C, u64 r, const Clk& ck, CT& ctr,
                      u32 aux = 0) {
  const u32 round = ck.round;
  using Cap = FastCaps<N>;
  constexpr u32 Q = N / 2 + 1;
  if constexpr (!kFastN<N>) {
    return false;
  } else {
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  const u32 par = round & 1u, ppar = par ^ 1u;
  const u64 cid = cid_of_n<N>(C, g);
  // ---- gather, level 1: independent loads
  RBE_RSTAMP(rt0);
  RBE_STAMP(t0);
  Hot h = load_hot(P, C, r, ck.tclk);
  Core c = P.core[r];
  u64 match[N], next[N];
  u32 st[N];
  // remote slots whose (match, next, state) changed this round: the scatter
  // stores only those (a heartbeat/ReadIndex round changes none), which saves
  // 2N scattered store requests per lane in the common case
  u32 rdirty = 0;
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    const RemoteMN x = P.rem[r * N + s];
    match[s] = x.match;
    next[s] = x.next;
    st[s] = P.rem_st[r * N + s];
  }
  u32 pcin[N];
  if constexpr (AUX) {  // the count words came with the work-list entry (inbound_aux)
#pragma unroll
    for (u32 s = 0; s < N; s++) pcin[s] = s == k ? 0u : aux_count_word<N>(aux, k, s);
  } else {
#pragma unroll
    for (u32 s = 0; s < N; s++) pcin[s] = s != k ? in_word<N>(P, g, s, k, round) : 0u;
  }
  // one row per other sender (row j is sender j + (j >= k)): no registers
  // for the lane's own slot, which is what keeps the step out of scratch.
  // With AUX the counts are known before any load, so the inbound messages
  // are part of the first gather level; otherwise they wait for the counts.
  LeadMsg in[N - 1][Cap::MAXM];
  auto load_inbox = [&]() {
#pragma unroll
    for (u32 j = 0; j + 1 < N; j++) {
      const u32 sj = j + (j >= k ? 1u : 0u);
      u32 pj = 0;
#pragma unroll
      for (u32 t = 0; t < N; t++)
        if (t == sj) pj = pcin[t];
      const u32 nbj = (pj >> 7) & 0x7Fu;
      const Msg* lst = &P.msgs[ppar][((g * N + sj) * N + k) * (u64)C.maxm];
#pragma unroll
      for (u32 i = 0; i < Cap::MAXM; i++) {
        in[j][i].w = 0xFFu;
        in[j][i].term = in[j][i].log_index = in[j][i].hint = in[j][i].hint_high = 0;
        if (i < nbj) in[j][i] = load_lead(&lst[C.maxm - 1u - i]);
      }
    }
  };
  if constexpr (AUX) load_inbox();
  // the isolation schedule and the Update record are read only when in use:
  // two of the lane's scattered lines saved in the steady state
  const u32 until = C.iso_period ? P.iso_until[g] : 0u;
  const u8 isom = C.iso_period ? P.iso_mask[g] : (u8)0;
  const u64 digest0 = TRACE ? P.upd[r].digest : 0;
  u32 cdirty = 0;  // Core chunks a proposal or the readIndex queue wrote (fast_finish)
  // ---- eligibility on level-1 data
  if (h.role != R_Leader) return false;
  if (h.flags & HF_SNAP_WORK) return false;  // compaction / SnapshotStatus: full table
  // membership: a changed voter set, a ConfigChange in the log or to apply,
  // or one to propose this round (full handler table)
  if (C.membership && ((c.members | c.cc_apply | c.mflags) != 0 ||
                       (C.cc_period && cc_selected(C, cid, round))))
    return false;
  // ext_commit: an Update whose unsaved entries left the in-memory log (Lane::run)
  if (C.ext_commit && c.saved_to + 1 < P.imark[r]) return false;
  if (h.flags & (HF_APPLY_PENDING | HF_IS_LTT)) return false;
  if (c.ltt != 0) return false;
  if (!ck.tick) return false;
  if (C.xfer_period && xfer_input(C, cid, round, k)) return false;
  // a queue past the register copy (or in pool pages: kRqExt), or one that
  // this round's ReadIndex could overflow, takes the full table
  if (c.rq_count >= Cap::RQ || c.rq_count >= C.rq_cap) return false;
  // the step's outputs stay within the planes' lists: ReadyToReads of the
  // queue (<= RQ), one dropped ReadIndex, two arena entries (rbe_spill.h)
  if (C.rtr_cap < Cap::RQ || C.ecap < 2) return false;
  // the apply range (< last + 2) stays in the ring window
  if (c.last_index + 1 - c.processed > C.ring) return false;
  u32 inp = wl_input(C, cid, round);
  // Host input (rbe_push_read_index / rbe_push_proposals): one ReadIndex, or
  // one inline non-ConfigChange entry, takes the same path as the workload's
  // (Lane::run reads it from Planes::ext; the entry stays in Planes::in_ents,
  // not the arena); anything else takes the full handler table.
  u64 xlo = 0, xhi = 0;
  u32 xlen = 16, xtype = E_Application;
  bool xin = false;
  if (C.ext_inputs) {
    const ExtIn* xp = &P.ext[r];
    const u32 xf = xp->flags;
    if (xf != 0) {
      if (inp != 0) return false;
      if (xf == EXT_READ) {
        xlo = xp->ctx_low;
        xhi = xp->ctx_high;
        inp = 2;
      } else if (xf == EXT_PROPOSE && xp->n_prop == 1) {
        const Ent e = P.in_ents[xp->prop_off];
        if ((e.type & ET_HEAP) || ent_type(e.type) == E_ConfigChange || e.len > 16) return false;
        xlo = e.lo;
        xhi = e.hi;
        xlen = e.len;
        xtype = e.type;
        inp = 1;
      } else {
        return false;
      }
      xin = true;
    }
  }
  u32 n_in = 0;
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    if (s == k) continue;
    const u32 na = pcin[s] & 0x7Fu, nb = (pcin[s] >> 7) & 0x7Fu;
    if (na != 0 || nb > Cap::MAXM) return false;
    n_in += nb;
  }
  // ---- gather, level 2: inbound message headers, readIndex queue
  RBE_STAMP(t1);
  // Loads only inside the branches; every use comes after the join, so no
  // branch waits for its own loads (a wait inside each conditional block
  // would serialise the message loads).
  if constexpr (!AUX) load_inbox();
  // the proposal's ring slot holds entry last + 1 - ring: it goes to the cold
  // log (rbe_spill.h) unless compacted; its record and the cold-log ref now
  const u64 lmark = C.snapshot_entries ? P.snp[r].marker : 0;
  const u64 ev_idx = c.last_index + 1 > C.ring ? c.last_index + 1 - C.ring : 0;
#ifdef RBE_DIAG_NO_EVICT  // timing-only build: the evicted entry is dropped (wrong below the ring)
  const bool ev = false;
#else
  const bool ev = inp == 1 && ev_idx > lmark;
#endif
  Ent ev_e;
  ColdRef ev_cr;
  ev_e.term = ev_e.lo = ev_e.hi = 0;
  ev_e.type = ev_e.len = 0;
  ev_cr.head = ev_cr.tail = 0;
  ev_cr.tail_pn = 0;
  if (ev) {
    const u64 es = (ev_idx & (u64)(C.ring - 1)) * C.n_rep + r;
    const Body eb = P.pay_ring[es];
    ev_e.term = P.term_ring[es];
    ev_e.type = eb.type;
    ev_e.len = eb.len;
    ev_e.lo = eb.lo;
    ev_e.hi = eb.hi;
    ev_cr = P.cold[r];
  }
  u64 rq_lo[Cap::RQ], rq_hi[Cap::RQ], rq_ix[Cap::RQ];
  u32 rq_fr[Cap::RQ], rq_cf[Cap::RQ];
  u32 rq_n = c.rq_count, rq_h = c.rq_head;
  auto rq_slot = [&](u32 i) -> u64 {
    u32 x = rq_h + i;
    if (x >= C.rq_cap) x -= C.rq_cap;
    return r * C.rq_cap + x;
  };
  u32 rq_w[Cap::RQ];  // from | confirmed << 8 (raw bytes 24..27 of the record)
#pragma unroll
  for (u32 i = 0; i < Cap::RQ; i++) {
    rq_lo[i] = rq_hi[i] = rq_ix[i] = 0;
    rq_w[i] = 0;
    if (i < rq_n) {
      const ReadReq* qp = &P.rq[rq_slot(i)];
      rq_lo[i] = qp->low;
      rq_hi[i] = qp->high;
      rq_ix[i] = qp->index;
      rq_w[i] = *(const u32*)&qp->from;
    }
  }
#pragma unroll
  for (u32 i = 0; i < Cap::RQ; i++) {
    rq_fr[i] = rq_w[i] & 0xFFu;
    rq_cf[i] = (rq_w[i] >> 8) & 0xFFu;
  }
  // queue entries (register index i, i.e. slot rq_h + i) this step wrote: only
  // those are stored back (a pop moves the head; the entries behind it keep
  // their slots)
  u32 rq_dm = 0;
  // eligibility of the inbox, then only the fields the handlers read stay live
  LeadIn inc[N - 1][Cap::MAXM];
  // With RBE_LDS_INBOX (N = 3 on the device) the kept fields move to LDS, one
  // column per lane (field-major, so a wave's 64 lanes hit consecutive banks),
  // and the rolled inbox loop reads its message from there by index: ~40
  // registers fewer through the compute phase, so the compiler need not spill,
  // and an LDS read waits on lgkmcnt, never behind the lane's stores (vmcnt).
#if defined(__HIP_DEVICE_COMPILE__) && RBE_LDS_INBOX
  constexpr bool kLdsIn = N == 3 || kFastWaves<N> == 1;
  constexpr u32 kLdsSlots = kLdsIn ? (N - 1) * Cap::MAXM : 1;
  constexpr u32 kLdsLanes = kLdsIn ? 256 : 1;
  __shared__ u32 s_in_w[kLdsSlots][kLdsLanes];
  __shared__ u64 s_in_a[kLdsSlots][kLdsLanes], s_in_b[kLdsSlots][kLdsLanes];
  const u32 lds_lane = kLdsIn ? threadIdx.x : 0u;
#else
  constexpr bool kLdsIn = false;
  u32 (*s_in_w)[1] = nullptr;
  u64 (*s_in_a)[1] = nullptr, (*s_in_b)[1] = nullptr;
  const u32 lds_lane = 0;
#endif
  u32 resp = 0;  // bit j: inbound sender j (slot order without k) sent something
#pragma unroll
  for (u32 j = 0; j + 1 < N; j++) {
#pragma unroll
    for (u32 i = 0; i < Cap::MAXM; i++) {
      const u32 t = in[j][i].w & 0xFFu;
      inc[j][i].w = in[j][i].w;
      inc[j][i].a = t == M_ReplicateResp ? in[j][i].log_index : in[j][i].hint;
      inc[j][i].b = in[j][i].hint_high;
      if (t == 0xFFu) continue;  // no message in this slot
      resp |= 1u << j;
      if (t != M_ReplicateResp && t != M_HeartbeatResp) return false;
      if (in[j][i].term != c.term) return false;
      if (t == M_ReplicateResp && (in[j][i].w >> 24)) return false;  // rejection: decreaseTo
    }
  }
  if constexpr (kLdsIn) {
#pragma unroll
    for (u32 j = 0; j + 1 < N; j++) {
#pragma unroll
      for (u32 i = 0; i < Cap::MAXM; i++) {
        s_in_w[j * Cap::MAXM + i][lds_lane] = inc[j][i].w;
        s_in_a[j * Cap::MAXM + i][lds_lane] = inc[j][i].a;
        s_in_b[j * Cap::MAXM + i][lds_lane] = inc[j][i].b;
      }
    }
  }
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    // every entry a Replicate of this round can carry is the one proposed
    // this round (so no ring read is needed after the first store) — or the
    // remote is paused (Wait / Snapshot: sendReplicateMessage sends nothing,
    // raft.go:758-765) and nothing from it arrives this round to unpause it
    // (the majority side's leader of a partitioned group)
    if (s == k || next[s] > c.last_index) continue;
    const u32 rs = st[s] & 3u;
    const bool paused = RBE_FAST_PAUSED && (rs == RS_Wait || rs == RS_Snapshot);
    if (!paused || (pcin[s] & 0x3FFFu) != 0) return false;
  }
  FastQ q;
  q.tick = h.q_tick;
  q.qs = h.q_quiesced_since;
  q.nas = h.q_no_activity_since;
  q.eqt = h.q_exit_quiesce_tick;
  q.qnew = false;
  {
    const bool idle = n_in == 0 && inp == 0;
    const bool q_at_tick = idle && C.quiesce &&
                           (q.qs > 0 || (q.tick + 1u - q.nas > C.election_rtt * 20));
    if (C.check_quorum && !q_at_tick && h.election_tick + 1u >= C.election_rtt) {
      // the tick reaches the check-quorum boundary: leaderHasQuorum (raft.go:
      // 378-388) counts self and the remotes active at the tick, i.e. active
      // now or answering in this round's inbox (both response handlers
      // setActive first).  Only a quorum that holds stays on the fast path.
      if (!RBE_FAST_CQ) return false;
      u32 act = 1;
#pragma unroll
      for (u32 s = 0; s < N; s++) {
        if (s == k) continue;
        const u32 j = s - (s > k ? 1u : 0u);
        act += ((st[s] >> 2) & 1u) | ((resp >> j) & 1u);
      }
      if (act < N / 2 + 1) return false;
    }
  }
  // ---- compute.  Every load above has completed before the first store
  // below: vmcnt counts loads and stores in order, so a wait for a load still
  // in flight after a store (the compiler is conservative inside the rolled
  // message loop) would also wait for that store's acknowledgement.
  asm volatile("" ::: "memory");
  rbe_wait_all_loads();
  RBE_STAMP(t2);
  u32 ev_fault = 0;
#if RBE_FAST_EV_EARLY
  // the step's first store: entry ev_idx into the cold log (also when the
  // proposal below does not append after all: a second copy of an entry the
  // ring still holds is harmless), so its registers are free from here on
  if (ev) {
    const u32 t0 = ev_cr.tail;
    ev_fault = cold_put(P, C, ev_cr, ev_idx, ev_e, par) ? 0u : F_NOMEM;
    if (ev_cr.tail != t0) {
      P.cold[r] = ev_cr;
      RBE_AUDIT(AS_COLD_REF, &P.cold[r], sizeof(ColdRef));
    }
  }
#endif
  FastOut<N, TRACE> o;
  o.r = r;
  o.g = g;
  o.k = k;
  o.par = par;
  o.self = k + 1;
  o.round_ = round;
  o.iso = round < until ? isom : (u8)0;
  o.pc = o.pc_hi = 0;
  o.fault = (h.flags & HF_FAULTED) ? P.upd[r].fault : 0u;  // rare: after the first fault
  o.n_msgs = o.n_rtr = o.n_drop_ri = 0;
  o.n_out = o.n_drop_msg = o.n_ent_out = 0;
  o.fault0 = o.fault;
  o.fault |= ev_fault;
  o.msg_hash = o.rtr_hash = o.drop_hash = 0;
  o.events = 0;
  stash_init(o.ost());
  o.term = c.term;
  u8 flags = h.flags;
  u32 etick = h.election_tick, htick = h.heartbeat_tick;
  const u64 committed0 = c.committed;
  const u64 last0 = c.last_index;
  ctr.v[C_STEPS]++;
  // arena of this round (Lane::arena_put / arena_log_range)
  Ent* arena = &P.arena[par][r * C.ecap];
  u32 arena_used = 0, seg_off = 0, seg_len = 0;
  u64 seg_lo = 0;
  // the entry proposed this round (index prop_idx), still in registers
  u64 prop_idx = 0, prop_lo = 0, prop_hi = 0;
  u32 prop_len = 16, prop_type = E_Application;

  // entryLog.term (logentry.go:142-161) without touching memory: a leader's
  // entries [lead_start, last] are of its term and earlier ones of a lower
  // term.  Every lookup here is either compared with the current term
  // (tryCommit, hasCommittedEntryAtCurrentTerm) or, by the eligibility rule
  // next[s] > last0, at an index >= lead_start (makeReplicateMessage), so
  // "lower" (0) is exact for every use.  The ring read the general Lane
  // performs is still counted and window-checked.
  // (an index below the ring is in the cold log, and of a lower term too)
  auto log_term = [&](u64 idx) -> u64 {
    if (idx > c.last_index || idx == 0) return 0;
    if (idx == c.last_index) return c.t_last;
    ctr.v[C_RING_ACCESS]++;
    return idx >= c.lead_start ? c.term : 0;
  };
  auto ent_at = [&](u64 idx) -> Ent {  // ring entry idx (registers when just proposed)
    // anything else is excluded by the eligibility rule next[s] > last0
    const bool hit = idx == prop_idx && prop_idx != 0;
    o.fault_if(!hit, F_UNSUPPORTED);
    Ent e;
    e.term = hit ? c.term : 0;
    e.type = hit ? prop_type : (u32)E_Application;
    e.len = hit ? prop_len : 0u;
    e.lo = hit ? prop_lo : 0;
    e.hi = hit ? prop_hi : 0;
    return e;
  };
  auto limit_count = [&](u64 lo, u64 hi) -> u64 {  // limitSize, entryutils.go:52-64
    const u64 n = hi - lo + 1;
    if (!C.heap_bytes && n * (128 + 16) <= C.max_entry_size) return n;
    u64 total = 128 + ent_at(lo).len;
    u64 inc = 1;
    for (; inc < n; inc++) {
      total += 128 + ent_at(lo + inc).len;
      if (total > C.max_entry_size) break;
    }
    return inc;
  };
  auto arena_log_range = [&](u64 lo, u32 cnt, u32* off) -> bool {  // Lane::arena_log_range
    if (seg_len && lo >= seg_lo && lo + cnt <= seg_lo + seg_len) {
      *off = seg_off + (u32)(lo - seg_lo);
      return true;
    }
    if (seg_len && lo >= seg_lo && lo <= seg_lo + seg_len && seg_off + seg_len == arena_used) {
      const u64 have_hi = seg_lo + seg_len;
      const u32 extra = (u32)(lo + cnt - have_hi);
      o.fault_if(arena_used + extra > C.ecap, F_ARENA);
      if (arena_used + extra > C.ecap) return false;
      for (u32 i = 0; i < extra; i++) {
        const u64 idx = have_hi + i;
        o.fault_if(c.last_index - idx >= C.ring, F_WINDOW);
        arena[arena_used + i] = ent_at(idx);
      }
      ctr.v[C_RING_ACCESS] += extra;
      arena_used += extra;
      seg_len += extra;
      *off = seg_off + (u32)(lo - seg_lo);
      return true;
    }
    o.fault_if(arena_used + cnt > C.ecap, F_ARENA);
    if (arena_used + cnt > C.ecap) return false;
    for (u32 i = 0; i < cnt; i++) {
      const u64 idx = lo + i;
      o.fault_if(c.last_index - idx >= C.ring, F_WINDOW);
      arena[arena_used + i] = ent_at(idx);
    }
    ctr.v[C_RING_ACCESS] += cnt;
    seg_lo = lo;
    seg_off = arena_used;
    seg_len = cnt;
    *off = arena_used;
    arena_used += cnt;
    return true;
  };
  auto try_update = [&](u64& mt, u64& nx, u32& sw, u64 idx) -> bool {  // remote.go:123-133
    ctr.v[C_REMOTE_TOUCH]++;
    if (nx < idx + 1) nx = idx + 1;
    if (mt < idx) {
      if ((sw & 3u) == RS_Wait) sw = (sw & ~3u) | RS_Retry;
      mt = idx;
      return true;
    }
    return false;
  };
  auto try_commit = [&]() -> bool {  // raft.go:886-907 + logentry.go:379-394
    u64 m[N];
#pragma unroll
    for (u32 s = 0; s < N; s++) m[s] = match[s];
#pragma unroll
    for (u32 pass = 0; pass < N; pass++) {
#pragma unroll
      for (u32 i = pass & 1u; i + 1 < N; i += 2) {
        const u64 a = m[i], b = m[i + 1];
        m[i] = a < b ? a : b;
        m[i + 1] = a < b ? b : a;
      }
    }
    ctr.v[C_REMOTE_TOUCH] += N;
    const u64 qv = m[N - Q];
    if (qv <= c.committed) return false;
    if (log_term(qv) != c.term) return false;
    o.fault_if(qv > c.last_index, F_PANIC);  // commitTo panics (logentry.go:324-333)
    if (qv > c.last_index) return true;
    c.committed = qv;
    return true;
  };
  // deferred fan-out state (Lane::rep_mask / hb_pending / rq_pending)
  u32 rep_mask = 0;
  bool hb_pending = false, rq_pending = false;
  u64 hb_lo = 0, hb_hi = 0, rq_plo = 0, rq_phi = 0;
  u32 rq_from = 0;
  auto send_replicate = [&](u32 s) {  // raft.go:758-792
    const u32 rs = st[s] & 3u;
    if (rs == RS_Wait || rs == RS_Snapshot) return;
    const u64 nx = next[s];
    Msg m = mk_msg(M_Replicate, s + 1);
    m.log_index = nx - 1;
    m.log_term = log_term(nx - 1);
    m.commit = c.committed;
    if (nx <= c.last_index) {
      const u64 cnt = limit_count(nx, c.last_index);
      u32 off = 0;
      if (arena_log_range(nx, (u32)cnt, &off)) {
        m.n_ent = (u16)cnt;
        m.ent_off = off;
      }
      // progress (remote.go:135-143)
      if (rs == RS_Replicate) next[s] = nx + cnt;
      else if (rs == RS_Retry) st[s] = (st[s] & ~3u) | RS_Wait;
      o.fault_if(rs != RS_Replicate && rs != RS_Retry, F_PANIC);
      rdirty |= 1u << s;
    }
    o.send(P, C, ctr, m, arena + m.ent_off);
  };
  auto rq_confirm = [&](u64 low, u64 high, u32 from) {  // readindex.go:77-116
    int pos = -1;
#pragma unroll
    for (u32 i = 0; i < Cap::RQ; i++)
      if (pos < 0 && i < rq_n && rq_lo[i] == low && rq_hi[i] == high) pos = (int)i;
    if (pos < 0) return;
    u64 sindex = 0;
    u32 conf = 0;
#pragma unroll
    for (u32 i = 0; i < Cap::RQ; i++)
      if ((int)i == pos) {
        rq_cf[i] |= 1u << (from - 1u);
        conf = rq_cf[i];
        sindex = rq_ix[i];
        rq_dm |= 1u << i;
      }
    ctr.v[C_RQ_TOUCH]++;
    if ((int)popc8(conf) + 1 < (int)Q) return;
    const u32 done = (u32)pos + 1;
#pragma unroll
    for (u32 i = 0; i < Cap::RQ; i++) {
      if (i >= done) continue;
      o.fault_if(rq_ix[i] > sindex, F_PANIC);
      if (rq_fr[i] == 0 || rq_fr[i] == o.self) {
        o.ready_to_read(P, C, ctr, sindex, rq_lo[i], rq_hi[i]);
      } else {
        Msg m = mk_msg(M_ReadIndexResp, rq_fr[i]);
        m.log_index = sindex;
        m.hint = low;
        m.hint_high = high;
        o.send(P, C, ctr, m, nullptr);
      }
    }
    ctr.v[C_RQ_TOUCH] += done;
    // pop `done` entries: shift the register queue down
#pragma unroll
    for (u32 i = 0; i < Cap::RQ; i++) {
      u64 a = 0, b = 0, x = 0;
      u32 f = 0, cf = 0;
#pragma unroll
      for (u32 j = 0; j < Cap::RQ; j++)
        if (j == i + done) {
          a = rq_lo[j];
          b = rq_hi[j];
          x = rq_ix[j];
          f = rq_fr[j];
          cf = rq_cf[j];
        }
      rq_lo[i] = a;
      rq_hi[i] = b;
      rq_ix[i] = x;
      rq_fr[i] = f;
      rq_cf[i] = cf;
    }
    rq_h += done;
    if (rq_h >= C.rq_cap) rq_h -= C.rq_cap;
    rq_n -= done;
    rq_dm >>= done;
  };
  auto fan_out = [&]() {
#pragma unroll
    for (u32 s = 0; s < N; s++)
      if (rep_mask & (1u << s)) send_replicate(s);
    rep_mask = 0;
    if (hb_pending) {
      hb_pending = false;
#pragma unroll
      for (u32 s = 0; s < N; s++) {
        if (s == k) continue;
        Msg m = mk_msg(M_Heartbeat, s + 1);  // raft.go:810-820
        m.commit = umin64(match[s], c.committed);
        m.hint = hb_lo;
        m.hint_high = hb_hi;
        o.send(P, C, ctr, m, nullptr);
      }
      ctr.v[C_REMOTE_TOUCH] += N - 1;
    }
    if (rq_pending) {
      rq_pending = false;
      rq_confirm(rq_plo, rq_phi, rq_from);
    }
  };

  // handleReadIndexRequests (node.go:1108-1118)
  if (inp == 2) {
    q.record_activity(C, M_ReadIndex);
    ctr.v[C_READS]++;
  }
  // handleReceivedMessages: senders in ascending order
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    if (s == k) continue;
    if (pcin[s] & 0x8000u) {  // Quiesce first in the sender's stream
      ctr.v[C_MSG_IN]++;
      q.try_enter(C);
    }
    // a rolled loop (the handler + fan-out body is too large to replicate
    // per message) reading the prefetched headers through a select chain,
    // so the register array is never indexed dynamically
    const u32 nb = (pcin[s] >> 7) & 0x7Fu;
    // this sender's row: s - 1 when s > k, else s (both compile-time here)
    const u32 jlo = s == 0 ? 0u : s - 1u;
    const u32 jhi = s + 1 >= N ? N - 2u : s;
    const bool use_lo = s > k;
    const u64 match0 = match[s], next0 = next[s];
    const u32 st0 = st[s];
#pragma unroll 1
    for (u32 i = 0; i < nb; i++) {
      LeadIn m;
      if constexpr (kLdsIn) {
        const u32 sl = (use_lo ? jlo : jhi) * Cap::MAXM + i;
        m.w = s_in_w[sl][lds_lane];
        m.a = s_in_a[sl][lds_lane];
        m.b = s_in_b[sl][lds_lane];
      } else {
        m = use_lo ? inc[jlo][0] : inc[jhi][0];
#pragma unroll
        for (u32 j = 1; j < Cap::MAXM; j++)
          if (i == j) m = use_lo ? inc[jlo][j] : inc[jhi][j];
      }
      ctr.v[C_MSG_IN]++;
      const u32 mtype = m.w & 0xFFu;
      if (mtype == M_HeartbeatResp && m.a > 0) q.record_activity(C, M_ReadIndex);
      else q.record_activity(C, mtype);
      st[s] |= 4u;  // setActive
      if (mtype == M_ReplicateResp) {  // raft.go:1667-1696 (accepted: rejections
        {                              // take the full table, see the gather)
          const u32 rs = st[s] & 3u;
          const bool paused = rs == RS_Wait || rs == RS_Snapshot;
          if (try_update(match[s], next[s], st[s], m.a)) {
            // respondedTo (remote.go:145-153); snapshotIndex is 0 on device
            const u32 rs2 = st[s] & 3u;
            if (rs2 == RS_Retry) {
              next[s] = match[s] + 1;
              st[s] = (st[s] & ~3u) | RS_Replicate;
            } else if (rs2 == RS_Snapshot) {
              next[s] = match[s] + 1;
              st[s] = (st[s] & ~3u) | RS_Retry;
            }
            if (try_commit()) rep_mask |= ((1u << N) - 1u) & ~(1u << k);
            else if (paused) rep_mask |= 1u << s;
          }
        }
      } else {  // HeartbeatResp, raft.go:1698-1710
        if ((st[s] & 3u) == RS_Wait) st[s] = (st[s] & ~3u) | RS_Retry;
        ctr.v[C_REMOTE_TOUCH]++;
        if (match[s] < c.last_index) rep_mask |= 1u << s;
        if (m.a != 0) {
          rq_pending = true;
          rq_plo = m.a;
          rq_phi = m.b;
          rq_from = s + 1;
        }
      }
      fan_out();
    }
    if (match[s] != match0 || next[s] != next0 || st[s] != st0) rdirty |= 1u << s;
  }
  // batchedReadIndex → Peer.ReadIndex → handleLeaderReadIndex (raft.go:1633-1665)
  if (inp == 2) {
    const u64 low = xin ? xlo : (((u64)(round + 1) << 32) | (u64)o.self);
    const u64 high = xin ? xhi : cid + 1;
    if (log_term(c.committed) != c.term) {
      o.dropped_read_index(P, C, ctr, low, high);
    } else {
      // readIndex.addRequest (readindex.go:43-67)
      bool dup = false;
#pragma unroll
      for (u32 i = 0; i < Cap::RQ; i++)
        if (i < rq_n && rq_lo[i] == low && rq_hi[i] == high) dup = true;
      if (!dup) {
        u64 back_ix = 0;
#pragma unroll
        for (u32 i = 0; i < Cap::RQ; i++)
          if (i + 1 == rq_n) back_ix = rq_ix[i];
        o.fault_if(rq_n > 0 && c.committed < back_ix, F_PANIC);
        o.fault_if(rq_n >= C.rq_cap, F_READQ);
        if (rq_n < C.rq_cap) {
#pragma unroll
          for (u32 i = 0; i < Cap::RQ; i++)
            if (i == rq_n) {
              rq_lo[i] = low;
              rq_hi[i] = high;
              rq_ix[i] = c.committed;
              rq_fr[i] = 0;
              rq_cf[i] = 0;
            }
          rq_dm |= 1u << rq_n;
          rq_n++;
          ctr.v[C_RQ_TOUCH]++;
        }
      }
      hb_pending = true;
      hb_lo = low;
      hb_hi = high;
    }
    fan_out();
  }
  // the tick (node.go:1384-1399 → raft.go:551-564, 592-629)
  RBE_STAMP(t3);
  q.increase_tick(C);
  const u32 qd = q.quiesced(C) ? 1u : 0u;
  ctr.v[C_QUIESCED_TICKS] += qd;
  ctr.v[C_ACTIVE_TICKS] += 1u - qd;
  if (qd) {
    flags |= HF_RAFT_QUIESCE;
    etick++;
  } else {
    flags &= (u8)~HF_RAFT_QUIESCE;
    etick++;  // leaderTick
    if (etick >= C.election_rtt) {
      etick = 0;
      if (C.check_quorum) {
        // handleLeaderCheckQuorum with the quorum eligibility established:
        // leaderHasQuorum clears the active flag of everything it counted
#pragma unroll
        for (u32 s = 0; s < N; s++) {
          if (st[s] & 4u) {
            st[s] &= ~4u;
            rdirty |= 1u << s;
          }
        }
      }
    }
    htick++;
    if (htick >= C.heartbeat_rtt) {
      htick = 0;
      // broadcastHeartbeatMessage (raft.go:824-832)
      u64 lo = 0, hi = 0;
#pragma unroll
      for (u32 i = 0; i < Cap::RQ; i++)
        if (i + 1 == rq_n) {
          lo = rq_lo[i];
          hi = rq_hi[i];
        }
      hb_pending = true;
      hb_lo = lo;
      hb_hi = hi;
    }
  }
  fan_out();
  // the proposal (handleProposals → Peer.ProposeEntries → handleLeaderPropose)
  if (inp == 1) {
    const u64 lo = xin ? xlo : wl_payload_lo(C.seed, cid, round), hi = xin ? xhi : mix64(lo);
    ctr.v[C_PROPOSALS]++;
    // the workload's entry is staged in the arena as the Propose message
    // carries it (term 0); the host's stays in Planes::in_ents (Lane::run)
    o.fault_if(!xin && arena_used + 1 > C.ecap, F_ARENA);
    if (xin || arena_used + 1 <= C.ecap) {
      if (!xin) {
        Ent e;
        e.term = 0;
        e.type = E_Application;
        e.len = 16;
        e.lo = lo;
        e.hi = hi;
        arena[arena_used] = e;
        arena_used++;
      }
      // appendEntries (raft.go:909-920)
      const u64 idx = c.last_index + 1;
      if (!RBE_FAST_EV_EARLY && ev) {  // the entry the slot held, into the cold log
        const u32 t0 = ev_cr.tail;
        o.fault_if(!cold_put(P, C, ev_cr, ev_idx, ev_e, par), F_NOMEM);
        if (ev_cr.tail != t0) {
      P.cold[r] = ev_cr;
      RBE_AUDIT(AS_COLD_REF, &P.cold[r], sizeof(ColdRef));
    }
      }
      const u64 sl = (idx & (u64)(C.ring - 1)) * C.n_rep + r;
      P.term_ring[sl] = c.term;
      RBE_AUDIT(AS_TERM, &P.term_ring[sl], 8);
      Body b;
      b.type = xtype;
      b.len = xlen;
      b.lo = lo;
      b.hi = hi;
      P.pay_ring[sl] = b;
      RBE_AUDIT(AS_PAY, &P.pay_ring[sl], sizeof(Body));
      ctr.v[C_RING_ACCESS]++;
      c.last_index = idx;
      c.t_last = c.term;
      cdirty |= 0xEu;
      prop_idx = idx;
      prop_lo = lo;
      prop_hi = hi;
      prop_len = xlen;
      prop_type = xtype;
#pragma unroll
      for (u32 s = 0; s < N; s++)
        if (s == k) try_update(match[s], next[s], st[s], c.last_index);
      rdirty |= 1u << k;
      rep_mask |= ((1u << N) - 1u) & ~(1u << k);
      fan_out();
    }
  }
  (void)last0;
  // ---- scatter
  RBE_STAMP(t4);
  if (xin) {  // the host input is consumed (Lane::run clears the record)
    ExtIn z{};
    P.ext[r] = z;
    RBE_AUDIT(AS_EXT, &P.ext[r], sizeof(ExtIn));
  }
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    RemoteMN x;
    x.match = match[s];
    x.next = next[s];
    if (rdirty & (1u << s)) {
      P.rem[r * N + s] = x;
      P.rem_st[r * N + s] = (u8)st[s];
      RBE_AUDIT(AS_REM, &P.rem[r * N + s], sizeof(RemoteMN));
      RBE_AUDIT(AS_REM_ST, &P.rem_st[r * N + s], 1);
    }
  }
  if (rq_dm) {
#pragma unroll
    for (u32 i = 0; i < Cap::RQ; i++) {
      if (i < rq_n && ((rq_dm >> i) & 1u)) {
        ReadReq x;
        x.low = rq_lo[i];
        x.high = rq_hi[i];
        x.index = rq_ix[i];
        x.from = (u8)rq_fr[i];
        x.confirmed = (u8)rq_cf[i];
        for (int j = 0; j < 6; j++) x.pad[j] = 0;
        P.rq[rq_slot(i)] = x;
        RBE_AUDIT(AS_RQ, &P.rq[rq_slot(i)], sizeof(ReadReq));
      }
    }
  }
  if ((u8)rq_h != c.rq_head || (u8)rq_n != c.rq_count) cdirty |= 4u;
  c.rq_head = (u8)rq_h;
  c.rq_count = (u8)rq_n;
  fast_finish<N, TRACE>(P, C, ctr, o, q, R_Leader, flags, h, c, etick, htick, committed0,
                        digest0, cdirty);
  RBE_STAMP(t5);
  RBE_RSTAMP(rt5);
  RBE_PHASE_ADD(0, 5, rt0, rt5);
  RBE_PHASE_ADD(0, 6, t0, t5);
  RBE_PHASE_ADD(0, 0, t0, t1);
  RBE_PHASE_ADD(0, 1, t1, t2);
  RBE_PHASE_ADD(0, 2, t2, t3);
  RBE_PHASE_ADD(0, 3, t3, t4);
  RBE_PHASE_ADD(0, 4, t4, t5);
  RBE_PHASE_ADD(0, 7, 0, 1);
  return true;
  }
}

// ---------------------------------------------------------------- follower
// One steady-state follower round: inbox from the known leader only
// (Replicate / Heartbeat / ReadIndexResp of the current term), no client
// input, a tick that does not start an election.
template <int N, bool TRACE, bool AUX = false, class CT>
RBE_HD bool foll_fast(const Planes& P, const Params& C, u64 r, const Clk& ck, CT& ctr,
                      u32 aux = 0) {
  const u32 round = ck.round;
  using Cap = FastCaps<N>;
  if constexpr (!kFastN<N>) {
    return false;
  } else {
  const u64 g = r / N;
  const u32 k = (u32)(r % N);
  const u32 par = round & 1u, ppar = par ^ 1u;
  // ---- gather, level 1
  RBE_RSTAMP(rt0);
  RBE_STAMP(t0);
  Hot h = load_hot(P, C, r, ck.tclk);
  Core c = P.core[r];
  u32 pcin[N];
  // With AUX the count words came with the work-list entry (inbound_aux):
  // the messages of the one sender that has any (the leader, checked below)
  // and the first entry of its arena are loaded in this first gather level.
  Msg raw[Cap::FMAXM];
  Ent spec0;
  u32 ls_a = 0xFFFFFFFFu;
  if constexpr (AUX) {
#pragma unroll
    for (u32 s = 0; s < N; s++) pcin[s] = s == k ? 0u : aux_count_word<N>(aux, k, s);
    u32 na_a = 0, n_a = 0;
#pragma unroll
    for (u32 s = N; s-- > 0;) {
      const u32 n = (pcin[s] & 0x7Fu) + ((pcin[s] >> 7) & 0x7Fu);
      if (s != k && n) {
        ls_a = s;
        na_a = pcin[s] & 0x7Fu;
        n_a = n;
      }
    }
    const u32 sa = ls_a < N ? ls_a : 0u;
    const Msg* la = &P.msgs[ppar][((g * N + sa) * N + k) * (u64)C.maxm];
#pragma unroll
    for (u32 i = 0; i < Cap::FMAXM; i++)
      if (i < n_a) raw[i] = la[i < na_a ? i : C.maxm - 1u - (i - na_a)];
    spec0.term = spec0.lo = spec0.hi = 0;
    spec0.type = spec0.len = 0;
    if (na_a > 0) spec0 = P.arena[ppar][(g * N + sa) * (u64)C.ecap];
  } else {
#pragma unroll
    for (u32 s = 0; s < N; s++) pcin[s] = s != k ? in_word<N>(P, g, s, k, round) : 0u;
  }
  // the isolation schedule and the Update record are read only when in use:
  // two of the lane's scattered lines saved in the steady state
  const u32 until = C.iso_period ? P.iso_until[g] : 0u;
  const u8 isom = C.iso_period ? P.iso_mask[g] : (u8)0;
  const u64 digest0 = TRACE ? P.upd[r].digest : 0;
  u32 cdirty = 0;  // Core chunks an append or a new leader wrote (fast_finish)
  if (h.role != R_Follower) return false;
  if (h.flags & HF_SNAP_WORK) return false;  // compaction / SnapshotStatus: full table
  if (C.membership && (c.members | c.cc_apply | c.mflags) != 0) return false;  // (lead_fast)
  if (C.ext_commit && c.saved_to + 1 < P.imark[r]) return false;  // (lead_fast)
  if (h.flags & (HF_APPLY_PENDING | HF_IS_LTT)) return false;
  if (c.ltt != 0) return false;
  if (!ck.tick) return false;
  if (C.xfer_period && xfer_input(C, cid_of_n<N>(C, g), round, k)) return false;
  if (C.ext_inputs && P.ext[r].flags) return false;
  // the step's ReadyToReads (one per ReadIndexResp) stay within the plane list
  if (C.rtr_cap < Cap::FMAXM) return false;
  const u32 ls = (u32)c.leader - 1u;  // leader slot (0xFFFFFFFF when no leader)
  u32 n_in = 0;
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    if (s == k) continue;
    const u32 n = (pcin[s] & 0x7Fu) + ((pcin[s] >> 7) & 0x7Fu);
    if (n && s != ls) return false;
    n_in += n;
  }
  if (n_in > Cap::FMAXM) return false;
  // ---- gather, level 2: the leader's messages (Replicate first, then the rest)
  RBE_STAMP(t1);
  InMsg in[Cap::FMAXM];
  u32 na = 0;
  const Msg* lst = &P.msgs[ppar][((g * N + (ls < N ? ls : 0)) * N + k) * (u64)C.maxm];
#pragma unroll
  for (u32 s = 0; s < N; s++)
    if (s == ls && s != k) na = pcin[s] & 0x7Fu;
  // loads only inside the branches, decoded after the join (see lead_fast);
  // with AUX they were issued in the first level from the same list (every
  // message came from ls, so ls_a == ls whenever n_in > 0)
  if constexpr (!AUX) {
#pragma unroll
    for (u32 i = 0; i < Cap::FMAXM; i++) {
      if (i < n_in) raw[i] = lst[i < na ? i : C.maxm - 1u - (i - na)];
    }
  } else {
    (void)ls_a;
  }
  // a Replicate may append at last + 1, whose ring slot holds entry last + 1
  // - ring: it goes to the cold log (rbe_spill.h) unless compacted; its
  // record and the cold-log ref now, with the messages
  const u64 lmark = C.snapshot_entries ? P.snp[r].marker : 0;
  const u64 ev_idx = c.last_index + 1 > C.ring ? c.last_index + 1 - C.ring : 0;
#ifdef RBE_DIAG_NO_EVICT
  const bool ev = false;
#else
  const bool ev = na > 0 && ev_idx > lmark;
#endif
  bool ev_app = false;
  Ent ev_e;
  ColdRef ev_cr;
  ev_e.term = ev_e.lo = ev_e.hi = 0;
  ev_e.type = ev_e.len = 0;
  ev_cr.head = ev_cr.tail = 0;
  ev_cr.tail_pn = 0;
  if (ev) {
    const u64 es = (ev_idx & (u64)(C.ring - 1)) * C.n_rep + r;
    const Body eb = P.pay_ring[es];
    ev_e.term = P.term_ring[es];
    ev_e.type = eb.type;
    ev_e.len = eb.len;
    ev_e.lo = eb.lo;
    ev_e.hi = eb.hi;
    ev_cr = P.cold[r];
  }
#pragma unroll
  for (u32 i = 0; i < Cap::FMAXM; i++) {
    if (i < n_in) in[i] = load_in(&raw[i]);
    else in[i].type = 0xFFu;
  }
#pragma unroll
  for (u32 i = 0; i < Cap::FMAXM; i++) {
    if (in[i].type == 0xFFu) continue;
    const u32 t = in[i].type;
    if (in[i].term != c.term) return false;
    if (t != M_Replicate && t != M_Heartbeat && t != M_ReadIndexResp) return false;
    if (in[i].n_ent == 0xFFFFu) return false;  // entries in the spill heap (load_in)
  }
  FastQ q;
  q.tick = h.q_tick;
  q.qs = h.q_quiesced_since;
  q.nas = h.q_no_activity_since;
  q.eqt = h.q_exit_quiesce_tick;
  q.qnew = false;
  {
    const bool idle = n_in == 0;
    const bool q_at_tick = idle && C.quiesce &&
                           (q.qs > 0 || (q.tick + 1u - q.nas > C.election_rtt * 20));
    if (n_in == 0 && !q_at_tick && h.election_tick + 1u >= h.rand_et) return false;
  }
  // ---- gather, level 3: the first entry of the first four Replicate messages
  // (a steady-state round carries up to three: commit broadcasts and resends
  // without entries, then the new proposal)
  Ent pre0, pre1, pre2, pre3;
  pre0.term = pre0.lo = pre0.hi = 0;
  pre0.type = pre0.len = 0;
  pre1 = pre2 = pre3 = pre0;
  {
    const Ent* ab = &P.arena[ppar][(g * N + (ls < N ? ls : 0)) * (u64)C.ecap];
    if constexpr (AUX) {  // the shared segment of a broadcast starts at offset 0
      if (na > 0 && n_in > 0 && in[0].n_ent > 0)
        pre0 = in[0].ent_off == 0 ? spec0 : ab[in[0].ent_off];
    } else {
      if (na > 0 && n_in > 0 && in[0].n_ent > 0) pre0 = ab[in[0].ent_off];
    }
    if (na > 1 && n_in > 1 && in[1].n_ent > 0) pre1 = ab[in[1].ent_off];
    if (na > 2 && n_in > 2 && in[2].n_ent > 0) pre2 = ab[in[2].ent_off];
    if (na > 3 && n_in > 3 && in[3].n_ent > 0) pre3 = ab[in[3].ent_off];
  }
  // Simulate the round's Replicate handling (handleReplicateMessage,
  // raft.go:1339-1372) on the log tail: admit the round only if every log
  // lookup hits t_last or lies past the tail and every appended entry is one
  // of the two prefetched, so nothing is read after the first store below.
  {
    u64 L = c.last_index, Cm = c.committed, T = c.t_last;
#pragma unroll
    for (u32 i = 0; i < Cap::FMAXM; i++) {
      if (in[i].type == 0xFFu) continue;
      const InMsg& m = in[i];
      if (m.type == M_Replicate) {
        if (m.log_index < Cm) continue;          // answered with committed
        if (m.log_index != L) return false;      // a ring lookup (or past the tail)
        if (m.log_term != T) continue;           // rejected: no lookups, no change
        if (m.n_ent > 1 || (m.n_ent == 1 && i >= 4)) return false;
        if (C.membership && m.n_ent == 1 &&      // a ConfigChange entry: full table
            ent_type(i == 0 ? pre0.type : (i == 1 ? pre1.type : (i == 2 ? pre2.type : pre3.type))) ==
                E_ConfigChange)
          return false;
        if (m.n_ent == 1) {                      // conflict at L + 1: append
          // a second append past the ring would evict an entry not loaded above
          if (L != c.last_index && L + 1 > C.ring) return false;
          T = i == 0 ? pre0.term : (i == 1 ? pre1.term : (i == 2 ? pre2.term : pre3.term));
          L = L + 1;
        }
        const u64 li = m.log_index + m.n_ent;
        const u64 x = li < m.commit ? li : m.commit;
        if (x > Cm && x <= L) Cm = x;
      } else if (m.type == M_Heartbeat) {
        if (m.commit > Cm && m.commit <= L) Cm = m.commit;
      }
    }
    // the apply range stays in the ring window
    if (L - c.processed > C.ring) return false;
    ev_app = ev && L > c.last_index;  // the append at last + 1 happens
  }
  // ---- compute.  Every load above has completed before the first store
  // below (vmcnt counts loads and stores in order; see lead_fast).
  asm volatile("" ::: "memory");
  rbe_wait_all_loads();
  RBE_STAMP(t2);
  u32 ev_fault = 0;
#if RBE_FAST_EV_EARLY
  if (ev_app) {  // the step's first store: the append's slot held entry ev_idx
    const u32 t0 = ev_cr.tail;
    ev_fault = cold_put(P, C, ev_cr, ev_idx, ev_e, par) ? 0u : F_NOMEM;
    if (ev_cr.tail != t0) {
      P.cold[r] = ev_cr;
      RBE_AUDIT(AS_COLD_REF, &P.cold[r], sizeof(ColdRef));
    }
  }
#endif
  FastOut<N, TRACE> o;
  o.r = r;
  o.g = g;
  o.k = k;
  o.par = par;
  o.self = k + 1;
  o.round_ = round;
  o.iso = round < until ? isom : (u8)0;
  o.pc = o.pc_hi = 0;
  o.fault = (h.flags & HF_FAULTED) ? P.upd[r].fault : 0u;  // rare: after the first fault
  o.n_msgs = o.n_rtr = o.n_drop_ri = 0;
  o.n_out = o.n_drop_msg = o.n_ent_out = 0;
  o.fault0 = o.fault;
  o.fault |= ev_fault;
  o.msg_hash = o.rtr_hash = o.drop_hash = 0;
  o.events = 0;
  stash_init(o.ost());
  o.term = c.term;
  u8 flags = h.flags;
  u32 etick = h.election_tick;
  const u32 htick = h.heartbeat_tick;
  const u64 committed0 = c.committed;
  ctr.v[C_STEPS]++;
  // entryLog.term (logentry.go:142-161) without touching memory: the
  // eligibility simulation above admits only rounds whose lookups hit the
  // log tail (t_last) or lie past it.
  auto log_term = [&](u64 idx) -> u64 {
    if (idx > c.last_index || idx == 0) return 0;
    if (idx == c.last_index) return c.t_last;
    const bool miss = c.last_index - idx >= C.ring;
    // a miss is F_WINDOW; a hit is excluded by the eligibility simulation
    o.fault_if(true, miss ? F_WINDOW : F_UNSUPPORTED);
    ctr.v[C_RING_ACCESS] += miss ? 0u : 1u;
    return 0;
  };
  auto commit_to = [&](u64 idx) {  // logentry.go:324-333
    if (idx <= c.committed) return;
    o.fault_if(idx > c.last_index, F_PANIC);
    if (idx > c.last_index) return;
    c.committed = idx;
  };
  const u32 lid = ls + 1;
  if (!RBE_FAST_EV_EARLY && ev_app) {  // the append's ring slot held entry ev_idx: into the cold log
    const u32 t0 = ev_cr.tail;
    o.fault_if(!cold_put(P, C, ev_cr, ev_idx, ev_e, par), F_NOMEM);
    if (ev_cr.tail != t0) {
      P.cold[r] = ev_cr;
      RBE_AUDIT(AS_COLD_REF, &P.cold[r], sizeof(ColdRef));
    }
  }
#pragma unroll
  for (u32 s = 0; s < N; s++) {
    if (s == k) continue;
    if (pcin[s] & 0x8000u) {  // Quiesce first in the sender's stream
      ctr.v[C_MSG_IN]++;
      q.try_enter(C);
    }
    if (s != ls) continue;
#pragma unroll
    for (u32 i = 0; i < Cap::FMAXM; i++) {
      if (in[i].type == 0xFFu) continue;
      const InMsg& m = in[i];
      ctr.v[C_MSG_IN]++;
      ctr.v[C_ENT_IN] += m.n_ent;
      if (m.type == M_Heartbeat && m.hint > 0) q.record_activity(C, M_ReadIndex);
      else q.record_activity(C, m.type);
      etick = 0;  // handleFollower{Replicate,Heartbeat,ReadIndexResp}: leader = from
      if (m.type == M_Replicate) {  // handleReplicateMessage, raft.go:1339-1372
        const Ent* ents = &P.arena[ppar][(g * N + s) * (u64)C.ecap + m.ent_off];
        (void)ents;
        auto ent = [&](u32 e) -> Ent {  // the eligibility simulation admits n_ent <= 1
          if (i == 1) return pre1;
          if (i == 2) return pre2;
          if (i == 3) return pre3;
          return pre0;
        };
        Msg resp = mk_msg(M_ReplicateResp, lid);
        if (m.log_index < c.committed) {
          resp.log_index = c.committed;
        } else if (log_term(m.log_index) == m.log_term) {
          // tryAppend / getConflictIndex (logentry.go:291-322)
          u64 conflict = 0;
          u32 ci = 0;
          for (u32 e = 0; e < m.n_ent; e++) {
            const u64 idx = m.log_index + 1 + e;
            if (log_term(idx) != ent(e).term) {
              conflict = idx;
              ci = e;
              break;
            }
          }
          if (conflict != 0) {
            o.fault_if(conflict <= c.committed, F_PANIC);
            if (conflict > c.committed) {
              o.fault_if(conflict - 1 >= 1 && conflict - 1 <= c.last_index &&
                             log_term(conflict - 1) > ent(ci).term,
                         F_PANIC);
              u64 tl = c.t_last;
              for (u32 e = ci; e < m.n_ent; e++) {
                const Ent x = ent(e);
                const u64 ai = m.log_index + 1 + e;
                const u64 sl = (ai & (u64)(C.ring - 1)) * C.n_rep + r;
                P.term_ring[sl] = x.term;
                RBE_AUDIT(AS_TERM, &P.term_ring[sl], 8);
                Body b;
                b.type = x.type;
                b.len = x.len;
                b.lo = x.lo;
                b.hi = x.hi;
                P.pay_ring[sl] = b;
                RBE_AUDIT(AS_PAY, &P.pay_ring[sl], sizeof(Body));
                ctr.v[C_RING_ACCESS]++;
                tl = x.term;
              }
              c.last_index = m.log_index + m.n_ent;
              c.t_last = tl;
              c.saved_to = umin64(c.saved_to, conflict - 1);
              cdirty |= 0xEu;
            }
          }
          const u64 last_idx = m.log_index + m.n_ent;
          commit_to(umin64(last_idx, m.commit));
          resp.log_index = last_idx;
        } else {
          resp.reject = 1;
          resp.log_index = m.log_index;
          resp.hint = c.last_index;
          o.event_if(true, EV_REPLICATION_REJECTED);
        }
        o.send(P, C, ctr, resp, nullptr);
      } else if (m.type == M_Heartbeat) {  // handleHeartbeatMessage, raft.go:1301-1309
        commit_to(m.commit);
        Msg resp = mk_msg(M_HeartbeatResp, lid);
        resp.hint = m.hint;
        resp.hint_high = m.hint_high;
        o.send(P, C, ctr, resp, nullptr);
      } else {  // ReadIndexResp, raft.go:1890-1898
        o.ready_to_read(P, C, ctr, m.log_index, m.hint, m.hint_high);
      }
    }
  }
  // the tick (raft.go:566-590, 623-629)
  RBE_STAMP(t3);
  q.increase_tick(C);
  const u32 qd = q.quiesced(C) ? 1u : 0u;
  ctr.v[C_QUIESCED_TICKS] += qd;
  ctr.v[C_ACTIVE_TICKS] += 1u - qd;
  if (qd) {
    flags |= HF_RAFT_QUIESCE;
    etick++;
  } else {
    flags &= (u8)~HF_RAFT_QUIESCE;
    etick++;  // nonLeaderTick; reaching the timeout is excluded above
    o.fault_if(etick >= h.rand_et, F_UNSUPPORTED);
  }
  const bool lchg = n_in && (u8)lid != c.leader;
  cdirty |= lchg ? 4u : 0u;
  o.event_if(lchg, EV_LEADER_UPDATED);
  c.leader = n_in ? (u8)lid : c.leader;
  fast_finish<N, TRACE>(P, C, ctr, o, q, R_Follower, flags, h, c, etick, htick, committed0,
                        digest0, cdirty);
  RBE_STAMP(t5);
  RBE_RSTAMP(rt5);
  RBE_PHASE_ADD(1, 5, rt0, rt5);
  RBE_PHASE_ADD(1, 6, t0, t5);
  RBE_PHASE_ADD(1, 0, t0, t1);
  RBE_PHASE_ADD(1, 1, t1, t2);
  RBE_PHASE_ADD(1, 2, t2, t3);
  RBE_PHASE_ADD(1, 4, t3, t5);
  RBE_PHASE_ADD(1, 7, 0, 1);
  return true;
  }
}

// the fast step of one role (k_round, k_fast_list)
template <int N, bool TRACE, int MODE, bool AUX = false, class CT>
RBE_HD bool step_fast(const Planes& P, const Params& C, u64 r, const Clk& ck, CT& ctr,
                      u32 aux = 0) {
  if constexpr (MODE == MODE_LEAD) return lead_fast<N, TRACE, AUX>(P, C, r, ck, ctr, aux);
  else return foll_fast<N, TRACE, AUX>(P, C, r, ck, ctr, aux);
}

}  // namespace rbe
