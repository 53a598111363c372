// rbe_spill.h — the spill tiers of the batched Raft step engine.
//
// The planes give every replica fixed capacities sized for the steady state:
// a term / payload ring of `ring` entries, `maxm` messages per (sender,
// destination) list, an `ecap`-entry arena for the entries its messages carry,
// `rq_cap` queued ReadIndex requests, `rtr_cap` ReadyToReads and `dri_cap`
// dropped ReadIndexes per step.  The reference has none of these limits, so a
// full plane spills here instead of faulting the replica:
//
//   1. the cold log — entryLog below the in-memory window, the ILogDB read path
//      of logentry.go:144-161 (term) and 186-246 (getEntriesFromLogDB): every
//      entry a ring write overwrites is evicted into the replica's chain of
//      pages of a device-wide page pool, and read back from there.  Pages at or
//      below the LogDB compaction marker are released (node_snapshot), a
//      restored snapshot releases them all.  Without snapshots the chain keeps
//      every entry, as dragonboat's LogDB does (SnapshotEntries = 0).
//   2. the readIndex queue beyond rq_cap (readindex.go:43-116 is unbounded):
//      the whole queue moves into pages of the same pool and returns to the
//      plane ring once it drains.
//   3. the round spill heap (one per round parity, reset every other round):
//      a message list past maxm moves there whole (a catch-up leader's
//      ReadIndexResps, a burst of Replicates), as do a message's entries past
//      the sender's ecap arena (a catch-up Replicate sized by MaxEntrySize,
//      raft.go:709-740 and limitSize, entryutils.go:50-64) and a step's
//      ReadyToReads / dropped ReadIndexes past rtr_cap / dri_cap.
//
// The plane keeps the first-tier form, so the steady-state kernels never look
// here: a spilled list's count word carries kCntSpill (and saturated counts,
// which every fast step declines), a spilled queue's Core::rq_count is kRqExt,
// and a message with entries in the heap carries kMsgXEnt.  Only exhaustion
// of a tier itself (cfg.pool_bytes, cfg.spill_bytes) is a fault: F_NOMEM.
//
// Concurrency.  Page allocation takes a page from the free stack of the other
// round parity (pages freed in the last round) by CAS, else from the bump
// counter; a page freed in a round of parity p goes to stack p.  No stack is
// pushed and popped in the same round, so the pops need no ABA guard.  A
// replica's chains are touched only by the lane stepping it.
#pragma once
#include "rbe_types.h"

namespace rbe {

// ---------------------------------------------------------------- atomics
// (the host build steps one replica at a time: plain operations)
RBE_HD u32 sp_atomic_add_u32(u32* p, u32 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  const u32 o = *p;
  *p = o + v;
  return o;
#endif
}
RBE_HD u64 sp_atomic_add_u64(u64* p, u64 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (u64)atomicAdd((unsigned long long*)p, (unsigned long long)v);
#else
  const u64 o = *p;
  *p = o + v;
  return o;
#endif
}
RBE_HD void sp_atomic_or_u32(u32* p, u32 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  *p |= v;
#endif
}
RBE_HD void sp_atomic_max_u64(u64* p, u64 v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicMax((unsigned long long*)p, (unsigned long long)v);
#else
  if (*p < v) *p = v;
#endif
}

// ---------------------------------------------------------------- page pool
template <class PL>
RBE_HD Ent* pool_ent(const PL& P, u32 page, u32 slot) {
  return &P.pool[(u64)page * kPageEnts + slot];
}
// a page for a step of round parity `par`; 0 when the pool is exhausted
template <class PL, class PA>
RBE_HD u32 pool_alloc(const PL& P, const PA& C, u32 par) {
  SpillCtl* s = P.sctl;
  u32* fh = &s->free_head[par ^ 1u];
#if defined(__HIP_DEVICE_COMPILE__)
  u32 h = __hip_atomic_load(fh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (h) {
    const u32 nx = P.pmeta[h].next;
    const u32 o = atomicCAS(fh, h, nx);
    if (o == h) break;
    h = o;
  }
#else
  const u32 h = *fh;
  if (h) *fh = P.pmeta[h].next;
#endif
  if (h) {
    sp_atomic_add_u32(&s->live, 1u);
    return h;
  }
  const u32 p = sp_atomic_add_u32(&s->bump, 1u);
  if (p >= C.pool_pages) {
    sp_atomic_or_u32(&s->oom, 1u);
    return 0;
  }
  sp_atomic_add_u32(&s->live, 1u);
  return p;
}
template <class PL>
RBE_HD void pool_free(const PL& P, u32 par, u32 page) {
  sp_atomic_add_u32(&P.sctl->live, ~0u);  // - 1
  u32* fh = &P.sctl->free_head[par];
#if defined(__HIP_DEVICE_COMPILE__)
  u32 h = __hip_atomic_load(fh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    P.pmeta[page].next = h;
    const u32 o = atomicCAS(fh, h, page);
    if (o == h) return;
    h = o;
  }
#else
  P.pmeta[page].next = *fh;
  *fh = page;
#endif
}

// ---------------------------------------------------------------- cold log
// The page of `cr` holding page number pn, or 0: walked from the nearer end
// (a catch-up reads just below the ring; a joining node from the bottom)
template <class PL>
RBE_HD u32 cold_find(const PL& P, const ColdRef& cr, u64 pn) {
  if (!cr.tail || pn > cr.tail_pn) return 0;
  if (cr.tail_pn - pn <= 8) {
    for (u32 p = cr.tail; p;) {
      const PoolMeta m = P.pmeta[p];
      if (m.pn == pn) return p;
      if (m.pn < pn) return 0;
      p = m.prev;
    }
    return 0;
  }
  for (u32 p = cr.head; p;) {
    const PoolMeta m = P.pmeta[p];
    if (m.pn == pn) return p;
    if (m.pn > pn) return 0;
    p = m.next;
  }
  return 0;
}
template <class PL>
RBE_HD bool cold_get(const PL& P, const ColdRef& cr, u64 idx, Ent* out) {
  const u32 p = cold_find(P, cr, idx / kPageEnts);
  if (!p) return false;
  *out = *pool_ent(P, p, (u32)(idx % kPageEnts));
  return true;
}
// Entry idx into the cold log (an eviction, or an entry written straight
// there); false when the pool is exhausted.  Evictions come in index order, so
// the common case is the tail page or a new one after it.
template <class PL, class PA>
RBE_HD bool cold_put(const PL& P, const PA& C, ColdRef& cr, u64 idx, const Ent& e, u32 par) {
  const u64 pn = idx / kPageEnts;
  u32 p = 0;
  if (cr.tail && pn == cr.tail_pn) {
    p = cr.tail;
  } else if (!cr.tail || pn > cr.tail_pn) {
    p = pool_alloc(P, C, par);
    if (!p) return false;
    PoolMeta m;
    m.pn = pn;
    m.prev = cr.tail;
    m.next = 0;
    P.pmeta[p] = m;
    RBE_AUDIT(AS_COLD_META, &P.pmeta[p], sizeof(PoolMeta) + (cr.tail ? 4 : 0));
    if (cr.tail) P.pmeta[cr.tail].next = p;
    else cr.head = p;
    cr.tail = p;
    cr.tail_pn = pn;
  } else {
    p = cold_find(P, cr, pn);
    if (!p) {  // below the tail and missing: a page inserted in order
      p = pool_alloc(P, C, par);
      if (!p) return false;
      u32 succ = cr.head;
      while (succ && P.pmeta[succ].pn < pn) succ = P.pmeta[succ].next;
      const u32 pred = succ ? P.pmeta[succ].prev : cr.tail;
      PoolMeta m;
      m.pn = pn;
      m.prev = pred;
      m.next = succ;
      P.pmeta[p] = m;
      if (succ) P.pmeta[succ].prev = p;
      if (pred) P.pmeta[pred].next = p;
      else cr.head = p;
    }
  }
  *pool_ent(P, p, (u32)(idx % kPageEnts)) = e;
  RBE_AUDIT(AS_COLD_ENT, pool_ent(P, p, (u32)(idx % kPageEnts)), sizeof(Ent));
  return true;
}
// Releases every page whose entries all lie at or below `upto` (LogDB.Compact
// to a marker; ~0 releases the whole chain)
template <class PL>
RBE_HD void cold_release(const PL& P, ColdRef& cr, u64 upto, u32 par) {
  while (cr.head) {
    const PoolMeta m = P.pmeta[cr.head];
    if (upto != ~0ull && (m.pn + 1) * kPageEnts - 1 > upto) break;
    pool_free(P, par, cr.head);
    cr.head = m.next;
    if (m.next) {
      P.pmeta[m.next].prev = 0;
    } else {
      cr.tail = 0;
      cr.tail_pn = 0;
    }
  }
}

// Log entry idx of replica r whose log ends at `last` (ring window [last -
// ring + 1, last], the cold log below), for code outside a Lane (host-driven
// commits, the payload-heap low mark, the host getters' gather kernel);
// false when it is in neither
RBE_HD bool log_ent_at(const Planes& P, const Params& C, u64 r, u64 last, u64 idx, Ent* out) {
  if (idx == 0 || idx > last) return false;
  if (last - idx < C.ring) {
    const u64 s = (idx & (u64)(C.ring - 1)) * C.n_rep + r;
    const Body b = P.pay_ring[s];
    out->term = P.term_ring[s];
    out->type = b.type;
    out->len = b.len;
    out->lo = b.lo;
    out->hi = b.hi;
    return true;
  }
  return cold_get(P, P.cold[r], idx, out);
}

// ---------------------------------------------------------------- round spill heap
// `bytes` of the round spill heap of parity `par`: its first 16-B granule, or
// ~0 when the heap is exhausted.  With rep_world > 1 (rbe_xchg.h) each rank
// allocates in its own 1/rep_world share, so the exchange can scatter a remote
// sender's spilled lists and entries at the granules the sender chose.
template <class PA>
RBE_HD u64 spill_share(const PA& C) {
  return C.rep_world > 1 ? C.spill_units / C.rep_world : C.spill_units;
}
template <class PL, class PA>
RBE_HD u64 spill_alloc(const PL& P, const PA& C, u32 par, u64 bytes) {
  const u64 n = (bytes + 15) / 16;
  const u64 share = spill_share(C);
  const u64 at = sp_atomic_add_u64(&P.sctl->used[par], n);
  if (at + n > share) {
    sp_atomic_or_u32(&P.sctl->oom, 2u << par);
    return ~0ull;
  }
  sp_atomic_max_u64(&P.sctl->peak[par], at + n);
  return (C.rep_world > 1 ? share * C.rep_rank : 0) + at;
}
template <class T, class PL>
RBE_HD T* spill_at(const PL& P, u32 par, u64 granule) {
  return (T*)(P.spill[par] + granule * 16);
}
// The round of parity `par` starts: the next round's heap (the other parity,
// whose contents the coming round reads as its inbox) starts empty once this
// round's readers are done; called by one thread of the round's first kernel
RBE_HD void spill_clear_next(const Planes& P, u32 par) { P.sctl->used[par ^ 1u] = 0; }

// ---------------------------------------------------------------- message lists
// count word bits (CntRow::w): A | B << 7 | kCntSpill | quiesce << 15
static constexpr u32 kCntSpill = 0x4000u;
static constexpr u32 kCntQ = 0x8000u;
// a spilled list's count word (saturated counts: every fast step declines it)
static constexpr u32 kCntSpilled = 0x7Fu | (0x7Fu << 7) | kCntSpill;
// message type of the record a spilled list leaves in its plane slot 0
// (hint = the list's granule in the spill heap, pad1 = its capacity,
// log_index / commit = its A / B counts), and of a stash chunk's link slot
static constexpr u8 M_SpillRef = 0xFE;
// Msg::pad0 of a message whose entries are in the round spill heap: ent_off is
// their first granule, pad1 their count (n_ent is min(count, 0xFFFF))
static constexpr u16 kMsgXEnt = 0x8000u;

RBE_HD u32 msg_nent(const Msg& m) { return (m.pad0 & kMsgXEnt) ? m.pad1 : (u32)m.n_ent; }
// the entries of message m, sent by replica rs in a round of parity par
RBE_HD const Ent* msg_ents(const Planes& P, const Params& C, u32 par, u64 rs, const Msg& m) {
  if (m.pad0 & kMsgXEnt) return spill_at<const Ent>(P, par, m.ent_off);
  return &P.arena[par][rs * C.ecap + m.ent_off];
}

// One (sender, destination) message list of round parity `par` as its readers
// see it: A (Replicate) messages in order at the front, then B from the back.
struct ListView {
  const Msg* base;
  u32 cap, na, nb;
  RBE_HD u32 n() const { return na + nb; }
  RBE_HD const Msg& at(u32 i) const { return base[i < na ? i : cap - 1u - (i - na)]; }
};
// `li` = (sender replica) * n + destination slot, `w` its count word
RBE_HD ListView list_view(const Planes& P, const Params& C, u32 par, u64 li, u32 w) {
  ListView v;
  const Msg* pl = &P.msgs[par][li * C.maxm];
  if (!(w & kCntSpill)) {
    v.base = pl;
    v.cap = C.maxm;
    v.na = w & 0x7Fu;
    v.nb = (w >> 7) & 0x7Fu;
  } else {
    const Msg h = pl[0];
    v.base = spill_at<const Msg>(P, par, h.hint);
    v.cap = h.pad1;
    v.na = (u32)h.log_index;
    v.nb = (u32)h.commit;
  }
  return v;
}

RBE_HD u32 list_len(const Planes& P, const Params& C, u32 par, u64 li, u32 w) {
  if (!(w & kCntSpill)) return (w & 0x7Fu) + ((w >> 7) & 0x7Fu);
  const Msg& h = P.msgs[par][li * C.maxm];
  return (u32)h.log_index + (u32)h.commit;
}

// A sender's messages past its full plane lists in one step, in emission
// order, in chunks of the round spill heap (the last slot of a full chunk
// links the next); outbox_relocate moves them into whole spilled lists at the
// step's end.
static constexpr u32 kStashChunk = 32;
struct OutStash {
  u64 head, cur;  // granules of the first and the current chunk
  u32 n;          // messages stashed
  u32 mask;       // destination slots with a stashed message
};
RBE_HD void stash_init(OutStash& s) {
  s.head = s.cur = 0;
  s.n = s.mask = 0;
}
template <class PL, class PA>
RBE_HD bool stash_put(const PL& P, const PA& C, u32 par, OutStash& s, const Msg& m) {
  const u32 i = s.n % (kStashChunk - 1u);
  if (i == 0) {
    const u64 g = spill_alloc(P, C, par, kStashChunk * sizeof(Msg));
    if (g == ~0ull) return false;
    if (s.n == 0) {
      s.head = g;
    } else {
      Msg link = {};
      link.type = M_SpillRef;
      link.hint = g;
      spill_at<Msg>(P, par, s.cur)[kStashChunk - 1u] = link;
    }
    s.cur = g;
  }
  spill_at<Msg>(P, par, s.cur)[i] = m;
  s.n++;
  s.mask |= 1u << (m.to - 1u);
  return true;
}
// The stashed messages in emission order: f(msg)
template <class PL, class F>
RBE_HD void stash_each(const PL& P, u32 par, const OutStash& s, F&& f) {
  u64 c = s.head;
  for (u32 t = 0; t < s.n; t++) {
    const u32 i = t % (kStashChunk - 1u);
    if (t > 0 && i == 0) c = spill_at<const Msg>(P, par, c)[kStashChunk - 1u].hint;
    f(spill_at<const Msg>(P, par, c)[i]);
  }
}
// The step's end: every list with stashed messages moves whole into the spill
// heap (plane part first, A in order at the front, B from the back).  The n
// count words of sender replica rs are the 16-bit fields of w_lo (destinations
// 0-3) and w_hi (4-7), rewritten for the moved lists (packed, so no register
// array is indexed at run time).  Returns F_NOMEM when the heap cannot take a
// list (it keeps its plane part).
template <class PL, class PA>
RBE_HD u32 outbox_relocate(const PL& P, const PA& C, u32 par, u64 rs, u32 n,
                           const OutStash& s, u64& w_lo, u64& w_hi) {
  u32 fault = 0;
  for (u32 d = 0; d < n; d++) {
    if (!((s.mask >> d) & 1u)) continue;
    // (values selected, never a reference to one of the two words: a
    // selected reference puts both in scratch memory)
    const bool lo = d < 4;
    const u32 sh = 16 * (d & 3u);
    const u32 w = (u32)(((lo ? w_lo : w_hi) >> sh) & 0xFFFFu);
    const u32 a0 = w & 0x7Fu, b0 = (w >> 7) & 0x7Fu;
    u32 na = a0, nb = b0;
    stash_each(P, par, s, [&](const Msg& m) {
      if (m.to == d + 1u) (m.type == M_Replicate ? na : nb)++;
    });
    const u32 cap = na + nb;
    const u64 gb = spill_alloc(P, C, par, (u64)cap * sizeof(Msg));
    if (gb == ~0ull) {
      fault |= F_NOMEM;
      continue;
    }
    Msg* blk = spill_at<Msg>(P, par, gb);
    Msg* pl = &P.msgs[par][(rs * n + d) * C.maxm];
    for (u32 i = 0; i < a0; i++) blk[i] = pl[i];
    for (u32 j = 0; j < b0; j++) blk[cap - 1u - j] = pl[C.maxm - 1u - j];
    u32 ia = a0, ib = b0;
    stash_each(P, par, s, [&](const Msg& m) {
      if (m.to != d + 1u) return;
      if (m.type == M_Replicate) blk[ia++] = m;
      else blk[cap - 1u - ib++] = m;
    });
    Msg h = {};
    h.type = M_SpillRef;
    h.hint = gb;
    h.pad1 = cap;
    h.log_index = na;
    h.commit = nb;
    pl[0] = h;
    const u64 keep = ~(0xFFFFull << sh), nw = (u64)((w & kCntQ) | kCntSpilled) << sh;
    w_lo = lo ? (w_lo & keep) | nw : w_lo;
    w_hi = lo ? w_hi : (w_hi & keep) | nw;
  }
  return fault;
}

// ---------------------------------------------------------------- output lists
// The ReadyToReads / dropped ReadIndexes of replica r's last step (n of them,
// written in a round of parity par): the plane list, or the spill heap block
// its slot 0 names (granule in index / low, when n exceeds the plane's capacity)
RBE_HD const RTR* rtr_list(const Planes& P, const Params& C, u64 r, u32 n, u32 par) {
  const RTR* pl = &P.rtr[r * C.rtr_cap];
  return n <= C.rtr_cap ? pl : spill_at<const RTR>(P, par, pl[0].index);
}
RBE_HD const DropRI* dri_list(const Planes& P, const Params& C, u64 r, u32 n, u32 par) {
  const DropRI* pl = &P.dri[r * C.dri_cap];
  return n <= C.dri_cap ? pl : spill_at<const DropRI>(P, par, pl[0].low);
}

// ---------------------------------------------------------------- readIndex queue
// Core::rq_count of a queue that moved into pool pages; the plane ring's slot 0
// then holds the queue's descriptor: low = head page | tail page << 32, high =
// offset in the head page | length << 32
static constexpr u8 kRqExt = 0xFF;
struct RqExt {
  u32 head, tail, off, n;
};
RBE_HD RqExt rq_ext_load(const Planes& P, const Params& C, u64 r) {
  const ReadReq d = P.rq[r * C.rq_cap];
  RqExt x;
  x.head = (u32)d.low;
  x.tail = (u32)(d.low >> 32);
  x.off = (u32)d.high;
  x.n = (u32)(d.high >> 32);
  return x;
}
RBE_HD void rq_ext_store(const Planes& P, const Params& C, u64 r, const RqExt& x) {
  ReadReq d = {};
  d.low = (u64)x.head | ((u64)x.tail << 32);
  d.high = (u64)x.off | ((u64)x.n << 32);
  P.rq[r * C.rq_cap] = d;
}
// entry i of a queue in pool pages
RBE_HD ReadReq* rq_ext_at(const Planes& P, const RqExt& x, u32 i) {
  u32 pos = x.off + i, p = x.head;
  while (pos >= kPageEnts) {
    p = P.pmeta[p].next;
    pos -= kPageEnts;
  }
  return (ReadReq*)pool_ent(P, p, pos);
}
// entry i (< length) of replica r's readIndex queue, wherever it lives
RBE_HD const ReadReq* rq_entry(const Planes& P, const Params& C, u64 r, const Core& c, u32 i) {
  if (c.rq_count == kRqExt) return rq_ext_at(P, rq_ext_load(P, C, r), i);
  u32 x = (u32)c.rq_head + i;
  if (x >= C.rq_cap) x -= C.rq_cap;
  return &P.rq[r * C.rq_cap + x];
}
RBE_HD u32 rq_length(const Planes& P, const Params& C, u64 r, const Core& c) {
  return c.rq_count == kRqExt ? rq_ext_load(P, C, r).n : (u32)c.rq_count;
}
template <class PL>
RBE_HD void rq_ext_free(const PL& P, const RqExt& x, u32 par) {
  for (u32 p = x.head; p;) {
    const u32 nx = p == x.tail ? 0u : P.pmeta[p].next;
    pool_free(P, par, p);
    p = nx;
  }
}

// ---------------------------------------------------------------- out of line
// The general step (Lane, rbe_step.h) calls the tiers through these `_ol`
// wrappers: each walk and allocation is compiled once there, as a real call
// (RBE_COLD), instead of being inlined into every log read and send of the
// handler table.  Inlined, the tiers doubled k_full_list's code and put it
// into scratch spills (C3 k_full_list 238 → 208 µs outlined).  The calls take
// values only (the tier pointers in a SpillRef, a ColdRef / OutStash / Msg by
// value, results returned by value), so no caller object has its address
// taken; inside, the templates above run on SpillP / SpillC, which hold just
// the tiers' fields.  The fast steps keep the inline forms: a call in their
// kernel costs more than the code it saves (measured: C4 k_fast_both +50%).
#if defined(__HIPCC__) || defined(__HIP__)
#define RBE_COLD __host__ __device__ inline __attribute__((noinline))
#else
#define RBE_COLD inline __attribute__((noinline))
#endif
// the tiers' fields of Planes / Params, for the templates above
struct SpillP {
  Ent* pool;
  PoolMeta* pmeta;
  SpillCtl* sctl;
  u8* spill[2];
  Msg* msgs[2];
};
struct SpillC {
  u64 spill_units;
  u32 pool_pages, rep_world, rep_rank, maxm;
};
struct SpillRef {
  SpillP P;
  SpillC C;
};
RBE_HD SpillRef spill_ref(const Planes& P, const Params& C) {
  SpillRef s;
  s.P.pool = P.pool;
  s.P.pmeta = P.pmeta;
  s.P.sctl = P.sctl;
  s.P.spill[0] = P.spill[0];
  s.P.spill[1] = P.spill[1];
  s.P.msgs[0] = P.msgs[0];
  s.P.msgs[1] = P.msgs[1];
  s.C.spill_units = C.spill_units;
  s.C.pool_pages = C.pool_pages;
  s.C.rep_world = C.rep_world;
  s.C.rep_rank = C.rep_rank;
  s.C.maxm = C.maxm;
  return s;
}
struct ColdGet {
  Ent e;
  u32 ok;
};
RBE_COLD ColdGet cold_get_o(SpillRef s, ColdRef cr, u64 idx) {
  ColdGet g;
  g.ok = cold_get(s.P, cr, idx, &g.e) ? 1u : 0u;
  return g;
}
struct ColdPut {
  ColdRef cr;
  u32 ok;
};
RBE_COLD ColdPut cold_put_o(SpillRef s, ColdRef cr, u64 idx, Ent e, u32 par) {
  ColdPut r;
  r.ok = cold_put(s.P, s.C, cr, idx, e, par) ? 1u : 0u;
  r.cr = cr;
  return r;
}
RBE_COLD ColdRef cold_release_o(SpillRef s, ColdRef cr, u64 upto, u32 par) {
  cold_release(s.P, cr, upto, par);
  return cr;
}
RBE_COLD u64 spill_alloc_o(SpillRef s, u32 par, u64 bytes) {
  return spill_alloc(s.P, s.C, par, bytes);
}
RBE_COLD u32 pool_alloc_o(SpillRef s, u32 par) {
  return pool_alloc(s.P, s.C, par);
}
RBE_COLD void pool_free_o(SpillRef s, u32 par, u32 page) {
  pool_free(s.P, par, page);
}
RBE_COLD void rq_ext_free_o(SpillRef s, RqExt q, u32 par) {
  rq_ext_free(s.P, q, par);
}
struct StashPut {
  OutStash st;
  u32 ok;
};
RBE_COLD StashPut stash_put_o(SpillRef s, u32 par, OutStash st, Msg m) {
  StashPut r;
  r.ok = stash_put(s.P, s.C, par, st, m) ? 1u : 0u;
  r.st = st;
  return r;
}
struct Reloc {
  u64 lo, hi;
  u32 fault;
};
RBE_COLD Reloc outbox_relocate_o(SpillRef s, u32 par, u64 rs, u32 n, OutStash st, u64 w_lo,
                                 u64 w_hi) {
  Reloc r;
  r.fault = outbox_relocate(s.P, s.C, par, rs, n, st, w_lo, w_hi);
  r.lo = w_lo;
  r.hi = w_hi;
  return r;
}
// the call sites' forms (the inline functions' signatures)
RBE_HD bool cold_get_ol(const Planes& P, const Params& C, const ColdRef& cr, u64 idx, Ent* out) {
  const ColdGet g = cold_get_o(spill_ref(P, C), cr, idx);
  *out = g.e;
  return g.ok != 0;
}
RBE_HD bool cold_put_ol(const Planes& P, const Params& C, ColdRef& cr, u64 idx, const Ent& e,
                        u32 par) {
  if (cr.tail && idx / kPageEnts == cr.tail_pn) {  // the tail page: inline
    P.pool[(u64)cr.tail * kPageEnts + idx % kPageEnts] = e;
    return true;
  }
  const ColdPut r = cold_put_o(spill_ref(P, C), cr, idx, e, par);
  cr = r.cr;
  return r.ok != 0;
}
RBE_HD void cold_release_ol(const Planes& P, const Params& C, ColdRef& cr, u64 upto, u32 par) {
  cr = cold_release_o(spill_ref(P, C), cr, upto, par);
}
RBE_HD u64 spill_alloc_ol(const Planes& P, const Params& C, u32 par, u64 bytes) {
  return spill_alloc_o(spill_ref(P, C), par, bytes);
}
RBE_HD u32 pool_alloc_ol(const Planes& P, const Params& C, u32 par) {
  return pool_alloc_o(spill_ref(P, C), par);
}
RBE_HD void pool_free_ol(const Planes& P, const Params& C, u32 par, u32 page) {
  pool_free_o(spill_ref(P, C), par, page);
}
RBE_HD void rq_ext_free_ol(const Planes& P, const Params& C, const RqExt& q, u32 par) {
  rq_ext_free_o(spill_ref(P, C), q, par);
}
RBE_HD bool stash_put_ol(const Planes& P, const Params& C, u32 par, OutStash& st, const Msg& m) {
  const StashPut r = stash_put_o(spill_ref(P, C), par, st, m);
  st = r.st;
  return r.ok != 0;
}
RBE_HD u32 outbox_relocate_ol(const Planes& P, const Params& C, u32 par, u64 rs, u32 n,
                              const OutStash& st, u64& w_lo, u64& w_hi) {
  const Reloc r = outbox_relocate_o(spill_ref(P, C), par, rs, n, st, w_lo, w_hi);
  w_lo = r.lo;
  w_hi = r.hi;
  return r.fault;
}

}  // namespace rbe
