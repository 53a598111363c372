// rbe_snap.h — byte layout of a group-range snapshot (rbe_export_groups /
// rbe_import_groups), shared by the HIP engine and the host build of the step.
//
// A snapshot is the complete protocol state of groups [first, first + count)
// between two rounds: every replica's raft/remote/readIndex/log-window rows and
// the group's in-flight network planes (count words, messages, Replicate
// entries of both parities), so that stepping an imported range produces the
// same rounds the exporting engine would have.  It is the state a dragonboat
// node keeps across a restart in *raft.Peer + LogDB (peer.go:64-87 Launch on an
// existing log; raft.go:283-330 loadState), restated for the SoA planes, and
// the hand-off a host slow path uses to run a rare handler on one group.
//
// Every plane is a set of rows whose per-group slice is contiguous: replica-
// and group-indexed planes are one row, the double-buffered network planes two
// rows (parity 0, 1), and the term/payload rings `ring` rows of pitch n_rep.
// A group range is therefore one 2-D copy per plane (hipMemcpy2DAsync on the
// device, a row loop on the host), and the snapshot body is the planes in the
// order below, rows in order, each row `count * group_bytes` bytes.
#pragma once

#include <cstring>

#include "rbe_step.h"

namespace rbe {

static constexpr u64 kSnapMagic = 0x31504E5345425255ull;  // "URBESNP1"
static constexpr int kSnapPlanes = 23;

struct SnapHeader {
  u64 magic;
  u32 abi, n, ring, rq_cap, maxm, ecap, rtr_cap, dri_cap;
  u32 round, hdr_bytes;
  u64 first, count;
  u64 body_bytes;
  u64 behavior;   // snap_behavior_hash of the writing configuration
  u64 tclk;       // ticks before `round` (Clk::tclk)
  u64 log_bytes;  // the log section after the planes (snap_log_*)
};
static_assert(sizeof(SnapHeader) == 96, "snapshot header layout");
// where the log section starts (16-B aligned after the planes)
inline u64 snap_log_at(u64 body_bytes) { return (sizeof(SnapHeader) + body_bytes + 15) & ~15ull; }

struct SnapPlane {
  u8* base;          // plane start
  u64 rows;          // 1, 2 (parities) or ring
  u64 pitch;         // bytes between rows
  u64 group_bytes;   // bytes of one group within a row
};

// The planes of P in snapshot order.
inline void snap_planes(const Planes& P, const Params& C, SnapPlane* out) {
  const u64 N = C.n, G = C.n_groups, R = C.n_rep;
  int i = 0;
  auto add = [&](const void* base, u64 rows, u64 pitch, u64 gb) {
    out[i++] = SnapPlane{(u8*)base, rows, pitch, gb};
  };
  add(P.hot, 1, R * sizeof(Hot), N * sizeof(Hot));
  add(P.core, 1, R * sizeof(Core), N * sizeof(Core));
  add(P.rem, 1, R * N * sizeof(RemoteMN), N * N * sizeof(RemoteMN));
  add(P.rem_st, 1, R * N, N * N);
  add(P.rq, 1, R * C.rq_cap * sizeof(ReadReq), N * C.rq_cap * sizeof(ReadReq));
  add(P.term_ring, C.ring, R * sizeof(u64), N * sizeof(u64));
  add(P.pay_ring, C.ring, R * sizeof(Body), N * sizeof(Body));
  // the network planes: parity 1 starts right after parity 0 (rbe_create)
  add(P.cnt[0], 2, R * sizeof(CntRow), N * sizeof(CntRow));
  add(P.msgs[0], 2, G * N * N * C.maxm * sizeof(Msg), N * N * C.maxm * sizeof(Msg));
  add(P.arena[0], 2, R * C.ecap * sizeof(Ent), N * C.ecap * sizeof(Ent));
  add(P.iso_mask, 1, G, 1);
  add(P.iso_until, 1, G * sizeof(u32), sizeof(u32));
  add(P.upd, 1, R * sizeof(Upd), N * sizeof(Upd));
  add(P.rtr, 1, R * C.rtr_cap * sizeof(RTR), N * C.rtr_cap * sizeof(RTR));
  add(P.dri, 1, R * C.dri_cap * sizeof(DropRI), N * C.dri_cap * sizeof(DropRI));
  add(P.ext, 1, R * sizeof(ExtIn), N * sizeof(ExtIn));
  add(P.idle, 1, R, N);
  add(P.applied, 1, R * sizeof(u64), N * sizeof(u64));
  if (C.snapshot_entries) {  // node snapshot / compaction state, remote snapshotIndex
    add(P.snp, 1, R * sizeof(SnapSt), N * sizeof(SnapSt));
    add(P.rem_snap, 1, R * N * sizeof(u64), N * N * sizeof(u64));
  }
  if (C.ext_commit || C.rl_max) add(P.imark, 1, R * sizeof(u64), N * sizeof(u64));  // inMemory markers
  if (C.rl_max) add(P.rl, 1, R * sizeof(RlSt), N * sizeof(RlSt));  // rate limiters
  if (C.membership) add(P.roles, 1, R * sizeof(u16), N * sizeof(u16));  // observers / witnesses
  // the per-replica fault words live in Hot/Core/Upd; nothing else is carried
  while (i < kSnapPlanes) out[i++] = SnapPlane{nullptr, 0, 0, 0};
}

inline u64 snap_body_bytes(const Planes& P, const Params& C, u64 count) {
  SnapPlane pl[kSnapPlanes];
  snap_planes(P, C, pl);
  u64 b = 0;
  for (int i = 0; i < kSnapPlanes && pl[i].rows; i++) b += pl[i].rows * pl[i].group_bytes * count;
  return b;
}

// Hash of every Params field that changes how a replica steps (timeouts,
// quorum check, quiesce, the injected PRNG seed, cluster-id mapping, entry
// size limit, workload, fault schedule, replica placement): a snapshot only
// resumes bit-exact under the configuration that wrote it, so import rejects
// a mismatch instead of diverging silently (SnapHeader::behavior).
inline u64 snap_behavior_hash(const Params& C) {
  const u64 f[] = {C.election_rtt, C.heartbeat_rtt, C.check_quorum, C.quiesce, C.seed,
                   C.cid_base, C.cid_stride, C.max_entry_size, C.wl_enabled, C.wl_start_round,
                   C.wl_stop_round, C.wl_active_mod, C.wl_read_permille, C.ext_inputs,
                   C.iso_period, C.iso_len, C.iso_mod, C.rep_world, C.rep_rank,
                   C.snapshot_entries, C.compaction_overhead, C.heap_bytes, C.ext_apply,
                   C.xfer_period, C.xfer_mod, C.ext_commit, C.membership, C.cc_period,
                   C.cc_mod, C.rl_max, C.n_voters, C.obs_slots, C.wit_slots};
  u64 h = 0x243F6A8885A308D3ull;
  for (u64 x : f) {
    h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
  }
  return h;
}

inline void snap_fill_header(const Params& C, u32 abi, u32 round, u32 tclk, u64 first, u64 count,
                             u64 body, SnapHeader* h) {
  *h = SnapHeader{};
  h->magic = kSnapMagic;
  h->abi = abi;
  h->n = C.n;
  h->ring = C.ring;
  h->rq_cap = C.rq_cap;
  h->maxm = C.maxm;
  h->ecap = C.ecap;
  h->rtr_cap = C.rtr_cap;
  h->dri_cap = C.dri_cap;
  h->round = round;
  h->hdr_bytes = sizeof(SnapHeader);
  h->first = first;
  h->count = count;
  h->body_bytes = body;
  h->behavior = snap_behavior_hash(C);
  h->tclk = tclk;
}

// 0 if the header describes a range this geometry can take, else RBE_E_INVALID.
inline int snap_check_header(const Params& C, u32 abi, const SnapHeader* h, u64 buf_bytes) {
  if (buf_bytes < sizeof(SnapHeader) || h->magic != kSnapMagic || h->abi != abi ||
      h->hdr_bytes != sizeof(SnapHeader))
    return -1;
  if (h->n != C.n || h->ring != C.ring || h->rq_cap != C.rq_cap || h->maxm != C.maxm ||
      h->ecap != C.ecap || h->rtr_cap != C.rtr_cap || h->dri_cap != C.dri_cap)
    return -1;
  if (h->behavior != snap_behavior_hash(C)) return -1;
  if (h->count == 0 || h->first >= C.n_groups || h->count > C.n_groups - h->first) return -1;
  if (buf_bytes < snap_log_at(h->body_bytes) + h->log_bytes) return -1;
  return 0;
}

// ---------------------------------------------------------------- the log section
// After the planes, 16-B aligned (snap_log_at): the spill-tier state that
// lives across rounds (rbe_spill.h), replica by replica of the range, each a
// SnapLogRec followed by its cold log's pages whole (SnapPage, in chain
// order) and then, for a readIndex queue that moved into pool pages
// (Core::rq_count == kRqExt), its requests in order.  The round spill heap
// is not carried: an export whose next round would read a spilled list or
// spilled entries, or whose last step's ReadyToReads / dropped ReadIndexes
// went past their planes, is refused (snap_round_spilled).
struct alignas(16) SnapLogRec {
  u32 n_pages, n_rq;
  u64 pad;
};
struct alignas(16) SnapPage {
  u64 pn, pad;
  Ent e[kPageEnts];
};

// The log section of replicas [r0, r0 + nr): its size, written at `out`
// unless null.  The accessor reads the source engine: cold(r) / core(r) /
// rq(r) (the queue descriptor) rows, meta(p) a page's PoolMeta, page(p, out)
// its kPageEnts entries.
template <class SRC>
u64 snap_log_write(const Params& C, u64 r0, u64 nr, SRC& s, u8* out) {
  u64 at = 0;
  for (u64 r = r0; r < r0 + nr; r++) {
    const ColdRef cr = s.cold(r);
    const Core c = s.core(r);
    SnapLogRec h = {};
    const u64 hat = at;
    at += sizeof(SnapLogRec);
    for (u32 p = cr.head; p;) {
      const PoolMeta m = s.meta(p);
      if (out) {
        SnapPage* sp = (SnapPage*)(out + at);
        sp->pn = m.pn;
        sp->pad = 0;
        s.page(p, sp->e);
      }
      at += sizeof(SnapPage);
      h.n_pages++;
      p = p == cr.tail ? 0u : m.next;
    }
    if (c.rq_count == kRqExt) {
      const RqExt x = s.rq(r);
      h.n_rq = x.n;
      u32 p = x.head, pos = x.off;
      Ent pg[kPageEnts];
      bool have = false;
      for (u32 i = 0; i < x.n; i++, pos++) {
        if (pos == kPageEnts) {
          p = s.meta(p).next;
          pos = 0;
          have = false;
        }
        if (out) {
          if (!have) s.page(p, pg);
          have = true;
          *(ReadReq*)(out + at) = *(const ReadReq*)&pg[pos];
        }
        at += sizeof(ReadReq);
      }
    }
    if (out) *(SnapLogRec*)(out + hat) = h;
  }
  (void)C;
  return at;
}

// A snapshot's log section checked against its planes before anything is
// imported: the offset of each of its nr replica records into rec_off; -1
// when a record runs past the section, or a replica's readIndex queue is in
// pool pages (Core::rq_count == kRqExt in the snapshot's Core rows) without
// requests in its record, or the other way round.
inline int snap_log_index(const Params& C, const u8* snap, u64 nr, u64* rec_off) {
  SnapHeader hd;
  memcpy(&hd, snap, sizeof(hd));
  const SnapHeader* h = &hd;
  const u8* sec = snap + snap_log_at(h->body_bytes);
  // the Core rows follow the Hot rows (snap_planes order)
  const u8* core = snap + sizeof(SnapHeader) + nr * sizeof(Hot);
  u64 at = 0;
  for (u64 i = 0; i < nr; i++) {
    if (at + sizeof(SnapLogRec) > h->log_bytes) return -1;
    SnapLogRec rec;
    memcpy(&rec, sec + at, sizeof(rec));
    Core c;
    memcpy(&c, core + i * sizeof(Core), sizeof(Core));
    if ((c.rq_count == kRqExt) != (rec.n_rq != 0)) return -1;
    const u64 sz = sizeof(SnapLogRec) + (u64)rec.n_pages * sizeof(SnapPage) +
                   (u64)rec.n_rq * sizeof(ReadReq);
    if (sz > h->log_bytes - at) return -1;
    rec_off[i] = at;
    at += sz;
  }
  (void)C;
  return at == h->log_bytes ? 0 : -1;
}

// Replica r's record of a log section (16-B aligned, at `rec`): rebuilds its
// cold log chain and its pool-page readIndex queue in this engine's pool
// (page allocation as in a round of parity `par`), after the planes were
// imported and r's old chains released (spill_replica_release).  Returns the
// record's size, or 0 when the pool is exhausted (*fault = F_NOMEM).
RBE_HD u64 snap_log_rebuild(const Planes& P, const Params& C, u64 r, const u8* rec, u32 par,
                            u32* fault) {
  const SnapLogRec h = *(const SnapLogRec*)rec;
  u64 at = sizeof(SnapLogRec);
  ColdRef cr;
  cr.head = cr.tail = 0;
  cr.tail_pn = 0;
  for (u32 i = 0; i < h.n_pages; i++, at += sizeof(SnapPage)) {
    const SnapPage* sp = (const SnapPage*)(rec + at);
    const u32 p = pool_alloc(P, C, par);
    if (!p) {
      P.cold[r] = cr;
      *fault = F_NOMEM;
      return 0;
    }
    PoolMeta m;
    m.pn = sp->pn;
    m.prev = cr.tail;
    m.next = 0;
    P.pmeta[p] = m;
    if (cr.tail) P.pmeta[cr.tail].next = p;
    else cr.head = p;
    cr.tail = p;
    cr.tail_pn = sp->pn;
    for (u32 j = 0; j < kPageEnts; j++) *pool_ent(P, p, j) = sp->e[j];
  }
  P.cold[r] = cr;
  if (h.n_rq) {
    RqExt x;
    x.head = x.tail = 0;
    x.off = 0;
    x.n = 0;
    for (u32 i = 0; i < h.n_rq; i++, at += sizeof(ReadReq)) {
      if (i % kPageEnts == 0) {
        const u32 p = pool_alloc(P, C, par);
        if (!p) {
          if (x.head) rq_ext_free(P, x, par);
          P.core[r].rq_count = 0;
          P.core[r].rq_head = 0;
          *fault = F_NOMEM;
          return 0;
        }
        P.pmeta[p].next = 0;
        if (x.tail) P.pmeta[x.tail].next = p;
        else x.head = p;
        x.tail = p;
      }
      *(ReadReq*)pool_ent(P, x.tail, i % kPageEnts) = *(const ReadReq*)(rec + at);
      x.n++;
    }
    rq_ext_store(P, C, r, x);
  }
  return at;
}

// Whether replica r's last step left state in the round spill heap that the
// snapshot cannot carry: a list the next round reads (count word with
// kCntSpill, stamp `round`), a message of those lists with entries in the
// heap, ReadyToReads / dropped ReadIndexes past the planes.  w[d] = r's count
// words for the next round (row_word of its outbox header of parity
// (round - 1) & 1), `lists` its N * maxm slots, `u` its Upd.
inline bool snap_round_spilled(const Params& C, const u32* w_in, const Msg* lists, const Upd& u) {
  if (u.n_rtr > C.rtr_cap || u.n_drop_ri > C.dri_cap) return true;
  for (u32 d = 0; d < C.n; d++) {
    const u32 w = w_in[d];
    if (w & kCntSpill) return true;
    const u32 na = w & 0x7Fu, nb = (w >> 7) & 0x7Fu;
    for (u32 i = 0; i < na + nb; i++) {
      const Msg& m = lists[d * C.maxm + (i < na ? i : C.maxm - 1u - (i - na))];
      if (m.pad0 & kMsgXEnt) return true;
    }
  }
  return false;
}

}  // namespace rbe
