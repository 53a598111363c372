// rbe_host.h — host-side staging of the node-layer inputs (rbe_push_*,
// rbe_request_leader_transfer, rbe_report_*, rbe_notify_applied), shared by
// the HIP engine and the test-only host build of the step.
//
// In dragonboat the node layer hands these to *raft.Peer one call at a time
// under raftMu (node.go:1030-1067 handleEvents → peer.go:106-315).  Here a call
// stages a whole batch host-side: it is checked completely before anything is
// staged (a bad replica or argument stages nothing), and the staged records go
// to the device in one copy plus one scatter launch when the next step starts.
// A replica takes one proposal batch, one ReadIndex ctx and one leader-transfer
// request per step, the way the node batches them (incomingProposals.get,
// node.go:1091-1106; batchedReadIndex, 1379-1382; pendingLeaderTransfer,
// 1069-1075): a second one is RBE_E_STATE instead of silently replacing the
// first.
#pragma once
#include <algorithm>
#include <cstring>
#include <functional>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/rbe.h"
#include "rbe_step.h"
#include "rbe_types.h"

namespace rbe {

// The group sizes the engine is built for (voting slots per group): every
// kernel and host routine templated on N is instantiated for each.
inline bool valid_n(u32 n) { return n >= 1 && n <= kMaxN; }
// f(std::integral_constant<int, N>()) for the runtime group size n (checked
// by the caller with valid_n; anything else takes N = 1)
template <typename F>
inline auto with_n(u32 n, F&& f) -> decltype(f(std::integral_constant<int, 1>())) {
  switch (n) {
    case 2: return f(std::integral_constant<int, 2>());
    case 3: return f(std::integral_constant<int, 3>());
    case 4: return f(std::integral_constant<int, 4>());
    case 5: return f(std::integral_constant<int, 5>());
    case 6: return f(std::integral_constant<int, 6>());
    case 7: return f(std::integral_constant<int, 7>());
    default: return f(std::integral_constant<int, 1>());
  }
}

// The spill tiers' sizes (rbe_spill.h): cfg.pool_bytes of page pool (0 = 8
// KiB per replica, at least 64 MiB and at most 32 GiB: four pages, 256
// entries of cold log, per replica on average) and cfg.spill_bytes of round
// spill heap per round parity (0 = 128 B per replica, at least 16 MiB, at most
// 4 GiB).  Shared with the test-only host build (tests/soa_cpu).
inline int spill_sizes(const rbe_config* cfg, Params* C) {
  const u64 R = C->n_rep, page = (u64)kPageEnts * sizeof(Ent);
  u64 pb = cfg->pool_bytes;
  if (!pb) pb = std::min(std::max(R * 8192ull, 64ull << 20), 32ull << 30);
  u64 pages = pb / page;
  if (pages < 2 || pages > 0xFFFFFFF0ull) return RBE_E_INVALID;
  C->pool_pages = (u32)pages;
  u64 sb = cfg->spill_bytes;
  const u64 W = C->rep_world > 1 ? C->rep_world : 1;  // (a share per rank: spill_alloc)
  if (!sb) sb = std::min(std::min(std::max(R * 128ull, 16ull << 20), 4ull << 30) * W, 0xFFFFFFF0ull * 16);
  const u64 units = sb / 16;
  if (units / W < 64 || units > 0xFFFFFFF0ull) return RBE_E_INVALID;  // granules are u32 in messages
  C->spill_units = units;
  return RBE_OK;
}

// Fingerprint of a Cmd longer than 16 bytes (Body/Ent lo when the bytes live in
// the payload heap): 64 bits over the zero-padded 8-byte words and the length.
// The trace digest folds it in place of the inline bytes, so the fingerprint
// stands for the payload in parity checks (oracle/harness.cpp restates it).
RBE_HD u64 cmd_fingerprint(const u8* b, u64 len) {
  u64 h = 0x243F6A8885A308D3ull ^ len;
  for (u64 i = 0; i < len; i += 8) {
    u64 w = 0;
    for (u64 j = 0; j < 8 && i + j < len; j++) w |= (u64)b[i + j] << (8 * j);
    h = mix64(h ^ w);
  }
  return mix64(h ^ (len << 1));
}
// Fingerprint of a payload-heap record (ET_HEAP): the Cmd's, extended by the
// session fields {Key, ClientID, SeriesID, RespondedTo} when any is non-zero
// (raft.pb.go:589-598; oracle/harness.cpp entry_fingerprint restates it).
RBE_HD u64 entry_fingerprint(const u64* meta, const u8* cmd, u64 len) {
  u64 h = cmd_fingerprint(cmd, len);
  if (meta[0] | meta[1] | meta[2] | meta[3])
    for (u64 i = 0; i < 4; i++) h = mix64(h ^ meta[i] ^ ((i + 1) << 60));
  return h;
}
// An rbe_entry that needs a heap record: a Cmd longer than 16 bytes, or any
// session field (requests.go:994-997 stamps them on every client proposal)
RBE_HD bool entry_needs_heap(const rbe_entry& e) {
  return e.cmd_len > 16 || (e.key | e.client_id | e.series_id | e.responded_to) != 0;
}
RBE_HD u64 heap_rec_bytes(u64 cmd_len) { return (kHeapHdr + cmd_len + 15) & ~15ull; }

// Payload heap (cfg.heap_bytes): one device byte ring shared by every group.
// An entry with a Cmd longer than 16 bytes or session fields is written there
// once, when it is staged, as a record {Key, ClientID, SeriesID, RespondedTo,
// Cmd}; every replica's log entry refers to it by (fingerprint, absolute
// position) in Body/Ent lo/hi with ET_HEAP in the type: a follower that
// appends the entry copies the reference, never the bytes (the Log Matching
// property makes the entry of an (index, term) the same on every replica).
// The host is the only writer, so positions are assigned here, in push order.
//
// Lifetime.  The heap never laps a record some replica may still need: a push
// that would overwrite one fails with RBE_E_NOMEM instead (the reference keeps
// an entry until it is saved and applied, inmemory.go:116-166, and in LogDB
// after that).  Live = referenced by an entry of some replica's log window
// above its group's low mark min over the group's replicas of min(savedTo,
// processed, applied) — what a replica of the group has not yet saved and
// applied, including entries a lagging follower has not received — or by a
// Propose in flight, or staged / uploaded by the last flush (`batch_lo`).  The
// engine computes the lowest live position on demand (`low_fn`, a device
// reduction), only when a push would cross the cached mark.  Bytes at a
// position older than one lap are still refused to readers (RBE_E_STATE, as
// ErrCompacted) and flagged F_WINDOW if a step ever tries to send them.
struct HostHeap {
  u64 cap = 0;       // bytes (0 = no heap: Cmd is at most 16 bytes, no session fields)
  u64 head = 0;      // next free absolute position
  u64 flushed = 0;   // positions below this are on the device
  u64 batch_lo = 0;  // first position of the last uploaded batch
  u64 round_lo = ~0ull;  // first position written straight to the device since the last
                         // step (rbe_wire_ingest); becomes batch_lo at the next step
  u64 live_lo = 0;   // cached: no live record below it (0 = unknown)
  std::vector<u8> stage;  // bytes of [flushed, head), position flushed at index 0
  // lowest position a live record of the device planes holds (~0 for none)
  std::function<int(u64*)> low_fn;
  // reserve len bytes (16-B aligned, never split across the end of the ring)
  u64 alloc(u64 len) {
    u64 p = head;
    if (p % cap + len > cap) p += cap - p % cap;
    head = p + ((len + 15) & ~15ull);
    return p;
  }
  bool valid(u64 pos, u64 len) const { return cap && pos + len <= head && head <= pos + cap; }
  u64 floor() const { return live_lo < batch_lo ? live_lo : batch_lo; }
  // room for `need` more bytes (alignment and the wrap skip included) without
  // lapping a live record; refreshes the live mark once when the cached one is short
  int room(u64 need) {
    if (need > cap) return RBE_E_NOMEM;
    if (head + need <= floor() + cap) return RBE_OK;
    if (low_fn) {
      u64 lo = ~0ull;
      const int rc = low_fn(&lo);
      if (rc) return rc;
      live_lo = lo < head ? lo : head;
    }
    return head + need <= floor() + cap ? RBE_OK : RBE_E_NOMEM;
  }
  // at a step: the batch uploaded (or written by the device) since the last
  // one stays live through it; the stage is empty
  void settle() {
    batch_lo = flushed < round_lo ? flushed : round_lo;
    round_lo = ~0ull;
    flushed = head;
  }
  // stage one record; returns its position
  u64 put_record(const u64* meta, const u8* cmd, u64 len) {
    const u64 pos = alloc(kHeapHdr + len);
    stage.resize(head - flushed, 0);
    u8* d = stage.data() + (pos - flushed);
    memcpy(d, meta, kHeapHdr);
    if (len) memcpy(d + kHeapHdr, cmd, len);
    return pos;
  }
  // `len` bytes of the record at `pos` from offset `off`, when still staged
  // (not yet uploaded); false when the caller must read the device copy
  bool read_staged(u64 pos, u64 off, u64 len, u8* dst) const {
    if (pos < flushed) return false;
    memcpy(dst, stage.data() + (pos - flushed) + off, len);
    return true;
  }
};

// Turn an rbe_entry with `cmd` (its Cmd bytes) into an arena/ring entry,
// staging a heap record when it needs one; the caller checked heap.room.
inline Ent stage_entry(HostHeap& heap, const rbe_entry& x, const u8* cmd) {
  Ent e;
  memset(&e, 0, sizeof(e));
  e.term = x.term;
  e.type = x.type & ET_TYPE_MASK;
  e.len = x.cmd_len;
  if (entry_needs_heap(x)) {
    const u64 meta[4] = {x.key, x.client_id, x.series_id, x.responded_to};
    e.type |= ET_HEAP;
    e.lo = entry_fingerprint(meta, cmd, x.cmd_len);
    e.hi = heap.put_record(meta, cmd, x.cmd_len);
  } else {
    u8 b[16];
    memset(b, 0, sizeof(b));
    if (x.cmd_len) memcpy(b, cmd, x.cmd_len);
    memcpy(&e.lo, b, 8);
    memcpy(&e.hi, b + 8, 8);
  }
  return e;
}

// The raftpb.Entry of a ring/arena entry, Index aside: type, Cmd length and
// the first 16 Cmd bytes, session fields; `rd(pos, off, len, dst)` reads heap
// record bytes (0, or RBE_E_STATE for an overwritten record).  With `cmd`
// non-null the whole Cmd is copied there.
template <typename RD>
inline int entry_out(const Ent& x, rbe_entry* o, u8* cmd, RD&& rd) {
  o->term = x.term;
  o->type = ent_type(x.type);
  o->cmd_len = x.len;
  memset(o->cmd, 0, sizeof(o->cmd));
  o->key = o->client_id = o->series_id = o->responded_to = 0;
  if (!ent_heap(x.type)) {
    u8 w[16];
    memcpy(w, &x.lo, 8);
    memcpy(w + 8, &x.hi, 8);
    memcpy(o->cmd, w, 16);
    if (cmd) memcpy(cmd, w, x.len);
    return RBE_OK;
  }
  u64 meta[4];
  int rc = rd(x.hi, 0, kHeapHdr, (u8*)meta);
  if (!rc && x.len) rc = rd(x.hi, kHeapHdr, x.len < 16 ? x.len : 16, o->cmd);
  if (!rc && cmd && x.len) rc = rd(x.hi, kHeapHdr, x.len, cmd);
  if (rc) return rc;
  o->key = meta[0];
  o->client_id = meta[1];
  o->series_id = meta[2];
  o->responded_to = meta[3];
  return RBE_OK;
}

// One staged replica-value pair into the planes (k_ext_scatter does the same)
RBE_HD void apply_pair(const Planes& P, u64 rep, u64 val) {
  if (rep >> 63) {
    Hot* h = &P.hot[rep & ~(1ull << 63)];
    h->flags = val ? (u8)(h->flags & ~HF_APPLY_HELD) : (u8)(h->flags | HF_APPLY_HELD);
  } else {
    P.applied[rep] = val;
  }
}

// The rbe_update of replica r after round `round` - 1 from its Upd, Core and
// Hot rows (rbe_get_updates).  A replica that made no Update-writing step in
// that round (an idle round finished in triage) has an empty Update.
// RBE_UF_HAS_UPDATE of update_view from the Upd record alone (the collect
// passes test every replica; a stale record, the common case, is one 16-B read)
RBE_HD bool upd_has(const Upd& d, u32 round) {
  if (!(round > 0 && d.round == round - 1)) return false;
  const u32 f = d.flags & ~UF_RANGES;
  if ((f & RBE_UF_STATE_CHANGED) || d.n_msgs || d.n_rtr ||
      (f & (RBE_UF_SENT_QUIESCE | RBE_UF_SNAPSHOT | RBE_UF_APPLIED | RBE_UF_HAS_UPDATE)))
    return true;
  return (d.flags & UF_RANGES) && (d.n_drop_ent || d.n_drop_ri || d.save_lo <= d.save_hi ||
                                   d.apply_lo <= d.apply_hi);
}
RBE_HD void update_view(const Upd& d, const Core& c, const Hot& h, u32 round, rbe_update& u) {
  u = rbe_update{};
  u.term = c.term;
  u.vote = c.vote;
  u.commit = c.committed;
  u.digest = d.digest;
  u.fault = d.fault;
  u.save_lo = u.apply_lo = 1;  // empty ranges unless the step wrote them
  u.save_hi = u.apply_hi = 0;
  if (round > 0 && d.round == round - 1) {
    if (d.flags & UF_RANGES) {  // chunks 0-2 of the record are this step's (Upd)
      u.save_lo = d.save_lo;
      u.save_hi = d.save_hi;
      u.apply_lo = d.apply_lo;
      u.apply_hi = d.apply_hi;
      u.n_dropped_entries = d.n_drop_ent;
      u.n_dropped_read_indexes = d.n_drop_ri;
    }
    u.n_messages = d.n_msgs;
    u.n_ready_to_read = d.n_rtr;
    u.flags = d.flags & ~UF_RANGES;
    u.events = d.events;
  }
  // Peer.HasUpdate (peer.go:253-280) and setFastApply / validateUpdate
  // (peer.go:209-245) on the range form
  const bool has = (u.flags & RBE_UF_STATE_CHANGED) || u.n_messages || u.n_ready_to_read ||
                   u.n_dropped_entries || u.n_dropped_read_indexes || u.save_lo <= u.save_hi ||
                   u.apply_lo <= u.apply_hi ||
                   (u.flags & (RBE_UF_SENT_QUIESCE | RBE_UF_SNAPSHOT | RBE_UF_APPLIED));
  if (has) u.flags |= RBE_UF_HAS_UPDATE;
  if (update_fast_apply((u.flags & RBE_UF_SNAPSHOT) != 0, u.save_lo, u.save_hi, u.apply_lo,
                        u.apply_hi))
    u.flags |= RBE_UF_FAST_APPLY;
  if (!update_valid(u.commit, u.save_lo, u.save_hi, u.apply_lo, u.apply_hi))
    u.fault |= RBE_FAULT_PANIC;
  u.role = h.role;
  u.leader_id = c.leader;
}
// An engine message in raftpb form (Update.Messages): its node ids (From, To,
// and the Hint of RequestVote / LeaderTransfer) from the internal ids of local
// group g, whose cluster id is `cid`
RBE_HD void msg_out(const Msg& m, u64 cid, const u64* ids, u32 n, u64 g, rbe_message& o) {
  o.type = m.type;
  o.reject = m.reject;
  o.to = ext_id(ids, n, g, m.to);
  o.from = ext_id(ids, n, g, m.from);
  o.cluster_id = cid;
  o.term = m.term;
  o.log_term = m.log_term;
  o.log_index = m.log_index;
  o.commit = m.commit;
  o.hint = hint_is_node(m.type) ? ext_id(ids, n, g, m.hint) : m.hint;
  o.hint_high = m.hint_high;
  o.n_entries = msg_nent(m);
  o.reserved = msg_reserved(m);
}
// an rbe_update's node ids (vote, leader) from the internal ids of group g
RBE_HD void update_ids(rbe_update& u, const u64* ids, u32 n, u64 g) {
  u.vote = ext_id(ids, n, g, u.vote);
  u.leader_id = ext_id(ids, n, g, u.leader_id);
}
// getUpdateCommit (peer.go:410-427) of an rbe_update: `applied` is the
// applied index the step ran with (GetUpdate's lastApplied), `term_of(i)` the
// term of log entry i (the last EntriesToSave entry)
// `snap_index`: the index of the Update's Snapshot (RBE_UF_SNAPSHOT), else 0
template <typename TermFn>
inline void update_commit_view(const rbe_update& u, u64 applied, u64 snap_index, TermFn&& term_of,
                               rbe_update_commit& o) {
  memset(&o, 0, sizeof(o));
  if (!(u.flags & RBE_UF_HAS_UPDATE)) return;
  o.ready_to_read = u.n_ready_to_read;
  o.last_applied = applied;
  u64 stable_log_to = 0;
  update_commit(u.save_lo, u.save_hi, u.apply_lo, u.apply_hi,
                (u.flags & RBE_UF_SNAPSHOT) ? snap_index : 0, &o.processed, &stable_log_to,
                &o.stable_snapshot_to);
  if (stable_log_to) {
    o.stable_log_to = stable_log_to;
    o.stable_log_term = term_of(u.save_hi);
  }
}

// One staged rbe_commit (Peer.Commit's log part, ext_commit mode); applied by
// commit_update (rbe_step.h) in k_ext_scatter / HostInputs::apply_host.
struct CommitRec {
  u64 r, stable_log_to, stable_log_term, processed, last_applied, stable_snapshot_to;
};

// The lowest payload-heap position the replicas of group g that this engine
// steps may still need (~0 for none), for HostHeap::room: the records of
// log-window entries above the group's low mark — min over those replicas of
// min(savedTo, processed, applied), and of a leader's remote match values
// (what its followers, here or behind the transport, have acknowledged) — and
// of the entries the Proposes of the last round's outboxes forward.  `round` is
// the round about to run.  One lane per group on the device (k_heap_low).
template <int N>
RBE_HD u64 heap_low_group(const Planes& P, const Params& C, u64 g, u32 round) {
  u64 mark = ~0ull;
  for (u32 k = 0; k < N; k++) {
    if (!owns_replica(C, g, k)) continue;
    const u64 r = g * N + k;
    const Core c = P.core[r];
    u64 m = c.saved_to < c.processed ? c.saved_to : c.processed;
    if (C.ext_apply && P.applied[r] < m) m = P.applied[r];
    if (P.hot[r].role == R_Leader)
      for (u32 s = 0; s < N; s++)
        if (s != k && P.rem[r * N + s].match < m) m = P.rem[r * N + s].match;
    if (m < mark) mark = m;
  }
  u64 lo = ~0ull;
  const u32 par = (round - 1u) & 1u;
  for (u32 k = 0; k < N; k++) {
    if (!owns_replica(C, g, k)) continue;
    const u64 r = g * N + k;
    const u64 last = P.core[r].last_index;
    u64 from = mark + 1;
    if (C.snapshot_entries && P.snp[r].marker + 1 > from) from = P.snp[r].marker + 1;
    for (u64 i = from; i <= last; i++) {  // the ring window and the cold log below it
      Ent e;
      if (log_ent_at(P, C, r, last, i, &e) && ent_heap(e.type) && e.hi < lo) lo = e.hi;
    }
    if (round == 0) continue;
    const CntRow row = P.cnt[par][r];
    for (u32 d = 0; d < N; d++) {
      const ListView lv = list_view(P, C, par, r * N + d, row_word(row, d, k, round));
      for (u32 i = 0; i < lv.n(); i++) {
        const Msg m = lv.at(i);
        if (m.type != M_Propose) continue;
        const Ent* es = msg_ents(P, C, par, r, m);
        for (u32 j = 0; j < msg_nent(m); j++)
          if (ent_heap(es[j].type) && es[j].hi < lo) lo = es[j].hi;
      }
    }
  }
  return lo;
}

// rbe_get_snapshot_state row: marker, marker term, snapshot index, snapshot
// term, reqSnapshotIndex, compactLogTo, the snapshot's and the state
// machine's membership (removed masks)
// The Snapshot of an Update (rbe_get_update_snapshots): index, term and packed
// membership of the snapshot a replica restored and holds in memory (it sits
// at the LogDB marker, SnapSt::upd_*), all zero when the Update carries none
inline void update_snapshot_row(const rbe_update& u, const SnapSt* s, u64* o) {
  o[0] = o[1] = o[2] = o[3] = 0;
  if (!s || !(u.flags & RBE_UF_HAS_UPDATE) || !(u.flags & RBE_UF_SNAPSHOT)) return;
  o[0] = s->marker;
  o[1] = s->marker_term;
  o[2] = pack_ms(s->upd_rem, s->upd_obs, s->upd_wit);
}
inline void snap_state_row(const SnapSt& s, u64* o) {
  o[0] = s.marker;
  o[1] = s.marker_term;
  o[2] = s.ss_index;
  o[3] = s.ss_term;
  o[4] = s.ss_req;
  o[5] = s.compact_to;
  o[6] = pack_ms(s.ss_rem, s.ss_obs, s.ss_wit);
  o[7] = pack_ms(s.sm_rem, s.sm_obs, s.sm_wit);
}

// Check a batch of entries whole: their types, and that the heap (if any
// needs it) can take them; sets *need to the heap bytes.  `cmd` null: each
// Cmd is the entry's inline cmd (at most 16 bytes).
inline int check_entries(const HostHeap& heap, u64 total, const rbe_entry* ents, const u8* cmd,
                         bool config_change_ok, u64* need) {
  u64 big = 0, maxrec = 0;
  for (u64 j = 0; j < total; j++) {
    const rbe_entry& e = ents[j];
    const u32 t = e.type;
    if (t > E_Metadata || (t == E_ConfigChange && !config_change_ok)) return RBE_E_INVALID;
    if (!cmd && e.cmd_len > 16) return RBE_E_INVALID;
    if (!entry_needs_heap(e)) continue;
    // a heap record takes at most a quarter of the heap (the ErrPayloadTooBig
    // check of requests.go:989-991, node.go:366-367)
    const u64 rb = heap_rec_bytes(e.cmd_len);
    if (heap.cap == 0 || e.cmd_len > heap.cap / 4) return RBE_E_INVALID;
    big += rb;
    if (rb > maxrec) maxrec = rb;
  }
  // one wrap skip at most (the batch is below a lap)
  *need = big ? big + maxrec : 0;
  return RBE_OK;
}

// Check an rbe_launch batch whole (rbe.h) and turn its entries into ring rows
// (terms, bodies) in batch order, staging heap records for the entries that
// need one; 0, RBE_E_INVALID or RBE_E_NOMEM (heap full of live records).
inline int launch_rows(const Params& C, HostHeap& heap, u64 n, const u64* replica,
                       const rbe_launch_state* st, const rbe_entry* ents, const u8* cmd,
                       std::vector<u64>& terms, std::vector<Body>& bodies) {
  if (n && (!replica || !st)) return RBE_E_INVALID;
  u64 total = 0;
  for (u64 i = 0; i < n; i++) {
    const rbe_launch_state& x = st[i];
    // a compacted LogDB (marker > 0) only with snapshots on; the entries lie
    // above the marker, the commit (loadState, raft.go:429-437) and the
    // snapshot at or above it, and Term(marker) is in the in-memory window
    const bool snap = x.marker || x.marker_term || x.snapshot_index || x.snapshot_term;
    if (snap && !C.snapshot_entries) return RBE_E_INVALID;
    if (x.marker > x.last_index || x.n_entries > x.last_index - x.marker ||
        x.commit < x.marker || x.snapshot_index < x.marker || x.snapshot_index > x.last_index ||
        (x.marker && !x.marker_term) || (x.snapshot_index && !x.snapshot_term))
      return RBE_E_INVALID;
    if (replica[i] >= C.n_rep || x.n_entries > x.last_index ||
        x.commit > x.last_index || x.vote > C.n || (x.last_index > x.marker && !x.n_entries))
      return RBE_E_INVALID;
    // the LogDB's membership (packed: slots not in Addresses | Observers << 8 |
    // Witnesses << 16), only with cfg.membership
    if (!ms_valid(x.removed, C.n) || (x.removed && !C.membership)) return RBE_E_INVALID;
    total += x.n_entries;
  }
  if (total && !ents) return RBE_E_INVALID;
  for (u64 j = 0, i = 0; i < n; i++) {
    const rbe_launch_state& x = st[i];
    for (u32 q = 0; q < x.n_entries; q++, j++) {
      const rbe_entry& e = ents[j];
      if (e.index != x.last_index - x.n_entries + 1 + q || e.term > x.term) return RBE_E_INVALID;
    }
  }
  u64 need = 0;
  int rc = check_entries(heap, total, ents, cmd, true, &need);
  if (rc) return rc;
  if (need && (rc = heap.room(need))) return rc;
  terms.resize(total);
  bodies.resize(total);
  u64 off = 0;
  for (u64 j = 0; j < total; j++) {
    const rbe_entry& e = ents[j];
    const Ent x = stage_entry(heap, e, cmd ? cmd + off : e.cmd);
    if (cmd) off += e.cmd_len;
    terms[j] = e.term;
    Body& b = bodies[j];
    b.type = x.type;
    b.len = x.len;
    b.lo = x.lo;
    b.hi = x.hi;
  }
  heap.live_lo = 0;  // restarted replicas may need older records again: recompute
  return RBE_OK;
}

// The input staged between two steps.  `Alloc` backs the three record
// vectors the upload copies whole (replicas, records, entries): the HIP engine
// gives them pinned host memory, so they go to the device without a host copy
// (rbe_engine.hip flush_inputs), the host build plain heap memory.
template <template <class> class Alloc>
struct HostInputsT {
  template <class T>
  using UpVec = std::vector<T, Alloc<T>>;
  u64 n_rep = 0;
  u32 n = 0;
  u32 in_cap = 0;
  // [n_rep] per replica: index into recs, valid when `gen` is the current
  // staging generation (so clear() bumps the generation instead of visiting
  // every staged replica), and the duplicate-check stamp of the current call,
  // side by side so a push touches one cache line per replica
  struct SlotMark {
    u32 slot, gen, mark;
  };
  std::vector<SlotMark> sm;
  u32 epoch = 0;
  u32 gen = 1;
  UpVec<u64> reps;    // staged replicas ...
  UpVec<ExtIn> recs;  // ... and their input records
  UpVec<Ent> ents;    // staged proposal entries (Planes::in_ents)
  // staged replica-value pairs: rbe_notify_applied values, and with bit 63 of
  // the replica word set, rbe_set_apply_ready flags (value 1 = ready)
  std::vector<u64> app_rep, app_val;
  struct AppSlot {
    u32 applied, ready, gen;  // index into app_rep (this generation), ~0u = none staged
  };
  std::vector<AppSlot> app_slot;  // [n_rep]
  std::vector<u64> applied;  // [n_rep] host mirror of Planes::applied (the host is its only writer)
  std::vector<CommitRec> commits;  // rbe_commit records for the next step, in call order
  std::vector<u8> committing;      // [n_rep] a commit is staged (one per replica per step)
  std::vector<SnapRec> snaps;      // rbe_snapshot_saved / rbe_compact, one record per replica
  std::vector<u32> snap_slot;      // [n_rep] index into snaps, ~0u = none
  const Params* owner = nullptr;  // replica-per-GPU mode: only owned replicas take input

  HostHeap heap;             // payload heap positions and staged bytes
  // [n_groups * n] node ids of the groups' slots (rbe_set_node_ids), empty =
  // slot s is node s + 1
  std::vector<u64> ids;

  const u64* id_table() const { return ids.empty() ? nullptr : ids.data(); }
  // rbe_set_node_ids: groups [first, first + count), n ids each, non-zero and
  // distinct within a group.  The engine's canonical node order is the slot
  // order: the reference visits its maps in Go's random order (raft.go:390-402,
  // 803, 836), so any fixed order is one of its executions; per (sender,
  // receiver) pair the message streams do not depend on it.
  int set_node_ids(u64 n_groups, u64 first, u64 count, const u64* v) {
    if (first > n_groups || count > n_groups - first || (count && !v)) return RBE_E_INVALID;
    for (u64 i = 0; i < count; i++)
      for (u32 s = 0; s < n; s++) {
        if (v[i * n + s] == 0) return RBE_E_INVALID;
        for (u32 t = 0; t < s; t++)
          if (v[i * n + t] == v[i * n + s]) return RBE_E_INVALID;
      }
    ensure_ids(n_groups);
    std::copy(v, v + count * n, ids.begin() + first * n);
    return RBE_OK;
  }
  void ensure_ids(u64 n_groups) {
    if (!ids.empty()) return;
    ids.resize(n_groups * n);
    for (u64 i = 0; i < n_groups * n; i++) ids[i] = i % n + 1;
  }
  // rbe_replace_node's checks on the host: replica[i] in range, at most one
  // per group, id[i] non-zero and not the id of another slot of the group, no
  // input staged for any replica of the group (RBE_E_STATE)
  int replace_args(u64 cnt, const u64* replica, const u64* id) const {
    if (cnt && (!replica || !id)) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++) {
      if (replica[i] >= n_rep || id[i] == 0) return RBE_E_INVALID;
      const u64 g = replica[i] / n;
      for (u64 j = 0; j < i; j++)
        if (replica[j] / n == g) return RBE_E_STATE;
      for (u32 s = 0; s < n; s++) {
        const u64 r = g * n + s;
        if (r != replica[i] && (ids.empty() ? s + 1 : ids[r]) == id[i]) return RBE_E_INVALID;
        if (slot_of(r) != ~0u || (app_slot[r].gen == gen && (app_slot[r].applied != ~0u ||
                                                              app_slot[r].ready != ~0u)) ||
            committing[r] || snap_slot[r] != ~0u)
          return RBE_E_STATE;
      }
    }
    return RBE_OK;
  }
  // the new node in replica r's slot: its id, and a state machine that has
  // applied nothing (the host mirror of Planes::applied)
  void assign_node(u64 n_groups, u64 r, u64 id) {
    ensure_ids(n_groups);
    ids[r] = id;
    applied[r] = 0;
  }
  // node id → internal id (slot + 1) in replica r's group; 0 when no slot has it
  u64 in_id(u64 r, u64 id) const {
    if (r >= n_rep || id == 0) return 0;
    if (ids.empty()) return id <= n ? id : 0;
    const u64* row = &ids[(r / n) * n];
    for (u32 s = 0; s < n; s++)
      if (row[s] == id) return s + 1;
    return 0;
  }
  // launch states with their votes (node ids) as internal ids; false when a
  // vote is not a slot of the replica's group (or the replica not a replica)
  bool map_votes(u64 cnt, const u64* replica, const rbe_launch_state* st,
                 std::vector<rbe_launch_state>& out) const {
    if (cnt && (!replica || !st)) return false;
    out.assign(st, st + cnt);
    for (u64 i = 0; i < cnt; i++)
      if (out[i].vote && (out[i].vote = in_id(replica[i], st[i].vote)) == 0) return false;
    return true;
  }
  // a batch of node ids of replica[i]'s groups; false when one is not a slot
  bool map_ids(u64 cnt, const u64* replica, const u64* node, std::vector<u64>& out) const {
    if (cnt && (!replica || !node)) return false;
    out.resize(cnt);
    for (u64 i = 0; i < cnt; i++)
      if ((out[i] = in_id(replica[i], node[i])) == 0) return false;
    return true;
  }

  void init(u64 n_rep_, u32 n_, u32 in_cap_, u64 heap_bytes = 0) {
    n_rep = n_rep_;
    n = n_;
    in_cap = in_cap_;
    heap.cap = heap_bytes;
    sm.assign(n_rep, SlotMark{~0u, 0u, 0u});
    applied.assign(n_rep, 0);
    committing.assign(n_rep, 0);
    snap_slot.assign(n_rep, ~0u);
    app_slot.assign(n_rep, AppSlot{~0u, ~0u, 0u});
  }
  bool empty() const {
    return reps.empty() && app_rep.empty() && heap.stage.empty() && commits.empty() &&
           snaps.empty();
  }
  void clear() {
    // a new generation: every slot of the last one reads as empty
    if (++gen == 0) {
      for (SlotMark& x : sm) x.gen = 0;
      for (AppSlot& x : app_slot) x.gen = 0;
      gen = 1;
    }
    reps.clear();
    recs.clear();
    ents.clear();
    app_rep.clear();
    app_val.clear();
    for (const CommitRec& c : commits) committing[c.r] = 0;
    commits.clear();
    for (const SnapRec& x : snaps) snap_slot[x.r] = ~0u;
    snaps.clear();
    heap.stage.clear();
    heap.settle();
  }
  u32 slot_of(u64 r) const { return sm[r].gen == gen ? sm[r].slot : ~0u; }
  ExtIn& rec(u64 r) {
    SlotMark& m = sm[r];
    if (m.gen != gen) {
      // (both vectors grow before the slot is marked: a failed allocation
      // leaves the staging as it was)
      reps.reserve(reps.size() + 1);
      recs.reserve(recs.size() + 1);
      m.gen = gen;
      m.slot = (u32)recs.size();
      reps.push_back(r);
      recs.emplace_back();
      memset(&recs.back(), 0, sizeof(ExtIn));
    }
    return recs[m.slot];
  }
  u32 staged_flags(u64 r) const {
    const u32 s = slot_of(r);
    return s == ~0u ? 0u : recs[s].flags;
  }
  // 0, or RBE_E_INVALID / RBE_E_STATE for the whole batch: every replica in
  // range, none twice in the batch, none with `flag` already staged
  int check_replicas(u64 cnt, const u64* replica, u32 flag) {
    int rc = check_range(cnt, replica);
    if (rc || !flag) return rc;
    return unique_replicas(cnt, replica, flag);
  }
  // RBE_E_STATE when a replica appears twice in the batch or already has
  // `flag` staged (0: only the first check); O(cnt) with the epoch stamps
  int unique_replicas(u64 cnt, const u64* replica, u32 flag) {
    if (++epoch == 0) {
      for (SlotMark& x : sm) x.mark = 0u;
      epoch = 1;
    }
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      if (sm[r].mark == epoch || (flag && (staged_flags(r) & flag))) return RBE_E_STATE;
      sm[r].mark = epoch;
    }
    return RBE_OK;
  }

  // Peer.ProposeEntries batches (peer.go:117-123): batch i holds n_ents[i]
  // entries for replica[i], whole raftpb.Entry values (Type, Key, ClientID,
  // SeriesID, RespondedTo; Index/Term are stamped by the leader, raft.go:
  // 909-920) with their Cmds concatenated in `cmd`.  Config changes go through
  // ProposeConfigChange.
  int push_entries(u64 cnt, const u64* replica, const u32* n_ents, const rbe_entry* pe,
                   const u8* cmd) {
    if (cnt && !n_ents) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, EXT_PROPOSE);
    if (rc) return rc;
    u64 total = 0, bytes = 0;
    for (u64 i = 0; i < cnt; i++) {
      if (n_ents[i] == 0 || n_ents[i] > 0xFFFFu) return RBE_E_INVALID;
      total += n_ents[i];
    }
    if (total && !pe) return RBE_E_INVALID;
    for (u64 j = 0; j < total; j++) bytes += pe[j].cmd_len;
    if (bytes && !cmd) return RBE_E_INVALID;
    u64 need = 0;
    const u8* cb = cmd ? cmd : (const u8*)"";
    if ((rc = check_entries(heap, total, pe, cb, false, &need))) return rc;
    if (ents.size() + total > in_cap) return RBE_E_NOMEM;
    if (need && (rc = heap.room(need))) return rc;
    // every allocation of the staging below happens here, before anything is
    // staged (a failure is RBE_E_NOMEM at the ABI with nothing staged)
    reps.reserve(reps.size() + cnt);
    recs.reserve(recs.size() + cnt);
    ents.reserve(ents.size() + total);
    heap.stage.reserve(heap.stage.size() + need + 16 * total);
    u64 j = 0, off = 0;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_PROPOSE;
      x.n_prop = n_ents[i];
      x.prop_off = (u32)ents.size();
      for (u32 t = 0; t < n_ents[i]; t++, j++) {
        rbe_entry y = pe[j];
        y.term = 0;  // stamped by the leader (appendEntries, raft.go:909-920)
        ents.push_back(stage_entry(heap, y, cb + off));
        off += y.cmd_len;
      }
    }
    return RBE_OK;
  }
  // rbe_push_proposals: the same without session fields
  int push_proposals(u64 cnt, const u64* replica, const u32* n_ents, const u32* type,
                     const u32* cmd_len, const u8* cmd) {
    if (cnt && (!n_ents || !type || !cmd_len)) return RBE_E_INVALID;
    u64 total = 0, bytes = 0;
    bool inline_only = true;
    for (u64 i = 0; i < cnt; i++) {
      if (n_ents[i] == 0 || n_ents[i] > 0xFFFFu) return RBE_E_INVALID;
      total += n_ents[i];
    }
    for (u64 j = 0; j < total; j++) {
      if (type[j] > E_Metadata || type[j] == E_ConfigChange) return RBE_E_INVALID;
      inline_only = inline_only && cmd_len[j] <= 16;
      bytes += cmd_len[j];
    }
    if (inline_only) return push_inline(cnt, replica, n_ents, type, cmd_len, cmd, total, bytes);
    std::vector<rbe_entry> pe(total);
    for (u64 j = 0; j < total; j++) {
      memset(&pe[j], 0, sizeof(rbe_entry));
      pe[j].type = type[j];
      pe[j].cmd_len = cmd_len[j];
    }
    return push_entries(cnt, replica, n_ents, pe.data(), cmd);
  }
  int push_read_index(u64 cnt, const u64* replica, const u64* lo, const u64* hi) {
    if (cnt && (!lo || !hi)) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (lo[i] == 0) return RBE_E_INVALID;  // ctx.Low is never 0 (requests.go:726)
    int rc = check_range(cnt, replica);
    if (rc) return rc;
    // one pass over the replicas: the duplicate checks and the staging
    // together, undone whole when a check fails (all-or-nothing)
    return stage_pass(cnt, replica, EXT_READ, [&](ExtIn& x, u64 i) {
      x.ctx_low = lo[i];
      x.ctx_high = hi[i];
    });
  }
  // every replica in range (and, replica-per-GPU, stepped here)
  int check_range(u64 cnt, const u64* replica) const {
    if (cnt && !replica) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++) {
      if (replica[i] >= n_rep) return RBE_E_INVALID;
      if (owner && !owns_replica(*owner, replica[i] / n, (u32)(replica[i] % n)))
        return RBE_E_INVALID;  // stepped by another engine
    }
    return RBE_OK;
  }
  // Stage `flag` for each replica (set(x, i) fills record x from input i) in
  // one pass, with check_replicas' duplicate checks: RBE_E_STATE, and nothing
  // staged, when a replica appears twice or already has `flag` staged
  template <class Set>
  int stage_pass(u64 cnt, const u64* replica, u32 flag, Set&& set) {
    if (++epoch == 0) {
      for (SlotMark& x : sm) x.mark = 0u;
      epoch = 1;
    }
    const size_t n0 = recs.size();
    recs.reserve(n0 + cnt);
    reps.reserve(reps.size() + cnt);
    undo.clear();
    undo.reserve(cnt);
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      if (i + 16 < cnt) __builtin_prefetch(&sm[replica[i + 16]], 1);
      SlotMark& m = sm[r];
      bool bad = m.mark == epoch;
      m.mark = epoch;
      if (!bad && m.gen == gen) {  // a record staged by another call: keep its old value
        ExtIn& x = recs[m.slot];
        bad = (x.flags & flag) != 0;
        if (!bad) {
          undo.push_back(std::make_pair(m.slot, x));
          x.flags |= flag;
          set(x, i);
        }
      } else if (!bad) {
        m.gen = gen;
        m.slot = (u32)recs.size();
        reps.push_back(r);
        recs.emplace_back();
        ExtIn& x = recs.back();
        memset(&x, 0, sizeof(ExtIn));
        x.flags = flag;
        set(x, i);
      }
      if (bad) {  // undo: the new records go, the old ones get their values back
        for (size_t q = n0; q < recs.size(); q++) sm[reps[q]].gen = 0;
        recs.resize(n0);
        reps.resize(n0);
        for (const auto& u : undo) recs[u.first] = u.second;
        undo.clear();
        return RBE_E_STATE;
      }
    }
    return RBE_OK;
  }
  // push_proposals when every Cmd is inline (at most 16 bytes, no session
  // fields): the entries go straight to ring form, in one pass with staging
  int push_inline(u64 cnt, const u64* replica, const u32* n_ents, const u32* type,
                  const u32* cmd_len, const u8* cmd, u64 total, u64 bytes) {
    if (bytes && !cmd) return RBE_E_INVALID;
    int rc = check_range(cnt, replica);
    if (rc) return rc;
    if (ents.size() + total > in_cap) return RBE_E_NOMEM;
    const size_t e0 = ents.size();
    ents.resize(e0 + total);
    Ent* out = ents.data() + e0;
    u64 j = 0, off = 0;
    for (u64 i = 0; i < cnt; i++)
      for (u32 t = 0; t < n_ents[i]; t++, j++) {
        Ent& e = out[j];
        e.term = 0;  // stamped by the leader (appendEntries, raft.go:909-920)
        e.type = type[j];
        e.len = cmd_len[j];
        u8 b[16] = {0};
        if (cmd_len[j]) memcpy(b, cmd + off, cmd_len[j]);
        memcpy(&e.lo, b, 8);
        memcpy(&e.hi, b + 8, 8);
        off += cmd_len[j];
      }
    u64 first = e0;
    try {
      rc = stage_pass(cnt, replica, EXT_PROPOSE, [&](ExtIn& x, u64 i) {
        x.n_prop = n_ents[i];
        x.prop_off = (u32)first;
        first += n_ents[i];
      });
    } catch (...) {  // (stage_pass allocates before it stages anything)
      ents.resize(e0);
      throw;
    }
    if (rc) ents.resize(e0);
    return rc;
  }
  std::vector<std::pair<u32, ExtIn>> undo;  // stage_pass: records to restore on failure
  int request_leader_transfer(u64 cnt, const u64* replica, const u64* target_id) {
    std::vector<u64> tv;  // NoNode panics (raft.go:1715), as does a node not in the group
    if (!map_ids(cnt, replica, target_id, tv)) return RBE_E_INVALID;
    const u64* target = tv.data();
    int rc = check_replicas(cnt, replica, EXT_XFER);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_XFER;
      x.xfer_target = (u8)target[i];
    }
    return RBE_OK;
  }
  int report_unreachable(u64 cnt, const u64* replica, const u64* node_id) {
    std::vector<u64> nv;
    if (!map_ids(cnt, replica, node_id, nv)) return RBE_E_INVALID;
    const u64* node = nv.data();
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_UNREACH;
      x.unreach |= (u8)(1u << (node[i] - 1));
    }
    return RBE_OK;
  }
  int report_snapshot_status(u64 cnt, const u64* replica, const u64* node_id, const u8* reject) {
    std::vector<u64> nv;
    if ((cnt && !reject) || !map_ids(cnt, replica, node_id, nv)) return RBE_E_INVALID;
    const u64* node = nv.data();
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      const u8 bit = (u8)(1u << (node[i] - 1));
      x.flags |= EXT_SNAPST;
      x.snap_nodes |= bit;
      x.snap_reject = (u8)(reject[i] ? (x.snap_reject | bit) : (x.snap_reject & ~bit));
    }
    return RBE_OK;
  }
  // rbe_propose_config_change / rbe_apply_config_change / rbe_reject_config_change
  int propose_config_change(u64 cnt, const u64* replica, const u32* type, const u64* node_id) {
    std::vector<u64> nv;
    if ((cnt && !type) || !map_ids(cnt, replica, node_id, nv)) return RBE_E_INVALID;
    const u64* node = nv.data();
    for (u64 i = 0; i < cnt; i++)
      if (type[i] > CC_AddWitness) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, EXT_CC_PROPOSE);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_CC_PROPOSE;
      x.pad[0] = (u64)type[i] | (node[i] << 8);
    }
    return RBE_OK;
  }
  // `ms_now[i]`: replica[i]'s raft membership now (packed, pack_ms), or null.
  // An AddObserver / AddWitness of another node that is a voter or in the
  // other set would put one node in two of raft's maps (raft.go:1159-1180
  // only checks its own map), which a slot cannot hold: RBE_E_INVALID.
  int apply_config_change(u64 cnt, const u64* replica, const u64* node_id, const u32* type,
                          bool reject, const u32* ms_now = nullptr) {
    if (cnt && !reject && (!type || !node_id)) return RBE_E_INVALID;
    std::vector<u64> nv(reject ? 0 : cnt);
    for (u64 i = 0; i < cnt && !reject; i++) {  // node id 0 = NoNode
      nv[i] = node_id[i] ? in_id(replica ? replica[i] : ~0ull, node_id[i]) : 0;
      if (type[i] > CC_AddWitness || (node_id[i] && !nv[i])) return RBE_E_INVALID;
      if (ms_now && nv[i] && nv[i] != replica[i] % n + 1 &&
          (type[i] == CC_AddObserver || type[i] == CC_AddWitness)) {
        // the membership the step applies it to: after a staged RestoreRemotes
        const u32 ms = (staged_flags(replica[i]) & EXT_RESTORE)
                           ? (u32)recs[slot_of(replica[i])].pad[2]
                           : ms_now[i];
        const u32 b = 1u << (nv[i] - 1);
        const bool voter = !(ms & b), obs = (ms >> 8) & b, wit = (ms >> 16) & b;
        if (voter || (type[i] == CC_AddObserver ? wit : obs)) return RBE_E_INVALID;
      }
    }
    const u64* node = nv.data();
    int rc = check_replicas(cnt, replica, EXT_CC_APPLY);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_CC_APPLY;
      x.pad[1] = reject ? (u64)(CCA_VALID | CCA_REJECT)
                        : (u64)(CCA_VALID | (type[i] << 3) | (u32)node[i]);
    }
    return RBE_OK;
  }
  // rbe_restore_remotes: replica[i]'s snapshot lists counts[3i] voters,
  // counts[3i + 1] observers and counts[3i + 2] witnesses, their node ids next in
  // `ids` in that order; staged packed (pack_ms)
  int restore_remotes(u64 cnt, const u64* replica, const u32* counts, const u64* vids) {
    if (cnt && !counts) return RBE_E_INVALID;
    std::vector<u64> rem(cnt);
    u64 j = 0;
    for (u64 i = 0; i < cnt; i++) {
      u32 sets[3] = {0, 0, 0}, listed = 0;
      for (u32 c = 0; c < 3; c++) {
        if (counts[3 * i + c] && !vids) return RBE_E_INVALID;
        for (u32 q = 0; q < counts[3 * i + c]; q++, j++) {
          const u64 x = in_id(replica ? replica[i] : ~0ull, vids[j]);
          if (!x || ((listed >> (x - 1)) & 1u)) return RBE_E_INVALID;  // each node in one set
          listed |= 1u << (x - 1);
          sets[c] |= 1u << (x - 1);
        }
      }
      rem[i] = pack_ms(((1u << n) - 1u) & ~sets[0], sets[1], sets[2]);
    }
    int rc = check_replicas(cnt, replica, EXT_RESTORE);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_RESTORE;
      x.pad[2] = rem[i];
    }
    return RBE_OK;
  }
  int notify_applied(u64 cnt, const u64* replica, const u64* value) {
    if (cnt && !value) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++)  // applied never moves backwards (node.go:911-913)
      if (value[i] < applied[replica[i]]) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      stage_pair(r, value[i], false);
      // a changed applied index is an event of the step (node.go:1033)
      if (value[i] != applied[r]) rec(r).flags |= EXT_APPLIED;
      applied[r] = value[i];
    }
    return RBE_OK;
  }
  int set_apply_ready(u64 cnt, const u64* replica, const u8* ready) {
    if (cnt && !ready) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) stage_pair(replica[i], ready[i] ? 1u : 0u, true);
    return RBE_OK;
  }
  // one staged pair per (replica, kind) between two steps, so no two lanes of
  // the scatter write one replica's row: a later call overwrites the value
  void stage_pair(u64 r, u64 v, bool ready) {
    AppSlot& a = app_slot[r];
    if (a.gen != gen) a = AppSlot{~0u, ~0u, gen};
    u32& slot = ready ? a.ready : a.applied;
    if (slot == ~0u) {
      slot = (u32)app_rep.size();
      app_rep.push_back(ready ? (r | (1ull << 63)) : r);
      app_val.push_back(v);
    } else {
      app_val[slot] = v;
    }
  }
  // rbe_snapshot_saved / rbe_compact (snapshot_entries with ext_apply): one of
  // each per replica per step; a snapshot no newer than the state machine's
  // applied index (what rbe_notify_applied reported), with its membership
  int snapshot_op(u64 cnt, const u64* replica, u32 kind, const u64* index, const u64* term,
                  const u32* removed, bool membership) {
    if (cnt && !index) return RBE_E_INVALID;
    if (kind == SR_SAVE && cnt && !term) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      if (index[i] == 0) return RBE_E_INVALID;
      if (kind == SR_SAVE) {
        const u32 rem = removed ? removed[i] : 0u;
        if (term[i] == 0 || index[i] > applied[replica[i]] || !ms_valid(rem, n) ||
            (rem && !membership))
          return RBE_E_INVALID;
      }
      const u32 s = snap_slot[replica[i]];
      if (s != ~0u && (snaps[s].kind & kind)) return RBE_E_STATE;
    }
    if ((rc = unique_replicas(cnt, replica, 0))) return rc;
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      if (snap_slot[r] == ~0u) {
        snap_slot[r] = (u32)snaps.size();
        snaps.push_back(SnapRec{r, 0, 0, 0, 0, 0});
      }
      SnapRec& x = snaps[snap_slot[r]];
      x.kind |= kind;
      if (kind == SR_SAVE) {
        x.index = index[i];
        x.term = term[i];
        x.rem = removed ? removed[i] : 0u;
      } else {
        x.compact_to = index[i];
      }
      rec(r);  // an (empty) input record wakes a sleeping group
    }
    return RBE_OK;
  }
  // rbe_commit: Peer.Commit's log part (rbe.h), checked whole, one per replica
  int commit(u64 cnt, const u64* replica, const rbe_update_commit* uc) {
    if (cnt && !uc) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++)
      if (committing[replica[i]]) return RBE_E_STATE;
    if ((rc = unique_replicas(cnt, replica, 0))) return rc;  // within the batch too
    for (u64 i = 0; i < cnt; i++) {
      committing[replica[i]] = 1;
      commits.push_back(CommitRec{replica[i], uc[i].stable_log_to, uc[i].stable_log_term,
                                  uc[i].processed, uc[i].last_applied,
                                  uc[i].stable_snapshot_to});
    }
    return RBE_OK;
  }
  // Write the staged input into host-resident planes (the test-only host build;
  // the HIP engine uploads the same vectors and scatters them on device).
  // resync the applied mirror after the plane was overwritten (snapshot import)
  void resync_applied(const u64* plane, u64 first, u64 count) {
    for (u64 i = 0; i < count; i++) applied[first + i] = plane[i];
  }
  void apply_host(const Planes& P, const Params& C_) {
    for (size_t i = 0; i < reps.size(); i++) {
      P.ext[reps[i]] = recs[i];
      P.gwake[reps[i] / n] = GW_AWAKE;  // input wakes a sleeping group
    }
    for (size_t i = 0; i < ents.size(); i++) P.in_ents[i] = ents[i];
    for (size_t i = 0; i < app_rep.size(); i++) apply_pair(P, app_rep[i], app_val[i]);
    for (const CommitRec& c : commits)
      commit_update(P, C_, c.r, c.stable_log_to, c.stable_log_term, c.processed, c.last_applied,
                    c.stable_snapshot_to);
    for (const SnapRec& x : snaps) snap_rec_apply(P, x);
  }
};
using HostInputs = HostInputsT<std::allocator>;

}  // namespace rbe
