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
#include <cstring>
#include <vector>

#include "../../include/rbe.h"
#include "rbe_step.h"
#include "rbe_types.h"

namespace rbe {

// Fingerprint of a Cmd longer than 16 bytes (Body/Ent lo when the bytes live in
// the payload heap): 64 bits over the zero-padded 8-byte words and the length.
// The trace digest folds it in place of the inline bytes, so the fingerprint
// stands for the payload in parity checks (oracle/harness.cpp restates it).
inline u64 cmd_fingerprint(const u8* b, u64 len) {
  u64 h = 0x243F6A8885A308D3ull ^ len;
  for (u64 i = 0; i < len; i += 8) {
    u64 w = 0;
    for (u64 j = 0; j < 8 && i + j < len; j++) w |= (u64)b[i + j] << (8 * j);
    h = mix64(h ^ w);
  }
  return mix64(h ^ (len << 1));
}

// Payload heap (cfg.heap_bytes): one device byte ring shared by every group.
// A Cmd longer than 16 bytes is written there once, when its proposal is
// staged, and every replica's log entry refers to it by (fingerprint, absolute
// heap position) in Body/Ent lo/hi: a follower that appends the entry copies
// the reference, never the bytes (the Log Matching property makes the bytes of
// an (index, term) the same on every replica).  The host is the only writer,
// so positions are assigned here, in push order.  Bytes at position p stay
// valid while head <= p + cap (a later lap overwrites them); a reader of an
// older entry gets RBE_E_STATE, the analog of ErrCompacted.
struct HostHeap {
  u64 cap = 0;      // bytes (0 = no heap: Cmd is at most 16 bytes)
  u64 head = 0;     // next free absolute position
  u64 flushed = 0;  // positions below this are on the device
  std::vector<u8> stage;  // bytes of [flushed, head), position flushed at index 0
  // reserve len bytes (16-B aligned, never split across the end of the ring)
  u64 alloc(u64 len) {
    u64 p = head;
    if (p % cap + len > cap) p += cap - p % cap;
    head = p + ((len + 15) & ~15ull);
    return p;
  }
  bool valid(u64 pos, u64 len) const { return cap && pos + len <= head && head <= pos + cap; }
};

// One staged replica-value pair into the planes (k_ext_scatter does the same)
RBE_HD void apply_pair(const Planes& P, u64 rep, u64 val) {
  if (rep >> 63) {
    Hot* h = &P.hot[rep & ~(1ull << 63)];
    h->flags = val ? (u8)(h->flags & ~HF_APPLY_HELD) : (u8)(h->flags | HF_APPLY_HELD);
  } else {
    P.applied[rep] = val;
  }
}

// Check an rbe_launch batch whole (rbe.h) and turn its entries into ring rows
// (terms, bodies) in batch order; 0 or RBE_E_INVALID.
// rbe_get_snapshot_state row: marker, marker term, snapshot index, snapshot
// term, reqSnapshotIndex, compactLogTo
inline void snap_state_row(const SnapSt& s, u64* o) {
  o[0] = s.marker;
  o[1] = s.marker_term;
  o[2] = s.ss_index;
  o[3] = s.ss_term;
  o[4] = s.ss_req;
  o[5] = s.compact_to;
}

inline int launch_rows(const Params& C, u64 n, const u64* replica, const rbe_launch_state* st,
                       const rbe_entry* ents, std::vector<u64>& terms, std::vector<Body>& bodies) {
  if (n && (!replica || !st)) return RBE_E_INVALID;
  // a restart carries no LogDB snapshot / compaction marker (SnapSt) yet
  if (n && C.snapshot_entries) return RBE_E_INVALID;
  u64 total = 0;
  std::vector<u8> seen;
  for (u64 i = 0; i < n; i++) {
    const rbe_launch_state& x = st[i];
    if (replica[i] >= C.n_rep || x.n_entries > C.ring || x.n_entries > x.last_index ||
        x.commit > x.last_index || x.vote > C.n || (x.last_index && !x.n_entries))
      return RBE_E_INVALID;
    total += x.n_entries;
  }
  if (total && !ents) return RBE_E_INVALID;
  for (u64 j = 0, i = 0; i < n; i++) {
    const rbe_launch_state& x = st[i];
    for (u32 q = 0; q < x.n_entries; q++, j++) {
      const rbe_entry& e = ents[j];
      if (e.index != x.last_index - x.n_entries + 1 + q || e.cmd_len > 16 || e.term > x.term)
        return RBE_E_INVALID;
    }
  }
  terms.resize(total);
  bodies.resize(total);
  for (u64 j = 0; j < total; j++) {
    const rbe_entry& e = ents[j];
    terms[j] = e.term;
    Body& b = bodies[j];
    b.type = e.type;
    b.len = e.cmd_len;
    memcpy(&b.lo, e.cmd, 8);
    memcpy(&b.hi, e.cmd + 8, 8);
  }
  return RBE_OK;
}

struct HostInputs {
  u64 n_rep = 0;
  u32 n = 0;
  u32 in_cap = 0;
  std::vector<u32> slot;    // [n_rep] index into recs, ~0u = nothing staged
  std::vector<u32> mark;    // [n_rep] duplicate check within one call (epoch stamps)
  u32 epoch = 0;
  std::vector<u64> reps;    // staged replicas ...
  std::vector<ExtIn> recs;  // ... and their input records
  std::vector<Ent> ents;    // staged proposal entries (Planes::in_ents)
  // staged replica-value pairs: rbe_notify_applied values, and with bit 63 of
  // the replica word set, rbe_set_apply_ready flags (value 1 = ready)
  std::vector<u64> app_rep, app_val;
  std::vector<u64> applied;  // [n_rep] host mirror of Planes::applied (the host is its only writer)

  HostHeap heap;             // payload heap positions and staged bytes

  void init(u64 n_rep_, u32 n_, u32 in_cap_, u64 heap_bytes = 0) {
    n_rep = n_rep_;
    n = n_;
    in_cap = in_cap_;
    heap.cap = heap_bytes;
    slot.assign(n_rep, ~0u);
    mark.assign(n_rep, 0u);
    applied.assign(n_rep, 0);
  }
  bool empty() const { return reps.empty() && app_rep.empty() && heap.stage.empty(); }
  void clear() {
    for (u64 r : reps) slot[r] = ~0u;
    reps.clear();
    recs.clear();
    ents.clear();
    app_rep.clear();
    app_val.clear();
    heap.stage.clear();
    heap.flushed = heap.head;
  }
  ExtIn& rec(u64 r) {
    if (slot[r] == ~0u) {
      slot[r] = (u32)recs.size();
      reps.push_back(r);
      ExtIn z;
      memset(&z, 0, sizeof(z));
      recs.push_back(z);
    }
    return recs[slot[r]];
  }
  u32 staged_flags(u64 r) const { return slot[r] == ~0u ? 0u : recs[slot[r]].flags; }
  // 0, or RBE_E_INVALID / RBE_E_STATE for the whole batch: every replica in
  // range, none twice in the batch, none with `flag` already staged
  int check_replicas(u64 cnt, const u64* replica, u32 flag) {
    if (cnt && !replica) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (replica[i] >= n_rep) return RBE_E_INVALID;
    if (!flag) return RBE_OK;
    if (++epoch == 0) {
      mark.assign(n_rep, 0u);
      epoch = 1;
    }
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      if (mark[r] == epoch || (staged_flags(r) & flag)) return RBE_E_STATE;
      mark[r] = epoch;
    }
    return RBE_OK;
  }

  int push_proposals(u64 cnt, const u64* replica, const u32* n_ents, const u32* type,
                     const u32* cmd_len, const u8* cmd) {
    if (cnt && (!n_ents || !type || !cmd_len)) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, EXT_PROPOSE);
    if (rc) return rc;
    u64 total = 0, bytes = 0;
    for (u64 i = 0; i < cnt; i++) {
      if (n_ents[i] == 0 || n_ents[i] > 0xFFFFu) return RBE_E_INVALID;
      total += n_ents[i];
    }
    u64 big = 0;  // heap bytes the batch needs (upper bound: alignment and lap skips)
    for (u64 j = 0; j < total; j++) {
      // Cmd is inline up to 16 bytes, longer ones need the payload heap and
      // may take at most a quarter of it (the ErrPayloadTooBig check of
      // requests.go:989-991, node.go:366-367); config changes go through ProposeConfigChange,
      // a membership path the device does not run
      if (type[j] == E_ConfigChange || type[j] > E_Metadata) return RBE_E_INVALID;
      if (cmd_len[j] > 16 && (heap.cap == 0 || (u64)cmd_len[j] > heap.cap / 4))
        return RBE_E_INVALID;
      if (cmd_len[j] > 16) big += (u64)cmd_len[j] + 16;
      bytes += cmd_len[j];
    }
    if (bytes && !cmd) return RBE_E_INVALID;
    if (ents.size() + total > in_cap) return RBE_E_NOMEM;
    // the bytes staged for one step must not lap the ring (they would
    // overwrite each other before the upload)
    if (big && heap.head - heap.flushed + 2 * big > heap.cap) return RBE_E_NOMEM;
    u64 j = 0, off = 0;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_PROPOSE;
      x.n_prop = n_ents[i];
      x.prop_off = (u32)ents.size();
      for (u32 t = 0; t < n_ents[i]; t++, j++) {
        Ent e;
        memset(&e, 0, sizeof(e));
        e.term = 0;  // stamped by the leader (appendEntries, raft.go:909-920)
        e.type = type[j];
        e.len = cmd_len[j];
        if (cmd_len[j] > 16) {
          // heap entry: lo = fingerprint, hi = absolute heap position
          const u64 pos = heap.alloc(cmd_len[j]);
          heap.stage.resize(heap.head - heap.flushed, 0);
          memcpy(heap.stage.data() + (pos - heap.flushed), cmd + off, cmd_len[j]);
          e.lo = cmd_fingerprint(cmd + off, cmd_len[j]);
          e.hi = pos;
        } else {
          u8 b[16];
          memset(b, 0, sizeof(b));
          if (cmd_len[j]) memcpy(b, cmd + off, cmd_len[j]);
          memcpy(&e.lo, b, 8);
          memcpy(&e.hi, b + 8, 8);
        }
        off += cmd_len[j];
        ents.push_back(e);
      }
    }
    return RBE_OK;
  }
  int push_read_index(u64 cnt, const u64* replica, const u64* lo, const u64* hi) {
    if (cnt && (!lo || !hi)) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (lo[i] == 0) return RBE_E_INVALID;  // ctx.Low is never 0 (requests.go:726)
    int rc = check_replicas(cnt, replica, EXT_READ);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_READ;
      x.ctx_low = lo[i];
      x.ctx_high = hi[i];
    }
    return RBE_OK;
  }
  int request_leader_transfer(u64 cnt, const u64* replica, const u64* target) {
    if (cnt && !target) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (target[i] < 1 || target[i] > n) return RBE_E_INVALID;  // NoNode panics, raft.go:1715
    int rc = check_replicas(cnt, replica, EXT_XFER);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_XFER;
      x.xfer_target = (u8)target[i];
    }
    return RBE_OK;
  }
  int report_unreachable(u64 cnt, const u64* replica, const u64* node) {
    if (cnt && !node) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (node[i] < 1 || node[i] > n) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++) {
      ExtIn& x = rec(replica[i]);
      x.flags |= EXT_UNREACH;
      x.unreach |= (u8)(1u << (node[i] - 1));
    }
    return RBE_OK;
  }
  int report_snapshot_status(u64 cnt, const u64* replica, const u64* node, const u8* reject) {
    if (cnt && (!node || !reject)) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++)
      if (node[i] < 1 || node[i] > n) return RBE_E_INVALID;
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
  int notify_applied(u64 cnt, const u64* replica, const u64* value) {
    if (cnt && !value) return RBE_E_INVALID;
    int rc = check_replicas(cnt, replica, 0);
    if (rc) return rc;
    for (u64 i = 0; i < cnt; i++)  // applied never moves backwards (node.go:911-913)
      if (value[i] < applied[replica[i]]) return RBE_E_INVALID;
    for (u64 i = 0; i < cnt; i++) {
      const u64 r = replica[i];
      app_rep.push_back(r);
      app_val.push_back(value[i]);
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
    for (u64 i = 0; i < cnt; i++) {
      app_rep.push_back(replica[i] | (1ull << 63));
      app_val.push_back(ready[i] ? 1u : 0u);
    }
    return RBE_OK;
  }
  // Write the staged input into host-resident planes (the test-only host build;
  // the HIP engine uploads the same vectors and scatters them on device).
  // resync the applied mirror after the plane was overwritten (snapshot import)
  void resync_applied(const u64* plane, u64 first, u64 count) {
    for (u64 i = 0; i < count; i++) applied[first + i] = plane[i];
  }
  void apply_host(const Planes& P) {
    for (size_t i = 0; i < reps.size(); i++) {
      P.ext[reps[i]] = recs[i];
      P.gwake[reps[i] / n] = GW_AWAKE;  // input wakes a sleeping group
    }
    for (size_t i = 0; i < ents.size(); i++) P.in_ents[i] = ents[i];
    for (size_t i = 0; i < app_rep.size(); i++) apply_pair(P, app_rep[i], app_val[i]);
  }
};

}  // namespace rbe
