// rbe_ingest.h — inbound MessageBatches straight into the plane slots
// (rbe_wire_ingest, SURVEY.md §8f rank 3: "inbound batches land directly in
// SoA").  The records rbe_wire_decode parses on the device are checked and
// scattered on the device too, into the inbox lists a local sender's step
// would have written: per (sender, destination) the Replicate messages in
// stream order at the front of the list, the rest at the back, the Quiesce
// notice bit, one round-stamped outbox header per sender named, the carried
// entries in the sender's arena, and the payload-heap records of entries with
// long Cmds or session fields.  This is Peer.Handle for remote senders
// (peer.go:186-198 via node.handleReceivedMessages, node.go:1030-1067; the
// transport's receive side, transport.go:318-350 handleRequest) with the same
// rules as rbe_push_messages (rbe_xchg.h messages_to_records), which remains
// the host-memory entry point.
//
// Pipeline (rbe_engine.hip rbe_wire_ingest):
//   decode           the rbe_wire_decode kernels, records left on the device
//   k_ing_key        lane per message: Peer.Handle filter + checks, list key,
//                    payload-heap bytes its entries need
//   radix sort       (list key, message index) pairs, stable: per list the
//                    stream order is kept
//   k_ing_walk<0>    lane per sender run: list capacities (maxm, ecap)
//   host             one read-back: errors, heap bytes → HostHeap::room
//   k_ing_walk<1>    lane per sender run: slots, entries, heap records, header
// All integer/byte work; HBM bound, no MFMA.  The same functions run on the
// host in the CPU test tier (tests/soa_cpu).
#pragma once
#include "rbe_xchg.h"

namespace rbe {

enum : u32 { ING_INVALID = 1u, ING_NOMEM = 2u };

// Does rbe_wire_encode put cell (g, k → d) on the wire?  Every cell with one
// replica set per engine; in replica mode (rep_world > 1) only the cells whose
// sender is stepped here and whose receiver is stepped elsewhere — by rank
// dst_rank when it is not negative (one stream per destination engine, as a
// transport keeps one connection per remote NodeHost, transport.go:400-441).
template <int N>
RBE_HD bool wire_cell_sent(const Params& C, int dst_rank, u64 g, u32 k, u32 d) {
  if (C.rep_world <= 1) return true;
  const u32 od = owner_of<N>(C, g, d);
  return owner_of<N>(C, g, k) == C.rep_rank && od != C.rep_rank &&
         (dst_rank < 0 || od == (u32)dst_rank);
}

// Sort key of a message that is dropped (a response from a node that is not a
// member of the group, as Peer.Handle drops it): past every list key.
RBE_HD u64 ing_drop_key(const Params& C) { return C.n_rep * (u64)C.n; }

// A decoded message's node ids (From, To, a RequestVote's / LeaderTransfer's
// Hint) as internal ids of the group its ClusterId names (rbe_set_node_ids;
// 0 = none of the group's slots, which ingest_check then drops or refuses)
template <int N>
RBE_HD void ingest_ids(const Params& C, const u64* ids, rbe_message& m) {
  if (!ids) return;
  const u64 cid = m.cluster_id, st = C.cid_stride ? C.cid_stride : 1;
  u64 g = 0;
  if (cid < C.cid_base || (cid - C.cid_base) % st != 0 ||
      !group_local(C, (cid - C.cid_base) / st, &g))
    return;  // refused by ingest_check
  m.from = int_id<N>(ids, g, m.from);
  m.to = int_id<N>(ids, g, m.to);
  if (hint_is_node(m.type)) m.hint = int_id<N>(ids, g, m.hint);
}

// Peer.Handle's filter and rbe_push_messages's checks for decoded message m
// (its entries at `ents`): the list key (g * N + from - 1) * N + to - 1, or
// the drop key; *err gets ING_INVALID / ING_NOMEM, *heap the payload-heap
// bytes its entries take (heap_rec_bytes per entry that needs a record).
// The group comes from Message.ClusterId (group g is cluster cid_base + g *
// cid_stride, as every engine API names it).
template <int N>
RBE_HD u64 ingest_check(const Params& C, u64 heap_cap, const rbe_message& m, const rbe_entry* ents,
                        u32* err, u64* heap) {
  *heap = 0;
  const u64 drop = ing_drop_key(C);
  if (m.type >= 26 || is_local_message(m.type)) {  // a local type is a caller bug (panics)
    *err |= ING_INVALID;
    return drop;
  }
  if ((m.from < 1 || m.from > N) && is_response_message(m.type) && m.n_entries == 0) return drop;
  const u64 cid = m.cluster_id;
  const u64 st = C.cid_stride ? C.cid_stride : 1;
  u64 g = 0;  // the local group of global group (cid - cid_base) / stride
  if (cid < C.cid_base || (cid - C.cid_base) % st != 0 ||
      !group_local(C, (cid - C.cid_base) / st, &g) || m.from < 1 || m.from > N || m.to < 1 ||
      m.to > N || m.from == m.to) {
    *err |= ING_INVALID;
    return drop;
  }
  const u32 s = (u32)m.from - 1u, d = (u32)m.to - 1u;
  if (owner_of<N>(C, g, s) == C.rep_rank || owner_of<N>(C, g, d) != C.rep_rank) {
    *err |= ING_INVALID;
    return drop;
  }
  const bool with_ents = m.type == M_Replicate || m.type == M_Propose;
  if (m.n_entries && (!with_ents || m.type == M_Quiesce)) {
    *err |= ING_INVALID;
    return drop;
  }
  if (m.n_entries > 0xFFFFu || m.n_entries > C.ecap) {
    *err |= ING_NOMEM;
    return drop;
  }
  u64 hb = 0;
  for (u32 j = 0; j < m.n_entries; j++) {
    const rbe_entry& e = ents[j];
    if (e.type > E_Metadata || (m.type == M_Replicate && e.index != m.log_index + 1 + j)) {
      *err |= ING_INVALID;
      return drop;
    }
    if (!entry_needs_heap(e)) continue;
    // a heap record takes at most a quarter of the heap (check_entries)
    if (heap_cap == 0 || e.cmd_len > heap_cap / 4) {
      *err |= ING_INVALID;
      return drop;
    }
    hb += heap_rec_bytes(e.cmd_len);
  }
  *heap = hb;
  return ((g * N + s) * N + d);
}

// One sender's run [p0, p1) of the sorted messages (every key of the run has
// the same sender replica sr = key / N; keys ascending, stream order within a
// key).  WRITE = false checks the list capacities only; WRITE = true builds
// the lists exactly as messages_to_records does and writes them into parity
// `par`: each message at its slot, its entries at the sender's next arena
// offsets, heap records at base + hscan[p] (16-B aligned, the batch's region
// does not cross the end of the ring), and the sender's outbox header stamped
// `round` with the count words of the lists named (0 for the others).
// Returns ING_NOMEM when a list would hold more than maxm messages or the
// sender more than ecap entries.
template <int N, bool WRITE>
RBE_HD u32 ingest_sender(const Planes& P, const Params& C, u32 par, u32 round, const u64* skey,
                         const u32* sidx, u64 p0, u64 p1, const rbe_message* msgs,
                         const rbe_entry* ents, const u64* ent0, const u64* cmd0, const u8* cmd,
                         u8* heap, u64 heap_cap, u64 base, const u64* hscan) {
  const u64 sr = skey[p0] / N;
  u32 words[N];
  for (int d = 0; d < N; d++) words[d] = 0;
  u32 used = 0;
  for (u64 p = p0; p < p1; p++) {
    const u64 key = skey[p];
    const u32 d = (u32)(key % N);
    const u32 j = sidx[p];
    const rbe_message& m = msgs[j];
    u32& w = words[d];
    if (m.type == M_Quiesce) {
      w |= 0x8000u;
      continue;
    }
    const u32 na = w & 0x7Fu, nb = (w >> 7) & 0x7Fu;
    if (na + nb >= C.maxm) return ING_NOMEM;
    u32 slot;
    if (m.type == M_Replicate) {
      slot = na;
      w += 1u;
    } else {
      slot = C.maxm - 1u - nb;
      w += 1u << 7;
    }
    const u32 ne = m.n_entries;
    if (ne && used + ne > C.ecap) return ING_NOMEM;
    if (!WRITE) {
      used += ne;
      continue;
    }
    Msg x = mk_msg(m.type, (u32)m.to);
    x.from = (u8)m.from;
    x.reject = (u8)(m.reject ? 1 : 0);
    x.term = m.term;
    x.log_term = m.log_term;
    x.log_index = m.log_index;
    x.commit = m.commit;
    x.hint = m.hint;
    x.hint_high = m.hint_high;
    if (ne) {
      x.n_ent = (u16)ne;
      x.ent_off = used;
      u64 hpos = base + hscan[p];
      const u8* cb = cmd + cmd0[j];
      for (u32 i = 0; i < ne; i++) {
        const rbe_entry& e = ents[ent0[j] + i];
        Ent y;
        y.term = e.term;
        y.type = e.type & ET_TYPE_MASK;
        y.len = e.cmd_len;
        if (entry_needs_heap(e)) {
          // the record {Key, ClientID, SeriesID, RespondedTo, Cmd} (HostHeap::put_record)
          const u64 meta[4] = {e.key, e.client_id, e.series_id, e.responded_to};
          u8* rec = heap + hpos % heap_cap;
          for (int q = 0; q < 4; q++) ((u64*)rec)[q] = meta[q];
          for (u32 b = 0; b < e.cmd_len; b++) rec[kHeapHdr + b] = cb[b];
          y.type |= ET_HEAP;
          y.lo = entry_fingerprint(meta, cb, e.cmd_len);
          y.hi = hpos;
          hpos += heap_rec_bytes(e.cmd_len);
        } else {
          u64 lo = 0, hi = 0;
          for (u32 b = 0; b < e.cmd_len && b < 16; b++) {
            if (b < 8) lo |= (u64)cb[b] << (8 * b);
            else hi |= (u64)cb[b] << (8 * (b - 8));
          }
          y.lo = lo;
          y.hi = hi;
        }
        P.arena[par][sr * C.ecap + used + i] = y;
        cb += e.cmd_len;
      }
      used += ne;
    }
    P.msgs[par][key * (u64)C.maxm + slot] = x;
  }
  if (WRITE) {
    CntRow row;
    row.stamp = round;
    for (int q = 0; q < 6; q++) row.w[q] = 0;
    for (int d = 0; d < N; d++)
      if ((u32)d != (u32)(sr % N)) row.w[cnt_widx((u32)d, (u32)(sr % N))] = (u16)words[d];
    P.cnt[par][sr] = row;
    P.gwake[sr / N] = GW_AWAKE;  // a message wakes the destination's group
  }
  return 0;
}

// Is sorted position p the first of its sender's run (and not dropped)?
RBE_HD bool ingest_run_start(const Params& C, const u64* skey, u64 p) {
  if (skey[p] >= ing_drop_key(C)) return false;
  return p == 0 || skey[p - 1] / C.n != skey[p] / C.n;
}
// end of the run that starts at p
RBE_HD u64 ingest_run_end(const Params& C, const u64* skey, u64 p, u64 n) {
  const u64 sr = skey[p] / C.n;
  u64 q = p + 1;
  while (q < n && skey[q] / C.n == sr) q++;
  return q;
}

}  // namespace rbe
