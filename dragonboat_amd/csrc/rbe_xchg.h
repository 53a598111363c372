// MI355X batched Raft step engine: replica-per-GPU mode.
//
// With rep_world > 1, replica k of group g is stepped on rank
// (g + k) % rep_world.  Every rank keeps the planes of all replicas (the
// ones it does not own are never stepped), so a round's messages can stay in
// the plane layout the step kernels read: after each round, every message,
// outbox-count word and Replicate entry that a rank's senders produced for a
// replica owned elsewhere is packed into fixed-size records, moved with one
// all-to-all (RCCL over xGMI on GPUs; gloo in the CPU tests), and scattered by
// the receiver into the same positions of its own planes.  Outbox headers are
// round-stamped (CntRow), so a remote sender that sent nothing leaves a stale
// header that reads as empty: silence needs no record and nothing is cleared.
// Record order is irrelevant: every record names its destination slot.
#pragma once
#include "rbe_fast.h"
#include "rbe_host.h"
#include "../../include/rbe.h"
#include <unordered_map>
#include <vector>

namespace rbe {

// stream ids of the exchange records
enum : u32 { XS_CNT = 0, XS_MSG = 1, XS_ENT = 2, XS_NUM = 3 };
constexpr u32 kXchgMaxWorld = 16;

struct alignas(16) XCnt {  // outbox header of sender replica g * N + s
  u64 key;                 // g * N + s
  u64 pad;
  CntRow row;
};
struct alignas(16) XMsg {  // one message of list (g, s, d) at `slot`
  u64 key;
  u64 slot;
  Msg m;
};
struct alignas(16) XEnt {  // one arena entry of sender replica g * N + s
  u64 key;                 // g * N + s
  u64 off;
  Ent e;
};
constexpr u64 kXRecBytes[XS_NUM] = {sizeof(XCnt), sizeof(XMsg), sizeof(XEnt)};
// XMsg::slot / XEnt::off of a record for the round spill heap (a list past
// maxm, entries past ecap): the rest is its granule, which lies in the
// sender rank's share of the heap (spill_alloc), free on every other rank
constexpr u64 kXSpill = 1ull << 63;

// rank that steps replica k of local group g (rep_world for a padding group
// of a compacted engine: nobody)
template <int N>
RBE_HD u32 owner_of(const Params& C, u64 g, u32 k) {
  const u64 gg = group_global(C, g);
  if (gg >= C.n_groups_glob) return C.rep_world;
  return (u32)((gg + k) % C.rep_world);
}
template <int N>
RBE_HD bool owned(const Params& C, u64 r) {
  if (C.rep_world <= 1) return true;
  return owner_of<N>(C, r / N, (u32)(r % N)) == C.rep_rank;
}

// Fixed-capacity layout (rbe_xchg_pack_fixed): every peer's chunk starts with
// this header, so the receiver learns the record counts from the data itself
// and the exchange needs no host-side count read: one all-to-all of equal
// chunks per round, capturable in a graph.
struct alignas(16) XHdr {
  u32 cnt[XS_NUM];  // records of each stream in this chunk (at most its capacity)
  u32 overflow;     // the sender had more than fit: the round takes a counted second pass
  u32 pad[12];
};
constexpr u64 kXHdrBytes = sizeof(XHdr);

// Byte offset of stream t of peer p in a pack buffer with per-peer, per-stream
// record capacities cap[t]; `hdr` header bytes open each peer's chunk (0 for
// the counted layout of rbe_xchg_pack, kXHdrBytes for the fixed one).
RBE_HD u64 xchg_chunk_bytes(const u64* cap, u64 hdr) {
  u64 per_peer = hdr;
  for (u32 i = 0; i < XS_NUM; i++) per_peer += cap[i] * kXRecBytes[i];
  return per_peer;
}
// The fixed layout's chunk of peer p in a buffer of rank `self`: every other
// peer's chunk is full size, the rank's own holds only its header (no record
// goes to oneself), so the all-to-all moves nothing it does not need
RBE_HD u64 xchg_fixed_off(const u64* cap, u32 p, u32 self) {
  const u64 cb = xchg_chunk_bytes(cap, kXHdrBytes);
  return p * cb - (p > self ? cb - kXHdrBytes : 0);
}
RBE_HD u64 xchg_region(const u64* cap, u32 p, u32 t, u64 hdr = 0, u32 self = 0) {
  u64 off = (hdr ? xchg_fixed_off(cap, p, self) : p * xchg_chunk_bytes(cap, 0)) + hdr;
  for (u32 i = 0; i < t; i++) off += cap[i] * kXRecBytes[i];
  return off;
}

// Records sender replica r (owned) produced in round `round` - 1 (parity
// `par`) for replicas owned elsewhere: its outbox header once per peer that
// owns a destination with a non-empty list, and those lists' messages and
// entries.  WRITE = false counts them into cnt[peer * XS_NUM + t]; WRITE =
// true writes them at slot base[peer * XS_NUM + t] + running index of the pack
// buffer (overflow past cap is counted, not written).
template <int N, bool WRITE>
RBE_HD void xchg_sender(const Planes& P, const Params& C, u64 r, u32 par, u32 round, u32* cnt,
                        const u32* base, u8* buf, const u64* cap, u64 hdr = 0) {
  const u64 g = r / N;
  const u32 s = (u32)(r % N);
  const CntRow row = P.cnt[par][r];
  u32 sent_to = 0;  // peers that have this header already
  for (u32 d = 0; d < N; d++) {
    if (d == s) continue;
    const u32 peer = owner_of<N>(C, g, d);
    if (peer == C.rep_rank) continue;
    const u64 gg = group_global(C, g);  // records carry global indexes
    const u64 key = (gg * N + s) * N + d;
    const u32 word = row_word(row, d, s, round);
    if (word == 0) continue;
    auto put = [&](u32 t) -> u8* {
      const u32 i = cnt[peer * XS_NUM + t]++;
      if (!WRITE) return nullptr;
      const u32 at = base[peer * XS_NUM + t] + i;
      if (at >= cap[t]) return nullptr;
      return buf + xchg_region(cap, peer, t, hdr, C.rep_rank) + (u64)at * kXRecBytes[t];
    };
    if (!((sent_to >> peer) & 1u)) {
      sent_to |= 1u << peer;
      if (u8* p = put(XS_CNT)) {
        XCnt x;
        x.key = gg * N + s;
        x.pad = 0;
        x.row = row;
        *(XCnt*)p = x;
      }
    }
    const u64 li = (g * N + s) * N + d;
    const ListView lv = list_view(P, C, par, li, word);  // local list (or its spilled block)
    const bool spl = (word & kCntSpill) != 0;
    const u64 blk = spl ? P.msgs[par][li * C.maxm].hint : 0;
    if (spl) {  // the plane slot 0 redirect record, as is
      if (u8* p = put(XS_MSG)) {
        XMsg x;
        x.key = key;
        x.slot = 0;
        x.m = P.msgs[par][li * C.maxm];
        *(XMsg*)p = x;
      }
    }
    for (u32 i = 0; i < lv.n(); i++) {
      const u32 bi = i < lv.na ? i : lv.cap - 1u - (i - lv.na);
      const Msg m = lv.base[bi];
      if (u8* p = put(XS_MSG)) {
        XMsg x;
        x.key = key;
        x.slot = spl ? kXSpill | (blk + (u64)bi * (sizeof(Msg) / 16)) : bi;
        x.m = m;
        *(XMsg*)p = x;
      }
      // the entries a Replicate carries live in the sender's arena, or past
      // it in the spill heap (msg_ents)
      const bool xe = (m.pad0 & kMsgXEnt) != 0;
      const u32 ne = msg_nent(m);
      for (u32 e = 0; e < ne; e++) {
        const u64 off = (u64)m.ent_off + e;
        if (!xe && off >= C.ecap) break;
        if (u8* p = put(XS_ENT)) {
          XEnt x;
          x.key = gg * N + s;
          x.off = xe ? kXSpill | ((u64)m.ent_off + (u64)e * (sizeof(Ent) / 16)) : off;
          x.e = xe ? spill_at<const Ent>(P, par, m.ent_off)[e] : P.arena[par][r * C.ecap + off];
          *(XEnt*)p = x;
        }
      }
    }
  }
}

// a record's global replica (or list, with `per` = N * N) key in this
// engine's local numbering (rep_compact); ~0 when it holds no such group
RBE_HD u64 xchg_local_key(const Params& C, u64 key, u64 per) {
  u64 g;
  if (!group_local(C, key / per, &g)) return ~0ull;
  return g * per + key % per;
}
RBE_HD void xchg_put_cnt(const Planes& P, const Params& C, u32 par, const XCnt& x) {
  const u64 key = xchg_local_key(C, x.key, C.n);
  if (key == ~0ull) return;
  P.cnt[par][key] = x.row;
  P.gwake[key / C.n] = GW_AWAKE;  // a message wakes the destination's group
}
RBE_HD void xchg_put_msg(const Planes& P, const Params& C, u32 par, const XMsg& x) {
  const u64 key = xchg_local_key(C, x.key, (u64)C.n * C.n);
  if (key == ~0ull) return;
  if (x.slot & kXSpill) *spill_at<Msg>(P, par, x.slot & ~kXSpill) = x.m;
  else P.msgs[par][key * (u64)C.maxm + x.slot] = x.m;
}
RBE_HD void xchg_put_ent(const Planes& P, const Params& C, u32 par, const XEnt& x) {
  const u64 key = xchg_local_key(C, x.key, C.n);
  if (key == ~0ull) return;
  if (x.off & kXSpill) *spill_at<Ent>(P, par, x.off & ~kXSpill) = x.e;
  else P.arena[par][key * C.ecap + x.off] = x.e;
}
// record i of stream t of source chunk p of a fixed-layout receive buffer, if
// the chunk holds it (returns false past the chunk's count); *overflow gets
// the chunk's overflow flag
RBE_HD bool xchg_put_fixed(const Planes& P, const Params& C, u32 par, const u8* recv,
                           const u64* cap, u32 p, u32 t, u64 i, u32* overflow) {
  const XHdr* h = (const XHdr*)(recv + xchg_fixed_off(cap, p, C.rep_rank));
  *overflow = h->overflow;
  if (i >= h->cnt[t]) return false;
  const u8* rec = recv + xchg_region(cap, p, t, kXHdrBytes, C.rep_rank) + i * kXRecBytes[t];
  if (t == XS_CNT) xchg_put_cnt(P, C, par, *(const XCnt*)rec);
  else if (t == XS_MSG) xchg_put_msg(P, C, par, *(const XMsg*)rec);
  else xchg_put_ent(P, C, par, *(const XEnt*)rec);
  return true;
}

// ------------------------------------------------ transport boundary (host)
// rbe_get_outbox / rbe_push_messages: the messages of one round in raftpb
// shape (rbe_message + rbe_entry), for replicas whose peers are stepped by
// another engine (another rank, or another host behind dragonboat's own
// transport).  Both directions reuse the exchange records above, so a pushed
// message lands in exactly the plane slot the sender's own step would have
// written.

// Sender replica r = g * N + k's messages of parity `par` as the transport
// sees them, destination by destination in ascending node id, each stream in
// the order the receiving step handles it (node.go:1030-1067 with the
// lockstep ordering of DESIGN.md §2): the Quiesce notice (node.go:873-886),
// Replicate messages (sent before persistence, node.go:897-905), the rest.
// A message's entries follow in `ents` (rbe_message.n_entries of them): a
// Replicate's with Index = LogIndex + 1 + i, a forwarded Propose's with Index
// 0 as the client proposed them (raft.go:1841-1853); their whole Cmds go to
// `cmd` back to back (when non-null).  row = the sender's outbox header of
// that round's parity, `round` the round that reads it, list(d) = host copies
// of the list to destination slot d in reading order (A, then B; a spilled
// list's from its spill heap block), ent(m, j) = entry j of message m (its
// sender's arena, or the spill heap: msg_ents); `rd` reads payload-heap record
// bytes (rbe_host.h entry_out).  Counts beyond the capacities are reported in
// *n_msg / *n_ent / *n_cmd and not written.  Returns RBE_OK or the reader's
// error (an overwritten record).
template <int N, typename LS, typename EA, typename RD>
int outbox_messages(const Params& C, u64 g, u32 k, const CntRow& row, u32 round, LS&& list,
                    EA&& ent, rbe_message* out, u32 cap, rbe_entry* ents, u32 ent_cap, u32* n_msg,
                    u32* n_ent, u8* cmd, u64 cmd_cap, u64* n_cmd, const u64* ids, RD&& rd) {
  const u64 cid = cid_of(C, g);
  u32 n = 0, ne = 0;
  u64 nc = 0;
  auto emit = [&](const Msg& m, u32 type, u32 to) {
    if (n < cap && out) {
      rbe_message& o = out[n];
      o = rbe_message{};
      Msg x = m;
      x.type = (u8)type;
      x.to = (u8)to;
      x.from = (u8)(k + 1);
      if (!(type == M_Replicate || type == M_Propose)) x.n_ent = 0;
      msg_out(x, cid, ids, N, g, o);
    }
    n++;
  };
  for (u32 d = 0; d < N; d++) {
    const u32 pc = row_word(row, d, k, round);
    if (pc & 0x8000u) {
      Msg q = mk_msg(M_Quiesce, d + 1);
      emit(q, M_Quiesce, d + 1);
    }
    if (!(pc & 0x7FFFu)) continue;
    for (const Msg& m : list(d)) {
      emit(m, m.type, d + 1);
      if (m.type != M_Replicate && m.type != M_Propose) continue;
      const bool xe = (m.pad0 & kMsgXEnt) != 0;
      for (u32 j = 0; j < msg_nent(m) && (xe || m.ent_off + j < C.ecap); j++) {
        const Ent x = ent(m, j);
        const bool room_c = cmd && nc + x.len <= cmd_cap;
        if (ents && ne < ent_cap) {
          rbe_entry& e = ents[ne];
          e = rbe_entry{};
          const int rc = entry_out(x, &e, room_c ? cmd + nc : nullptr, rd);
          if (rc) return rc;
          e.index = m.type == M_Replicate ? m.log_index + 1 + j : 0;
        } else if (room_c) {
          rbe_entry e;
          const int rc = entry_out(x, &e, cmd + nc, rd);
          if (rc) return rc;
        }
        ne++;
        nc += x.len;
      }
    }
  }
  *n_msg = n;
  *n_ent = ne;
  if (n_cmd) *n_cmd = nc;
  return RBE_OK;
}

// The inverse for one round's inbound batch: message i of group group[i]
// from node msgs[i].from (a replica this engine does not step) to node
// msgs[i].to (one it does), carrying msgs[i].n_entries entries taken in order
// from `ents` with their Cmds back to back in `cmd` (null: each entry's inline
// cmd, at most 16 bytes).  Per (sender, destination) the Replicate messages
// keep their order in the A list, the others in the B list, and a Quiesce
// message sets the notice bit, exactly the layout a local sender's step
// writes.  Replicate and forwarded Propose messages carry entries (raft.go:
// 1841-1853); entries with Cmds over 16 bytes or session fields are staged in
// this engine's payload heap.  Each sender named gets one outbox header
// stamped for `round` (the round that reads them); a sender not named keeps a
// stale header, which reads as empty.  Checked whole before anything is
// staged: RBE_OK, RBE_E_INVALID (ids, ownership, entry indexes or types) or
// RBE_E_NOMEM (more than maxm messages in one list, more than ecap entries
// from one sender, or no heap room).
template <int N>
int messages_to_records(const Params& C, HostHeap& heap, u32 round, u64 n, const u64* group,
                        const rbe_message* msgs, const rbe_entry* ents, const u8* cmd,
                        std::vector<XCnt>& oc, std::vector<XMsg>& om, std::vector<XEnt>& oe,
                        const u64* ids = nullptr) {
  u64 total = 0;
  for (u64 i = 0; i < n; i++) total += msgs[i].n_entries;
  if (total && !ents) return RBE_E_INVALID;
  u64 need = 0;
  int rc = check_entries(heap, total, ents, cmd, true, &need);
  if (rc) return rc;
  auto pass = [&](bool write) -> int {
    std::unordered_map<u64, u32> words;  // list key → count word
    std::vector<u64> order;              // list keys in first-use order
    std::unordered_map<u64, u32> used;   // sender replica → arena entries used
    u64 ei = 0, coff = 0;
    for (u64 i = 0; i < n; i++) {
      rbe_message m = msgs[i];
      const u64 g = group[i];
      if (ids && g < C.n_groups) {  // node ids → internal ids (rbe_set_node_ids)
        m.from = int_id<N>(ids, g, m.from);
        m.to = int_id<N>(ids, g, m.to);
        if (hint_is_node(m.type)) m.hint = int_id<N>(ids, g, m.hint);
      }
      // Peer.Handle (peer.go:186-198): a local message type is a caller bug (the
      // reference panics); a response from a node that is not a member of the
      // group is dropped.  Other messages from non-members cannot be held by a
      // slot-indexed group and are refused.
      if (m.type >= 26 || is_local_message(m.type)) return RBE_E_INVALID;
      if ((m.from < 1 || m.from > N) && is_response_message(m.type) && m.n_entries == 0) continue;
      if (g >= C.n_groups || m.from < 1 || m.from > N || m.to < 1 || m.to > N || m.from == m.to)
        return RBE_E_INVALID;
      const u32 s = (u32)m.from - 1u, d = (u32)m.to - 1u;
      if (owner_of<N>(C, g, s) == C.rep_rank || owner_of<N>(C, g, d) != C.rep_rank)
        return RBE_E_INVALID;
      const u64 key = (group_global(C, g) * N + s) * N + d;  // records carry global indexes
      auto it = words.find(key);
      if (it == words.end()) {
        it = words.emplace(key, 0u).first;
        order.push_back(key);
      }
      u32& w = it->second;
      if (m.type == M_Quiesce) {
        if (m.n_entries) return RBE_E_INVALID;
        w |= 0x8000u;
        continue;
      }
      const bool with_ents = m.type == M_Replicate || m.type == M_Propose;
      if (m.n_entries && !with_ents) return RBE_E_INVALID;
      const u32 na = w & 0x7Fu, nb = (w >> 7) & 0x7Fu;
      if (na + nb >= C.maxm) return RBE_E_NOMEM;
      XMsg x;
      x.key = key;
      x.m = mk_msg(m.type, m.to);
      x.m.from = (u8)m.from;
      x.m.reject = (u8)(m.reject ? 1 : 0);
      x.m.term = m.term;
      x.m.log_term = m.log_term;
      x.m.log_index = m.log_index;
      x.m.commit = m.commit;
      x.m.hint = m.hint;
      x.m.hint_high = m.hint_high;
      // an InstallSnapshot's snapshot membership (rbe_message.reserved, msg_reserved)
      if (m.type == M_InstallSnapshot) {
        if (!ms_valid(m.reserved, N)) return RBE_E_INVALID;
        x.m.pad0 = (u16)(m.reserved & 0xFFu);
        x.m.pad1 = (m.reserved >> 8) & 0xFFFFu;
      }
      if (m.type == M_Replicate) {
        x.slot = na;
        w += 1u;
      } else {
        x.slot = C.maxm - 1u - nb;
        w += 1u << 7;
      }
      if (with_ents && m.n_entries) {
        const u64 sr = group_global(C, g) * N + s;
        u32& off = used[sr];
        if (m.n_entries > 0xFFFFu || off + m.n_entries > C.ecap) return RBE_E_NOMEM;
        x.m.n_ent = (u16)m.n_entries;
        x.m.ent_off = off;
        for (u32 j = 0; j < m.n_entries; j++, ei++) {
          const rbe_entry& e = ents[ei];
          if (m.type == M_Replicate && e.index != m.log_index + 1 + j) return RBE_E_INVALID;
          const u8* cb = cmd ? cmd + coff : e.cmd;
          coff += cmd ? e.cmd_len : 0;
          if (!write) continue;
          XEnt y;
          y.key = sr;
          y.off = off + j;
          y.e = stage_entry(heap, e, cb);
          oe.push_back(y);
        }
        off += m.n_entries;
      }
      if (write) om.push_back(x);
    }
    if (!write) return RBE_OK;
    // one stamped header per sender with the words of all its lists
    std::unordered_map<u64, size_t> hdr;  // sender replica → index in oc
    for (u64 key : order) {
      const u64 sr = key / N;
      const u32 d = (u32)(key % N);
      auto it = hdr.find(sr);
      if (it == hdr.end()) {
        XCnt c;
        c.key = sr;
        c.pad = 0;
        c.row.stamp = round;
        for (int w = 0; w < 6; w++) c.row.w[w] = 0;
        it = hdr.emplace(sr, oc.size()).first;
        oc.push_back(c);
      }
      oc[it->second].row.w[cnt_widx(d, (u32)(sr % N))] = (u16)words[key];
    }
    return RBE_OK;
  };
  if ((rc = pass(false))) return rc;
  if (need && (rc = heap.room(need))) return rc;
  return pass(true);
}

}  // namespace rbe
