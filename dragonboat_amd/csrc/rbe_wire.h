// rbe_wire.h — the transport's wire format over the engine's outbox planes,
// shared by the device codec (rbe_wire_kernels.h) and the test-only host build.
//
// What a dragonboat node puts on a TCP connection for Raft traffic
// (internal/transport/tcp.go:149-185 writeMessage): the 2-byte magic 0xAE7D,
// an 18-byte requestHeader (method 100, payload size, header crc32, payload
// crc32; big endian; tcp.go:80-91), then a marshaled raftpb.MessageBatch
// (raft.pb.go:2415-2443): its Requests as protobuf Messages (2230-2294), each
// embedding a Snapshot (2140-2217) and its log entries in colfer form
// (raftpb/raft_optimized.go:161-295), then DeploymentId, SourceAddress, BinVer.
//
// The engine's frame is one MessageBatch per (sender slot k, destination slot
// d, range of `groups_per_batch` groups): every message the replicas k of
// those groups sent to their replicas d in the last round, group by group, each
// replica's in transport order (Quiesce notice, Replicate, the rest; the order
// rbe_get_outbox reports).  InstallSnapshot messages never travel in a
// MessageBatch (transport.go:400-403: they go through the snapshot chunk
// stream), so they are counted and left out.  Entries carry every field:
// Index, Term, Type, the session fields and Cmd (a payload-heap record's from
// the heap, rbe_types.h ET_HEAP); a Replicate's are numbered LogIndex + 1 + i,
// a forwarded Propose's keep Index 0 (raft.go:1841-1853).
//
// One function, wire_cell, both sizes and writes a (group, k, d) cell, so the
// size pass and the write pass cannot disagree.
#pragma once

#include "rbe_step.h"

namespace rbe {

static constexpr u32 kWireHeader = 20;  // magic + requestHeader
static constexpr u32 kWireMethod = 100;  // tcp.go raftType
static constexpr u32 kWireCrcPoly = 0xEDB88320u;

RBE_HD u32 wsov(u64 x) {  // sovRaft (raft.pb.go:2879-2887)
  u32 n = 1;
  while (x >= 0x80) {
    x >>= 7;
    n++;
  }
  return n;
}
RBE_HD u32 wput(u8* o, u64 x) {  // encodeVarintRaft (raft.pb.go:2559-2567)
  u32 i = 0;
  while (x >= 0x80) {
    o[i++] = (u8)(x | 0x80);
    x >>= 7;
  }
  o[i++] = (u8)x;
  return i;
}
// colfer u64 field (raft_optimized.go:164-178): absent when 0, 9 bytes from 2^49
RBE_HD u32 colfer_u64_size(u64 x) { return x >= (1ull << 49) ? 9u : (x ? 1u + wsov(x) : 0u); }
RBE_HD u32 colfer_u64_put(u8* o, u32 field, u64 x) {
  if (x >= (1ull << 49)) {
    o[0] = (u8)(field | 0x80);
    for (u32 b = 0; b < 8; b++) o[1 + b] = (u8)(x >> (56 - 8 * b));
    return 9;
  }
  if (!x) return 0;
  o[0] = (u8)field;
  return 1 + wput(o + 1, x);
}
// Entry.Size (raft_optimized.go:79-153); meta = {Key, ClientID, SeriesID,
// RespondedTo}
RBE_HD u32 wire_entry_size(u64 index, u64 term, u32 type, const u64* meta, u32 len) {
  u32 l = 1 + colfer_u64_size(term) + colfer_u64_size(index);
  if (type) l += 1 + wsov(type);
  for (u32 f = 0; f < 4; f++) l += colfer_u64_size(meta[f]);
  if (len) l += 1 + wsov(len) + len;
  return l;
}
// The wire view of an arena entry: its session fields and where its Cmd bytes
// are (the inline lo/hi words in `inl`, or the heap record after its header)
struct WireEnt {
  u64 meta[4];
  u8 inl[16];
  const u8* cmd;
};
RBE_HD void wire_ent_view(const Ent& x, const u8* heap, u64 heap_cap, WireEnt& v) {
  if (ent_heap(x.type) && heap_cap) {
    const u8* rec = heap + x.hi % heap_cap;
    const u64* h = (const u64*)rec;  // records are 16-B aligned
    for (u32 f = 0; f < 4; f++) v.meta[f] = h[f];
    v.cmd = rec + kHeapHdr;
  } else {
    for (u32 f = 0; f < 4; f++) v.meta[f] = 0;
    for (u32 b = 0; b < 16; b++) v.inl[b] = (u8)((b < 8 ? x.lo : x.hi) >> (8 * (b & 7)));
    v.cmd = v.inl;
  }
}
// Entry.marshalTo (raft_optimized.go:161-295)
RBE_HD u32 wire_entry_put(u8* o, u64 index, u64 term, u32 type, const WireEnt& v, u32 len) {
  u32 i = colfer_u64_put(o, 0, term);
  i += colfer_u64_put(o + i, 1, index);
  if (type) {
    o[i++] = 2;
    i += wput(o + i, type);
  }
  for (u32 f = 0; f < 4; f++) i += colfer_u64_put(o + i, 3 + f, v.meta[f]);
  if (len) {
    o[i++] = 7;
    i += wput(o + i, len);
    for (u32 b = 0; b < len; b++) o[i + b] = v.cmd[b];
    i += len;
  }
  o[i++] = 0x7F;
  return i;
}

// The Snapshot embedded in every MessageBatch message (no InstallSnapshot
// travels there): Filepath "", FileSize 0, Index 0, Term 0, Membership
// {ConfigChangeId 0}, Dummy, ClusterId, Type, Imported, OnDiskIndex, Witness.
static constexpr u32 kWireEmptySnap = 24;
RBE_HD u32 wire_empty_snap_put(u8* o) {
  const u8 b[kWireEmptySnap] = {0x12, 0, 0x18, 0, 0x20, 0, 0x28, 0, 0x32, 2, 0x08, 0,
                                0x48, 0, 0x50, 0, 0x58, 0, 0x60, 0, 0x68, 0, 0x70, 0};
  for (u32 i = 0; i < kWireEmptySnap; i++) o[i] = b[i];
  return kWireEmptySnap;
}

// Message.MarshalTo (raft.pb.go:2230-2294) of one outbox message, as a
// MessageBatch request (tag 0x0a + length); `out` null = size only.  An entry
// whose heap record a later lap overwrote (position below heap_head - cap)
// counts in *n_bad and is encoded from whatever the heap holds: the caller
// refuses the whole encode then.
RBE_HD u32 wire_message(const Msg& m, u32 type, u64 to, u64 from, u64 cid, const Ent* ents,
                        const u8* heap, u64 heap_cap, u64 heap_head, u8* out, u32* n_bad) {
  const u32 ne = type == M_Replicate || type == M_Propose ? msg_nent(m) : 0u;
  u32 body = 1 + wsov(type) + 1 + wsov(to) + 1 + wsov(from) + 1 + wsov(cid) + 1 + wsov(m.term) +
             1 + wsov(m.log_term) + 1 + wsov(m.log_index) + 1 + wsov(m.commit) + 2 + 1 +
             wsov(m.hint) + 1 + 1 + kWireEmptySnap + 1 + wsov(m.hint_high);
  for (u32 j = 0; j < ne; j++) {
    const Ent& x = ents[j];
    const u64 idx = type == M_Replicate ? m.log_index + 1 + j : 0;
    WireEnt v;
    wire_ent_view(x, heap, heap_cap, v);
    if (ent_heap(x.type) && (!heap_cap || x.hi + heap_cap < heap_head)) (*n_bad)++;
    const u32 es = wire_entry_size(idx, x.term, ent_type(x.type), v.meta, x.len);
    body += 1 + wsov(es) + es;
  }
  const u32 total = 1 + wsov(body) + body;
  if (!out) return total;
  u32 i = 0;
  out[i++] = 0x0A;
  i += wput(out + i, body);
  out[i++] = 0x08;
  i += wput(out + i, type);
  out[i++] = 0x10;
  i += wput(out + i, to);
  out[i++] = 0x18;
  i += wput(out + i, from);
  out[i++] = 0x20;
  i += wput(out + i, cid);
  out[i++] = 0x28;
  i += wput(out + i, m.term);
  out[i++] = 0x30;
  i += wput(out + i, m.log_term);
  out[i++] = 0x38;
  i += wput(out + i, m.log_index);
  out[i++] = 0x40;
  i += wput(out + i, m.commit);
  out[i++] = 0x48;
  out[i++] = m.reject ? 1 : 0;
  out[i++] = 0x50;
  i += wput(out + i, m.hint);
  for (u32 j = 0; j < ne; j++) {
    const Ent& x = ents[j];
    const u64 idx = type == M_Replicate ? m.log_index + 1 + j : 0;
    WireEnt v;
    wire_ent_view(x, heap, heap_cap, v);
    out[i++] = 0x5A;
    i += wput(out + i, wire_entry_size(idx, x.term, ent_type(x.type), v.meta, x.len));
    i += wire_entry_put(out + i, idx, x.term, ent_type(x.type), v, x.len);
  }
  out[i++] = 0x62;
  out[i++] = (u8)kWireEmptySnap;
  i += wire_empty_snap_put(out + i);
  out[i++] = 0x68;
  i += wput(out + i, m.hint_high);
  return i;
}

// The requests replica (g, k) sent replica (g, d) in the round that produced
// header `row` (written as round `round` - 1, parity (round - 1) & 1): their
// bytes (written at `out` unless null); *n_msgs / *n_is count the messages
// encoded and the InstallSnapshots left out, *n_bad the entries whose heap
// record is gone (rbe_wire_encode fails then).
template <int N>
RBE_HD u32 wire_cell(const Planes& P, const Params& C, const u8* heap, u64 heap_head, u64 g, u32 k,
                     u32 d, u32 round, u8* out, u32* n_msgs, u32* n_is, u32* n_bad) {
  const u32 par = (round - 1u) & 1u;
  const u64 r = g * N + k;
  const u64 cid = cid_of(C, g);
  const u32 pc = row_word(P.cnt[par][r], d, k, round);
  u32 bytes = 0, nm = 0, ni = 0, bad = 0;
  // Message.To / From (and a RequestVote's / LeaderTransfer's Hint) as node ids
  const u64 to_id = ext_id(P.node_ids, N, g, d + 1), from_id = ext_id(P.node_ids, N, g, k + 1);
  if (pc & 0x8000u) {  // sendEnterQuiesceMessages (node.go:873-886)
    Msg q;
    q.type = (u8)M_Quiesce;
    q.from = q.to = q.reject = 0;
    q.n_ent = 0;
    q.pad0 = 0;
    q.ent_off = q.pad1 = 0;
    q.term = q.log_term = q.log_index = q.commit = q.hint = q.hint_high = 0;
    bytes += wire_message(q, M_Quiesce, to_id, from_id, cid, nullptr, heap, C.heap_bytes,
                          heap_head, out ? out + bytes : nullptr, &bad);
    nm++;
  }
  // (the plane list or, past maxm, the spill heap's: rbe_spill.h)
  const ListView lst = list_view(P, C, par, r * N + d, pc);
  for (u32 i = 0; i < lst.n(); i++) {
    Msg m = lst.at(i);
    if (m.type == M_InstallSnapshot) {
      ni++;
      continue;
    }
    const Ent* ents = msg_ents(P, C, par, r, m);
    if (hint_is_node(m.type)) m.hint = ext_id(P.node_ids, N, g, m.hint);
    bytes += wire_message(m, m.type, to_id, from_id, cid, ents, heap, C.heap_bytes,
                          heap_head, out ? out + bytes : nullptr, &bad);
    nm++;
  }
  *n_msgs = nm;
  *n_is = ni;
  *n_bad = bad;
  return bytes;
}

// MessageBatch trailer (raft.pb.go:2432-2441): DeploymentId, SourceAddress, BinVer
RBE_HD u32 wire_trailer(u64 deployment_id, const u8* addr, u32 addr_len, u32 bin_ver, u8* out) {
  const u32 n = 1 + wsov(deployment_id) + 1 + wsov(addr_len) + addr_len + 1 + wsov(bin_ver);
  if (!out) return n;
  u32 i = 0;
  out[i++] = 0x10;
  i += wput(out + i, deployment_id);
  out[i++] = 0x1A;
  i += wput(out + i, addr_len);
  for (u32 b = 0; b < addr_len; b++) out[i++] = addr[b];
  out[i++] = 0x20;
  i += wput(out + i, bin_ver);
  return i;
}

// ---------------------------------------------------------------- crc32 (IEEE)
// crc32.ChecksumIEEE; segments are combined with zlib's crc32_combine
// (multmodp / x2nmodp over the reflected polynomial).
RBE_HD u32 crc_table_entry(u32 i) {
  u32 c = i;
  for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ kWireCrcPoly : c >> 1;
  return c;
}
RBE_HD u32 crc32_update(u32 crc, const u8* p, u64 n, const u32* table) {
  u32 c = ~crc;
  for (u64 i = 0; i < n; i++) c = table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return ~c;
}
RBE_HD constexpr u32 crc_multmodp(u32 a, u32 b) {
  u32 m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1u)) == 0) break;
    }
    m >>= 1;
    b = (b & 1u) ? (b >> 1) ^ kWireCrcPoly : b >> 1;
  }
  return p;
}
// x2n[k] = x^(2^k) mod P, evaluated at compile time
struct CrcX2n {
  u32 v[32];
};
constexpr CrcX2n crc_x2n_make() {
  CrcX2n t{};
  t.v[0] = 1u << 30;
  for (int k = 1; k < 32; k++) t.v[k] = crc_multmodp(t.v[k - 1], t.v[k - 1]);
  return t;
}
static constexpr CrcX2n kCrcX2n = crc_x2n_make();
RBE_HD u32 crc32_combine(u32 crc1, u32 crc2, u64 len2, const u32* x2n) {
  u32 p = 1u << 31;  // x^(8 len2) mod P
  u32 k = 3;
  while (len2) {
    if (len2 & 1u) p = crc_multmodp(x2n[k & 31], p);
    len2 >>= 1;
    k++;
  }
  return crc_multmodp(p, crc1) ^ crc2;
}
// requestHeader.encode (tcp.go:80-91) after the magic, for a payload of
// `size` bytes with crc32 `pcrc`
RBE_HD void wire_header_put(u8* o, u64 size, u32 pcrc, const u32* table) {
  o[0] = 0xAE;
  o[1] = 0x7D;
  u8* h = o + 2;
  h[0] = (u8)(kWireMethod >> 8);
  h[1] = (u8)kWireMethod;
  for (u32 b = 0; b < 8; b++) h[2 + b] = (u8)(size >> (56 - 8 * b));
  for (u32 b = 0; b < 4; b++) h[10 + b] = 0;
  for (u32 b = 0; b < 4; b++) h[14 + b] = (u8)(pcrc >> (24 - 8 * b));
  const u32 hc = crc32_update(0, h, 18, table);
  for (u32 b = 0; b < 4; b++) h[10 + b] = (u8)(hc >> (24 - 8 * b));
}

// ---------------------------------------------------------------- decode
// sequential reader over one frame's payload
struct WireRd {
  const u8* p;
  u64 n, i;
  bool bad;
  RBE_HD u8 byte() {
    if (i >= n) {
      bad = true;
      return 0;
    }
    return p[i++];
  }
  RBE_HD u64 varint() {  // protobuf varint (Message.Unmarshal)
    u64 x = 0;
    for (u32 s = 0; s < 64; s += 7) {
      const u8 b = byte();
      x |= (u64)(b & 0x7F) << s;
      if (b < 0x80 || bad) return x;
    }
    bad = true;
    return x;
  }
  // skipRaft (raft.pb.go): a length or fixed width past the end is
  // ErrInvalidLength / io.ErrUnexpectedEOF; compared as "l > n - i" so a
  // length near 2^64 cannot wrap the position
  RBE_HD void advance(u64 l) {
    if (i > n || l > n - i) {
      bad = true;
      i = n;
    } else {
      i += l;
    }
  }
  RBE_HD void skip(u32 wt) {
    if (wt == 0) varint();
    else if (wt == 1) advance(8);
    else if (wt == 2) advance(varint());
    else if (wt == 5) advance(4);
    else bad = true;
  }
};

// Entry.unmarshal (raft_optimized.go:303-651) of [rd.i, end)
RBE_HD void wire_entry_get(WireRd& rd, u64 end, rbe_entry* e, u8* cmd) {
  u64 vals[7] = {0, 0, 0, 0, 0, 0, 0};
  u8 h = rd.byte();
  for (u32 f = 0; f < 7; f++) {
    if (h == f) {
      u64 x = 0;
      if (f == 2) {
        x = rd.varint();
      } else {
        for (u32 s = 0;; s += 7) {
          const u8 b = rd.byte();
          if (b < 0x80 || s == 56) {
            x |= (u64)b << s;
            break;
          }
          x |= (u64)(b & 0x7F) << s;
        }
      }
      vals[f] = x;
      h = rd.byte();
    } else if (h == (f | 0x80)) {
      u64 x = 0;
      if (f == 2) {
        x = (u64)(u32)(0u - (u32)rd.varint());
      } else {
        for (int b = 0; b < 8; b++) x = (x << 8) | rd.byte();
      }
      vals[f] = x;
      h = rd.byte();
    }
  }
  u32 len = 0;
  if (h == 7) {
    const u64 l = rd.varint();
    if (rd.i > end || l > end - rd.i) rd.bad = true;
    len = rd.bad ? 0u : (u32)l;
    for (u32 b = 0; b < len && !rd.bad; b++) {
      const u8 x = rd.byte();
      if (cmd) cmd[b] = x;
      if (e && b < 16) e->cmd[b] = x;
    }
    h = rd.byte();
  }
  if (h != 0x7F || rd.i != end) rd.bad = true;
  if (e) {
    e->term = vals[0];
    e->index = vals[1];
    e->type = (u32)vals[2];
    e->cmd_len = len;
    e->key = vals[3];
    e->client_id = vals[4];
    e->series_id = vals[5];
    e->responded_to = vals[6];
  }
}

// Message.Unmarshal (raft_optimized.go:654-979) of [rd.i, end); entries to
// ents[0..] and their Cmds to cmd[cmd_at..]; returns entries, *cmd_at advanced
RBE_HD u32 wire_message_get(WireRd& rd, u64 end, rbe_message* m, rbe_entry* ents, u8* cmd,
                            u64* cmd_at) {
  u64 f[14] = {0};
  u32 ne = 0;
  while (rd.i < end && !rd.bad) {
    const u64 tag = rd.varint();
    const u32 fn = (u32)(tag >> 3), wt = (u32)(tag & 7);
    if (fn >= 1 && fn <= 13 && fn != 11 && fn != 12 && wt == 0) {
      f[fn] = rd.varint();
    } else if (fn == 11 && wt == 2) {
      const u64 l = rd.varint();
      if (rd.bad || rd.i > end || l > end - rd.i) {
        rd.bad = true;
        break;
      }
      const u64 e_end = rd.i + l;
      // Cmd length first (the colfer walk below writes at cmd + *cmd_at)
      rbe_entry tmp;
      rbe_entry* e = ents ? &ents[ne] : &tmp;
      for (int b = 0; b < 16; b++) e->cmd[b] = 0;
      wire_entry_get(rd, e_end, e, cmd ? cmd + *cmd_at : nullptr);
      *cmd_at += e->cmd_len;
      ne++;
    } else {
      rd.skip(wt);  // the embedded Snapshot included: no InstallSnapshot here
    }
  }
  if (rd.i != end) rd.bad = true;
  if (m) {
    m->type = (u32)f[1];
    m->to = f[2];
    m->from = f[3];
    m->cluster_id = f[4];
    m->term = f[5];
    m->log_term = f[6];
    m->log_index = f[7];
    m->commit = f[8];
    m->reject = f[9] != 0;
    m->hint = f[10];
    m->hint_high = f[13];
    m->n_entries = ne;
    m->reserved = 0;
  }
  return ne;
}

}  // namespace rbe
