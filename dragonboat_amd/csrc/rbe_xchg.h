// MI355X batched Raft step engine: replica-per-GPU mode.
//
// With rep_world > 1, replica k of group g is stepped on rank
// (g + k) % rep_world.  Every rank keeps the planes of all replicas (the
// ones it does not own are never stepped), so a round's messages can stay in
// the plane layout the step kernels read: after each round, every message,
// outbox-count word and Replicate entry that a rank's senders produced for a
// replica owned elsewhere is packed into fixed-size records, moved with one
// all-to-all (RCCL over xGMI on GPUs; gloo in the CPU tests), and scattered by
// the receiver into the same positions of its own planes.  The receiver first
// clears the count words of its remote senders for that parity, so silence
// (no record) reads as an empty list.  Record order is irrelevant: every
// record names its destination slot.
#pragma once
#include "rbe_step.h"

namespace rbe {

// stream ids of the exchange records
enum : u32 { XS_CNT = 0, XS_MSG = 1, XS_ENT = 2, XS_NUM = 3 };
constexpr u32 kXchgMaxWorld = 16;

struct alignas(16) XCnt {  // outbox-count word of list (g, s, d)
  u64 key;                 // (g * N + s) * N + d
  u64 word;
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

template <int N>
RBE_HD u32 owner_of(const Params& C, u64 g, u32 k) {
  return (u32)((g + k) % C.rep_world);
}
template <int N>
RBE_HD bool owned(const Params& C, u64 r) {
  if (C.rep_world <= 1) return true;
  return owner_of<N>(C, r / N, (u32)(r % N)) == C.rep_rank;
}

// Byte offset of stream t of peer p in a pack buffer with per-peer, per-stream
// record capacities cap[t].
RBE_HD u64 xchg_region(const u64* cap, u32 p, u32 t) {
  u64 per_peer = 0;
  for (u32 i = 0; i < XS_NUM; i++) per_peer += cap[i] * kXRecBytes[i];
  u64 off = p * per_peer;
  for (u32 i = 0; i < t; i++) off += cap[i] * kXRecBytes[i];
  return off;
}

// Records sender replica r (owned) produced in parity `par` for replicas
// owned elsewhere.  WRITE = false counts them into cnt[peer * XS_NUM + t];
// WRITE = true writes them at slot base[peer * XS_NUM + t] + running index
// of the pack buffer (overflow past cap is counted, not written).
template <int N, bool WRITE>
RBE_HD void xchg_sender(const Planes& P, const Params& C, u64 r, u32 par, u32* cnt, const u32* base,
                        u8* buf, const u64* cap) {
  const u64 g = r / N;
  const u32 s = (u32)(r % N);
  for (u32 d = 0; d < N; d++) {
    if (d == s) continue;
    const u32 peer = owner_of<N>(C, g, d);
    if (peer == C.rep_rank) continue;
    const u64 key = (g * N + s) * N + d;
    const u32 word = P.cnt[par][key];
    if (word == 0) continue;
    auto put = [&](u32 t) -> u8* {
      const u32 i = cnt[peer * XS_NUM + t]++;
      if (!WRITE) return nullptr;
      const u32 at = base[peer * XS_NUM + t] + i;
      if (at >= cap[t]) return nullptr;
      return buf + xchg_region(cap, peer, t) + (u64)at * kXRecBytes[t];
    };
    if (u8* p = put(XS_CNT)) {
      XCnt x;
      x.key = key;
      x.word = word;
      *(XCnt*)p = x;
    }
    const u32 na = word & 0x7Fu, nb = (word >> 7) & 0x7Fu;
    const Msg* lst = &P.msgs[par][key * (u64)C.maxm];
    for (u32 i = 0; i < na + nb; i++) {
      const u32 slot = i < na ? i : C.maxm - 1u - (i - na);
      const Msg m = lst[slot];
      if (u8* p = put(XS_MSG)) {
        XMsg x;
        x.key = key;
        x.slot = slot;
        x.m = m;
        *(XMsg*)p = x;
      }
      // the entries a Replicate carries live in the sender's arena
      for (u32 e = 0; e < m.n_ent; e++) {
        const u64 off = (u64)m.ent_off + e;
        if (off >= C.ecap) break;
        if (u8* p = put(XS_ENT)) {
          XEnt x;
          x.key = r;
          x.off = off;
          x.e = P.arena[par][r * C.ecap + off];
          *(XEnt*)p = x;
        }
      }
    }
  }
}

// Before the scatter: the count words of parity `par` of every list whose
// sender is remote and whose destination replica r is owned here.
template <int N>
RBE_HD void xchg_clear(const Planes& P, const Params& C, u64 r, u32 par) {
  const u64 g = r / N;
  const u32 d = (u32)(r % N);
  for (u32 s = 0; s < N; s++) {
    if (s == d || owner_of<N>(C, g, s) == C.rep_rank) continue;
    P.cnt[par][(g * N + s) * N + d] = 0;
  }
}

RBE_HD void xchg_put_cnt(const Planes& P, const Params& C, u32 par, const XCnt& x) {
  P.cnt[par][x.key] = (u16)x.word;
}
RBE_HD void xchg_put_msg(const Planes& P, const Params& C, u32 par, const XMsg& x) {
  P.msgs[par][x.key * (u64)C.maxm + x.slot] = x.m;
}
RBE_HD void xchg_put_ent(const Planes& P, const Params& C, u32 par, const XEnt& x) {
  P.arena[par][x.key * C.ecap + x.off] = x.e;
}

}  // namespace rbe
