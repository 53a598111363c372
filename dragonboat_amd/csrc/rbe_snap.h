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

#include "rbe_types.h"

namespace rbe {

static constexpr u64 kSnapMagic = 0x31504E5345425255ull;  // "URBESNP1"
static constexpr int kSnapPlanes = 23;

struct SnapHeader {
  u64 magic;
  u32 abi, n, ring, rq_cap, maxm, ecap, rtr_cap, dri_cap;
  u32 round, hdr_bytes;
  u64 first, count;
  u64 body_bytes;
  u64 behavior;  // snap_behavior_hash of the writing configuration
  u64 tclk;      // ticks before `round` (Clk::tclk)
};
static_assert(sizeof(SnapHeader) == 88, "snapshot header layout");

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
  if (buf_bytes < sizeof(SnapHeader) + h->body_bytes) return -1;
  return 0;
}

}  // namespace rbe
