// TEST-ONLY host build of the device step function (dragonboat_amd/csrc/rbe_step.h).
//
// The CPU test tier has no GPU, so the SoA protocol logic that k_step<N> runs
// on MI355X is compiled here for the host and diffed against the oracle
// harness round by round (tests/test_soa_cpu_parity.py).  This library is
// never loaded by the dragonboat_amd package or by any -m gpu test: the GPU
// parity tests call libdragonboat_amd.so through the C ABI.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../dragonboat_amd/csrc/rbe_fast.h"
#include "../../dragonboat_amd/csrc/rbe_host.h"
#include "../../dragonboat_amd/csrc/rbe_snap.h"
#include "../../dragonboat_amd/csrc/rbe_xchg.h"
#include "../../dragonboat_amd/csrc/rbe_wire.h"
#include "../../dragonboat_amd/csrc/rbe_ingest.h"
#include "../../include/rbe.h"

using namespace rbe;

#ifdef RBE_STORE_AUDIT
namespace rbe {
bool g_audit_on = false;
u64 g_store_audit[AS_NUM][2];
}  // namespace rbe
static u64 g_audit_steps, g_audit_leads, g_audit_declined;
// address trace: (item, site, address, bytes) per store while tracing, the
// item being the step's position in the round's fast list (leaders first)
static bool g_audit_tracing;
static u64 g_audit_item;
static std::vector<u64> g_audit_trace;
namespace rbe {
void audit_store(u32 site, const void* at, u64 bytes) {
  if (!g_audit_tracing) return;
  const u64 rec[4] = {g_audit_item, site, (u64)(uintptr_t)at, bytes};
  g_audit_trace.insert(g_audit_trace.end(), rec, rec + 4);
}
}  // namespace rbe
extern "C" void soa_audit_trace(int on) {
  g_audit_tracing = on != 0;
  if (on) g_audit_trace.clear();
}
extern "C" uint64_t soa_audit_trace_get(uint64_t* out, uint64_t max_recs) {
  const u64 n = g_audit_trace.size() / 4;
  if (out) memcpy(out, g_audit_trace.data(), 32 * (n < max_recs ? n : max_recs));
  return n;
}
// out: AS_NUM (count, bytes) pairs, then fast steps, leader steps, declines
extern "C" void soa_store_audit(uint64_t* out, int reset) {
  for (u32 i = 0; i < AS_NUM; i++) {
    out[2 * i] = g_store_audit[i][0];
    out[2 * i + 1] = g_store_audit[i][1];
  }
  out[2 * AS_NUM] = g_audit_steps;
  out[2 * AS_NUM + 1] = g_audit_leads;
  out[2 * AS_NUM + 2] = g_audit_declined;
  if (reset) {
    for (u32 i = 0; i < AS_NUM; i++) g_store_audit[i][0] = g_store_audit[i][1] = 0;
    g_audit_steps = g_audit_leads = g_audit_declined = 0;
  }
}
#endif

struct SoaEngine {
  Params C;
  Planes P;
  std::vector<std::vector<uint8_t>> bufs;
  std::vector<void*> cbufs;  // calloc'd (the spill tiers: zero pages mapped on first touch)
  ~SoaEngine() {
    for (void* p : cbufs) free(p);
  }
  u32 round = 0;
  u32 tclk = 0;
  u32 scan_at = 0;  // the host's last scan round (k_triage list mode: Lists::scan_round)
  HostInputs hin;
  u64 counters[C_NUM] = {0};
  bool full_only = false;
  int staged = 0;  // 4: the fast steps take the inbound counts from the summary word (inbound_aux)
  u64 slow_total = 0;
  std::vector<u8> heap;  // payload heap (cfg.heap_bytes), as on the device
  u64 heap_head = 0;     // Planes::heap_head
  u32 xflag = 0;         // fixed-layout exchange overflow (rbe_xchg_status)
  std::vector<u8> iso_bits;  // replica mode: ORed leader bits of the epoch round iso_round
  u32 iso_round = ~0u;
};

// heap record bytes as rbe_engine.hip read_heap reads them
static int soa_read_heap(SoaEngine* e, u64 pos, u64 off, u64 len, u8* dst) {
  const HostHeap& h = e->hin.heap;
  if (!h.valid(pos, off + len)) return RBE_E_STATE;
  if (h.read_staged(pos, off, len, dst)) return RBE_OK;
  for (u64 i = 0; i < len; i++) dst[i] = e->heap[(pos + off + i) % h.cap];
  return RBE_OK;
}

template <typename T>
static T* alloc(SoaEngine* e, u64 n) {
  e->bufs.emplace_back(n * sizeof(T) + 64, 0);
  return (T*)e->bufs.back().data();
}
template <typename T>
static T* calloc_t(SoaEngine* e, u64 n) {
  void* p = calloc(n * sizeof(T) + 64, 1);
  e->cbufs.push_back(p);
  return (T*)p;
}

template <int N>
static void run_round(SoaEngine* e, bool tick = true) {
  const Clk ck{e->round, e->tclk, tick ? 1u : 0u};
  spill_clear_next(e->P, e->round & 1u);  // (k_triage's first thread on the device)
  if (!e->hin.empty()) {  // the HIP engine uploads and scatters the same records
    HostHeap& hp = e->hin.heap;
    for (u64 p = hp.flushed; p < hp.head; p++) e->heap[p % hp.cap] = hp.stage[p - hp.flushed];
    e->heap_head = hp.head;
    e->hin.apply_host(e->P, e->C);
    e->hin.clear();
  } else {
    e->hin.heap.settle();
  }
  if (e->C.iso_period && e->round > 0 && e->round % e->C.iso_period == 0) {
    if (e->C.rep_world > 1) {  // the ORed leader bits of every rank (soa_set_iso_leaders)
      if (e->iso_round != e->round) abort();
      for (u64 g = 0; g < e->C.n_groups; g++) {
        const u64 gg = group_global(e->C, g);
        if (gg < e->C.n_groups_glob) iso_apply(e->P, e->C, g, e->round, e->iso_bits[gg]);
      }
    } else {
      for (u64 g = 0; g < e->C.n_groups; g++) iso_group<N>(e->P, e->C, g, e->round);
    }
  }
  // the GPU pipeline, sequentially: triage → leader fast list → follower fast
  // list → full list (k_triage / k_fast_list / k_full_list)
  StepCounters c;
  std::vector<u64> lists[3];
  const u32 n = e->C.n;
  const bool shortcut = !e->C.trace && e->C.quiesce && !e->full_only;
  // k_triage's list mode (one replica set per engine) sees a sleeping group
  // only on scan rounds; replica mode scans every round
  const bool scan = e->C.rep_world > 1 || e->round == e->scan_at || forced_round(e->C, e->round);
  for (u64 g = 0; g < e->C.n_groups; g++) {
    // group sleep as k_triage runs it (rbe_step.h)
    const u8 gw = e->P.gwake[g];
    if (shortcut && !(gw & GW_AWAKE) &&
        (!scan || !group_forced(e->C, e->C.cid_base + g * e->C.cid_stride, e->round))) {
      memset(&c, 0, sizeof(c));
      u32 own = 0;
      for (u32 k = 0; k < n; k++) own += owned<N>(e->C, g * n + k) ? 1u : 0u;
      group_sleep_round(gw, own, ck, c);
      for (int i = 0; i < C_NUM; i++) e->counters[i] += c.v[i];
      continue;
    }
    u32 leaders = 0, busy = 0;
    for (u64 r = g * n; r < (g + 1) * n; r++) {
      if (!owned<N>(e->C, r)) continue;
      memset(&c, 0, sizeof(c));
      u32 cls = T_FULL;
      bool done = false;
      if (!e->full_only) {
        const u8 ib = e->P.idle[r];
        const u32 inb = inbound_bits<N>(e->P, r, e->round);
        leaders += (ib & IB_LEAD) ? 1u : 0u;
        if (!e->C.trace && e->C.quiesce && triage_lazy<N>(e->P, e->C, r, ck, ib, inb & 1u, c)) {
          cls = T_DONE;
          done = true;
        } else if (inb & 2u) {  // messages: the role decides the list (as triage_replica would)
          cls = e->C.rl_max ? T_FULL : class_of_role(idle_role(ib));
        } else {
          cls = e->C.trace ? triage_replica<N, true>(e->P, e->C, r, ck, c)
                           : triage_replica<N, false>(e->P, e->C, r, ck, c);
        }
      }
      busy += done ? 0u : 1u;
      if (cls != T_DONE) lists[cls - 1].push_back(r);
      for (int i = 0; i < C_NUM; i++) e->counters[i] += c.v[i];
    }
    if (shortcut) {
      const u32 tr = group_transition(e->C, e->C.cid_base + g * e->C.cid_stride, e->round,
                                      (gw & GW_AWAKE) != 0, busy);
      if (tr == GS_SLEEP) e->P.gwake[g] = group_sleep_byte(leaders);
      if (tr == GS_WAKE) e->P.gwake[g] = GW_AWAKE;
    }
  }
#ifdef RBE_STORE_AUDIT
  g_audit_on = true;
  g_audit_steps += lists[0].size() + lists[1].size();
  g_audit_leads += lists[0].size();
#endif
#ifdef RBE_STORE_AUDIT
  g_audit_item = 0;
#endif
  for (int li = 0; li < 2; li++) {
    for (u64 r : lists[li]) {
      memset(&c, 0, sizeof(c));
      bool ok;
      if (e->staged == 4) {  // counts from the work-list summary word (k_fast_both)
        const u32 g = (u32)(r / N), k = (u32)(r % N);
        u16 w[N];
        inbound_load<N>(e->P, g, k, e->round, w);
        const u32 aux = inbound_aux<N>(w, k, e->round);
        if (li == 0)
          ok = e->C.trace
                   ? step_fast<N, true, MODE_LEAD, true>(e->P, e->C, r, ck, c, aux)
                   : step_fast<N, false, MODE_LEAD, true>(e->P, e->C, r, ck, c, aux);
        else
          ok = e->C.trace
                   ? step_fast<N, true, MODE_FOLL, true>(e->P, e->C, r, ck, c, aux)
                   : step_fast<N, false, MODE_FOLL, true>(e->P, e->C, r, ck, c, aux);
      } else if (li == 0) {
        ok = e->C.trace ? step_fast<N, true, MODE_LEAD>(e->P, e->C, r, ck, c)
                        : step_fast<N, false, MODE_LEAD>(e->P, e->C, r, ck, c);
      } else {
        ok = e->C.trace ? step_fast<N, true, MODE_FOLL>(e->P, e->C, r, ck, c)
                        : step_fast<N, false, MODE_FOLL>(e->P, e->C, r, ck, c);
      }
      if (!ok) lists[2].push_back(r);
      for (int i = 0; i < C_NUM; i++) e->counters[i] += c.v[i];
#ifdef RBE_STORE_AUDIT
      g_audit_item++;
#endif
    }
  }
#ifdef RBE_STORE_AUDIT
  g_audit_on = false;
  g_audit_declined += lists[2].size();
#endif
  std::vector<u64>& slow = lists[2];
  for (u64 r : slow) {
    memset(&c, 0, sizeof(c));
    if (e->C.trace) step_replica<N, true>(e->P, e->C, r, ck, c);
    else step_replica<N, false>(e->P, e->C, r, ck, c);
    for (int i = 0; i < C_NUM; i++) e->counters[i] += c.v[i];
  }
  e->slow_total += slow.size();
  e->round++;
  if (tick) e->tclk++;
}

extern "C" {

void* soa_create(const rbe_config* cfg) {
  SoaEngine* e = new SoaEngine();
  Params& C = e->C;
  memset(&C, 0, sizeof(C));
  C.n = cfg->n_replicas;
  C.n_groups = cfg->n_groups;
  C.n_rep = C.n_groups * C.n;
  C.cid_base = cfg->cid_base ? cfg->cid_base : 1;
  C.cid_stride = cfg->cid_stride ? cfg->cid_stride : 1;
  C.seed = cfg->seed;
  C.max_entry_size = cfg->max_entry_size ? cfg->max_entry_size : (64ull << 20);
  C.ring = cfg->ring ? cfg->ring : 64;
  C.rq_cap = cfg->rq_cap ? cfg->rq_cap : 8;
  C.maxm = cfg->maxm ? cfg->maxm : 12;
  C.ecap = cfg->ecap ? cfg->ecap : 32;
  C.rtr_cap = cfg->rtr_cap ? cfg->rtr_cap : 8;
  C.dri_cap = cfg->dri_cap ? cfg->dri_cap : 8;
  C.election_rtt = cfg->election_rtt;
  C.heartbeat_rtt = cfg->heartbeat_rtt;
  C.check_quorum = cfg->check_quorum;
  C.quiesce = cfg->quiesce;
  C.trace = cfg->trace;
  C.wl_enabled = cfg->wl_enabled;
  C.wl_start_round = cfg->wl_start_round;
  C.wl_stop_round = cfg->wl_stop_round;
  C.wl_active_mod = cfg->wl_active_mod;
  C.wl_read_permille = cfg->wl_read_permille;
  C.ext_inputs = cfg->ext_inputs;
  C.ext_apply = cfg->ext_apply;
  C.ext_commit = cfg->ext_commit;
  C.membership = cfg->membership;
  C.cc_period = cfg->cc_period;
  C.cc_mod = cfg->cc_mod ? cfg->cc_mod : 1;
  C.in_cap = cfg->in_cap ? cfg->in_cap : (u32)(cfg->n_groups > 1024 ? cfg->n_groups : 1024);
  C.xfer_period = cfg->xfer_period;
  C.xfer_mod = cfg->xfer_mod;
  C.iso_period = cfg->iso_period;
  C.iso_len = cfg->iso_len;
  C.iso_mod = cfg->iso_mod;
  C.rep_world = cfg->rep_world > 1 ? cfg->rep_world : 1;
  C.rep_rank = cfg->rep_rank;
  rep_compact_setup(C, cfg->rep_compact != 0);
  C.snapshot_entries = cfg->snapshot_entries;
  C.compaction_overhead = cfg->compaction_overhead;
  C.rl_max = cfg->max_inmem_log_size;
  C.n_voters = cfg->n_voters ? cfg->n_voters : C.n;
  C.obs_slots = cfg->observer_slots;
  C.wit_slots = cfg->witness_slots;
  const u32 spare = ((1u << (C.n & 31)) - 1u) & ~((1u << (C.n_voters & 31)) - 1u);
  if (!valid_n(C.n) || C.n_voters > C.n || (C.n_voters < C.n && !C.membership) ||
      ((C.obs_slots | C.wit_slots) & ~spare) || (C.obs_slots & C.wit_slots) ||
      ((C.obs_slots | C.wit_slots) && !C.membership)) {
    delete e;
    return nullptr;
  }
  const u64 N = C.n, G = C.n_groups, R = C.n_rep;
  Planes& P = e->P;
  P.hot = alloc<Hot>(e, R);
  P.core = alloc<Core>(e, R);
  P.rem = alloc<RemoteMN>(e, R * N);
  P.rem_st = alloc<u8>(e, R * N);
  P.rq = alloc<ReadReq>(e, R * C.rq_cap);
  P.term_ring = alloc<u64>(e, (u64)C.ring * R);
  P.pay_ring = alloc<Body>(e, (u64)C.ring * R);
  // parity 1 follows parity 0 in one allocation, as on the device (rbe_snap.h)
  P.cnt[0] = alloc<CntRow>(e, 2 * R);
  P.cnt[1] = P.cnt[0] + R;
  P.msgs[0] = alloc<Msg>(e, 2 * G * N * N * C.maxm);
  P.msgs[1] = P.msgs[0] + G * N * N * C.maxm;
  P.arena[0] = alloc<Ent>(e, 2 * R * C.ecap);
  P.arena[1] = P.arena[0] + R * C.ecap;
  P.iso_mask = alloc<u8>(e, G);
  P.idle = alloc<u8>(e, R);
  P.iso_until = alloc<u32>(e, G);
  P.upd = alloc<Upd>(e, R);
  P.rtr = alloc<RTR>(e, R * C.rtr_cap);
  P.dri = alloc<DropRI>(e, R * C.dri_cap);
  P.ext = alloc<ExtIn>(e, R);
  P.in_ents = alloc<Ent>(e, C.in_cap);
  P.applied = alloc<u64>(e, R);
  P.gwake = alloc<u8>(e, G);
  memset(P.gwake, GW_AWAKE, G);  // every group starts awake
  P.snp = C.snapshot_entries ? alloc<SnapSt>(e, R) : nullptr;
  P.rem_snap = C.snapshot_entries ? alloc<u64>(e, R * N) : nullptr;
  P.imark = (C.ext_commit || C.rl_max) ? alloc<u64>(e, R) : nullptr;
  P.rl = C.rl_max ? alloc<RlSt>(e, R) : nullptr;
  P.roles = C.membership ? alloc<u16>(e, R) : nullptr;
  // spill tiers (rbe_spill.h), sized as the HIP engine sizes them
  if (C.rq_cap >= kRqExt || spill_sizes(cfg, &C)) {
    delete e;
    return nullptr;
  }
  P.pool = calloc_t<Ent>(e, (u64)C.pool_pages * kPageEnts);
  P.pmeta = calloc_t<PoolMeta>(e, C.pool_pages);
  P.cold = alloc<ColdRef>(e, R);
  P.spill[0] = calloc_t<u8>(e, 2 * C.spill_units * 16);
  P.spill[1] = P.spill[0] + C.spill_units * 16;
  P.sctl = calloc_t<SpillCtl>(e, 1);
  P.sctl->bump = 1;
  C.heap_bytes = (cfg->heap_bytes + 255) & ~255ull;
  e->heap.assign(C.heap_bytes, 0);
  e->hin.init(R, C.n, C.in_cap, C.heap_bytes);
  e->hin.owner = C.rep_world > 1 ? &e->C : nullptr;
  if (C.heap_bytes) {
    P.heap_head = &e->heap_head;
    e->hin.heap.low_fn = [e](u64* lo) -> int {  // k_heap_low, group by group
      u64 m = ~0ull;
      for (u64 g = 0; g < e->C.n_groups; g++) {
        u64 x = with_n(e->C.n, [&](auto NN) {
          return heap_low_group<decltype(NN)::value>(e->P, e->C, g, e->round);
        });
        if (x < m) m = x;
      }
      *lo = m;
      return RBE_OK;
    };
  }
  P.counters = nullptr;
  P.node_ids = nullptr;  // slot s is node s + 1 until soa_set_node_ids
  P.ids_n = (u32)N;
  for (u64 r = 0; r < R; r++) {
    with_n(N, [&](auto NN) { launch_replica<decltype(NN)::value>(P, C, r); });
  }
  return e;
}

void soa_destroy(void* h) { delete (SoaEngine*)h; }

// rbe_spill_stats on the host build
void soa_spill_stats(void* h, uint64_t* out) {
  SoaEngine* e = (SoaEngine*)h;
  const SpillCtl& s = *e->P.sctl;
  out[0] = s.live;
  out[1] = e->C.pool_pages - 1;
  out[2] = std::max(s.peak[0], s.peak[1]) * 16;
  out[3] = e->C.spill_units * 16;
  out[4] = s.oom;
}

// rbe_get_entry_cmds: Cmd bytes of entries [lo, hi] of a replica, inline or
// from the payload heap
int soa_get_entry_cmds(void* h, uint64_t replica, uint64_t lo, uint64_t hi, uint8_t* buf,
                       uint64_t cap, uint64_t* offsets) {
  SoaEngine* e = (SoaEngine*)h;
  const Params& C = e->C;
  if (replica >= C.n_rep || lo == 0 || hi < lo) return RBE_E_INVALID;
  const Core& c = e->P.core[replica];
  if (hi > c.last_index) return RBE_E_INVALID;
  std::vector<Ent> en(hi - lo + 1);
  for (u64 i = lo; i <= hi; i++)  // the ring window and the cold log (rbe_spill.h)
    if (!log_ent_at(e->P, C, replica, c.last_index, i, &en[i - lo])) return RBE_E_STATE;
  u64 off = 0;
  for (u64 i = lo; i <= hi; i++) {
    offsets[i - lo] = off;
    off += en[i - lo].len;
  }
  offsets[hi - lo + 1] = off;
  if (off > cap) return RBE_E_NOMEM;
  for (u64 i = lo; i <= hi; i++) {
    const Ent& b = en[i - lo];
    u8* d = buf + offsets[i - lo];
    if (!ent_heap(b.type)) {
      u8 w[16];
      memcpy(w, &b.lo, 8);
      memcpy(w + 8, &b.hi, 8);
      memcpy(d, w, b.len);
    } else if (b.len) {
      const int rc = soa_read_heap(e, b.hi, kHeapHdr, b.len, d);
      if (rc) return rc;
    }
  }
  return RBE_OK;
}
// rbe_get_entries: every raftpb.Entry field of entries [lo, hi] of a replica
int soa_get_entries(void* h, uint64_t replica, uint64_t lo, uint64_t hi, rbe_entry* out) {
  SoaEngine* e = (SoaEngine*)h;
  const Params& C = e->C;
  if (replica >= C.n_rep || lo == 0 || hi < lo) return RBE_E_INVALID;
  const Core& c = e->P.core[replica];
  if (hi > c.last_index) return RBE_E_INVALID;
  auto rd = [e](u64 pos, u64 off, u64 len, u8* dst) { return soa_read_heap(e, pos, off, len, dst); };
  for (u64 i = lo; i <= hi; i++) {
    Ent x;  // the ring window and the cold log (rbe_spill.h)
    if (!log_ent_at(e->P, C, replica, c.last_index, i, &x)) return RBE_E_STATE;
    rbe_entry& o = out[i - lo];
    memset(&o, 0, sizeof(o));
    const int rc = entry_out(x, &o, nullptr, rd);
    if (rc) return rc;
    o.index = i;
  }
  return RBE_OK;
}
void soa_set_full_only(void* h, int v) { ((SoaEngine*)h)->full_only = v != 0; }
void soa_set_staged(void* h, int v) { ((SoaEngine*)h)->staged = v; }
uint64_t soa_slow_total(void* h) { return ((SoaEngine*)h)->slow_total; }
uint64_t soa_sleeping_groups(void* h) {  // groups asleep after the last round (group sleep)
  SoaEngine* e = (SoaEngine*)h;
  uint64_t n = 0;
  for (u64 g = 0; g < e->C.n_groups; g++) n += (e->P.gwake[g] & GW_AWAKE) ? 0 : 1;
  return n;
}

void soa_run(void* h, uint32_t rounds) {
  SoaEngine* e = (SoaEngine*)h;
  for (u32 i = 0; i < rounds; i++) {
    with_n(e->C.n, [&](auto NN) { run_round<decltype(NN)::value>(e); });
  }
}

// rbe_step_ex (RBE_STEP_NO_TICK = 1)
void soa_step_ex(void* h, uint32_t flags) {
  SoaEngine* e = (SoaEngine*)h;
  const bool tick = (flags & 1u) == 0;
  with_n(e->C.n, [&](auto NN) { run_round<decltype(NN)::value>(e, tick); });
}

// rbe_push_* / rbe_request_leader_transfer / rbe_report_* / rbe_notify_applied
// through the same staging code (rbe_host.h) as the HIP engine
int soa_push_proposals(void* h, uint64_t n, const uint64_t* replica, const uint32_t* n_ents,
                       const uint32_t* type, const uint32_t* cmd_len, const uint8_t* cmd) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.push_proposals(n, replica, n_ents, type, cmd_len, cmd);
}
int soa_propose_entries(void* h, uint64_t n, const uint64_t* replica, const uint32_t* n_ents,
                        const rbe_entry* ents, const uint8_t* cmd) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.push_entries(n, replica, n_ents, ents, cmd);
}
// rbe_launch on the host build (same checks and per-replica restart)
int soa_launch(void* h, uint64_t n, const uint64_t* replica, const rbe_launch_state* st_ids,
               const rbe_entry* ents, const uint8_t* cmd) {
  SoaEngine* e = (SoaEngine*)h;
  std::vector<rbe_launch_state> stv;  // votes as internal ids
  if (!e->hin.map_votes(n, replica, st_ids, stv)) return RBE_E_INVALID;
  const rbe_launch_state* st = stv.data();
  if (n && replica) {
    std::vector<u64> v(replica, replica + n);
    std::sort(v.begin(), v.end());
    if (std::adjacent_find(v.begin(), v.end()) != v.end()) return RBE_E_INVALID;
  }
  std::vector<u64> terms;
  std::vector<Body> bodies;
  int rc = launch_rows(e->C, e->hin.heap, n, replica, st, ents, cmd, terms, bodies);
  if (rc) return rc;
  const u32 ppar = (e->round & 1u) ^ 1u;
  u64 off = 0;
  for (u64 i = 0; i < n; i++) {
    const rbe_launch_state& x = st[i];
    const u64* t = terms.data() + off;
    const Body* b = bodies.data() + off;
    with_n(e->C.n, [&](auto NN) {
      relaunch_replica<decltype(NN)::value>(e->P, e->C, replica[i], x.term, x.vote, x.commit,
                                            x.last_index, x.n_entries, t, b, ppar, e->tclk,
                                            x.marker, x.marker_term, x.snapshot_index,
                                            x.snapshot_term, x.removed);
    });
    e->P.gwake[replica[i] / e->C.n] = GW_AWAKE;
    off += x.n_entries;
  }
  e->scan_at = e->round;  // as rbe_launch: the next round scans every group
  return RBE_OK;
}

int soa_set_apply_ready(void* h, uint64_t n, const uint64_t* replica, const uint8_t* ready) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.set_apply_ready(n, replica, ready);
}
int soa_push_read_index(void* h, uint64_t n, const uint64_t* replica, const uint64_t* lo,
                        const uint64_t* hi) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.push_read_index(n, replica, lo, hi);
}
int soa_request_leader_transfer(void* h, uint64_t n, const uint64_t* replica,
                                const uint64_t* target) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.request_leader_transfer(n, replica, target);
}
int soa_report_unreachable(void* h, uint64_t n, const uint64_t* replica, const uint64_t* node) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.report_unreachable(n, replica, node);
}
int soa_report_snapshot_status(void* h, uint64_t n, const uint64_t* replica, const uint64_t* node,
                               const uint8_t* reject) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.report_snapshot_status(n, replica, node, reject);
}
int soa_notify_applied(void* h, uint64_t n, const uint64_t* replica, const uint64_t* applied) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_apply) return RBE_E_STATE;
  return e->hin.notify_applied(n, replica, applied);
}
// membership inputs on the host build
int soa_propose_config_change(void* h, uint64_t n, const uint64_t* replica, const uint32_t* type,
                              const uint64_t* node) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.propose_config_change(n, replica, type, node);
}
int soa_apply_config_change(void* h, uint64_t n, const uint64_t* replica, const uint64_t* node,
                            const uint32_t* type) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.membership || !e->C.ext_apply) return RBE_E_STATE;
  std::vector<u32> ms(n);
  for (u64 i = 0; i < n && replica; i++) {
    if (replica[i] >= e->C.n_rep) return RBE_E_INVALID;
    const Core& c = e->P.core[replica[i]];
    const u32 x = (c.mflags & MB_ROLES) ? e->P.roles[replica[i]] : 0u;
    ms[i] = pack_ms(c.members & MB_REMOVED, x & 0xFFu, x >> 8);
  }
  return e->hin.apply_config_change(n, replica, node, type, false, ms.data());
}
int soa_reject_config_change(void* h, uint64_t n, const uint64_t* replica) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.apply_config_change(n, replica, nullptr, nullptr, true);
}
int soa_snapshot_saved(void* h, uint64_t n, const uint64_t* replica, const uint64_t* index,
                       const uint64_t* term, const uint32_t* removed) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.snapshot_entries || !e->C.ext_apply) return RBE_E_STATE;
  return e->hin.snapshot_op(n, replica, SR_SAVE, index, term, removed, e->C.membership != 0);
}
int soa_compact(void* h, uint64_t n, const uint64_t* replica, const uint64_t* to) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.snapshot_entries || !e->C.ext_apply) return RBE_E_STATE;
  return e->hin.snapshot_op(n, replica, SR_COMPACT, to, nullptr, nullptr, false);
}
// rbe_replace_node on the host build: the same checks (slot_referenced) and
// the same new node (join_replica)
int soa_replace_node(void* h, uint64_t n, const uint64_t* replica, const uint64_t* node_id) {
  SoaEngine* e = (SoaEngine*)h;
  int rc = e->hin.replace_args(n, replica, node_id);
  if (rc) return rc;
  if (!e->C.membership || e->C.rep_world > 1 || e->C.cc_period || e->C.xfer_period)
    return RBE_E_STATE;
  for (u64 i = 0; i < n; i++) {
    bool refd = false;
    with_n(e->C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      refd = slot_referenced<N>(e->P, e->C, replica[i] / N, (u32)(replica[i] % N), e->round);
    });
    if (refd) return RBE_E_STATE;
  }
  const u32 ppar = (e->round & 1u) ^ 1u;
  for (u64 i = 0; i < n; i++) {
    e->hin.assign_node(e->C.n_groups, replica[i], node_id[i]);
    with_n(e->C.n, [&](auto NN) {
      constexpr int N = decltype(NN)::value;
      join_replica<N>(e->P, e->C, replica[i], ppar, e->tclk);
      e->P.gwake[replica[i] / N] = GW_AWAKE;
    });
  }
  e->P.node_ids = e->hin.id_table();
  e->scan_at = e->round;  // as rbe_launch: the next round scans every group
  return RBE_OK;
}

int soa_set_node_ids(void* h, uint64_t first, uint64_t count, const uint64_t* ids) {
  SoaEngine* e = (SoaEngine*)h;
  if (e->round != 0) return RBE_E_STATE;
  int rc = e->hin.set_node_ids(e->C.n_groups, first, count, ids);
  if (rc) return rc;
  e->P.node_ids = e->hin.id_table();  // the host build's planes are host memory
  return RBE_OK;
}
int soa_restore_remotes(void* h, uint64_t n, const uint64_t* replica, const uint32_t* counts,
                        const uint64_t* ids) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.membership || !e->C.ext_inputs) return RBE_E_STATE;
  return e->hin.restore_remotes(n, replica, counts, ids);
}
// rbe_commit / rbe_get_update_commits on the host build
int soa_commit(void* h, uint64_t n, const uint64_t* replica, const rbe_update_commit* uc) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_commit) return RBE_E_STATE;
  return e->hin.commit(n, replica, uc);
}
int soa_get_update_commits(void* h, uint64_t first, uint64_t count, rbe_update_commit* out) {
  SoaEngine* e = (SoaEngine*)h;
  if (!e->C.ext_commit) return RBE_E_STATE;
  if (!out || first + count > e->C.n_rep) return RBE_E_INVALID;
  for (u64 i = 0; i < count; i++) {
    const u64 r = first + i;
    rbe_update u;
    update_view(e->P.upd[r], e->P.core[r], e->P.hot[r], e->round, u);
    auto term_of = [&](u64 idx) -> u64 {
      const Core& c = e->P.core[r];
      if (idx == c.last_index) return c.t_last;
      Ent x;
      return log_ent_at(e->P, e->C, r, c.last_index, idx, &x) ? x.term : 0;
    };
    const u64 si = e->C.snapshot_entries ? e->P.snp[r].marker : 0;
    update_commit_view(u, e->P.applied[r], si, term_of, out[i]);
  }
  return RBE_OK;
}
// rbe_get_update_snapshots on the host build
int soa_get_update_snapshots(void* h, uint64_t first, uint64_t count, uint64_t* out4) {
  SoaEngine* e = (SoaEngine*)h;
  if (!out4 || first + count > e->C.n_rep) return RBE_E_INVALID;
  for (u64 i = 0; i < count; i++) {
    const u64 r = first + i;
    rbe_update u;
    update_view(e->P.upd[r], e->P.core[r], e->P.hot[r], e->round, u);
    update_snapshot_row(u, e->C.snapshot_entries ? &e->P.snp[r] : nullptr, out4 + 4 * i);
  }
  return RBE_OK;
}

// rbe_wire_encode on the host build: the same wire_cell / trailer / header
// functions the device passes run, batch by batch, into `out` (cap bytes);
// frames as rbe_wire_frame.  Returns total bytes (or -1 when cap is short).
int64_t soa_wire_encode(void* h, uint64_t deployment_id, uint32_t bin_ver, uint32_t gpb,
                        const char* const* addr, uint8_t* out, uint64_t cap,
                        rbe_wire_frame* frames, uint32_t* n_frames, int32_t dst_rank) {
  SoaEngine* e = (SoaEngine*)h;
  const Params& C = e->C;
  const u32 N = C.n;
  if (!gpb) gpb = (u32)C.n_groups;
  u32 table[256];
  for (u32 i = 0; i < 256; i++) table[i] = crc_table_entry(i);
  std::vector<u8> buf;
  u32 nf = 0;
  for (u32 p = 0; p < N * (N - 1); p++) {
    const u32 k = p / (N - 1), dd = p % (N - 1), d = dd >= k ? dd + 1 : dd;
    const u32 alen = addr && addr[k] ? (u32)strlen(addr[k]) : 0;
    for (u64 g0 = 0; g0 < C.n_groups; g0 += gpb) {
      const u64 g1 = g0 + gpb < C.n_groups ? g0 + gpb : C.n_groups;
      std::vector<u8> pay;
      u32 nm = 0;
      for (u64 g = g0; g < g1; g++) {
        u32 cm = 0, ci = 0, bad = 0;
        u32 b = 0;
        if (!with_n(N, [&](auto NN) { return wire_cell_sent<decltype(NN)::value>(C, dst_rank, g, k, d); }))
          continue;
        const u8* hp = e->heap.data();
        const u64 hh = e->hin.heap.flushed;
        b = with_n(N, [&](auto NN) {
          return wire_cell<decltype(NN)::value>(e->P, C, hp, hh, g, k, d, e->round, nullptr, &cm,
                                                &ci, &bad);
        });
        if (bad) return -2;  // rbe_wire_encode: RBE_E_STATE
        if (!cm) continue;
        const size_t at = pay.size();
        pay.resize(at + b);
        with_n(N, [&](auto NN) {
          return wire_cell<decltype(NN)::value>(e->P, C, hp, hh, g, k, d, e->round,
                                                pay.data() + at, &cm, &ci, &bad);
        });
        nm += cm;
      }
      if (!nm) continue;
      const u8* a = (const u8*)(alen ? addr[k] : "");
      const u32 tl = wire_trailer(deployment_id, a, alen, bin_ver, nullptr);
      const size_t at = pay.size();
      pay.resize(at + tl);
      wire_trailer(deployment_id, a, alen, bin_ver, pay.data() + at);
      const size_t fo = buf.size();
      buf.resize(fo + kWireHeader + pay.size());
      memcpy(buf.data() + fo + kWireHeader, pay.data(), pay.size());
      wire_header_put(buf.data() + fo, pay.size(), crc32_update(0, pay.data(), pay.size(), table),
                      table);
      if (frames) {
        rbe_wire_frame& f = frames[nf];
        f.offset = fo;
        f.bytes = kWireHeader + pay.size();
        f.first_group = g0;
        f.src = k;
        f.dst = d;
        f.n_messages = nm;
        f.n_groups = (u32)(g1 - g0);
      }
      nf++;
    }
  }
  *n_frames = nf;
  if (buf.size() > cap) return -1;
  if (!buf.empty()) memcpy(out, buf.data(), buf.size());
  return (int64_t)buf.size();
}

}  // extern "C"

// rbe_wire_ingest on the host build: frames checked and walked on the host
// (the device's k_wire_verify / k_wire_bounds rules for well-formed streams),
// messages parsed with the device's wire_message_get, then the same
// ingest_check / ingest_sender functions the device kernels run, in the
// order of a stable sort by list key.  stats6 as rbe_wire_ingest_stats.
template <int N>
static int soa_ingest_t(SoaEngine* e, const uint8_t* d, uint64_t bytes, uint64_t* st) {
  const Params& C = e->C;
  u32 table[256];
  for (u32 i = 0; i < 256; i++) table[i] = crc_table_entry(i);
  std::vector<std::pair<u64, u64>> pos;  // message bodies
  for (u64 i = 0; i < bytes;) {
    if (bytes - i < kWireHeader || d[i] != 0xAE || d[i + 1] != 0x7D) return RBE_E_CORRUPT;
    u64 size = 0;
    for (int b = 0; b < 8; b++) size = (size << 8) | d[i + 4 + b];
    if (size == 0 || size > bytes - i - kWireHeader) return RBE_E_CORRUPT;
    u8 hb[18];
    memcpy(hb, d + i + 2, 18);
    const u32 inc = ((u32)hb[10] << 24) | ((u32)hb[11] << 16) | ((u32)hb[12] << 8) | hb[13];
    const u32 pc = ((u32)hb[14] << 24) | ((u32)hb[15] << 16) | ((u32)hb[16] << 8) | hb[17];
    hb[10] = hb[11] = hb[12] = hb[13] = 0;
    const u64 off = i + kWireHeader;
    if (crc32_update(0, hb, 18, table) != inc || (((u32)hb[0] << 8) | hb[1]) != kWireMethod ||
        crc32_update(0, d + off, size, table) != pc)
      return RBE_E_CORRUPT;
    WireRd rd{d + off, size, 0, false};
    while (rd.i < size && !rd.bad) {
      const u64 tag = rd.varint();
      const u32 fn = (u32)(tag >> 3), wt = (u32)(tag & 7);
      if (fn == 1 && wt == 2) {
        const u64 l = rd.varint();
        if (rd.bad || l > size - rd.i) return RBE_E_CORRUPT;
        pos.emplace_back(off + rd.i, l);
        rd.i += l;
      } else {
        rd.skip(wt);
      }
    }
    if (rd.bad) return RBE_E_CORRUPT;
    st[0]++;
    i = off + size;
  }
  const u64 tm = pos.size();
  std::vector<u64> ent0(tm + 1, 0), cmd0(tm + 1, 0);
  for (u64 j = 0; j < tm; j++) {
    WireRd rd{d, pos[j].first + pos[j].second, pos[j].first, false};
    u64 cb = 0;
    const u32 ne = wire_message_get(rd, pos[j].first + pos[j].second, nullptr, nullptr, nullptr, &cb);
    if (rd.bad) return RBE_E_CORRUPT;
    ent0[j + 1] = ent0[j] + ne;
    cmd0[j + 1] = cmd0[j] + cb;
  }
  std::vector<rbe_message> msgs(tm);
  std::vector<rbe_entry> ents(ent0[tm] + 1);
  std::vector<u8> cmd(cmd0[tm] + 1);
  for (u64 j = 0; j < tm; j++) {
    WireRd rd{d, pos[j].first + pos[j].second, pos[j].first, false};
    u64 cb = cmd0[j];
    wire_message_get(rd, pos[j].first + pos[j].second, &msgs[j], ents.data() + ent0[j], cmd.data(),
                     &cb);
  }
  st[1] = tm;
  st[3] = ent0[tm];
  st[4] = cmd0[tm];
  if (!tm) return RBE_OK;
  HostHeap& H = e->hin.heap;
  std::vector<u64> key(tm), hb(tm);
  u32 err = 0;
  for (u64 j = 0; j < tm; j++) {
    u32 x = 0;
    ingest_ids<N>(C, e->hin.id_table(), msgs[j]);
    key[j] = ingest_check<N>(C, H.cap, msgs[j], ents.data() + ent0[j], &x, &hb[j]);
    err |= x;
    if (!x && key[j] == ing_drop_key(C)) st[2]++;
  }
  if (err & ING_INVALID) return RBE_E_INVALID;
  if (err & ING_NOMEM) return RBE_E_NOMEM;
  std::vector<u32> sidx(tm);
  for (u64 j = 0; j < tm; j++) sidx[j] = (u32)j;
  std::stable_sort(sidx.begin(), sidx.end(), [&](u32 a, u32 b) { return key[a] < key[b]; });
  std::vector<u64> skey(tm), hs(tm);
  u64 need = 0;
  for (u64 p = 0; p < tm; p++) {
    skey[p] = key[sidx[p]];
    hs[p] = need;
    need += hb[sidx[p]];
  }
  auto walk = [&](bool write, u64 base) {
    u32 x = 0;
    for (u64 p = 0; p < tm; p++) {
      if (!ingest_run_start(C, skey.data(), p)) continue;
      const u64 q = ingest_run_end(C, skey.data(), p, tm);
      if (write)
        x |= ingest_sender<N, true>(e->P, C, (e->round - 1) & 1u, e->round, skey.data(),
                                    sidx.data(), p, q, msgs.data(), ents.data(), ent0.data(),
                                    cmd0.data(), cmd.data(), e->heap.data(), H.cap, base, hs.data());
      else
        x |= ingest_sender<N, false>(e->P, C, (e->round - 1) & 1u, e->round, skey.data(),
                                     sidx.data(), p, q, msgs.data(), ents.data(), ent0.data(),
                                     cmd0.data(), cmd.data(), nullptr, H.cap, base, hs.data());
    }
    return x;
  };
  if (walk(false, 0)) return RBE_E_NOMEM;
  st[5] = need;
  u64 base = 0;
  if (need) {
    for (u64 p = H.flushed; p < H.head; p++) e->heap[p % H.cap] = H.stage[p - H.flushed];
    const u64 skip = H.head % H.cap + need > H.cap ? H.cap - H.head % H.cap : 0;
    const int rc = H.room(need + skip);
    if (rc) return rc;
    if (H.flushed < H.round_lo) H.round_lo = H.flushed;
    H.stage.clear();
    base = H.head + skip;
    H.head = base + need;
    H.flushed = H.head;
    e->heap_head = H.head;
  }
  walk(true, base);
  return RBE_OK;
}
extern "C" int soa_wire_ingest(void* h, const uint8_t* data, uint64_t bytes, uint64_t* stats6) {
  SoaEngine* e = (SoaEngine*)h;
  memset(stats6, 0, 6 * sizeof(u64));
  if (e->round == 0) return RBE_E_INVALID;
  if (e->C.rep_world <= 1) return RBE_E_STATE;
  return with_n(e->C.n, [&](auto NN) {
    return soa_ingest_t<decltype(NN)::value>(e, data, bytes, stats6);
  });
}

extern "C" {

// rbe_iso_leaders / rbe_set_iso_leaders on the host build
int soa_iso_leaders(void* h, uint8_t* out, uint32_t* epoch) {
  SoaEngine* e = (SoaEngine*)h;
  const Params& C = e->C;
  *epoch = C.iso_period && e->round > 0 && e->round % C.iso_period == 0 ? 1u : 0u;
  if (!*epoch || !out) return RBE_OK;
  memset(out, 0, C.n_groups_glob);
  for (u64 g = 0; g < C.n_groups; g++) {
    const u64 gg = group_global(C, g);  // exchanged by global group
    if (gg >= C.n_groups_glob) continue;
    out[gg] = (u8)with_n(C.n, [&](auto NN) {
      return (u32)iso_leader_bits<decltype(NN)::value>(e->P, C, g);
    });
  }
  return RBE_OK;
}
int soa_rate_limited(void* h, uint64_t first, uint64_t count, uint8_t* limited,
                     uint64_t* size) {
  SoaEngine* e = (SoaEngine*)h;
  if (count == 0 || first >= e->C.n_rep || count > e->C.n_rep - first) return RBE_E_INVALID;
  if (!e->P.rl) return RBE_E_STATE;
  for (u64 i = 0; i < count; i++) {
    RlSt s = e->P.rl[first + i];  // a copy: the query's gc is not kept (unobservable)
    if (limited) limited[i] = rl_limited(s, e->C.rl_max) ? 1 : 0;
    if (size) size[i] = s.size;
  }
  return RBE_OK;
}
int soa_local_groups(void* h, uint64_t* n_local, uint64_t* global_of) {
  SoaEngine* e = (SoaEngine*)h;
  *n_local = e->C.n_groups;
  if (global_of)
    for (u64 g = 0; g < e->C.n_groups; g++) {
      const u64 gg = group_global(e->C, g);
      global_of[g] = gg < e->C.n_groups_glob ? gg : ~0ull;
    }
  return RBE_OK;
}
int soa_set_iso_leaders(void* h, const uint8_t* bits) {
  SoaEngine* e = (SoaEngine*)h;
  e->iso_bits.assign(bits, bits + e->C.n_groups_glob);
  e->iso_round = e->round;
  return RBE_OK;
}

void soa_snapshot_state(void* h, uint64_t* out8) {
  SoaEngine* e = (SoaEngine*)h;
  for (u64 r = 0; r < e->C.n_rep; r++) {
    if (e->P.snp) snap_state_row(e->P.snp[r], out8 + 8 * r);
    else memset(out8 + 8 * r, 0, 8 * sizeof(u64));
  }
}

void soa_counters(void* h, uint64_t* out) {
  SoaEngine* e = (SoaEngine*)h;
  for (int i = 0; i < C_NUM; i++) out[i] = e->counters[i];
}

void soa_views(void* h, rbe_replica_view* out) {
  SoaEngine* e = (SoaEngine*)h;
  const u32 N = e->C.n;
  for (u64 i = 0; i < e->C.n_rep; i++) {
    rbe_replica_view& v = out[i];
    memset(&v, 0, sizeof(v));
    const Hot hh = materialize_hot(e->P.hot[i], e->C, e->tclk);
    const Core& c = e->P.core[i];
    v.term = c.term;
    v.vote = ext_id(e->hin.id_table(), N, i / N, c.vote);
    v.leader_id = ext_id(e->hin.id_table(), N, i / N, c.leader);
    v.committed = c.committed;
    v.last_index = c.last_index;
    v.processed = c.processed;
    v.saved_to = c.saved_to;
    v.digest = e->P.upd[i].digest;
    v.role = hh.role;
    v.election_tick = hh.election_tick;
    v.heartbeat_tick = hh.heartbeat_tick;
    v.rand_election_timeout = hh.rand_et;
    v.q_tick = hh.q_tick;
    v.q_quiesced_since = hh.q_quiesced_since;
    v.q_no_activity_since = hh.q_no_activity_since;
    v.q_exit_quiesce_tick = hh.q_exit_quiesce_tick;
    v.raft_quiesce = (hh.flags & HF_RAFT_QUIESCE) ? 1 : 0;
    v.rq_count = rq_length(e->P, e->C, i, c);
    v.votes_resp = hh.votes_resp;
    v.votes_granted = hh.votes_granted;
    v.events = (e->round > 0 && e->P.upd[i].round == e->round - 1) ? e->P.upd[i].events : 0u;
    v.removed = c.members & MB_REMOVED;
    if (c.mflags & MB_ROLES) {  // Planes::roles is only current while MB_ROLES is set
      v.observers = e->P.roles[i] & 0xFFu;
      v.witnesses = e->P.roles[i] >> 8;
    }
    if (hh.role == R_Leader) {
      for (u32 s = 0; s < N && s < 8; s++) {
        // remotes, observers and witnesses
        if ((v.removed >> s) & ~((v.observers | v.witnesses) >> s) & 1u) continue;
        v.match[s] = e->P.rem[i * N + s].match;
        v.next[s] = e->P.rem[i * N + s].next;
        v.rstate[s] = e->P.rem_st[i * N + s] & 3;
        v.ractive[s] = (e->P.rem_st[i * N + s] >> 2) & 1;
      }
    }
  }
}

uint32_t soa_faults(void* h, uint64_t* n_faulty) {
  SoaEngine* e = (SoaEngine*)h;
  uint32_t o = 0;
  uint64_t n = 0;
  for (u64 i = 0; i < e->C.n_rep; i++) {
    if (e->P.upd[i].fault) n++;
    o |= e->P.upd[i].fault;
  }
  *n_faulty = n;
  return o;
}

}  // extern "C"

// replica-per-GPU exchange on the host build (same record format and the same
// rbe_xchg.h functions as the device kernels)
template <int N>
static int soa_xchg_pack_t(SoaEngine* e, uint8_t* buf, const uint64_t* cap, uint32_t* counts) {
  const u32 par = (e->round - 1) & 1u, nc = e->C.rep_world * XS_NUM;
  for (u32 i = 0; i < nc; i++) counts[i] = 0;
  std::vector<u32> cnt(nc), base(nc);
  for (u64 r = 0; r < e->C.n_rep; r++) {
    if (!owned<N>(e->C, r)) continue;
    for (u32 i = 0; i < nc; i++) cnt[i] = 0;
    xchg_sender<N, false>(e->P, e->C, r, par, e->round, cnt.data(), nullptr, nullptr, cap);
    for (u32 i = 0; i < nc; i++) {
      base[i] = counts[i];
      counts[i] += cnt[i];
      cnt[i] = 0;
    }
    xchg_sender<N, true>(e->P, e->C, r, par, e->round, cnt.data(), base.data(), buf, cap);
  }
  for (u32 i = 0; i < nc; i++)
    if (counts[i] > cap[i % XS_NUM]) return -3;
  return 0;
}
template <int N>
static void soa_xchg_unpack_t(SoaEngine* e, const XCnt* c, uint64_t nc, const XMsg* m, uint64_t nm,
                              const XEnt* x, uint64_t ne) {
  const u32 par = (e->round - 1) & 1u;
  for (u64 i = 0; i < nc; i++) xchg_put_cnt(e->P, e->C, par, c[i]);
  for (u64 i = 0; i < nm; i++) xchg_put_msg(e->P, e->C, par, m[i]);
  for (u64 i = 0; i < ne; i++) xchg_put_ent(e->P, e->C, par, x[i]);
}
// fixed layout (rbe_xchg_pack_fixed / rbe_xchg_unpack_fixed) on the host build
template <int N>
static void soa_xchg_pack_fixed_t(SoaEngine* e, uint8_t* buf, const uint64_t* cap) {
  const u32 par = (e->round - 1) & 1u, nc = e->C.rep_world * XS_NUM;
  std::vector<u32> counts(nc, 0), cnt(nc), base(nc);
  for (u64 r = 0; r < e->C.n_rep; r++) {
    if (!owned<N>(e->C, r)) continue;
    for (u32 i = 0; i < nc; i++) cnt[i] = 0;
    xchg_sender<N, false>(e->P, e->C, r, par, e->round, cnt.data(), nullptr, nullptr, cap,
                          kXHdrBytes);
    for (u32 i = 0; i < nc; i++) {
      base[i] = counts[i];
      counts[i] += cnt[i];
      cnt[i] = 0;
    }
    xchg_sender<N, true>(e->P, e->C, r, par, e->round, cnt.data(), base.data(), buf, cap,
                         kXHdrBytes);
  }
  for (u32 p = 0; p < e->C.rep_world; p++) {
    XHdr hd;
    memset(&hd, 0, sizeof(hd));
    for (u32 t = 0; t < XS_NUM; t++) {
      const u32 n = counts[p * XS_NUM + t];
      hd.cnt[t] = n < cap[t] ? n : (u32)cap[t];
      if (n > cap[t]) hd.overflow = 1;
    }
    if (hd.overflow) e->xflag = 1;
    memcpy(buf + xchg_fixed_off(cap, p, e->C.rep_rank), &hd, sizeof(hd));
  }
}
extern "C" void soa_xchg_pack_fixed(void* h, uint8_t* buf, const uint64_t* cap) {
  SoaEngine* e = (SoaEngine*)h;
  with_n(e->C.n, [&](auto NN) { soa_xchg_pack_fixed_t<decltype(NN)::value>(e, buf, cap); });
}
extern "C" void soa_xchg_unpack_fixed(void* h, const uint8_t* recv, const uint64_t* cap) {
  SoaEngine* e = (SoaEngine*)h;
  const u32 par = (e->round - 1) & 1u;
  for (u32 t = 0; t < XS_NUM; t++)
    for (u32 p = 0; p < e->C.rep_world; p++)
      for (u64 i = 0; i < cap[t]; i++) {
        u32 ovf = 0;
        const bool put = xchg_put_fixed(e->P, e->C, par, recv, cap, p, t, i, &ovf);
        if (ovf) e->xflag = 1;
        if (!put) break;
      }
}
extern "C" uint32_t soa_xchg_status(void* h) {  // read-and-clear, as rbe_xchg_status
  SoaEngine* e = (SoaEngine*)h;
  const u32 f = e->xflag;
  e->xflag = 0;
  return f;
}

extern "C" int soa_xchg_pack(void* h, uint8_t* buf, const uint64_t* cap, uint32_t* counts) {
  SoaEngine* e = (SoaEngine*)h;
  if (e->C.heap_bytes) return RBE_E_STATE;  // as rbe_xchg_pack: heap positions are local
  return with_n(e->C.n, [&](auto NN) {
    return soa_xchg_pack_t<decltype(NN)::value>(e, buf, cap, counts);
  });
}
extern "C" void soa_xchg_unpack(void* h, const void* c, uint64_t nc, const void* m, uint64_t nm,
                                const void* x, uint64_t ne) {
  SoaEngine* e = (SoaEngine*)h;
  with_n(e->C.n, [&](auto NN) {
    soa_xchg_unpack_t<decltype(NN)::value>(e, (const XCnt*)c, nc, (const XMsg*)m, nm,
                                           (const XEnt*)x, ne);
  });
}

// transport boundary on the host build (rbe_get_outbox / rbe_push_messages)
extern "C" int soa_get_outbox(void* h, uint64_t replica, rbe_message* out, uint32_t cap,
                              uint32_t* n_out, rbe_entry* ents, uint32_t ent_cap,
                              uint32_t* n_ents, uint8_t* cmd, uint64_t cmd_cap,
                              uint64_t* cmd_bytes) {
  SoaEngine* e = (SoaEngine*)h;
  if (replica >= e->C.n_rep || e->round == 0) return RBE_E_INVALID;
  const u32 N = e->C.n, par = (e->round - 1) & 1u;
  const u64 g = replica / N;
  const u32 k = (u32)(replica % N);
  const CntRow& row = e->P.cnt[par][replica];
  const u32 rd = e->round;
  std::vector<Msg> lv;
  auto list = [&](u32 d) -> const std::vector<Msg>& {
    const ListView v = list_view(e->P, e->C, par, replica * N + d, row_word(row, d, k, rd));
    lv.clear();
    for (u32 i = 0; i < v.n(); i++) lv.push_back(v.at(i));
    return lv;
  };
  auto ent = [&](const Msg& m, u32 j) { return msg_ents(e->P, e->C, par, replica, m)[j]; };
  auto hr = [e](u64 pos, u64 off, u64 len, u8* dst) { return soa_read_heap(e, pos, off, len, dst); };
  return with_n(N, [&](auto NN) {
    return outbox_messages<decltype(NN)::value>(e->C, g, k, row, rd, list, ent, out, cap, ents,
                                                ent_cap, n_out, n_ents, cmd, cmd_cap, cmd_bytes,
                                                e->hin.id_table(), hr);
  });
}
template <int N>
static int soa_push_t(SoaEngine* e, uint64_t n, const uint64_t* group, const rbe_message* msgs,
                      const rbe_entry* ents, const uint8_t* cmd) {
  std::vector<XCnt> c;
  std::vector<XMsg> m;
  std::vector<XEnt> x;
  const int rc =
      messages_to_records<N>(e->C, e->hin.heap, e->round, n, group, msgs, ents, cmd, c, m, x,
                             e->hin.id_table());
  if (rc) return rc;
  soa_xchg_unpack_t<N>(e, c.data(), c.size(), m.data(), m.size(), x.data(), x.size());
  return RBE_OK;
}
extern "C" int soa_push_messages(void* h, uint64_t n, const uint64_t* group,
                                 const rbe_message* msgs, const rbe_entry* ents,
                                 const uint8_t* cmd) {
  SoaEngine* e = (SoaEngine*)h;
  if (e->round == 0) return RBE_E_INVALID;
  if (e->C.rep_world <= 1) return RBE_E_STATE;
  return with_n(e->C.n, [&](auto NN) {
    return soa_push_t<decltype(NN)::value>(e, n, group, msgs, ents, cmd);
  });
}

// Group-range snapshots in the engine's byte layout (rbe_export_groups /
// rbe_import_groups run the same plane walk with hipMemcpy2DAsync).
extern "C" uint64_t soa_snapshot_bytes(void* h, uint64_t count) {
  SoaEngine* e = (SoaEngine*)h;
  return sizeof(SnapHeader) + snap_body_bytes(e->P, e->C, count);
}

// the log section's source (rbe_snap.h snap_log_write): the planes themselves
struct SnapLogHost {
  const Planes& P;
  const Params& C;
  ColdRef cold(u64 r) { return P.cold[r]; }
  Core core(u64 r) { return P.core[r]; }
  RqExt rq(u64 r) { return rq_ext_load(P, C, r); }
  PoolMeta meta(u32 p) { return P.pmeta[p]; }
  void page(u32 p, Ent* out) { memcpy(out, pool_ent(P, p, 0), kPageEnts * sizeof(Ent)); }
};
static bool soa_range_spilled(SoaEngine* e, u64 first, u64 count) {
  if (e->round == 0) return false;
  const u32 N = e->C.n, par = (e->round - 1) & 1u;
  for (u64 r = first * N; r < (first + count) * N; r++) {
    u32 w[8];
    for (u32 d = 0; d < N; d++) w[d] = row_word(e->P.cnt[par][r], d, (u32)(r % N), e->round);
    if (snap_round_spilled(e->C, w, e->P.msgs[par] + r * N * e->C.maxm, e->P.upd[r])) return true;
  }
  return false;
}
extern "C" uint64_t soa_export_bytes(void* h, uint64_t first, uint64_t count) {
  SoaEngine* e = (SoaEngine*)h;
  SnapLogHost src{e->P, e->C};
  return snap_log_at(snap_body_bytes(e->P, e->C, count)) +
         snap_log_write(e->C, first * e->C.n, count * e->C.n, src, nullptr);
}

extern "C" int soa_export_groups(void* h, uint64_t first, uint64_t count, void* buf, uint64_t cap) {
  SoaEngine* e = (SoaEngine*)h;
  if (count == 0 || first >= e->C.n_groups || count > e->C.n_groups - first) return RBE_E_INVALID;
  if (soa_range_spilled(e, first, count)) return RBE_E_STATE;
  const u64 body = snap_body_bytes(e->P, e->C, count);
  SnapLogHost src{e->P, e->C};
  const u64 r0 = first * e->C.n, nr = count * e->C.n;
  const u64 lb = snap_log_write(e->C, r0, nr, src, nullptr);
  if (cap < snap_log_at(body) + lb) return RBE_E_NOMEM;
  SnapHeader hd;
  snap_fill_header(e->C, RBE_ABI_VERSION, e->round, e->tclk, first, count, body, &hd);
  hd.log_bytes = lb;
  memcpy(buf, &hd, sizeof(hd));
  memset((u8*)buf + sizeof(hd) + body, 0, snap_log_at(body) - sizeof(hd) - body);
  snap_log_write(e->C, r0, nr, src, (u8*)buf + snap_log_at(body));
  SnapPlane pl[kSnapPlanes];
  snap_planes(e->P, e->C, pl);
  u8* dst = (u8*)buf + sizeof(SnapHeader);
  for (int i = 0; i < kSnapPlanes && pl[i].rows; i++) {
    const u64 w = count * pl[i].group_bytes;
    for (u64 row = 0; row < pl[i].rows; row++, dst += w)
      memcpy(dst, pl[i].base + row * pl[i].pitch + first * pl[i].group_bytes, w);
  }
  return RBE_OK;
}

extern "C" int soa_import_groups(void* h, const void* buf, uint64_t bytes, uint32_t flags) {
  SoaEngine* e = (SoaEngine*)h;
  SnapHeader hd;
  if (bytes < sizeof(hd)) return RBE_E_INVALID;
  memcpy(&hd, buf, sizeof(hd));
  if (snap_check_header(e->C, RBE_ABI_VERSION, &hd, bytes) ||
      hd.body_bytes != snap_body_bytes(e->P, e->C, hd.count))
    return RBE_E_INVALID;
  const bool resume = (flags & RBE_IMPORT_RESUME) != 0;
  if (resume && (hd.first != 0 || hd.count != e->C.n_groups)) return RBE_E_INVALID;
  if (!resume && hd.round != e->round) return RBE_E_STATE;
  const u64 r0 = hd.first * e->C.n, nr = hd.count * e->C.n;
  std::vector<u64> rec_off(nr);
  if (snap_log_index(e->C, (const u8*)buf, nr, rec_off.data())) return RBE_E_INVALID;
  const u32 spar = e->round & 1u;  // (as rbe_import_groups)
  for (u64 i = 0; i < nr; i++) spill_replica_release(e->P, e->C, r0 + i, spar);
  SnapPlane pl[kSnapPlanes];
  snap_planes(e->P, e->C, pl);
  const u8* src = (const u8*)buf + sizeof(SnapHeader);
  for (int i = 0; i < kSnapPlanes && pl[i].rows; i++) {
    const u64 w = hd.count * pl[i].group_bytes;
    for (u64 row = 0; row < pl[i].rows; row++, src += w)
      memcpy(pl[i].base + row * pl[i].pitch + hd.first * pl[i].group_bytes, src, w);
  }
  {  // the log section, 16-B aligned for the record reads
    std::vector<u64> sec((hd.log_bytes + 15) / 8 + 2);
    u8* s = (u8*)(((uintptr_t)sec.data() + 15) & ~(uintptr_t)15);
    memcpy(s, (const u8*)buf + snap_log_at(hd.body_bytes), hd.log_bytes);
    u32 f = 0;
    for (u64 i = 0; i < nr; i++) snap_log_rebuild(e->P, e->C, r0 + i, s + rec_off[i], spar ^ 1u, &f);
    if (f) return RBE_E_NOMEM;
  }
  e->hin.resync_applied(e->P.applied + hd.first * e->C.n, hd.first * e->C.n, hd.count * e->C.n);
  memset(e->P.gwake + hd.first, GW_AWAKE, hd.count);  // imported groups start awake
  if (resume) {
    e->round = hd.round;
    e->scan_at = hd.round;
    e->tclk = (u32)hd.tclk;
  }
  return RBE_OK;
}

// ---------------------------------------------------------------- quiesce FSM
// The device-side quiesce manager restatements (Lane::q_* used by the full
// handler table, FastQ used by the fast steps), driven op by op so the
// reference's quiesce_test.go vectors pin them directly (tests/test_quiesce.py).
struct SoaQuiesce {
  Params C;
  Planes P;
  StepCounters ctr;
  Lane<3, false, MODE_FULL>* lane;
  FastQ fq;
  int which;  // 0 = Lane, 1 = FastQ
};
extern "C" void* soa_quiesce_new(uint64_t election_tick, int enabled, int which) {
  auto* s = new SoaQuiesce();
  memset(&s->C, 0, sizeof(s->C));
  memset(&s->P, 0, sizeof(s->P));
  memset(&s->ctr, 0, sizeof(s->ctr));
  s->C.election_rtt = (u32)(election_tick / 2);  // node.go:165 electionTick = 2 x ElectionRTT
  s->C.quiesce = enabled ? 1 : 0;
  s->lane = new Lane<3, false, MODE_FULL>(s->P, s->C, 0, Clk{0, 0, 1}, s->ctr);
  s->lane->q_tick = s->lane->q_qs = s->lane->q_nas = s->lane->q_eqt = 0;
  s->lane->q_new = false;
  s->fq.tick = s->fq.qs = s->fq.nas = s->fq.eqt = 0;
  s->fq.qnew = false;
  s->which = which;
  return s;
}
extern "C" void soa_quiesce_free(void* h) {
  auto* s = (SoaQuiesce*)h;
  delete s->lane;
  delete s;
}
// same op codes as orc_quiesce_op (oracle/oracle_capi.cpp)
extern "C" uint64_t soa_quiesce_op(void* h, int op, uint64_t a) {
  auto* s = (SoaQuiesce*)h;
  auto& L = *s->lane;
  auto& q = s->fq;
  const bool lane = s->which == 0;
  switch (op) {
    case 0:
      if (lane) L.q_increase_tick();
      else q.increase_tick(s->C);
      return lane ? L.q_tick : q.tick;
    case 1:
      if (lane) L.q_record_activity((u32)a);
      else q.record_activity(s->C, (u32)a);
      return 0;
    case 2:
      if (lane) L.q_try_enter();
      else q.try_enter(s->C);
      return 0;
    case 3: return (lane ? L.q_quiesced() : q.quiesced(s->C)) ? 1 : 0;
    case 4: return (lane ? L.q_new_to_quiesce() : q.new_to_quiesce(s->C)) ? 1 : 0;
    case 5: return lane ? L.q_threshold() : s->C.election_rtt * 20;
    case 6: return lane ? L.q_tick : q.tick;
    case 7: return lane ? L.q_nas : q.nas;
    case 8: return lane ? L.q_qs : q.qs;
    case 9: return lane ? L.q_eqt : q.eqt;
    case 10: {
      bool v = lane ? L.q_new : q.qnew;
      if (lane) L.q_new = false;
      else q.qnew = false;
      return v ? 1 : 0;
    }
    case 11: s->C.quiesce = a ? 1 : 0; return 0;
    default: return ~0ull;
  }
}

// ---------------------------------------------------------------- Update helpers
// the engine's range-form restatements of getUpdateCommit / validateUpdate /
// setFastApply (rbe_step.h update_*), same fn codes as orc_update_fn
extern "C" int soa_update_fn(int fn, uint64_t commit, uint64_t apply_lo, uint64_t apply_hi,
                             uint64_t save_lo, uint64_t save_hi, uint64_t snap_index,
                             uint64_t* out3) {
  if (fn == 0) {
    update_commit(save_lo, save_hi, apply_lo, apply_hi, snap_index, &out3[0], &out3[1], &out3[2]);
    return 0;
  }
  if (fn == 1) return update_valid(commit, save_lo, save_hi, apply_lo, apply_hi) ? 0 : -1;
  if (fn == 2) {
    out3[0] = update_fast_apply(snap_index != 0, save_lo, save_hi, apply_lo, apply_hi) ? 1 : 0;
    return 0;
  }
  return -2;
}
