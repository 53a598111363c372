// rbe_wire_kernels.h — device codec of the transport wire format (rbe_wire.h):
// encode the last round's outbox into framed MessageBatches, decode framed
// MessageBatches into raftpb-form records.  Included by rbe_engine.hip only.
//
// Encode is four passes over HBM, all byte/integer work (no MFMA):
//   k_wire_size   one lane per (group, k, d) cell: bytes + messages of the cell
//   k_wire_batch  one block per batch: exclusive scan of its cells' bytes
//   k_wire_frames one block: frame offsets, the compacted frame index
//   k_wire_write  one lane per cell: the cell's requests at their offset;
//                 one lane per batch: the trailer
//   k_wire_crc    one block per frame: payload crc32 by segments combined
//                 with crc32_combine, then the header
// Decode: k_wire_verify (block per frame: both crc32s), k_wire_bounds (block
// per frame: where its requests are), k_wire_parse (lane per message: count,
// device scan, then the records).
#pragma once

#include "rbe_wire.h"
#include "rbe_ingest.h"

namespace rbe {

struct WireArgs {
  u64 deployment_id;
  u32 bin_ver, gpb;      // groups per batch
  u32 nchunks, npairs;   // batches = npairs * nchunks
  u32 round;
  u64 heap_head;         // payload heap head at the last upload (lapped-record check)
  int32_t dst_rank;      // replica mode: receivers of this rank only (-1: every remote rank)
  u32 pad;
  u32 alen[kMaxN];
  u8 addr[kMaxN][48];        // source address of each slot
};

struct WireFrame {  // mirrors rbe_wire_frame (include/rbe.h)
  u64 offset, bytes, first_group;
  u32 src, dst, n_messages, n_groups;
};

struct WireBufs {
  u32* cell_bytes;  // [npairs * n_groups]
  u32* cell_msgs;
  u32* cell_off;    // offset in its batch's payload
  u64* batch_pay;   // [nbatch] payload bytes (0 = no message)
  u32* batch_msgs;
  u32* batch_is;
  u64* frame_off;   // [nbatch]
  WireFrame* frames;  // compacted, non-empty batches
  u64* totals;      // [0] bytes, [1] frames, [2] messages, [3] InstallSnapshots left out,
                    // [4] entries whose heap record a later lap overwrote
};

RBE_HD void wire_pair(u32 N, u32 p, u32* k, u32* d) {
  *k = p / (N - 1u);
  const u32 dd = p % (N - 1u);
  *d = dd >= *k ? dd + 1u : dd;
}

template <int N>
__global__ __launch_bounds__(256) void k_wire_size(Planes P, Params C, WireArgs A, WireBufs B,
                                                   const u8* heap) {
  const u64 c = (u64)blockIdx.x * 256 + threadIdx.x;
  if (c >= (u64)A.npairs * C.n_groups) return;
  const u32 p = (u32)(c / C.n_groups);
  const u64 g = c % C.n_groups;
  u32 k, d;
  wire_pair(N, p, &k, &d);
  if (!wire_cell_sent<N>(C, A.dst_rank, g, k, d)) {
    B.cell_bytes[c] = 0;
    B.cell_msgs[c] = 0;
    return;
  }
  u32 nm = 0, ni = 0, bad = 0;
  const u32 b = wire_cell<N>(P, C, heap, A.heap_head, g, k, d, A.round, nullptr, &nm, &ni, &bad);
  B.cell_bytes[c] = b;
  B.cell_msgs[c] = nm | (ni << 16);
  if (bad) atomicAdd((unsigned long long*)&B.totals[4], (unsigned long long)bad);
}

// block-wide exclusive scan of one value per thread; returns this thread's
// prefix and the block total in *total
__device__ __forceinline__ u64 block_scan_u64(u64 v, u64* total, u64* s_tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  u64 x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const u64 y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  u64 base = 0, t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
    if (i < w) base += s_tmp[i];
    t += s_tmp[i];
  }
  __syncthreads();
  *total = t;
  return base + x - v;
}

__global__ __launch_bounds__(256) void k_wire_batch(Params C, WireArgs A, WireBufs B) {
  __shared__ u64 s_tmp[4];
  const u32 bt = blockIdx.x;
  const u32 p = bt / A.nchunks, ch = bt % A.nchunks;
  const u64 g0 = (u64)ch * A.gpb;
  const u64 g1 = g0 + A.gpb < C.n_groups ? g0 + A.gpb : C.n_groups;
  const u64 base = (u64)p * C.n_groups;
  u64 carry = 0, msgs = 0, is = 0;
  for (u64 g = g0; g < g1; g += 256) {
    const u64 gi = g + threadIdx.x;
    u64 v = 0;
    u32 mm = 0;
    if (gi < g1) {
      v = B.cell_bytes[base + gi];
      mm = B.cell_msgs[base + gi];
    }
    u64 tot = 0;
    const u64 pre = block_scan_u64(v, &tot, s_tmp);
    if (gi < g1) B.cell_off[base + gi] = (u32)(carry + pre);
    carry += tot;
    u64 t2 = 0;
    block_scan_u64((u64)(mm & 0xFFFFu) | ((u64)(mm >> 16) << 32), &t2, s_tmp);
    msgs += t2 & 0xFFFFFFFFull;
    is += t2 >> 32;
  }
  if (threadIdx.x == 0) {
    u32 k, d;
    wire_pair(C.n, p, &k, &d);
    B.batch_pay[bt] = msgs ? carry + wire_trailer(A.deployment_id, A.addr[k], A.alen[k], A.bin_ver,
                                                  nullptr)
                           : 0;
    B.batch_msgs[bt] = (u32)msgs;
    B.batch_is[bt] = (u32)is;
  }
}

// Batches of more than kWireBatchSeg groups are scanned by segments, one
// block each (k_wire_batch_part: offsets within the segment and its totals),
// then per batch the segments' totals (k_wire_batch_fix) and the segment bases
// added to the offsets (k_wire_batch_add), instead of one block walking the
// whole batch
static constexpr u32 kWireBatchSeg = 4096;
__global__ __launch_bounds__(256) void k_wire_batch_part(Params C, WireArgs A, WireBufs B,
                                                         u64* seg_tot) {
  __shared__ u64 s_tmp[4];
  const u32 bt = blockIdx.x, sgi = blockIdx.y;
  const u32 p = bt / A.nchunks, ch = bt % A.nchunks;
  const u64 b0 = (u64)ch * A.gpb;
  const u64 b1 = b0 + A.gpb < C.n_groups ? b0 + A.gpb : C.n_groups;
  const u64 g0 = b0 + (u64)sgi * kWireBatchSeg;
  const u64 g1 = g0 + kWireBatchSeg < b1 ? g0 + kWireBatchSeg : b1;
  const u64 base = (u64)p * C.n_groups;
  u64 carry = 0, mi = 0;
  for (u64 g = g0; g < g1; g += 256) {  // uniform over the block (empty past b1)
    const u64 gi = g + threadIdx.x;
    u64 v = 0;
    u32 mm = 0;
    if (gi < g1) {
      v = B.cell_bytes[base + gi];
      mm = B.cell_msgs[base + gi];
    }
    u64 tot = 0;
    const u64 pre = block_scan_u64(v, &tot, s_tmp);
    if (gi < g1) B.cell_off[base + gi] = (u32)(carry + pre);
    carry += tot;
    u64 t2 = 0;
    block_scan_u64((u64)(mm & 0xFFFFu) | ((u64)(mm >> 16) << 32), &t2, s_tmp);
    mi += t2;
  }
  if (threadIdx.x == 0) {
    seg_tot[2 * ((u64)bt * gridDim.y + sgi)] = carry;
    seg_tot[2 * ((u64)bt * gridDim.y + sgi) + 1] = mi;  // messages | InstallSnapshots << 32
  }
}
__global__ __launch_bounds__(256) void k_wire_batch_fix(Params C, WireArgs A, WireBufs B,
                                                        u64* seg_tot, u32 nseg) {
  __shared__ u64 s_tmp[4];
  const u32 bt = blockIdx.x;
  u64 carry = 0, mi = 0;
  for (u32 s0 = 0; s0 < nseg; s0 += 256) {
    const u32 sgi = s0 + threadIdx.x;
    u64* t = &seg_tot[2 * ((u64)bt * nseg + sgi)];
    const u64 v = sgi < nseg ? t[0] : 0, m = sgi < nseg ? t[1] : 0;
    u64 tot = 0, t2 = 0;
    const u64 pre = block_scan_u64(v, &tot, s_tmp);
    block_scan_u64(m, &t2, s_tmp);
    if (sgi < nseg) t[0] = carry + pre;  // the segment's base within the batch
    carry += tot;
    mi += t2;
  }
  if (threadIdx.x == 0) {
    const u64 msgs = mi & 0xFFFFFFFFull;
    u32 k, d;
    wire_pair(C.n, bt / A.nchunks, &k, &d);
    B.batch_pay[bt] = msgs ? carry + wire_trailer(A.deployment_id, A.addr[k], A.alen[k], A.bin_ver,
                                                  nullptr)
                           : 0;
    B.batch_msgs[bt] = (u32)msgs;
    B.batch_is[bt] = (u32)(mi >> 32);
  }
}
__global__ __launch_bounds__(256) void k_wire_batch_add(Params C, WireArgs A, WireBufs B,
                                                        const u64* seg_tot) {
  const u32 bt = blockIdx.x, sgi = blockIdx.y;
  if (sgi == 0) return;
  const u64 add = seg_tot[2 * ((u64)bt * gridDim.y + sgi)];
  const u32 p = bt / A.nchunks, ch = bt % A.nchunks;
  const u64 b0 = (u64)ch * A.gpb;
  const u64 b1 = b0 + A.gpb < C.n_groups ? b0 + A.gpb : C.n_groups;
  const u64 g0 = b0 + (u64)sgi * kWireBatchSeg;
  const u64 g1 = g0 + kWireBatchSeg < b1 ? g0 + kWireBatchSeg : b1;
  const u64 base = (u64)p * C.n_groups;
  for (u64 gi = g0 + threadIdx.x; gi < g1; gi += 256) B.cell_off[base + gi] += (u32)add;
}

__global__ __launch_bounds__(256) void k_wire_frames(Params C, WireArgs A, WireBufs B,
                                                     u32 nbatch) {
  __shared__ u64 s_tmp[4];
  u64 carry = 0, fcarry = 0, msgs = 0, is = 0;
  for (u32 b0 = 0; b0 < nbatch; b0 += 256) {
    const u32 b = b0 + threadIdx.x;
    u64 fb = 0, ne = 0;
    if (b < nbatch && B.batch_msgs[b]) {
      fb = kWireHeader + B.batch_pay[b];
      ne = 1;
    }
    u64 tot = 0, ftot = 0;
    const u64 off = block_scan_u64(fb, &tot, s_tmp);
    const u64 fi = block_scan_u64(ne, &ftot, s_tmp);
    if (b < nbatch) {
      B.frame_off[b] = carry + off;
      if (ne) {
        const u32 p = b / A.nchunks, ch = b % A.nchunks;
        u32 k, d;
        wire_pair(C.n, p, &k, &d);
        WireFrame f;
        f.offset = carry + off;
        f.bytes = fb;
        f.first_group = (u64)ch * A.gpb;
        const u64 g1 = f.first_group + A.gpb < C.n_groups ? f.first_group + A.gpb : C.n_groups;
        f.src = k;
        f.dst = d;
        f.n_messages = B.batch_msgs[b];
        f.n_groups = (u32)(g1 - f.first_group);
        B.frames[fcarry + fi] = f;
      }
    }
    u64 t3 = 0;
    block_scan_u64(b < nbatch ? ((u64)B.batch_msgs[b] | ((u64)B.batch_is[b] << 32)) : 0, &t3,
                   s_tmp);
    msgs += t3 & 0xFFFFFFFFull;
    is += t3 >> 32;
    carry += tot;
    fcarry += ftot;
  }
  if (threadIdx.x == 0) {
    B.totals[0] = carry;
    B.totals[1] = fcarry;
    B.totals[2] = msgs;
    B.totals[3] = is;
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_wire_write(Planes P, Params C, WireArgs A, WireBufs B,
                                                    const u8* heap, u8* out) {
  const u64 c = (u64)blockIdx.x * 256 + threadIdx.x;
  if (c >= (u64)A.npairs * C.n_groups) return;
  if ((B.cell_msgs[c] & 0xFFFFu) == 0) return;
  const u32 p = (u32)(c / C.n_groups);
  const u64 g = c % C.n_groups;
  const u32 bt = p * A.nchunks + (u32)(g / A.gpb);
  u32 k, d;
  wire_pair(N, p, &k, &d);
  u32 nm = 0, ni = 0, bad = 0;
  wire_cell<N>(P, C, heap, A.heap_head, g, k, d, A.round,
               out + B.frame_off[bt] + kWireHeader + B.cell_off[c], &nm, &ni, &bad);
}

__global__ __launch_bounds__(256) void k_wire_trailers(Params C, WireArgs A, WireBufs B,
                                                       u32 nbatch, u8* out) {
  const u32 b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nbatch || !B.batch_msgs[b]) return;
  u32 k, d;
  wire_pair(C.n, b / A.nchunks, &k, &d);
  const u32 tl = wire_trailer(A.deployment_id, A.addr[k], A.alen[k], A.bin_ver, nullptr);
  wire_trailer(A.deployment_id, A.addr[k], A.alen[k], A.bin_ver,
               out + B.frame_off[b] + kWireHeader + B.batch_pay[b] - tl);
}

// crc32 of [p, p + n) by one lane, reading 16-B aligned words (the bytes
// outside [p, p + n) of the first and last word are read, not used)
__device__ u32 crc32_words(u32 crc, const u8* p, u64 n, const u32* table) {
  // table: 4 x 256 (slicing-by-4: table[k][i] = crc of byte i followed by k zeros)
  if (!n) return crc;
  u32 c = ~crc;
  const u8* a = (const u8*)((u64)p & ~15ull);
  u32 o = (u32)(p - a);
  u64 left = n;
  while (left) {
    const uint4 w = *(const uint4*)a;
    const u32 ws[4] = {w.x, w.y, w.z, w.w};
    if (o == 0 && left >= 16) {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const u32 x = c ^ ws[q];
        c = table[768 + (x & 0xFFu)] ^ table[512 + ((x >> 8) & 0xFFu)] ^
            table[256 + ((x >> 16) & 0xFFu)] ^ table[x >> 24];
      }
      left -= 16;
    } else {
      for (; o < 16 && left; o++, left--) {
        const u8 b = (u8)(ws[o >> 2] >> (8 * (o & 3)));
        c = table[(c ^ b) & 0xFFu] ^ (c >> 8);
      }
    }
    a += 16;
    o = 0;
  }
  return ~c;
}

// the 4 x 256 slicing table in LDS (one block of 256 threads)
__device__ __forceinline__ void crc_tables_lds(u32* t) {
  const u32 i = threadIdx.x;
  u32 v = crc_table_entry(i);
  t[i] = v;
  for (int k = 1; k < 4; k++) {
    v = (v >> 8) ^ crc_table_entry(v & 0xFFu);
    t[256 * k + i] = v;
  }
}

// crc32 of [p, p + n) by this block: one contiguous segment per thread.
// crc32_combine(c1, c2, l2) = c1 · x^(8 l2) ^ c2 is linear, so the whole
// crc is the XOR over segments of each segment's crc shifted to the end,
// c_t · x^(8 (n - hi_t)): every lane shifts its own crc (a few multmodp over
// the set bits of its distance to the end) and the block XOR-reduces, with no
// serial combine tree.
__device__ u32 block_crc32(const u8* p, u64 n, const u32* table, const u32* x2n, u32* s_crc) {
  const u32 T = blockDim.x, t = threadIdx.x;
  const u64 seg = (n + T - 1) / T;
  const u64 lo = seg * t < n ? seg * t : n;
  const u64 hi = lo + seg < n ? lo + seg : n;
  u32 c = crc32_words(0, p + lo, hi - lo, table);
  u64 rest = n - hi;
  if (c && rest) {
    u32 sh = 1u << 31;  // x^(8 rest) mod P
    for (u32 k = 3; rest; rest >>= 1, k++)
      if (rest & 1u) sh = crc_multmodp(x2n[k & 31], sh);
    c = crc_multmodp(sh, c);
  }
  for (int o = 32; o; o >>= 1) c ^= __shfl_xor(c, o, 64);
  if ((t & 63u) == 0) s_crc[t >> 6] = c;
  __syncthreads();
  u32 r = 0;
  for (u32 w = 0; w < T / 64; w++) r ^= s_crc[w];
  __syncthreads();
  return r;
}

// one block per frame whose payload is at most `big` bytes: its crc32 and header
__global__ __launch_bounds__(256) void k_wire_crc(WireBufs B, u8* out, u64 big) {
  __shared__ u32 s_table[1024], s_x2n[32], s_crc[256];
  const WireFrame f = B.frames[blockIdx.x];
  const u64 n = f.bytes - kWireHeader;
  if (n > big) return;  // (the whole block) k_wire_crc_seg / k_wire_crc_fin take it
  crc_tables_lds(s_table);
  if (threadIdx.x < 32) s_x2n[threadIdx.x] = kCrcX2n.v[threadIdx.x];
  __syncthreads();
  u8* fp = out + f.offset;
  const u32 c = block_crc32(fp + kWireHeader, n, s_table, s_x2n, s_crc);
  if (threadIdx.x == 0) wire_header_put(fp, n, c, s_table);
}
// A bigger frame's payload crc by 64 KiB segments, one block each, shifted to
// the payload's end and XORed into acc[frame] (crc32_combine is linear, as in
// block_crc32); then one lane per big frame writes its header.
struct WireEncSeg {
  u32 frame, pad;
  u64 start;  // payload offset of the segment
};
static constexpr u64 kWireEncSeg = 65536;
__global__ __launch_bounds__(256) void k_wire_crc_seg(WireBufs B, const WireEncSeg* seg, u32* acc,
                                                      const u8* out) {
  __shared__ u32 s_table[1024], s_x2n[32], s_crc[256];
  crc_tables_lds(s_table);
  if (threadIdx.x < 32) s_x2n[threadIdx.x] = kCrcX2n.v[threadIdx.x];
  __syncthreads();
  const WireEncSeg sg = seg[blockIdx.x];
  const WireFrame f = B.frames[sg.frame];
  const u64 n = f.bytes - kWireHeader;
  const u64 lo = sg.start, hi = n - lo < kWireEncSeg ? n : lo + kWireEncSeg;
  u32 c = block_crc32(out + f.offset + kWireHeader + lo, hi - lo, s_table, s_x2n, s_crc);
  if (threadIdx.x == 0) {
    u64 rest = n - hi;
    if (c && rest) {
      u32 sh = 1u << 31;  // x^(8 rest) mod P
      for (u32 k = 3; rest; rest >>= 1, k++)
        if (rest & 1u) sh = crc_multmodp(s_x2n[k & 31], sh);
      c = crc_multmodp(sh, c);
    }
    if (c) atomicXor(&acc[sg.frame], c);
  }
}
__global__ __launch_bounds__(256) void k_wire_crc_fin(WireBufs B, const u32* bigf, u32 nbig,
                                                      const u32* acc, u8* out) {
  __shared__ u32 s_table[1024];
  crc_tables_lds(s_table);
  __syncthreads();
  const u32 i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nbig) return;
  const WireFrame f = B.frames[bigf[i]];
  wire_header_put(out + f.offset, f.bytes - kWireHeader, acc[bigf[i]], s_table);
}

// ---------------------------------------------------------------- decode
struct WireIn {  // one inbound frame
  u64 offset, size;  // payload offset in the device copy, payload bytes
  u64 msg0;          // its first request in the output
  u64 pos0;          // its first slot in the single-pass position area
  u64 pad0;
  u32 n_msgs, pos_cap;  // requests; slots reserved for them (single pass)
  u32 crc_want, crc_acc;  // big frames: the header's payload crc; the XOR of the chunks' shifted crcs
  u32 status;  // 0 ok, 1 header crc, 2 payload crc, 3 malformed, 4 more requests than slots
  u32 pad;
};

// One block per frame of [f0, f0 + grid): both crc32s.  A frame longer than
// `big` has its header checked here and its payload crc left to
// k_wire_chunk_crc (many blocks per frame) and k_wire_crc_check.
__global__ __launch_bounds__(256) void k_wire_verify(const u8* data, WireIn* fr, u32 f0, u64 big) {
  __shared__ u32 s_table[1024], s_x2n[32], s_crc[256];
  crc_tables_lds(s_table);
  if (threadIdx.x < 32) s_x2n[threadIdx.x] = kCrcX2n.v[threadIdx.x];
  __syncthreads();
  const u32 fi = f0 + blockIdx.x;
  WireIn f = fr[fi];
  const bool chunked = f.size > big;
  const u32 c = chunked ? 0u : block_crc32(data + f.offset, f.size, s_table, s_x2n, s_crc);
  if (threadIdx.x == 0) {
    const u8* h = data + f.offset - 18;
    u8 hb[18];
    for (int i = 0; i < 18; i++) hb[i] = h[i];
    const u32 inc = ((u32)hb[10] << 24) | ((u32)hb[11] << 16) | ((u32)hb[12] << 8) | hb[13];
    hb[10] = hb[11] = hb[12] = hb[13] = 0;
    const u32 pc = ((u32)hb[14] << 24) | ((u32)hb[15] << 16) | ((u32)hb[16] << 8) | hb[17];
    u32 st = 0;
    // requestHeader.decode (tcp.go:93-112): the header crc, then the method —
    // a MessageBatch frame is raftType (100); snapshotType frames carry chunks
    const u32 method = ((u32)hb[0] << 8) | hb[1];
    if (crc32_update(0, hb, 18, s_table) != inc) st = 1;
    else if (method != 100u) st = 3;
    else if (!chunked && pc != c) st = 2;
    fr[fi].status = st;
    if (chunked) fr[fi].crc_want = pc;
  }
}

// A big frame's payload crc by 64 KiB segments, one block each: the
// segment's crc shifted to the frame's end (crc32_combine is linear, as in
// block_crc32) XORed into crc_acc; then one lane per frame compares.
static constexpr u32 kWireCrcSeg = 65536;
struct WireSeg {
  u32 frame, start;
};
__global__ __launch_bounds__(256) void k_wire_chunk_crc(const u8* data, WireIn* fr,
                                                        const WireSeg* seg) {
  __shared__ u32 s_table[1024], s_x2n[32], s_crc[256];
  crc_tables_lds(s_table);
  if (threadIdx.x < 32) s_x2n[threadIdx.x] = kCrcX2n.v[threadIdx.x];
  __syncthreads();
  const WireSeg sg = seg[blockIdx.x];
  const WireIn f = fr[sg.frame];
  const u64 lo = sg.start, hi = f.size - lo < kWireCrcSeg ? f.size : lo + kWireCrcSeg;
  u32 c = block_crc32(data + f.offset + lo, hi - lo, s_table, s_x2n, s_crc);
  if (threadIdx.x == 0) {
    u64 rest = f.size - hi;
    if (c && rest) {
      u32 sh = 1u << 31;  // x^(8 rest) mod P
      for (u32 k = 3; rest; rest >>= 1, k++)
        if (rest & 1u) sh = crc_multmodp(s_x2n[k & 31], sh);
      c = crc_multmodp(sh, c);
    }
    if (c) atomicXor(&fr[sg.frame].crc_acc, c);
  }
}
__global__ __launch_bounds__(64) void k_wire_crc_check(WireIn* fr, const u32* bigf, u32 nbig) {
  const u32 i = blockIdx.x * 64 + threadIdx.x;
  if (i >= nbig) return;
  WireIn& f = fr[bigf[i]];
  if (f.status == 0 && f.crc_acc != f.crc_want) f.status = 2;
}

// Decode is parallel per message: one block per frame finds the top-level
// requests of its MessageBatch (MessageBatch.Unmarshal, raft_optimized.go:
// 1051-1204: field 1 = a Message, 2-4 the trailer) in LDS windows;
// then one lane per message parses it (Message.Unmarshal), first counting its
// entries and Cmd bytes (scanned on the device for the output offsets), then
// writing the records.
struct WireMsgPos {
  u64 at, len;  // Message body [at, at + len) in the device copy of the input
};

// pass 0: count the frame's requests; pass 1: record where each one is (at
// msg0); pass 2: both at once into the frame's pos_cap slots from pos0 (the
// default: one walk; a frame with more requests than slots reports status 4
// and the caller walks twice).
// One block per frame: the block (one wave) stages an 8 KB window of the payload in LDS
// (coalesced), one lane walks the top-level fields inside it, and the window
// moves to wherever the walk stops (a field header near the window's end, or
// a request longer than the window, which is skipped without being read).
__device__ __forceinline__ u32 uni32(u32 x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ u64 uni64(u64 x) {
  return ((u64)uni32((u32)(x >> 32)) << 32) | uni32((u32)x);
}
static constexpr u32 kWireWin = 8192;
static constexpr u32 kWireWalkBlock = 64;
__global__ __launch_bounds__(kWireWalkBlock) void k_wire_bounds(const u8* data, WireIn* fr, int pass,
                                                     WireMsgPos* pos, u64 big, u32 f0) {
  __shared__ __attribute__((aligned(16))) u8 s_buf[kWireWin + 16];
  __shared__ u64 s_at, s_nm;
  __shared__ u32 s_state;  // 0 walking, 1 done, 2 bad
  const u32 fi = f0 + blockIdx.x;
  const WireIn f = fr[fi];
  if (f.status || f.size > big) return;  // a big frame is walked by chunks (below)
  const u8* p = data + f.offset;
  const u64 n = uni64(f.size);
  if (threadIdx.x == 0) {
    s_at = 0;
    s_nm = 0;
    s_state = 0;
  }
  __syncthreads();
  while (s_state == 0) {
    // 16-B aligned words from the one holding byte `base`, all in flight at once
    const u64 base = uni64(s_at);
    const u8* a0 = (const u8*)((u64)(p + base) & ~15ull);
    const u32 sh = (u32)((p + base) - a0);
    const u64 avail = n - base < kWireWin - sh ? n - base : kWireWin - sh;
    const u32 nw = (u32)((sh + avail + 15) / 16);
#pragma unroll
    for (u32 it = 0; it < kWireWin / 16 / kWireWalkBlock; it++) {
      const u32 wi = it * kWireWalkBlock + threadIdx.x;
      if (wi < nw) ((uint4*)s_buf)[wi] = ((const uint4*)a0)[wi];
    }
    __syncthreads();
    {
      // Every lane of the wave runs the walk with the same values (each LDS
      // read goes through readfirstlane), so the compiler keeps the walk in
      // scalar registers and scalar branches: a single-lane vector walk paid
      // a full wave issue for every instruction.
      u64 i = uni64(base), nm = uni64(s_nm);
      u32 st = 0;
      const u64 wend = base + avail;
      // a field header (tag + length, <= 20 bytes) must lie in the window
      // unless the frame ends first (s_buf indexed directly: LDS reads, not
      // flat loads through a captured pointer)
      for (;;) {
        if (i >= n) {
          st = 1;
          break;
        }
        if (i + 20 > wend && wend < n) break;  // move the window to i
        if (i + 8 <= wend) {
          // the usual request header (1-2 byte tag, length in the next bytes)
          // from 8 bytes taken with three aligned 4-byte LDS reads
          const u32 x = (u32)(i - base) + sh;
          const u32* w4 = (const u32*)s_buf;
          const u32 a = uni32(w4[x >> 2]), b = uni32(w4[(x >> 2) + 1]),
                    c = uni32(w4[(x >> 2) + 2]);
          const u32 s8 = (x & 3u) * 8u;
          const u64 lo = (u64)a | ((u64)b << 32);
          const u64 w8 = s8 ? (lo >> s8) | ((u64)c << (64 - s8)) : lo;
          u32 tb = 0;
          u64 tg = 0;
          if ((w8 & 0x80) == 0) {
            tg = w8 & 0x7F;
            tb = 1;
          } else if ((w8 & 0x8000) == 0) {
            tg = (w8 & 0x7F) | (((w8 >> 8) & 0x7F) << 7);
            tb = 2;
          }
          if (tb && (tg & 7) == 2) {
            u64 v = 0;
            u32 lb = 0;
            for (u32 k = 0; k < 6 && tb + k < 8; k++) {
              const u32 by = (u32)(w8 >> (8 * (tb + k))) & 0xFFu;
              v |= (u64)(by & 0x7F) << (7 * k);
              if (by < 0x80) {
                lb = k + 1;
                break;
              }
            }
            if (lb) {
              const u64 q = i + tb + lb;
              if (v > n - q) {
                st = 2;
                break;
              }
              if ((tg >> 3) == 1) {
                if (threadIdx.x == 0) {
                  if (pass == 1) pos[f.msg0 + nm] = WireMsgPos{f.offset + q, v};
                  else if (pass == 2 && nm < f.pos_cap) pos[f.pos0 + nm] = WireMsgPos{f.offset + q, v};
                }
                nm++;
              }
              i = q + v;
              continue;
            }
          }
        }
        u64 tag = 0;
        bool ok = false;
        u64 q = i;
        for (u32 bs = 0; bs < 64 && q < wend; bs += 7) {
          const u8 b = (u8)uni32(s_buf[(u32)(q++ - base) + sh]);
          tag |= (u64)(b & 0x7F) << bs;
          if (b < 0x80) {
            ok = true;
            break;
          }
        }
        if (!ok) {
          st = 2;
          break;
        }
        const u32 fn = (u32)(tag >> 3), wt = (u32)(tag & 7);
        if (wt == 0 || wt == 2) {
          u64 v = 0;
          ok = false;
          for (u32 bs = 0; bs < 64 && q < wend; bs += 7) {
            const u8 b = (u8)uni32(s_buf[(u32)(q++ - base) + sh]);
            v |= (u64)(b & 0x7F) << bs;
            if (b < 0x80) {
              ok = true;
              break;
            }
          }
          if (!ok) {
            st = 2;
            break;
          }
          if (wt == 2) {
            if (v > n - q) {
              st = 2;
              break;
            }
            if (fn == 1) {
              if (threadIdx.x == 0) {
                if (pass == 1) pos[f.msg0 + nm] = WireMsgPos{f.offset + q, v};
                else if (pass == 2 && nm < f.pos_cap) pos[f.pos0 + nm] = WireMsgPos{f.offset + q, v};
              }
              nm++;
            }
            q += v;
          }
        } else if (wt == 1 || wt == 5) {
          q += wt == 1 ? 8 : 4;
          if (q > n) {
            st = 2;
            break;
          }
        } else {
          st = 2;
          break;
        }
        i = q;
      }
      __syncthreads();  // every lane has read the window before lane 0 moves it
      if (threadIdx.x == 0) {
        s_at = i;
        s_nm = nm;
        s_state = st;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (s_state == 2) {
      fr[fi].status = 3;
    } else if (pass != 1) {
      fr[fi].n_msgs = (u32)s_nm;
      if (pass == 2 && s_nm > f.pos_cap) fr[fi].status = 4;
    }
  }
}

// ------------------------------------------------- big frames, walked by chunks
// A frame longer than the engine's walk threshold (rbe_engine.hip, wire_big) is
// cut into kWireChunk-byte chunks and its top level walked in three launches,
// so the walk no longer runs one field at a time across the whole frame:
//   k_wire_chunk_exit  block per chunk: for EVERY byte position p of the
//                      chunk, where the field walk started at p leaves the
//                      chunk (its exit) and how many requests it passes —
//                      each position's next field (wire_field_end) in LDS,
//                      then pointer doubling over the chunk (log2 steps)
//   k_wire_hop         lane per frame: the true walk from position 0, one
//                      exit per chunk (a frame of 7 MB: ~900 hops, not ~130k
//                      field headers); each chunk's entry and request base
//   k_wire_chunk_emit  block per chunk: the walk from the chunk's entry to
//                      its end, request positions written at their base
// Same rules and the same results as k_wire_bounds (MessageBatch.Unmarshal,
// raft_optimized.go:1051-1204; skipRaft for the trailer fields).
static constexpr u32 kWireChunk = 8192;
static constexpr u32 kWireNone = 0xFFFFFFFFu;  // exit of a malformed walk; entry of an unvisited chunk
struct WireChunk {
  u32 frame, start;  // the frame's index, the chunk's first payload byte
};
// One top-level field at payload position i (< n), bytes read through at(q):
// its end, or ~0 when malformed (k_wire_bounds' rules); a request (field 1,
// length-delimited) sets *req and its body start.
template <class At>
RBE_HD u64 wire_field_end(At at, u64 i, u64 n, u64* body, bool* req) {
  u64 q = i, tag = 0;
  bool ok = false;
  for (u32 bs = 0; bs < 64 && q < n; bs += 7) {
    const u8 b = at(q++);
    tag |= (u64)(b & 0x7F) << bs;
    if (b < 0x80) {
      ok = true;
      break;
    }
  }
  if (!ok) return ~0ull;
  const u32 wt = (u32)(tag & 7);
  if (wt == 0 || wt == 2) {
    u64 v = 0;
    ok = false;
    for (u32 bs = 0; bs < 64 && q < n; bs += 7) {
      const u8 b = at(q++);
      v |= (u64)(b & 0x7F) << bs;
      if (b < 0x80) {
        ok = true;
        break;
      }
    }
    if (!ok) return ~0ull;
    if (wt == 2) {
      if (v > n - q) return ~0ull;
      *body = q;
      *req = (tag >> 3) == 1;
      q += v;
    }
    return q;
  }
  if (wt == 1 || wt == 5) {
    q += wt == 1 ? 8 : 4;
    return q > n ? ~0ull : q;
  }
  return ~0ull;
}

__global__ __launch_bounds__(256) void k_wire_chunk_exit(const u8* data, const WireIn* fr,
                                                         const WireChunk* ch, u32* exitv,
                                                         u16* cntv) {
  constexpr u32 kPer = kWireChunk / 256;
  __shared__ __attribute__((aligned(16))) u8 s_b[kWireChunk + 32];
  __shared__ u32 s_x[kWireChunk];
  __shared__ u16 s_c[kWireChunk];
  const WireChunk c = ch[blockIdx.x];
  const WireIn f = fr[c.frame];
  if (f.status) return;
  const u64 n = f.size;
  const u32 cb = c.start;
  const u32 ce = (u32)(n - cb < kWireChunk ? n : cb + kWireChunk);
  // bytes [cb, ce + 32) (or to the frame's end): a field header that starts
  // in the chunk is at most 20 bytes
  const u32 le = (u32)(n - ce < 32 ? n : ce + 32);
  const u8* p = data + f.offset;
  for (u32 j = threadIdx.x; j < le - cb; j += 256) s_b[j] = p[cb + j];
  __syncthreads();
  auto at = [&](u64 q) { return s_b[(u32)q - cb]; };
#pragma unroll
  for (u32 k = 0; k < kPer; k++) {
    const u32 j = threadIdx.x + k * 256;
    if (j < ce - cb) {
      u64 body = 0;
      bool req = false;
      const u64 e = wire_field_end(at, cb + j, n, &body, &req);
      s_x[j] = e == ~0ull ? kWireNone : (u32)e;
      s_c[j] = req ? 1 : 0;
    }
  }
  __syncthreads();
  // pointer doubling: each pass composes every position's walk with the walk
  // from where it stops, until every walk has left the chunk (or failed)
  for (;;) {
    u32 nx[kPer];
    u32 nc[kPer];
    bool chg = false;
#pragma unroll
    for (u32 k = 0; k < kPer; k++) {
      const u32 j = threadIdx.x + k * 256;
      nx[k] = kWireNone;
      nc[k] = 0;
      if (j < ce - cb) {
        const u32 x = s_x[j];
        nx[k] = x;
        nc[k] = s_c[j];
        if (x != kWireNone && x < ce) {
          nx[k] = s_x[x - cb];
          nc[k] += s_c[x - cb];
          chg = true;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (u32 k = 0; k < kPer; k++) {
      const u32 j = threadIdx.x + k * 256;
      if (j < ce - cb) {
        s_x[j] = nx[k];
        s_c[j] = (u16)nc[k];
      }
    }
    if (!__syncthreads_or(chg)) break;
  }
  for (u32 j = threadIdx.x; j < ce - cb; j += 256) {
    exitv[f.offset + cb + j] = s_x[j];
    cntv[f.offset + cb + j] = s_c[j];
  }
}

// one lane per big frame (bigf: frame indexes, chunk0: each one's first chunk)
__global__ __launch_bounds__(64) void k_wire_hop(WireIn* fr, const u32* bigf, const u32* chunk0,
                                                 const u32* exitv, const u16* cntv, u32* ent,
                                                 u32* base) {
  if (threadIdx.x) return;
  const u32 fi = bigf[blockIdx.x];
  const WireIn f = fr[fi];
  if (f.status) return;
  const u32 c0 = chunk0[blockIdx.x];
  u64 e = 0, run = 0;
  bool bad = false;
  while (e < f.size) {
    const u32 c = c0 + (u32)(e / kWireChunk);
    const u32 x = exitv[f.offset + e];
    const u32 k = cntv[f.offset + e];
    ent[c] = (u32)e;
    base[c] = (u32)run;
    if (x == kWireNone) {
      bad = true;
      break;
    }
    run += k;
    e = x;
  }
  if (bad) {
    fr[fi].status = 3;
  } else {
    fr[fi].n_msgs = (u32)run;
    if (run > f.pos_cap) fr[fi].status = 4;
  }
}

// pass 2: positions into the frame's single-pass slots; pass 1: at msg0
__global__ __launch_bounds__(64) void k_wire_chunk_emit(const u8* data, const WireIn* fr,
                                                        const WireChunk* ch, const u32* ent,
                                                        const u32* base, int pass,
                                                        WireMsgPos* pos) {
  __shared__ __attribute__((aligned(16))) u8 s_b[kWireChunk + 32];
  const WireChunk c = ch[blockIdx.x];
  const WireIn f = fr[c.frame];
  const u32 e0 = ent[blockIdx.x];
  if (f.status || e0 == kWireNone) return;
  const u64 n = f.size;
  const u32 cb = c.start;
  const u32 ce = (u32)(n - cb < kWireChunk ? n : cb + kWireChunk);
  const u32 le = (u32)(n - ce < 32 ? n : ce + 32);
  const u8* p = data + f.offset;
  for (u32 j = threadIdx.x; j < le - cb; j += 64) s_b[j] = p[cb + j];
  __syncthreads();
  auto at = [&](u64 q) { return (u8)uni32(s_b[(u32)q - cb]); };
  u64 i = e0;
  u32 m = base[blockIdx.x];
  while (i < ce) {  // every field here is well formed: k_wire_hop walked it
    u64 body = 0;
    bool req = false;
    const u64 e = wire_field_end(at, i, n, &body, &req);
    if (req) {
      if (threadIdx.x == 0) {
        if (pass == 1) pos[f.msg0 + m] = WireMsgPos{f.offset + body, e - body};
        else if (m < f.pos_cap) pos[f.pos0 + m] = WireMsgPos{f.offset + body, e - body};
      }
      m++;
    }
    i = e;
  }
}

// Decode without a read-back in the middle (rbe_wire_ingest): the kernels
// after the walk are launched for capacities the host chose beforehand, read
// the true counts from the device, and raise WD_RETRY in `flags` instead of
// writing past a capacity (the host then decodes again with the counts it
// reads back); WD_CORRUPT reports a frame the walk refused.
enum : u32 { WD_CORRUPT = 1u, WD_RETRY = 2u };
// One block: each frame's first request (msg0, an exclusive scan of n_msgs in
// frame order), the total at tot[0], and the frames' statuses folded into flags.
__global__ __launch_bounds__(256) void k_wire_frames_scan(WireIn* fr, u32 nf, u64 cap_m, u64* tot,
                                                          u32* flags) {
  __shared__ u64 s_tmp[4];
  u64 carry = 0;
  u32 fl = 0;
  for (u32 b0 = 0; b0 < nf; b0 += 256) {
    const u32 i = b0 + threadIdx.x;
    u64 x = 0;
    if (i < nf) {
      const u32 st = fr[i].status;
      if (st == 4) fl |= WD_RETRY;
      else if (st) fl |= WD_CORRUPT;
      x = st ? 0 : fr[i].n_msgs;
    }
    u64 t = 0;
    const u64 pre = block_scan_u64(x, &t, s_tmp);
    if (i < nf) fr[i].msg0 = carry + pre;
    carry += t;
  }
  if (fl) atomicOr(flags, fl);
  if (threadIdx.x == 0) {
    tot[0] = carry;
    if (carry > cap_m) atomicOr(flags, WD_RETRY);
  }
}

// a frame's single-pass positions to their place in request order (at most
// cap_m positions in all: past it the decode is retried)
// (grid: frames x blocks per frame)
__global__ __launch_bounds__(256) void k_wire_compact(const WireIn* fr, const WireMsgPos* pos,
                                                      WireMsgPos* out, u64 cap_m) {
  const WireIn f = fr[blockIdx.x];
  if (f.status) return;
  for (u32 j = blockIdx.y * 256 + threadIdx.x; j < f.n_msgs && f.msg0 + j < cap_m;
       j += 256 * gridDim.y)
    out[f.msg0 + j] = pos[f.pos0 + j];
}

// pass 0: entries and Cmd bytes of each message; pass 1: the records.  With
// `dtm` (the no-read-back decode) nm is the launched capacity and *dtm the
// messages: pass 0 zeroes the counts past *dtm (so the scans over nm stay
// exact), pass 1 writes nothing when the scanned totals (*te, *tc) exceed the
// record capacities cap_e / cap_c, and nothing after a refused frame.
__global__ __launch_bounds__(256) void k_wire_parse(const u8* data, const WireMsgPos* pos,
                                                    u64 nm, int pass, u64* ecnt, u64* ccnt,
                                                    rbe_message* msgs, rbe_entry* ents, u8* cmd,
                                                    u32* err, const u64* dtm = nullptr,
                                                    const u64* te = nullptr, const u64* tc = nullptr,
                                                    u64 cap_e = 0, u64 cap_c = 0,
                                                    u32* flags = nullptr) {
  const u64 j = (u64)blockIdx.x * 256 + threadIdx.x;
  if (j >= nm) return;
  if (dtm) {
    if (*flags) return;
    if (j >= *dtm) {
      if (!pass) ecnt[j] = ccnt[j] = 0;
      return;
    }
    if (pass && (*te > cap_e || *tc > cap_c)) {
      if (j == 0) atomicOr(flags, WD_RETRY);
      return;
    }
  }
  const WireMsgPos q = pos[j];
  WireRd rd{data, q.at + q.len, q.at, false};
  u64 cb = pass ? ccnt[j] : 0;
  const u32 ne = wire_message_get(rd, q.at + q.len, pass ? &msgs[j] : nullptr,
                                  pass ? &ents[ecnt[j]] : nullptr, pass ? cmd : nullptr, &cb);
  if (rd.bad) {
    atomicOr(err, 1u);
    return;
  }
  if (!pass) {
    ecnt[j] = ne;
    ccnt[j] = cb;
  }
}

// exclusive scan of v[0, n) in place (three launches: block sums, their scan
// by one block, the adds); top must hold grid + 1 words, top[grid] = total
__global__ __launch_bounds__(256) void k_scan_blocks(u64* v, u64 n, u64* top) {
  __shared__ u64 s_tmp[4];
  const u64 j = (u64)blockIdx.x * 256 + threadIdx.x;
  const u64 x = j < n ? v[j] : 0;
  u64 t = 0;
  const u64 pre = block_scan_u64(x, &t, s_tmp);
  if (j < n) v[j] = pre;
  if (threadIdx.x == 0) top[blockIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_scan_top(u64* top, u32 nb) {
  __shared__ u64 s_tmp[4];
  u64 carry = 0;
  for (u32 b0 = 0; b0 < nb; b0 += 256) {
    const u32 b = b0 + threadIdx.x;
    const u64 x = b < nb ? top[b] : 0;
    u64 t = 0;
    const u64 pre = block_scan_u64(x, &t, s_tmp);
    if (b < nb) top[b] = carry + pre;
    carry += t;
  }
  if (threadIdx.x == 0) top[nb] = carry;
}
__global__ __launch_bounds__(256) void k_scan_add(u64* v, u64 n, const u64* top) {
  const u64 j = (u64)blockIdx.x * 256 + threadIdx.x;
  if (j < n) v[j] += top[blockIdx.x];
}

}  // namespace rbe

// ---------------------------------------------------------------- ingest
// rbe_wire_ingest (rbe_ingest.h): decoded records → inbox plane slots.
namespace rbe {

// With `dtm` (the no-read-back decode) nm is the launched capacity: the
// positions past *dtm become drop keys (sorted last, never listed or counted)
template <int N>
__global__ __launch_bounds__(256) void k_ing_key(Params C, u64 heap_cap, rbe_message* msgs,
                                                 const rbe_entry* ents, const u64* ent0, u64 nm,
                                                 u64* key, u32* idx, u64* hb, u32* err,
                                                 unsigned long long* ndrop, const u64* ids,
                                                 const u64* dtm = nullptr,
                                                 const u32* flags = nullptr) {
  const u64 j = (u64)blockIdx.x * 256 + threadIdx.x;
  if (j >= nm) return;
  if (dtm && (j >= *dtm || *flags)) {
    key[j] = ing_drop_key(C);
    idx[j] = (u32)j;
    hb[j] = 0;
    return;
  }
  u32 e = 0;
  u64 h = 0;
  if (ids) {  // node ids → internal ids, in place for the walk that scatters them
    rbe_message m = msgs[j];
    ingest_ids<N>(C, ids, m);
    msgs[j] = m;
  }
  const u64 k = ingest_check<N>(C, heap_cap, msgs[j], ents + ent0[j], &e, &h);
  key[j] = k;
  idx[j] = (u32)j;
  hb[j] = h;
  if (e) atomicOr(err, e);
  else if (k == ing_drop_key(C)) atomicAdd(ndrop, 1ull);
}

// heap bytes in sorted order (scanned next into each message's heap offset)
__global__ __launch_bounds__(256) void k_ing_gather(const u32* sidx, const u64* hb, u64* hs, u64 nm) {
  const u64 p = (u64)blockIdx.x * 256 + threadIdx.x;
  if (p < nm) hs[p] = hb[sidx[p]];
}

template <int N, bool WRITE>
__global__ __launch_bounds__(256) void k_ing_walk(Planes P, Params C, u32 par, u32 round,
                                                  const u64* skey, const u32* sidx, u64 nm,
                                                  const rbe_message* msgs, const rbe_entry* ents,
                                                  const u64* ent0, const u64* cmd0, const u8* cmd,
                                                  u8* heap, u64 heap_cap, u64 base, const u64* hs,
                                                  u32* err, const u32* gate = nullptr) {
  const u64 p = (u64)blockIdx.x * 256 + threadIdx.x;
  if (p >= nm || !ingest_run_start(C, skey, p)) return;
  // the writing walk of the no-read-back ingest: nothing at all when the
  // checking walk or the decode found anything (all-or-nothing)
  if (WRITE && gate && (gate[0] | gate[1])) return;
  const u64 q = ingest_run_end(C, skey, p, nm);
  const u32 e = ingest_sender<N, WRITE>(P, C, par, round, skey, sidx, p, q, msgs, ents, ent0, cmd0,
                                        cmd, heap, heap_cap, base, hs);
  if (e) atomicOr(err, e);
}

}  // namespace rbe
