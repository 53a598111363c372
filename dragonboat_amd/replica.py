"""Replica-per-GPU mode: the host side of the
cross-rank message exchange.

With `rep_world = W > 1`, replica k of group g is stepped on rank (g + k) % W,
so the messages a Raft round produces between replicas of one group cross
ranks.  In dragonboat they would leave through the transport
(node.go:888-905 `sendMessages` → nodehost.go:1724 `sendMessage` →
transport.go:392-557); here one round's cross-rank traffic moves as one
all-to-all after the round:

  1. `rbe_xchg_pack` (device): every owned sender packs the count words,
     messages and Replicate entries it produced for replicas owned elsewhere
     into fixed-size records, bucketed per destination rank and stream;
  2. the per-(peer, stream) record counts go out with one small all-to-all;
  3. the records go out with one `all_to_all_single` (RCCL over xGMI with the
     nccl backend; gloo in the CPU tests and the one-GPU two-process test,
     staged through host memory);
  4. `rbe_xchg_unpack` (device): clears the remote senders' count words of the
     round and scatters the received records into the same plane positions.

Records name their destination slot, so order within a stream is free and
the round that follows is bit-identical to a single-rank run of all replicas
(tests/test_replica_gloo.py, tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

from .engine import xchg_record_bytes

# the fixed-capacity layout's chunk header (rbe_xchg.h XHdr)
XHDR_BYTES = 64

STREAMS = 3  # count words, messages, entries


def initial_caps(n_rep: int, n: int, world: int) -> List[int]:
    """Per-(peer, stream) record capacities to start with.  The count stream
    is bounded by the lists from owned senders to one peer; messages and
    entries start at one per list and grow on demand (ReplicaExchange.grow)."""
    lists = -(-n_rep * max(n - 1, 1) // world) + 64
    return [lists, lists, lists // 2 + 64]


class ReplicaExchange:
    """Drives the exchange of one engine (the HIP `Engine`, or the host build
    used by the CPU tests — anything with `xchg_pack`/`xchg_unpack`).

    `buf_device` is where the pack buffer lives (the engine's GPU, or "cpu"
    for the host build); `comm_device` is where the collectives run ("cuda:i"
    for RCCL, "cpu" for gloo).  When they differ, records are staged through
    the comm device."""

    def __init__(self, engine, group=None, buf_device="cpu", comm_device="cpu",
                 caps: Optional[Sequence[int]] = None, fixed: bool = False):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.eng = engine
        self.group = group
        self.world = int(engine.cfg.rep_world)
        self.rank = int(engine.cfg.rep_rank)
        if self.world < 2:
            raise ValueError("replica exchange needs rep_world >= 2")
        if dist.get_world_size(group) != self.world or dist.get_rank(group) != self.rank:
            raise ValueError(f"process group (rank {dist.get_rank(group)} of "
                             f"{dist.get_world_size(group)}) does not match the engine's "
                             f"rep_rank {self.rank} of rep_world {self.world}")
        self.rec = xchg_record_bytes()
        n = int(engine.cfg.n_replicas)
        # caps: the fixed chunks' per-stream capacities (equal on every rank);
        # ccaps: the counted exchange's regions (this rank's own, grown on demand)
        self.caps = list(caps) if caps else initial_caps(int(engine.cfg.n_groups) * n, n,
                                                         self.world)
        self.ccaps = list(self.caps)
        self.buf_device = torch.device(buf_device)
        self.comm_device = torch.device(comm_device)
        self.bytes_sent = 0
        self.records_sent = [0] * STREAMS
        # fixed: equal chunks with a count header per peer, no host-side count
        # read (rbe_xchg_pack_fixed).  A round whose records did not fit its
        # chunks (the headers say so on every rank) is repaired by a counted
        # exchange of the same round (exchange_fixed): never invalid
        self.fixed = fixed
        self.repaired = 0  # fixed rounds that took the counted second pass
        # per stream, over the counted exchanges since reset_peak: the most
        # records one (rank, peer) pair moved, and the sum / number of such
        # counts (what to_fixed sizes the chunks by)
        self.peak = [0] * STREAMS
        self.csum = [0] * STREAMS
        self.cn = 0
        self.cbuf = None
        self._alloc()

    # --- layout: per peer p, streams t = 0..2, cap[t] records each (rbe_xchg.h xchg_region)
    def _per_peer(self, caps=None) -> int:
        return sum(c * b for c, b in zip(self.caps if caps is None else caps, self.rec))

    def _region(self, p: int, t: int) -> int:  # (the counted layout)
        return p * self._per_peer(self.ccaps) + sum(self.ccaps[i] * self.rec[i] for i in range(t))

    def _alloc(self):
        """The fixed layout's send / receive chunks (fixed mode): a full chunk
        per peer, a header-only one for this rank itself (rbe_xchg.h
        xchg_fixed_off), so the all-to-all moves nothing it does not need."""
        if not self.fixed:
            return
        per = self._per_peer() + XHDR_BYTES
        self.splits = [XHDR_BYTES if p == self.rank else per for p in range(self.world)]
        self.buf = self.torch.empty(sum(self.splits), dtype=self.torch.uint8,
                                    device=self.buf_device)
        self.recv = self.torch.empty_like(self.buf, device=self.comm_device)
        self.recv_buf = self.recv if self.comm_device == self.buf_device else \
            self.torch.empty_like(self.buf)

    def _calloc(self):
        """The counted layout's pack buffer (its regions grow on demand)."""
        need = self.world * self._per_peer(self.ccaps)
        if self.cbuf is None or self.cbuf.numel() < need:
            self.cbuf = self.torch.empty(need, dtype=self.torch.uint8, device=self.buf_device)

    def exchange_fixed(self):
        """One round's exchange without reading counts on the host: pack into
        equal chunks (headers carry the counts), one all_to_all_single, unpack.
        With the buffers on the engine's GPU and RCCL, the collective is
        enqueued on the engine's own stream, so nothing waits on the host."""
        torch, dist = self.torch, self.dist
        self.eng.xchg_pack_fixed(self.buf.data_ptr(), self.caps)
        if self.buf_device.type == "cuda" and self.comm_device == self.buf_device:
            s = torch.cuda.ExternalStream(self.eng.stream_handle(), device=self.buf_device)
            with torch.cuda.stream(s):
                dist.all_to_all_single(self.recv, self.buf, output_split_sizes=self.splits,
                                       input_split_sizes=self.splits, group=self.group)
        else:  # gloo: staged through host memory
            if self.buf_device.type == "cuda":
                self.eng.sync()
            send = self.buf if self.buf.device == self.comm_device else self.buf.to(self.comm_device)
            dist.all_to_all_single(self.recv, send, output_split_sizes=self.splits,
                                   input_split_sizes=self.splits, group=self.group)
            if self.recv_buf is not self.recv:
                self.recv_buf.copy_(self.recv)
                torch.cuda.current_stream(self.buf_device).synchronize()
        self.bytes_sent += self.buf.numel() - XHDR_BYTES  # (the own header stays local)
        self.eng.xchg_unpack_fixed(self.recv_buf.data_ptr(), self.caps)
        # one 4-byte read (rbe_xchg_status, read-and-clear): set on every rank
        # alike when any rank's records outgrew a chunk this round, because
        # every chunk header reaches every rank.  The outboxes of the round
        # are intact until the next step, so a counted exchange of the same
        # round delivers every record again, each to its own slot (idempotent)
        if self.eng.xchg_status():
            self.repaired += 1
            self.exchange(stats=False)

    def check(self) -> int:
        """The number of fixed rounds repaired by a counted second pass."""
        return self.repaired

    def reset_peak(self):
        self.peak = [0] * STREAMS
        self.csum = [0] * STREAMS
        self.cn = 0

    def to_fixed(self, margin: float = 1.25):
        """Switch to the fixed-capacity exchange with chunks sized from the
        counted rounds seen since reset_peak: every (peer, stream) capacity is
        `margin` times the MEAN count of one (rank, peer) pair over those
        rounds and all ranks (plus a small floor), so the bytes moved per round
        stay near `margin` times the records.  A round above that is repaired
        by a counted second pass (exchange_fixed), so the chunks need not hold
        the peak.  Collective: every rank calls it (the chunk size must agree)."""
        t = self.torch.tensor(self.peak + self.csum + [self.cn], dtype=self.torch.int64,
                              device=self.comm_device)
        mx = t.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX, group=self.group)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        self.peak = [int(x) for x in mx[:STREAMS].tolist()]
        tot, n = t[STREAMS:2 * STREAMS].tolist(), max(1, int(t[-1]))
        self.mean = [x / n for x in tot]
        self.caps = [int(m * margin) + 64 for m in self.mean]
        self.fixed = True
        self._alloc()

    def pad_ratio(self) -> float:
        """Bytes of one fixed chunk (one peer) over the bytes of the mean
        counted round's records to one peer since reset_peak."""
        mean = getattr(self, "mean", self.peak)
        rec = sum(m * b for m, b in zip(mean, self.rec))
        return (self._per_peer() + XHDR_BYTES) / rec if rec else float("inf")

    def fixed_bytes_per_round(self) -> int:
        """Bytes one fixed-layout exchange moves from this rank (all peers)."""
        return (self.world - 1) * (self._per_peer() + XHDR_BYTES)

    def grow(self, counts: Sequence[int]):
        need = [max(counts[p * STREAMS + t] for p in range(self.world)) for t in range(STREAMS)]
        self.ccaps = [max(c, n + n // 4 + 64) for c, n in zip(self.ccaps, need)]
        self._calloc()

    def exchange(self, stats: bool = True):
        """Move the last round's cross-rank records with their counts read on
        the host (call after every round; exchange_fixed calls it for a round
        its chunks could not hold, with stats=False)."""
        torch, dist = self.torch, self.dist
        self._calloc()
        fits, counts = self.eng.xchg_pack(self.cbuf.data_ptr(), self.ccaps)
        if not fits:
            self.grow(counts)
            fits, counts = self.eng.xchg_pack(self.cbuf.data_ptr(), self.ccaps)
            if not fits:
                raise RuntimeError("replica exchange: pack overflow after growing")
        W, S = self.world, STREAMS
        if stats:
            self.cn += W - 1
            for t in range(S):
                c = [counts[p * S + t] for p in range(W) if p != self.rank]
                self.peak[t] = max([self.peak[t]] + c)
                self.csum[t] += sum(c)
        send_cnt = torch.tensor(counts, dtype=torch.int64, device=self.comm_device)
        recv_cnt = torch.empty_like(send_cnt)
        dist.all_to_all_single(recv_cnt, send_cnt, group=self.group)
        rc = recv_cnt.tolist()
        # compact the populated prefix of every (peer, stream) region
        parts, out_split = [], []
        for p in range(W):
            nbytes = 0
            for t in range(S):
                b = counts[p * S + t] * self.rec[t]
                if b:
                    o = self._region(p, t)
                    parts.append(self.cbuf[o:o + b])
                    nbytes += b
            out_split.append(nbytes)
        send = torch.cat(parts) if parts else torch.empty(0, dtype=torch.uint8,
                                                          device=self.buf_device)
        if send.device != self.comm_device:
            send = send.to(self.comm_device)
        in_split = [sum(rc[p * S + t] * self.rec[t] for t in range(S)) for p in range(W)]
        recv = torch.empty(sum(in_split), dtype=torch.uint8, device=self.comm_device)
        dist.all_to_all_single(recv, send, output_split_sizes=in_split,
                               input_split_sizes=out_split, group=self.group)
        self.bytes_sent += sum(out_split)
        if stats:
            for t in range(S):
                self.records_sent[t] += sum(counts[p * S + t] for p in range(W))
        # per stream: the records of every source rank, back to back
        streams: List[List] = [[] for _ in range(S)]
        at = 0
        for p in range(W):
            for t in range(S):
                b = rc[p * S + t] * self.rec[t]
                if b:
                    streams[t].append(recv[at:at + b])
                at += b
        cat = []
        for t in range(S):
            x = torch.cat(streams[t]) if streams[t] else torch.empty(0, dtype=torch.uint8,
                                                                     device=self.comm_device)
            if x.device != self.buf_device:
                x = x.to(self.buf_device)
            cat.append(x)
        if self.buf_device.type == "cuda":
            torch.cuda.current_stream(self.buf_device).synchronize()
        n = [cat[t].numel() // self.rec[t] for t in range(S)]
        self.eng.xchg_unpack(cat[0].data_ptr(), n[0], cat[1].data_ptr(), n[1],
                             cat[2].data_ptr(), n[2])

    def iso_sync(self):
        """Before an isolation-schedule epoch round (cfg.iso_period): the
        leader bits of every rank's replicas, ORed (a sum: each replica has
        one owner) and handed to the engine (rbe_iso_leaders /
        rbe_set_iso_leaders).  A no-op on other rounds."""
        bits = self.eng.iso_leaders()
        if bits is None:
            return
        t = self.torch.from_numpy(bits.astype("int32")).to(self.comm_device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        self.eng.set_iso_leaders(t.cpu().numpy().astype("uint8"))

    def step(self):
        """One round of the owned replicas (the exchange of the round before
        must have run)."""
        self.iso_sync()
        self.eng.step()

    def run(self, rounds: int):
        """`rounds` lockstep rounds of the owned replicas, exchanging after each."""
        for _ in range(rounds):
            self.step()
            if self.fixed:
                self.exchange_fixed()
            else:
                self.exchange()
        self.check()
