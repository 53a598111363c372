"""TEST INFRASTRUCTURE — CPU restatement of the reference's transport wire
format, the checker for the device codec (dragonboat_amd/csrc/rbe_wire.h).
Only tests/ may import it.

What it restates:
- protobuf varints: encodeVarintRaft / sovRaft (raftpb/raft.pb.go:2559-2567, 2879-2887);
- raftpb.Message.MarshalTo / Size (raft.pb.go:2230-2294, 2748-2773) with the
  embedded Snapshot (2140-2217, 2716-2746) and its Membership (2017-2089,
  2657-2690);
- raftpb.Entry in colfer form, marshalTo / Size (raftpb/raft_optimized.go:79-295);
- raftpb.MessageBatch.MarshalTo (raft.pb.go:2415-2443);
- the TCP frame: magic 0xAE7D, the 18-byte requestHeader (method, size,
  header crc, payload crc, big endian) and the IEEE crc32 of the payload
  (internal/transport/tcp.go:44-110, 149-185);
- the decoders: Message.Unmarshal (raft_optimized.go:654-979), Entry.unmarshal
  (303-651), MessageBatch.Unmarshal (1051-1204), requestHeader.decode
  (tcp.go:93-116).

Parity pin: the reference holds no byte-level golden vectors for these types
(raftpb/raft_test.go checks round trips and size bounds only), so the
restatement is pinned by the published algorithms' own check values (CRC-32
"123456789" = 0xCBF43926; the protobuf varint examples 1 = 01, 150 = 96 01,
300 = AC 02), by zlib's crc32 as an independent implementation, and by
encode -> decode round trips; the byte layout is "parity unpinned" against
reference-produced bytes (no Go toolchain here).
"""
from __future__ import annotations

MAGIC = b"\xAE\x7D"
RAFT_TYPE = 100          # tcp.go:61 raftType
HEADER_SIZE = 18         # tcp.go:60 requestHeaderSize
INSTALL_SNAPSHOT = 16    # raftpb MessageType (raft.pb.go:23-51)

# ------------------------------------------------------------------ crc32 (IEEE)
_POLY = 0xEDB88320
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32(data: bytes, crc: int = 0) -> int:
    """crc32.ChecksumIEEE (reflected, init/xorout 0xFFFFFFFF)."""
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _multmodp(a: int, b: int) -> int:
    """a * b mod P in the reflected GF(2) representation (zlib crc32.c multmodp)."""
    m, p = 1 << 31, 0
    while True:
        if a & m:
            p ^= b
            if (a & (m - 1)) == 0:
                break
        m >>= 1
        b = (b >> 1) ^ _POLY if b & 1 else b >> 1
    return p


_X2N = [1 << 30]
for _k in range(1, 32):
    _X2N.append(_multmodp(_X2N[-1], _X2N[-1]))


def x2nmodp(n: int, k: int) -> int:
    p = 1 << 31
    while n:
        if n & 1:
            p = _multmodp(_X2N[k & 31], p)
        n >>= 1
        k += 1
    return p


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    """crc32 of A||B from crc32(A), crc32(B), len(B) (zlib crc32_combine)."""
    return _multmodp(x2nmodp(len2, 3), crc1) ^ crc2


# ------------------------------------------------------------------ varints
def sov(x: int) -> int:
    n = 1
    while x >= 0x80:
        x >>= 7
        n += 1
    return n


def put_varint(out: bytearray, x: int):
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)


def get_varint(buf: bytes, i: int):
    x, shift = 0, 0
    while True:
        if shift >= 64:
            raise ValueError("varint overflow")
        if i >= len(buf):
            raise ValueError("unexpected EOF")
        b = buf[i]
        i += 1
        x |= (b & 0x7F) << shift
        if b < 0x80:
            return x & 0xFFFFFFFFFFFFFFFF, i
        shift += 7


# ------------------------------------------------------------------ colfer Entry
def _colfer_u64(out: bytearray, field: int, x: int):
    if x >= 1 << 49:
        out.append(field | 0x80)
        out += x.to_bytes(8, "big")
    elif x != 0:
        out.append(field)
        put_varint(out, x)


def entry_bytes(e: dict) -> bytes:
    """Entry.marshalTo (raft_optimized.go:161-295): fields 0-6 when non-zero,
    Cmd (7) when non-empty, then 0x7f."""
    out = bytearray()
    _colfer_u64(out, 0, e.get("term", 0))
    _colfer_u64(out, 1, e.get("index", 0))
    t = e.get("type", 0)
    if t != 0:  # EntryType is int32; the engine's types are non-negative
        out.append(2)
        put_varint(out, t)
    _colfer_u64(out, 3, e.get("key", 0))
    _colfer_u64(out, 4, e.get("client_id", 0))
    _colfer_u64(out, 5, e.get("series_id", 0))
    _colfer_u64(out, 6, e.get("responded_to", 0))
    cmd = e.get("cmd", b"")
    if cmd:
        out.append(7)
        put_varint(out, len(cmd))
        out += cmd
    out.append(0x7F)
    return bytes(out)


def entry_decode(data: bytes) -> dict:
    """Entry.unmarshal (raft_optimized.go:303-651)."""
    e = {"term": 0, "index": 0, "type": 0, "key": 0, "client_id": 0, "series_id": 0,
         "responded_to": 0, "cmd": b""}
    names = ["term", "index", "type", "key", "client_id", "series_id", "responded_to"]
    i = 0
    h = data[i]
    i += 1
    for f, name in enumerate(names):
        if h == f:
            if f == 2:
                x, i = get_varint(data, i)
                e[name] = x
            else:  # colfer u64: the 9th byte carries 8 bits
                x, shift = 0, 0
                while True:
                    b = data[i]
                    i += 1
                    if b < 0x80 or shift == 56:
                        x |= b << shift
                        break
                    x |= (b & 0x7F) << shift
                    shift += 7
                e[name] = x
            h = data[i]
            i += 1
        elif h == (f | 0x80):
            if f == 2:
                x, i = get_varint(data, i)
                e[name] = (-x) & 0xFFFFFFFF
            else:
                e[name] = int.from_bytes(data[i:i + 8], "big")
                i += 8
            h = data[i]
            i += 1
    if h == 7:
        n, i = get_varint(data, i)
        end = _take(data, i, n)
        e["cmd"] = bytes(data[i:end])
        i = end
        h = data[i]
        i += 1
    if h != 0x7F:
        raise ValueError(f"colfer: bad header {h:#x}")
    return e


# ------------------------------------------------------------------ Message
def _field_varint(out: bytearray, tag: int, x: int):
    out.append(tag)
    put_varint(out, x)


def snapshot_bytes(index: int = 0, term: int = 0, filepath: str = "", file_size: int = 0) -> bytes:
    """Snapshot.MarshalTo (raft.pb.go:2140-2217) with no membership, checksum
    or flags: the Snapshot every non-InstallSnapshot message embeds (empty), or
    getMaxSizedMsg's (raftpb/raft_test.go:319-346: path, size, index, term)."""
    out = bytearray()
    fp = filepath.encode()
    out.append(0x12)                 # Filepath
    put_varint(out, len(fp))
    out += fp
    _field_varint(out, 0x18, file_size)  # FileSize
    _field_varint(out, 0x20, index)  # Index
    _field_varint(out, 0x28, term)   # Term
    out += b"\x32\x02\x08\x00"      # Membership{ConfigChangeId: 0}
    out += b"\x48\x00"              # Dummy
    _field_varint(out, 0x50, 0)      # ClusterId
    _field_varint(out, 0x58, 0)      # Type
    out += b"\x60\x00"              # Imported
    _field_varint(out, 0x68, 0)      # OnDiskIndex
    out += b"\x70\x00"              # Witness
    return bytes(out)


def message_bytes(m: dict, entries: list, snapshot: bytes = None) -> bytes:
    """Message.MarshalTo (raft.pb.go:2230-2294); `snapshot` the marshaled
    Snapshot field (default: the empty one)."""
    out = bytearray()
    _field_varint(out, 0x08, m["type"])
    _field_varint(out, 0x10, m["to"])
    _field_varint(out, 0x18, m["from"])
    _field_varint(out, 0x20, m["cluster_id"])
    _field_varint(out, 0x28, m["term"])
    _field_varint(out, 0x30, m["log_term"])
    _field_varint(out, 0x38, m["log_index"])
    _field_varint(out, 0x40, m["commit"])
    out += b"\x48" + (b"\x01" if m["reject"] else b"\x00")
    _field_varint(out, 0x50, m["hint"])
    for e in entries:
        eb = entry_bytes(e)
        out.append(0x5A)
        put_varint(out, len(eb))
        out += eb
    sb = snapshot_bytes() if snapshot is None else snapshot
    out.append(0x62)
    put_varint(out, len(sb))
    out += sb
    _field_varint(out, 0x68, m["hint_high"])
    return bytes(out)


def batch_bytes(msgs: list, deployment_id: int, source_address: str, bin_ver: int) -> bytes:
    """MessageBatch.MarshalTo (raft.pb.go:2415-2443); msgs = [(message, entries)]."""
    out = bytearray()
    for m, ents in msgs:
        mb = message_bytes(m, ents)
        out.append(0x0A)
        put_varint(out, len(mb))
        out += mb
    _field_varint(out, 0x10, deployment_id)
    a = source_address.encode()
    out.append(0x1A)
    put_varint(out, len(a))
    out += a
    _field_varint(out, 0x20, bin_ver)
    return bytes(out)


SNAPSHOT_TYPE = 200      # tcp.go:62 snapshotType


def request_header_encode(method: int, size: int, crc: int) -> bytes:
    """requestHeader.encode (tcp.go:80-91): method, size, a zero crc slot, the
    payload crc; then the IEEE crc32 of those 18 bytes goes into the slot."""
    h = bytearray(HEADER_SIZE)
    h[0:2] = method.to_bytes(2, "big")
    h[2:10] = size.to_bytes(8, "big")
    h[14:18] = crc.to_bytes(4, "big")
    h[10:14] = crc32(bytes(h)).to_bytes(4, "big")
    return bytes(h)


def request_header_decode(buf: bytes):
    """requestHeader.decode (tcp.go:93-112): None when the header crc fails or
    the method is neither raftType nor snapshotType, else (method, size, crc)."""
    if len(buf) < HEADER_SIZE:
        return None
    h = bytearray(buf[:HEADER_SIZE])
    inc = int.from_bytes(h[10:14], "big")
    h[10:14] = b"\0\0\0\0"
    if crc32(bytes(h)) != inc:
        return None
    method = int.from_bytes(h[0:2], "big")
    if method not in (RAFT_TYPE, SNAPSHOT_TYPE):
        return None
    return method, int.from_bytes(h[2:10], "big"), int.from_bytes(h[14:18], "big")


def frame(payload: bytes) -> bytes:
    """writeMessage (tcp.go:149-185): magic, requestHeader.encode (80-91), payload."""
    return MAGIC + request_header_encode(RAFT_TYPE, len(payload), crc32(payload)) + payload


# ------------------------------------------------------------------ size bounds
ENTRY_NON_CMD_FIELDS_SIZE = 16 * 8  # settings.EntryNonCmdFieldsSize (soft.go:20)


def entry_size_upper_limit(cmd_len: int) -> int:
    """Entry.SizeUpperLimit (raft_optimized.go:71-76)."""
    return ENTRY_NON_CMD_FIELDS_SIZE + cmd_len


def message_size_upper_limit(entry_cmd_lens: list, snapshot: bytes = None) -> int:
    """Message.SizeUpperLimit (raft_optimized.go:1204-1216): 16 x 12 for the
    scalar fields, the Snapshot's own size, 16 + the bound of every entry."""
    sb = snapshot_bytes() if snapshot is None else snapshot
    return 16 * 12 + len(sb) + sum(16 + entry_size_upper_limit(n) for n in entry_cmd_lens)


def batch_size_upper_limit(source_address: str, message_bounds: list) -> int:
    """MessageBatch.SizeUpperLimit (raft_optimized.go:1218-1227)."""
    return 16 * 3 + len(source_address) + sum(16 + b for b in message_bounds)


def _take(buf: bytes, i: int, n: int) -> int:
    """The end of an n-byte field at i: ErrInvalidLength / io.ErrUnexpectedEOF
    when it runs past the buffer (raft.pb.go skipRaft and the field reads)."""
    if n > len(buf) - i:
        raise ValueError("invalid length")
    return i + n


def _skip_field(buf: bytes, i: int, wt: int) -> int:  # skipRaft
    if wt == 0:
        _, i = get_varint(buf, i)
    elif wt == 1:
        i = _take(buf, i, 8)
    elif wt == 2:
        n, i = get_varint(buf, i)
        i = _take(buf, i, n)
    elif wt == 5:
        i = _take(buf, i, 4)
    else:
        raise ValueError(f"bad wire type {wt}")
    return i


def snapshot_decode(buf: bytes) -> tuple:
    """(index, term) of an embedded Snapshot; other fields skipped."""
    i, index, term = 0, 0, 0
    while i < len(buf):
        tag, i = get_varint(buf, i)
        f, wt = tag >> 3, tag & 7
        if f == 4 and wt == 0:
            index, i = get_varint(buf, i)
        elif f == 5 and wt == 0:
            term, i = get_varint(buf, i)
        else:
            i = _skip_field(buf, i, wt)
    return index, term


MESSAGE_FIELDS = {1: "type", 2: "to", 3: "from", 4: "cluster_id", 5: "term", 6: "log_term",
                  7: "log_index", 8: "commit", 9: "reject", 10: "hint", 13: "hint_high"}


def message_decode(buf: bytes) -> tuple:
    """Message.Unmarshal (raft_optimized.go:654-979): (message dict, entries)."""
    m = {v: 0 for v in MESSAGE_FIELDS.values()}
    m["snapshot"] = (0, 0)
    ents, i = [], 0
    while i < len(buf):
        tag, i = get_varint(buf, i)
        f, wt = tag >> 3, tag & 7
        if f in MESSAGE_FIELDS and wt == 0:
            x, i = get_varint(buf, i)
            m[MESSAGE_FIELDS[f]] = x
        elif f == 11 and wt == 2:
            n, i = get_varint(buf, i)
            end = _take(buf, i, n)
            ents.append(entry_decode(buf[i:end]))
            i = end
        elif f == 12 and wt == 2:
            n, i = get_varint(buf, i)
            end = _take(buf, i, n)
            m["snapshot"] = snapshot_decode(buf[i:end])
            i = end
        else:
            i = _skip_field(buf, i, wt)
    m["reject"] = int(m["reject"] != 0)
    return m, ents


def batch_decode(buf: bytes) -> dict:
    """MessageBatch.Unmarshal (raft_optimized.go:1051-1204)."""
    out = {"requests": [], "deployment_id": 0, "source_address": "", "bin_ver": 0}
    i = 0
    while i < len(buf):
        tag, i = get_varint(buf, i)
        f, wt = tag >> 3, tag & 7
        if f == 1 and wt == 2:
            n, i = get_varint(buf, i)
            end = _take(buf, i, n)
            out["requests"].append(message_decode(buf[i:end]))
            i = end
        elif f == 2 and wt == 0:
            out["deployment_id"], i = get_varint(buf, i)
        elif f == 3 and wt == 2:
            n, i = get_varint(buf, i)
            out["source_address"] = buf[i:i + n].decode()
            i += n
        elif f == 4 and wt == 0:
            out["bin_ver"], i = get_varint(buf, i)
        else:
            i = _skip_field(buf, i, wt)
    return out


def frames_decode(data: bytes) -> list:
    """readMessage (tcp.go:187-244) over back-to-back frames: the payloads, each
    checked against its header and payload crc32."""
    out, i = [], 0
    while i < len(data):
        if data[i:i + 2] != MAGIC:
            raise ValueError("bad magic")
        h = bytearray(data[i + 2:i + 2 + HEADER_SIZE])
        inc = int.from_bytes(h[10:14], "big")
        h[10:14] = b"\0\0\0\0"
        if crc32(bytes(h)) != inc:
            raise ValueError("header crc")
        if int.from_bytes(h[0:2], "big") != RAFT_TYPE:
            raise ValueError("method")
        size = int.from_bytes(h[2:10], "big")
        p = data[i + 2 + HEADER_SIZE:i + 2 + HEADER_SIZE + size]
        if crc32(p) != int.from_bytes(h[14:18], "big"):
            raise ValueError("payload crc")
        out.append(p)
        i += 2 + HEADER_SIZE + size
    return out
