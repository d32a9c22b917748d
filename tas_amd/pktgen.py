"""Seeded synthetic packet batches (BASELINE.md / SURVEY.md section 8d).

All randomness is splitmix64 with a fixed seed, so CPU oracle, GPU kernels,
tests and bench see identical bytes.  Frame layout follows the reference's TX
segment builder, flow_tx_segment() (/root/reference/tas/fast/fast_flows.c:877-955):
14 B Ethernet + 20 B IPv4 (IHL 5) + 20 B TCP + 12 B timestamp option
(10 B + 2 B pad) + payload; ip.len = 52 + payload; a frame starts at the mbuf
data room (BUFFER_SIZE 2048, tas/fast/internal.h:34).  The checksum fields are
filled with random bytes on purpose: tcp_checksums() must treat them as zero.
"""
from __future__ import annotations

import numpy as np

SEED = 0x7A5C_5EED_2026_0001
MTU_MIX = (64, 576, 1500, 9000)
ETH_LEN, IP_LEN, TCP_LEN, TS_OPT_LEN = 14, 20, 20, 12
HDRS_LEN = ETH_LEN + IP_LEN + TCP_LEN + TS_OPT_LEN  # 66, fast_flows.c:887-888
TCP_MSS = 1448                                      # fast_flows.c:37
MBUF_ROOM = 2048                                    # tas/fast/internal.h:34

_C1 = np.uint64(0x9E3779B97F4A7C15)
_C2 = np.uint64(0xBF58476D1CE4E5B9)
_C3 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """n outputs of splitmix64 (Steele/Lea/Flood 2014) from `seed`, skipping `start`."""
    i = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * _C1
        z = (z ^ (z >> np.uint64(30))) * _C2
        z = (z ^ (z >> np.uint64(27))) * _C3
        z = z ^ (z >> np.uint64(31))
    return z


def random_bytes(seed: int, nbytes: int, start_word: int = 0) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8, start_word)
    return words.view(np.uint8)[:nbytes].copy()


def raw_uniform(n: int, length: int = 1500, seed: int = SEED) -> tuple[np.ndarray, int]:
    """n packed payloads of `length` bytes (stride == length). Returns (buf, stride)."""
    return random_bytes(seed, n * length), length


def mixed_lengths(n: int, seed: int = SEED, sizes=MTU_MIX) -> np.ndarray:
    r = splitmix64(seed ^ 0x51ED, n)
    return np.asarray(sizes, dtype=np.uint32)[(r % np.uint64(len(sizes))).astype(np.int64)]


def raw_mixed(n: int, seed: int = SEED, sizes=MTU_MIX, align: int = 16, odd: bool = False):
    """Mixed-MTU RAW batch in random order.  Offsets are `align`-aligned
    (odd=True: lengths +/- 1 and offsets shifted by a random byte, for parity
    of the odd-start / odd-tail paths).  Returns (buf, offsets u64, lengths u32)."""
    lens = mixed_lengths(n, seed, sizes).astype(np.int64)
    if odd:
        jitter = (splitmix64(seed ^ 0x0DD, n) % np.uint64(3)).astype(np.int64) - 1
        lens = np.maximum(lens + jitter, 0)
        shift = (splitmix64(seed ^ 0x5A1F, n) % np.uint64(16)).astype(np.int64)
    else:
        shift = np.zeros(n, np.int64)
    slot = (lens + shift + align - 1) // align * align
    offs = np.zeros(n, np.int64)
    np.cumsum(slot[:-1], out=offs[1:])
    offs += shift
    total = int(offs[-1] + lens[-1]) if n else 0
    buf = random_bytes(seed ^ 0xB0F, total + 16)
    return buf, offs.astype(np.uint64), lens.astype(np.uint32)


def tcp4_frames(n: int, payload=TCP_MSS, stride: int = MBUF_ROOM, seed: int = SEED,
                ip_total_len=None) -> np.ndarray:
    """n TAS TX data segments at `stride` (one mbuf data room each).
    `payload` is an int or a per-frame array; `ip_total_len` overrides ip.len
    (e.g. 65535 for the TSO config, where stride must hold 14 + 65535 bytes)."""
    payload = np.broadcast_to(np.asarray(payload, dtype=np.int64), (n,))
    if ip_total_len is None:
        tl = HDRS_LEN - ETH_LEN + payload
    else:
        tl = np.broadcast_to(np.asarray(ip_total_len, dtype=np.int64), (n,))
    assert int((ETH_LEN + tl).max(initial=0)) <= stride or n == 0
    buf = random_bytes(seed, n * stride)
    f = buf.reshape(n, stride)
    h = random_bytes(seed ^ 0x4EAD, n * 16).reshape(n, 16)  # per-frame header entropy
    f[:, 12] = 0x08
    f[:, 13] = 0x00                                   # eth.type = IP
    ip = ETH_LEN
    f[:, ip + 0] = 0x45                               # v4, IHL 5
    f[:, ip + 1] = h[:, 0] & 0x3                      # tos: ECN bits only
    f[:, ip + 2] = (tl >> 8) & 0xFF
    f[:, ip + 3] = tl & 0xFF                          # ip.len
    f[:, ip + 4] = 0
    f[:, ip + 5] = 3                                  # ip.id = 3 (fast_flows.c:898)
    f[:, ip + 6] = 0
    f[:, ip + 7] = 0
    f[:, ip + 8] = 0xFF                               # ttl
    f[:, ip + 9] = 6                                  # proto TCP
    # ip.chksum (ip+10..11) keeps random bytes
    f[:, ip + 12: ip + 20] = h[:, 1:9]                # src, dst
    t = ETH_LEN + IP_LEN
    f[:, t + 12] = (5 + TS_OPT_LEN // 4) << 4          # hdrlen 8 words
    f[:, t + 13] = 0x18                               # PSH|ACK
    # tcp.chksum (t+16..17) keeps random bytes
    f[:, t + 18] = 0
    f[:, t + 19] = 0                                  # urgp
    o = t + TCP_LEN
    f[:, o + 0] = 8
    f[:, o + 1] = 10                                  # TS option kind/len
    f[:, o + 10] = 0
    f[:, o + 11] = 0                                  # pad
    return buf


# struct tasx_tx_seg (include/tasx_xsum.h), 32 bytes
TX_SEG_DTYPE = np.dtype([("frame_off", "<u8"), ("tx_base", "<u8"), ("tx_len", "<u4"), ("pos", "<u4"),
                         ("payload", "<u2"), ("hdrs_len", "<u2"), ("room", "<u4")])


def tx_segments(n: int, payload=TCP_MSS, stride: int = MBUF_ROOM, seed: int = SEED,
                nflows: int | None = None, tx_len: int = 16384, odd: bool = False,
                make_shm: bool = True, room: int = 0):
    """n TX data segments the way fast_flows_qman -> flow_tx_segment() builds
    them (/root/reference/tas/fast/fast_flows.c:877-955): headers filled (as
    tcp4_frames), payload still to be read from the flow's circular TX buffer.
    Segment i belongs to flow i % nflows; a flow's segments read consecutive
    payload from a random start position, wrapping at tx_len.  odd=True gives
    odd buffer lengths and odd, unaligned buffer bases.  room: the
    descriptors' room field (TAS passes its mbuf data room, e.g. the stride).
    Returns (shm u8, frames u8, segs TX_SEG_DTYPE, shm_bytes)."""
    payload = np.broadcast_to(np.asarray(payload, dtype=np.int64), (n,)).copy()
    nflows = nflows or max(1, n // 8)
    tlen = np.full(nflows, tx_len, np.int64)
    if odd:
        tlen -= (splitmix64(seed ^ 0x0DDF, nflows) % np.uint64(7)).astype(np.int64)
    assert int(payload.max(initial=0)) <= int(tlen.min(initial=tx_len))
    slot = tlen + (16 if odd else 0)
    base = np.zeros(nflows, np.int64)
    np.cumsum(slot[:-1], out=base[1:])
    if odd:
        base += (splitmix64(seed ^ 0xBA5E, nflows) % np.uint64(16)).astype(np.int64)
    shm_bytes = int(base[-1] + tlen[-1]) + 16 if nflows else 16
    start = (splitmix64(seed ^ 0x5747, nflows) % tlen.astype(np.uint64)).astype(np.int64)
    flow = np.arange(n, dtype=np.int64) % nflows
    # bytes the flow sent before segment i: exclusive cumsum within each flow
    order = np.lexsort((np.arange(n), flow))
    ps = payload[order]
    cs = np.cumsum(ps) - ps
    first = np.r_[True, flow[order][1:] != flow[order][:-1]] if n else np.zeros(0, bool)
    grp0 = np.maximum.accumulate(np.where(first, np.arange(n), 0)) if n else np.zeros(0, np.int64)
    before = np.empty(n, np.int64)
    before[order] = cs - cs[grp0]
    segs = np.zeros(n, TX_SEG_DTYPE)
    segs["frame_off"] = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    segs["tx_base"] = base[flow]
    segs["tx_len"] = tlen[flow]
    segs["pos"] = (start[flow] + before) % tlen[flow]
    segs["payload"] = payload
    segs["hdrs_len"] = HDRS_LEN
    segs["room"] = room  # the mbuf data room the build may rewrite (0: frame bytes only)
    frames = tcp4_frames(n, payload, stride, seed)
    shm = random_bytes(seed ^ 0x7E5B, shm_bytes) if make_shm else None
    return shm, frames, segs, shm_bytes


# ---------------------------------------------------------------------------
# RX flow lookup inputs (fast_flows_packet_fss, tas/fast/fast_flows.c:1084-1163)

FLOWST_SIZE = 128     # sizeof(struct flextcp_pl_flowst), include/tas_memif.h:231-317
FLOWST_KEY_OFF = 32   # local_ip, remote_ip, local_port, remote_port (:248-252)
FLOWHT_NBSZ = 4       # FLEXNIC_PL_FLOWHT_NBSZ (:187)
FLOWHTE_VALID = 1 << 31
FLOWHTE_POSSHIFT = 29


def flow_keys(nflows: int, seed: int = SEED) -> np.ndarray:
    """nflows distinct 12-byte keys in flow-state order: local_ip, remote_ip
    (network order), local_port, remote_port."""
    raw = random_bytes(seed ^ 0xF10E, nflows * 16).reshape(nflows, 16)[:, :12].copy()
    raw[:, 0:4] = np.frombuffer(np.arange(nflows, dtype=">u4").tobytes(), np.uint8).reshape(nflows, 4)
    raw[:, 0] |= 0x0A                                  # distinct local ips (10.x.y.z-ish)
    return raw


def flow_state(keys: np.ndarray, seed: int = SEED) -> np.ndarray:
    """The flow-state array (FLOWST_SIZE bytes per flow, random other fields)
    with each flow's key at FLOWST_KEY_OFF."""
    n = len(keys)
    fs = random_bytes(seed ^ 0xF57A, n * FLOWST_SIZE).reshape(n, FLOWST_SIZE)
    fs[:, FLOWST_KEY_OFF:FLOWST_KEY_OFF + 12] = keys
    return fs.reshape(-1)


def flow_table(hashes: np.ndarray, ht_entries: int, fids=None) -> tuple[np.ndarray, np.ndarray]:
    """flowht for flows with the given hashes: each goes to the first free of
    its FLOWHT_NBSZ entries (h + d) % ht_entries with d in the POSSHIFT bits,
    as flow_slot_alloc() places it when no displacement is needed
    (tas/slow/nicif.c:603-622, :241-244).  Flows whose bucket is full are left
    out.  Returns (flowht u32[2 * ht_entries], inserted mask)."""
    ht = np.zeros(2 * ht_entries, np.uint32)
    fids = np.arange(len(hashes)) if fids is None else np.asarray(fids)
    ok = np.zeros(len(hashes), bool)
    for i, (h, fid) in enumerate(zip(np.asarray(hashes, np.uint64), fids)):
        for d in range(FLOWHT_NBSZ):
            k = int((int(h) + d) & 0xFFFFFFFF) % ht_entries
            if not ht[2 * k] & FLOWHTE_VALID:
                ht[2 * k] = FLOWHTE_VALID | (d << FLOWHTE_POSSHIFT) | int(fid)
                ht[2 * k + 1] = int(h)
                ok[i] = True
                break
    return ht, ok


def rx_frames(keys: np.ndarray, stride: int = MBUF_ROOM, seed: int = SEED) -> np.ndarray:
    """One received TCP frame per key, as the peer sends it: ip.src = the
    flow's remote ip, ip.dst = local ip, tcp.src = remote port, tcp.dst =
    local port (the key fast_flows_packet_fss builds, :1097-1101).  Only the
    first 64 bytes of each frame are filled (headers); the rest is random."""
    n = len(keys)
    f = tcp4_frames(n, payload=0, stride=stride, seed=seed)
    set_flow_keys(f, keys, stride)
    return f


def set_flow_keys(frames: np.ndarray, keys: np.ndarray, stride: int) -> None:
    """Write each flow key into its frame's headers as the peer sends it
    (rx_frames' mapping), in place; checksums are not updated."""
    n = len(keys)
    f = frames[:n * stride].reshape(n, stride)
    ip, t = ETH_LEN, ETH_LEN + IP_LEN
    f[:, ip + 16: ip + 20] = keys[:, 0:4]
    f[:, ip + 12: ip + 16] = keys[:, 4:8]
    f[:, t + 2: t + 4] = keys[:, 8:10]
    f[:, t: t + 2] = keys[:, 10:12]


def kat_frame() -> bytearray:
    """The window-update segment built by the reference unit test
    test_rxbump_fc_reopen_notx (tests/tas_unit/fastpath.c:18-22,68-89,187-207
    -> fast_flows_bump -> flow_tx_segment, fast_flows.c:886-928): zero MACs,
    10.1.2.1:23456 -> 10.1.2.3:12345, seq 0, ack 0, wnd 1024, ip.id 3, TTL 255,
    ip.len 52, TS opt val 0 ecr 0, no payload.  66 bytes."""
    f = bytearray(HDRS_LEN)
    f[12:14] = b"\x08\x00"
    ip = ETH_LEN
    f[ip] = 0x45
    f[ip + 2: ip + 4] = (52).to_bytes(2, "big")
    f[ip + 4: ip + 6] = (3).to_bytes(2, "big")
    f[ip + 8] = 0xFF
    f[ip + 9] = 6
    f[ip + 12: ip + 16] = bytes([10, 1, 2, 1])
    f[ip + 16: ip + 20] = bytes([10, 1, 2, 3])
    t = ETH_LEN + IP_LEN
    f[t: t + 2] = (23456).to_bytes(2, "big")
    f[t + 2: t + 4] = (12345).to_bytes(2, "big")
    f[t + 12: t + 14] = ((8 << 12) | 0x18).to_bytes(2, "big")
    f[t + 14: t + 16] = (1024).to_bytes(2, "big")
    f[t + 20] = 8
    f[t + 21] = 10
    return f


# expected results for kat_frame(): network-order bytes a3 bb / cf d7
# (hand-derived in SURVEY.md section 8c; stored as native LE u16)
KAT_IP_CHKSUM = 0xBBA3
KAT_TCP_CHKSUM = 0xD7CF
