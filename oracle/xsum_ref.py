"""TEST INFRASTRUCTURE ONLY -- independent numpy restatement of the checksum path.

This second restatement is written from RFC 1071 arithmetic (exact integer sum
of little-endian 16-bit words, then the closed form of the end-around-carry
fold) rather than from DPDK's loop structure, so that it cross-checks
`oracle/tasx_oracle.c` instead of repeating it.  It follows the same reference
semantics:

* rte_raw_cksum (DPDK 19.11 rte_ip.h): folded, not
  inverted; 0 only for an all-zero buffer, otherwise in [1, 0xffff].
* rte_ipv4_cksum (a3), rte_ipv4_phdr_cksum (a4), rte_ipv4_udptcp_cksum (a5).
* tcp_checksums flag-off branch, /root/reference tas/fast/fast_flows.c:1058-1069.
* network_ip_phdr_xsum, /root/reference tas/fast/network.h:157-173.

Only tests/ (and tests/golden/gen_golden.py) import this module.  Parity status:
see oracle/tasx_oracle.h -- the reference's own tests pin no checksum value.
"""
from __future__ import annotations

import numpy as np

PKT_TX_TCP_SEG = 1 << 50


def _fold_exact(total: int) -> int:
    """Closed form of repeated 16-bit end-around folding of a non-negative sum."""
    if total == 0:
        return 0
    return ((total - 1) % 0xFFFF) + 1


def word_sum(buf) -> int:
    """Exact integer sum of LE u16 words counted from the buffer start; an odd
    tail byte is the low byte of a zero-padded word."""
    b = np.frombuffer(bytes(buf), dtype=np.uint8)
    if b.size & 1:
        b = np.concatenate([b, np.zeros(1, np.uint8)])
    return int(b.view("<u2").astype(np.int64).sum())


def raw_cksum(buf) -> int:
    return _fold_exact(word_sum(buf))


def ipv4_cksum(ip: bytes) -> int:
    c = raw_cksum(ip[:20])
    return c if c == 0xFFFF else (~c) & 0xFFFF


def ipv4_phdr_cksum(ip: bytes, ol_flags: int = 0) -> int:
    tl = (ip[2] << 8) | ip[3]
    l4 = 0 if (ol_flags & PKT_TX_TCP_SEG) else ((tl - 20) & 0xFFFF)
    psd = bytes(ip[12:20]) + bytes([0, ip[9], l4 >> 8, l4 & 0xFF])
    return raw_cksum(psd)


def ipv4_udptcp_cksum(ip: bytes, l4: bytes) -> int:
    l3 = (ip[2] << 8) | ip[3]
    if l3 < 20:
        return 0
    c = raw_cksum(l4[: l3 - 20]) + ipv4_phdr_cksum(ip, 0)
    c = (c >> 16) + (c & 0xFFFF)
    c = (~c) & 0xFFFF
    return 0xFFFF if c == 0 else c


def tcp_checksums(frame: bytearray, ip_off: int = 14, l4_off: int = 34) -> tuple[int, int]:
    """In-place flag-off branch of tcp_checksums(); returns (ip.chksum, tcp.chksum)
    as the native u16 values the reference stores."""
    frame[ip_off + 10: ip_off + 12] = b"\0\0"
    frame[l4_off + 16: l4_off + 18] = b"\0\0"
    ip = bytes(frame[ip_off: ip_off + 20])
    ipc = ipv4_cksum(ip)
    frame[ip_off + 10: ip_off + 12] = ipc.to_bytes(2, "little")
    tl = (frame[ip_off + 2] << 8) | frame[ip_off + 3]
    l4 = bytes(frame[l4_off: l4_off + max(tl - 20, 0)])
    tcpc = ipv4_udptcp_cksum(bytes(frame[ip_off: ip_off + 20]), l4)
    frame[l4_off + 16: l4_off + 18] = tcpc.to_bytes(2, "little")
    return ipc, tcpc


def ip_phdr_xsum(ip_src_be: int, ip_dst_be: int, proto: int, l3_paylen: int) -> int:
    s = (ip_src_be & 0xFFFF) + (ip_src_be >> 16) + (ip_dst_be & 0xFFFF) + (ip_dst_be >> 16)
    s += proto << 8
    s += ((l3_paylen & 0xFF) << 8) | (l3_paylen >> 8)
    return _fold_exact(s)


def raw_batch(buf: np.ndarray, offsets, lengths) -> np.ndarray:
    """Vectorised-by-packet reference for RAW batches (uint16 per packet)."""
    out = np.empty(len(offsets), np.uint16)
    mv = memoryview(np.ascontiguousarray(buf, dtype=np.uint8))
    for i, (o, n) in enumerate(zip(offsets, lengths)):
        out[i] = raw_cksum(mv[int(o): int(o) + int(n)])
    return out


def ipv4_hdr_verify(ip: bytes) -> bool:
    """Receive-side header check: the 20-byte header (checksum included) folds to 0xffff."""
    return raw_cksum(ip[:20]) == 0xFFFF


def ipv4_udptcp_cksum_verify(ip: bytes, l4: bytes) -> bool:
    """DPDK 21.11 rte_ipv4_udptcp_cksum_verify for IHL 5 (published algorithm)."""
    l3 = (ip[2] << 8) | ip[3]
    if l3 < 20:
        return False
    c = raw_cksum(l4[: l3 - 20]) + ipv4_phdr_cksum(ip, 0)
    c = (c >> 16) + (c & 0xFFFF)
    return c == 0xFFFF


def tcp4_verify(frame: bytes, ip_off: int = 14, l4_off: int = 34) -> int:
    ip = bytes(frame[ip_off: ip_off + 20])
    tl = (ip[2] << 8) | ip[3]
    v = 1 if ipv4_hdr_verify(ip) else 0
    if ipv4_udptcp_cksum_verify(ip, bytes(frame[l4_off: l4_off + max(tl - 20, 0)])):
        v |= 2
    if (ip[0] & 0x0F) != 5:
        v |= 4
    return v


def flow_tx_read(shm, tx_base: int, tx_len: int, pos: int, n: int) -> bytes:
    """flow_tx_read(), /root/reference tas/fast/fast_flows.c:833-846."""
    mv = memoryview(shm)
    if pos + n <= tx_len:
        return bytes(mv[tx_base + pos: tx_base + pos + n])
    part = tx_len - pos
    return bytes(mv[tx_base + pos: tx_base + tx_len]) + bytes(mv[tx_base: tx_base + n - part])


def tx_segment(shm, shm_len: int, frames: np.ndarray, segs: np.ndarray, ip_off: int = 14,
               l4_off: int = 34) -> np.ndarray:
    """flow_tx_segment()'s payload copy + tcp_checksums() per descriptor, in
    place on `frames` (uint8); returns ip.chksum | tcp.chksum << 16 per segment,
    0 for a descriptor dma_read()'s assertions would reject."""
    out = np.zeros(len(segs), np.uint32)
    shm = np.ascontiguousarray(shm, dtype=np.uint8)
    for i, d in enumerate(segs):
        fo, tb, tlen, pos, pay, hl = (int(d["frame_off"]), int(d["tx_base"]), int(d["tx_len"]),
                                      int(d["pos"]), int(d["payload"]), int(d["hdrs_len"]))
        if not ((pay == 0 or pos < tlen) and pay <= tlen and tb <= shm_len and tlen <= shm_len - tb
                and hl >= l4_off + 20):
            continue
        if pay:
            frames[fo + hl: fo + hl + pay] = np.frombuffer(flow_tx_read(shm, tb, tlen, pos, pay), np.uint8)
        fr = bytearray(frames[fo: fo + max(l4_off + 18, ip_off + 20, hl + pay,
                                           ip_off + ((int(frames[fo + ip_off + 2]) << 8) | int(frames[fo + ip_off + 3])))])
        ipc, tcpc = tcp_checksums(fr, ip_off, l4_off)
        frames[fo: fo + len(fr)] = np.frombuffer(bytes(fr), np.uint8)
        out[i] = ipc | (tcpc << 16)
    return out


# ---------------------------------------------------------------------------
# RX flow lookup

CRC32C_POLY = 0x82F63B78


def crc32c(data: bytes, crc: int = 0) -> int:
    """CRC32C bit by bit from the polynomial definition (reflected, no pre/post
    inversion: the SSE4.2 crc32 instruction; DPDK crc32c_sse42_u32/_u64)."""
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (CRC32C_POLY if crc & 1 else 0)
    return crc


def flow_hash(frame, ip_off: int = 14, l4_off: int = 34) -> int:
    """flow_hash() of the key fast_flows_packet_fss() builds
    (/root/reference tas/fast/fast_flows.c:1078-1082, :1097-1101): bytes
    ip.dest, ip.src, tcp.dest, tcp.src."""
    f = bytes(frame)
    key = f[ip_off + 16: ip_off + 20] + f[ip_off + 12: ip_off + 16] + f[l4_off + 2: l4_off + 4] + f[l4_off: l4_off + 2]
    return crc32c(key, 0)


def flow_lookup(frame, flowht: np.ndarray, flowst: bytes, fs_num: int, ip_off: int = 14, l4_off: int = 34,
                fs_stride: int = 128, fs_key_off: int = 32) -> tuple[int, int]:
    """fast_flows_packet_fss() for one frame (:1127-1162): (hash, flow id or 0xffffffff)."""
    f = bytes(frame)
    h = flow_hash(f, ip_off, l4_off)
    want = f[ip_off + 16: ip_off + 20] + f[ip_off + 12: ip_off + 16] + f[l4_off + 2: l4_off + 4] + f[l4_off: l4_off + 2]
    ent = len(flowht) // 2
    for j in range(4):
        k = ((h + j) & 0xFFFFFFFF) % ent
        ffid, eh = int(flowht[2 * k]), int(flowht[2 * k + 1])
        fid = ffid & ((1 << 29) - 1)
        if not (ffid & 0x80000000) or eh != h or fid >= fs_num:
            continue
        o = fid * fs_stride + fs_key_off
        if bytes(flowst[o: o + 12]) == want:
            return h, fid
    return h, 0xFFFFFFFF
