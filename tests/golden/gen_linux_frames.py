"""Golden TCP/IPv4 frames checksummed by the Linux TCP/IP stack.

The reference pins its software checksums (TAS run with --fp-no-xsumoffload)
the same way in its end-to-end test: tests/full/fulltest.c:103 starts TAS on a
DPDK tap vdev whose other end is the Linux stack, which drops every segment
whose IPv4 or TCP checksum is wrong, so the test's connections only complete
if TAS's checksums are right.  Here one TCP connection runs over a TUN device
between the Linux stack (10.77.0.1, a listening socket in this process) and
this script (10.77.0.2, speaking TCP by hand through the TUN fd):

* "linux" frames: every IPv4 packet the kernel sends -- the SYN-ACK, its ACKs,
  and data segments of many lengths (full 1448-byte MSS segments with the
  timestamp option, i.e. TAS's 1514-byte frame, and odd short ones).  A TUN
  device without TUNSETOFFLOAD offers no checksum offload, so the kernel
  computes both checksums in software (validate_xmit_skb -> skb_checksum_help,
  ip_send_check): these are Linux's own values.
* "accepted" frames: the segments this script sent, checksummed by the C
  oracle (oracle_tcp_checksums, the tcp_checksums restatement) and accepted
  by the kernel -- it verifies both checksums of every received segment and
  the listening socket receives exactly the bytes sent.

Each packet is stored as a TAS frame (14 zero Ethernet bytes, IPv4 at 14, TCP
at 34) in a 2048-byte mbuf room, with its length and origin.  The tests take
the checksum fields out and recompute them with the oracle and the GPU kernels
(tests/test_linux_frames.py).  Needs root and /dev/net/tun
(this build container, not the GPU box); sequence numbers and timestamps differ
per run, so the committed file is one run's capture.

    python tests/golden/gen_linux_frames.py
"""
from __future__ import annotations

import fcntl
import os
import select
import socket
import struct
import sys
import threading
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

from oracle.oracle_lib import Oracle  # noqa: E402  (the generator's checksum source for its own segments)
from tas_amd import pktgen  # noqa: E402

TUNSETIFF, IFF_TUN, IFF_NO_PI = 0x400454CA, 0x0001, 0x1000
SIOCSIFADDR, SIOCSIFNETMASK, SIOCSIFFLAGS, SIOCSIFMTU = 0x8916, 0x891C, 0x8914, 0x8922
IFF_UP, IFF_RUNNING = 0x1, 0x40
IFNAME = b"tasxgold0"
LINUX_IP, PEER_IP = "10.77.0.1", "10.77.0.2"
LPORT, PPORT = 5555, 40000
ROOM = pktgen.MBUF_ROOM
# segment payload lengths this script sends (odd, even, tiny, full MSS)
SEND_LENS = [1, 2, 3, 5, 16, 17, 63, 64, 65, 127, 255, 256, 511, 999, 1000, 1447, 1448, 700, 1201, 1448]
# what the Linux side writes back (TCP_NODELAY: one segment per write when the
# window allows; the 24,000-byte write goes out as full MSS segments)
ECHO_WRITES = [1, 2, 3, 7, 100, 513, 1447, 24000, 4097, 9]
FIN, SYN, RST, PSH, ACK = 0x01, 0x02, 0x04, 0x08, 0x10


def ifreq_addr(name: bytes, ip: str) -> bytes:
    return struct.pack("16sH2s4s8s", name, socket.AF_INET, b"\0\0", socket.inet_aton(ip), b"\0" * 8)


def tun_open() -> int:
    fd = os.open("/dev/net/tun", os.O_RDWR)
    fcntl.ioctl(fd, TUNSETIFF, struct.pack("16sH", IFNAME, IFF_TUN | IFF_NO_PI))
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    fcntl.ioctl(s, SIOCSIFADDR, ifreq_addr(IFNAME, LINUX_IP))
    fcntl.ioctl(s, SIOCSIFNETMASK, ifreq_addr(IFNAME, "255.255.255.0"))
    fcntl.ioctl(s, SIOCSIFMTU, struct.pack("16si", IFNAME, 1500))
    fcntl.ioctl(s, SIOCSIFFLAGS, struct.pack("16sH", IFNAME, IFF_UP | IFF_RUNNING))
    s.close()
    return fd


class Peer:
    """The TCP end at PEER_IP, one segment at a time through the TUN fd."""

    def __init__(self, fd: int, orc: Oracle):
        self.fd, self.orc = fd, orc
        self.snd_nxt = 0x1000_0000
        self.rcv_nxt = 0
        self.ts_recent = 0
        self.ip_id = 1
        self.frames: list[tuple[bytes, str]] = []   # (IPv4 packet, origin)

    def send(self, flags: int, payload: bytes = b"", syn_opts: bool = False) -> None:
        tsval = int(time.monotonic() * 1000) & 0xFFFFFFFF
        if syn_opts:   # MSS 1460, NOP NOP, TS (kind 8 len 10)
            opts = struct.pack("!BBH", 2, 4, 1460) + b"\x01\x01" + struct.pack("!BBII", 8, 10, tsval, 0)
        else:          # NOP NOP TS: TAS's 12-byte option block (fast_flows.c:887-888)
            opts = b"\x01\x01" + struct.pack("!BBII", 8, 10, tsval, self.ts_recent)
        thl = 20 + len(opts)
        tcp = struct.pack("!HHIIHHHH", PPORT, LPORT, self.snd_nxt, self.rcv_nxt if flags & ACK else 0,
                          (thl // 4) << 12 | flags, 65535, 0xDEAD, 0) + opts + payload
        ip = struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(tcp), self.ip_id, 0x4000, 64, 6, 0xBEEF,
                         socket.inet_aton(PEER_IP), socket.inet_aton(LINUX_IP))
        self.ip_id += 1
        frame = bytearray(14) + bytearray(ip + tcp)
        self.orc.tcp_checksums(frame)   # ip.chksum, tcp.chksum by the oracle
        pkt = bytes(frame[14:])
        os.write(self.fd, pkt)
        self.frames.append((pkt, "accepted"))
        self.snd_nxt = (self.snd_nxt + len(payload) + (1 if flags & (SYN | FIN) else 0)) & 0xFFFFFFFF

    def recv(self, timeout: float = 1.0) -> bytes | None:
        r, _, _ = select.select([self.fd], [], [], timeout)
        if not r:
            return None
        pkt = os.read(self.fd, 65536)
        if len(pkt) < 40 or pkt[0] != 0x45 or pkt[9] != 6:
            return b""   # not ours (IPv6 router solicitations and the like)
        self.frames.append((pkt, "linux"))
        seq, _ack = struct.unpack("!II", pkt[24:32])
        flags = pkt[33]
        thl = (pkt[32] >> 4) * 4
        paylen = struct.unpack("!H", pkt[2:4])[0] - 20 - thl
        opts = pkt[40:20 + thl]
        i = 0
        while i < len(opts):   # the peer's TSval, echoed as TSecr
            k = opts[i]
            if k == 0:
                break
            if k == 1:
                i += 1
                continue
            ln = opts[i + 1]
            if k == 8 and ln == 10:
                self.ts_recent = struct.unpack("!I", opts[i + 2:i + 6])[0]
            i += max(ln, 2)
        end = (seq + paylen + (1 if flags & (SYN | FIN) else 0)) & 0xFFFFFFFF
        if flags & SYN:
            self.rcv_nxt = end
        elif seq == self.rcv_nxt and (paylen or flags & FIN):
            self.rcv_nxt = end
        return pkt


def server(ready: threading.Event, got: dict) -> None:
    ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind((LINUX_IP, LPORT))
    ls.listen(1)
    ls.settimeout(10)
    ready.set()
    c, _ = ls.accept()
    c.settimeout(10)
    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    want = sum(SEND_LENS)
    data = b""
    while len(data) < want:
        d = c.recv(65536)
        if not d:
            break
        data += d
    got["received"] = data
    rnd = pktgen.random_bytes(0x11AB, sum(ECHO_WRITES)).tobytes()
    pos = 0
    for n in ECHO_WRITES:
        c.sendall(rnd[pos:pos + n])
        pos += n
        time.sleep(0.02)
    got["sent"] = rnd
    time.sleep(0.3)
    c.close()
    ls.close()


def main() -> None:
    orc = Oracle()
    fd = tun_open()
    try:
        peer = Peer(fd, orc)
        ready, got = threading.Event(), {}
        th = threading.Thread(target=server, args=(ready, got), daemon=True)
        th.start()
        ready.wait(5)
        peer.send(SYN, syn_opts=True)
        while True:   # the SYN-ACK
            pkt = peer.recv(3.0)
            if pkt is None:
                raise SystemExit("no SYN-ACK: the kernel dropped the SYN (checksum?) or the TUN is not up")
            if pkt and pkt[33] & (SYN | ACK) == SYN | ACK:
                break
        peer.send(ACK)
        payload = pktgen.random_bytes(0x5EED, sum(SEND_LENS)).tobytes()
        pos = 0
        for n in SEND_LENS:
            peer.send(PSH | ACK, payload[pos:pos + n])
            pos += n
            while peer.recv(0.05) is not None:
                pass
        # the Linux side's writes: ACK every data segment as it arrives
        idle = 0
        while idle < 8 and not (peer.frames and peer.frames[-1][1] == "linux" and peer.frames[-1][0][33] & FIN):
            pkt = peer.recv(0.25)
            if pkt is None:
                idle += 1
                continue
            if pkt and len(pkt) > 52 + 0 and struct.unpack("!H", pkt[2:4])[0] > 20 + (pkt[32] >> 4) * 4:
                peer.send(ACK)
        peer.send(FIN | ACK)
        while peer.recv(0.3) is not None:
            pass
        th.join(5)
    finally:
        os.close(fd)
    if got.get("received") != payload:
        raise SystemExit("the kernel did not deliver the bytes sent: an oracle-checksummed segment was dropped")
    frames = peer.frames
    n = len(frames)
    buf = np.zeros((n, ROOM), np.uint8)
    lens = np.zeros(n, np.uint32)
    origin = np.zeros(n, np.uint8)   # 0 = linux, 1 = accepted (oracle-checksummed, accepted by Linux)
    for i, (pkt, who) in enumerate(frames):
        buf[i, 14:14 + len(pkt)] = np.frombuffer(pkt, np.uint8)
        lens[i] = 14 + len(pkt)
        origin[i] = 0 if who == "linux" else 1
    out = HERE / "linux_frames.npz"
    np.savez_compressed(out, frames=buf.reshape(-1), lens=lens, origin=origin)
    nl = int((origin == 0).sum())
    big = int(((origin == 0) & (lens == 1514)).sum())
    print(f"{out.name}: {n} frames ({nl} from Linux, {big} of them 1514-byte MSS segments; "
          f"{n - nl} oracle-checksummed segments accepted; {len(got['received'])} bytes delivered)")


if __name__ == "__main__":
    main()
