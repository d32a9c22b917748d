"""Generate the committed golden fixtures for the checksum path.

Inputs are seeded (splitmix64, tas_amd/pktgen.py) plus hand-built edge cases;
expected outputs come from the independent numpy restatement
(oracle/xsum_ref.py).  The C oracle and the GPU kernels are both checked
against these files by tests/.  No reference-produced output exists for this
path (the reference's tests pin no checksum value; DPDK is not vendored), so
the only external anchors are the RFC 1071 section 3 vector and the unit-test
frame KAT (kat.json).

    python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))

from oracle import xsum_ref as R  # noqa: E402
from tas_amd import pktgen  # noqa: E402

SEED = 0x601D_F1C5


def raw_fixture():
    """RAW rte_raw_cksum vectors: lengths 0..192 at every start offset mod 16,
    plus long / special buffers."""
    rng_bytes = pktgen.random_bytes(SEED, 1 << 16)
    chunks, offs, lens = [], [], []
    pos = 0

    def add(payload: bytes, shift: int):
        nonlocal pos
        pad = (-pos) % 16 + shift
        chunks.append(np.zeros(pad, np.uint8))
        pos += pad
        offs.append(pos)
        lens.append(len(payload))
        chunks.append(np.frombuffer(payload, np.uint8).copy())
        pos += len(payload)

    k = 0
    for L in range(0, 193):
        add(bytes(rng_bytes[k:k + L]), L % 16)
        k = (k + 97) % 60000
    for L in (1499, 1500, 1501, 9000, 8999):
        for shift in (0, 1, 7):
            add(bytes(rng_bytes[k:k + L]), shift)
            k = (k + 131) % 50000
    # special values
    add(bytes(64), 0)                 # all zero -> 0
    add(bytes(1), 3)                  # single zero byte -> 0
    add(b"\xff" * 64, 0)              # all 0xff -> 0xffff
    add(b"\xff" * 63, 5)              # odd all-0xff
    add(bytes([0, 1, 0xF2, 3, 0xF4, 0xF5, 0xF6, 0xF7]), 0)   # RFC 1071 section 3
    add(bytes([0, 1, 0xF2, 3, 0xF4, 0xF5, 0xF6, 0xF7]), 1)   # same, odd start
    # sums that fold to exactly 0xffff without being zero
    add(b"\x01\x00\xfe\xff", 0)
    add(b"\x01\x00\xfe\xff", 9)
    chunks.append(np.zeros(16, np.uint8))
    buf = np.concatenate(chunks)
    offs = np.asarray(offs, np.uint64)
    lens = np.asarray(lens, np.uint32)
    exp = R.raw_batch(buf, offs, lens)
    return dict(buf=buf, offsets=offs, lengths=lens, expected=exp)


def _set_word(f: bytearray, pos: int, w: int):
    f[pos: pos + 2] = (w & 0xFFFF).to_bytes(2, "little")


def tcp4_fixture():
    """TCP4 frames at a 1520 B stride (tests also shift them to odd starts): payloads 0..1448 (sampled), ACK-sized
    datagrams, l3 < 20, the 0 -> 0xffff rules, and odd frame starts."""
    stride = 1520  # holds the 1514 B maximum frame; 16-byte multiple
    payloads = list(range(0, 24)) + list(range(24, 1449, 97)) + [1447, 1448]
    n_rand = len(payloads)
    frames = pktgen.tcp4_frames(n_rand, payload=np.asarray(payloads), stride=stride, seed=SEED)
    frames = frames.reshape(n_rand, stride)
    extra = []

    def mk(payload: int, seed: int) -> bytearray:
        return bytearray(pktgen.tcp4_frames(1, payload=payload, stride=stride, seed=seed).tobytes())

    # total_length below 20: udptcp -> 0 (DPDK 19.11); ip checksum still computed
    for tl in (0, 1, 19, 20, 21, 36, 37, 38):
        f = mk(100, SEED + tl)
        f[16:18] = tl.to_bytes(2, "big")
        extra.append(f)
    # tcp checksum result 0 -> 0xffff: fix the last payload word so that
    # (L4 sum + pseudo header) == 0 mod 0xffff
    for payload in (2, 100, 1448):
        f = mk(payload, SEED ^ payload)
        tl = 52 + payload
        last = 34 + (tl - 20) - 2
        _set_word(f, last, 0)
        g = bytearray(f)
        g[24:26] = b"\0\0"
        g[50:52] = b"\0\0"
        s = R.word_sum(bytes(g[34:34 + tl - 20])) + R.ipv4_phdr_cksum(bytes(g[14:34]))
        w = (-s) % 0xFFFF
        # the word is at an even L4 offset: LE value w
        _set_word(f, last, w if w else 0xFFFF)
        extra.append(f)
    # ip header whose raw sum folds to 0xffff (kept as 0xffff, not inverted to 0)
    for k in range(2):
        f = mk(64 + k, SEED ^ (0x77 + k))
        g = bytearray(f[14:34])
        g[10:12] = b"\0\0"
        g[4:6] = b"\0\0"
        s = R.word_sum(bytes(g))
        _set_word(f, 14 + 4, (-s) % 0xFFFF or 0xFFFF)
        extra.append(f)
    # all-zero header + zero payload: raw ip sum 0 -> ~0 = 0xffff
    z = bytearray(stride)
    z[16:18] = (40).to_bytes(2, "big")
    extra.append(z)
    ex = np.frombuffer(b"".join(bytes(e) for e in extra), np.uint8).reshape(len(extra), stride)
    allf = np.concatenate([frames, ex]).reshape(-1)
    n = allf.size // stride
    offs = np.arange(n, dtype=np.uint64) * stride
    exp = np.empty(2 * n, np.uint16)
    for i in range(n):
        fr = bytearray(allf[i * stride:(i + 1) * stride].tobytes())
        a, b = R.tcp_checksums(fr)
        exp[2 * i], exp[2 * i + 1] = a, b
    return dict(frames=allf, offsets=offs, stride=np.uint64(stride),
                expected=exp)


def txseg_fixture():
    """Fused TX segment build (flow_tx_read + tcp_checksums, SURVEY.md section 8f
    row 1): odd-length / odd-based circular TX buffers small enough that many
    payloads wrap, plus rejected descriptors, zero payloads, other header
    lengths and ip.total_length that disagrees with the payload."""
    stride = 1536
    pay = np.asarray([0, 1, 2, 15, 16, 17, 100, 1447, 1448] + list(range(200, 1449, 97)))
    n_reg = len(pay)
    shm, frames, segs, shm_len = pktgen.tx_segments(n_reg, payload=pay, stride=stride, seed=SEED,
                                                    nflows=5, tx_len=1600, odd=True)
    segs = list(segs)
    fr = [bytearray(frames[i * stride:(i + 1) * stride].tobytes()) for i in range(n_reg)]

    def add(f: bytearray, d):
        d = d.copy()
        d["frame_off"] = len(fr) * stride
        fr.append(f)
        segs.append(d)

    base = segs[7]  # a full-MSS segment
    f0 = fr[7]
    d = base.copy(); d["payload"] = 0; d["pos"] = d["tx_len"] + 3          # no payload: pos unused
    g = bytearray(f0); g[16:18] = (52).to_bytes(2, "big"); add(g, d)
    d = base.copy(); d["pos"] = d["tx_len"]; d["payload"] = 5; add(bytearray(f0), d)    # rejected
    d = base.copy(); d["payload"] = d["tx_len"] + 1; add(bytearray(f0), d)              # rejected
    d = base.copy(); d["tx_base"] = shm_len - d["tx_len"] + 1; add(bytearray(f0), d)    # rejected
    d = base.copy(); d["hdrs_len"] = 53; add(bytearray(f0), d)                           # rejected
    for delta in (7, -100):                                         # ip.len disagrees
        g = bytearray(f0); g[16:18] = (52 + int(base["payload"]) + delta).to_bytes(2, "big")
        add(g, base)
    g = bytearray(f0); g[16:18] = (10).to_bytes(2, "big"); add(g, base)      # total_length < 20
    for hl in (54, 67, 80):                                         # other header lengths
        d = base.copy(); d["hdrs_len"] = hl; d["payload"] = 1400
        g = bytearray(f0); g[16:18] = (hl - 14 + 1400).to_bytes(2, "big"); add(g, d)
    d = base.copy(); d["pos"] = d["tx_len"] - 1; d["payload"] = 300   # wraps after 1 byte
    g = bytearray(f0); g[16:18] = (52 + 300).to_bytes(2, "big"); add(g, d)
    d = base.copy(); d["pos"] = 0; d["payload"] = d["tx_len"] if d["tx_len"] <= 1448 else 1448
    g = bytearray(f0); g[16:18] = (52 + int(d["payload"])).to_bytes(2, "big"); add(g, d)
    segs = np.asarray(segs, pktgen.TX_SEG_DTYPE)
    frames_in = np.frombuffer(b"".join(bytes(x) for x in fr), np.uint8).copy()
    frames_out = frames_in.copy()
    exp = R.tx_segment(shm, shm_len, frames_out, segs)
    return dict(shm=shm, shm_len=np.uint64(shm_len), frames_in=frames_in, segs=segs.view(np.uint8),
                frames_out=frames_out, expected=exp)


def flow_fixture():
    """RX flow lookup (fast_flows_packet_fss + CRC32C flow_hash, SURVEY.md
    section 8f row 4): a small, crowded table (61 entries, not a power of two,
    so probes wrap and buckets fill), frames for inserted flows, for flows whose
    bucket was full, for unknown keys, and planted entries that must be
    skipped: same hash but another flow's key, invalid bit clear, flow id past
    the flow-state array."""
    nflows, ent, stride = 48, 61, 128
    keys = pktgen.flow_keys(nflows, seed=SEED)
    fs = pktgen.flow_state(keys, seed=SEED)
    hashes = np.asarray([R.crc32c(bytes(k), 0) for k in keys], np.uint64)
    ht, ok = pktgen.flow_table(hashes, ent)
    unknown = pktgen.flow_keys(8, seed=SEED ^ 0x5555)
    unknown[:, 0] ^= 0x80
    fkeys = np.concatenate([keys, unknown])
    frames = pktgen.rx_frames(fkeys, stride=stride, seed=SEED).reshape(len(fkeys), stride)
    # planted entries: for three unknown keys, fill their whole bucket with
    # entries carrying their hash -- flow 0 (wrong key), invalid, past the array
    for u, kind in zip(range(3), ("wrong_key", "invalid", "past_end")):
        h = R.crc32c(bytes(unknown[u]), 0)
        for d in range(4):
            k = ((h + d) & 0xFFFFFFFF) % ent
            fid = {"wrong_key": 0, "invalid": 1, "past_end": nflows + 5}[kind]
            ht[2 * k] = (0 if kind == "invalid" else pktgen.FLOWHTE_VALID) | fid
            ht[2 * k + 1] = h
    exp_h = np.empty(len(fkeys), np.uint32)
    exp_f = np.empty(len(fkeys), np.uint32)
    for i in range(len(fkeys)):
        exp_h[i], exp_f[i] = R.flow_lookup(frames[i].tobytes(), ht, fs.tobytes(), nflows)
    return dict(frames=frames.reshape(-1), stride=np.uint64(stride), flowht=ht, flowst=fs,
                fs_num=np.uint32(nflows), expected_hash=exp_h, expected_fid=exp_f)


def main():
    raw = raw_fixture()
    np.savez_compressed(HERE / "raw_vectors.npz", **raw)
    tcp = tcp4_fixture()
    np.savez_compressed(HERE / "tcp4_vectors.npz", **tcp)
    kat = {
        "rfc1071_sec3": {"bytes": "0001f203f4f5f6f7", "raw_cksum_be": "ddf2",
                         "raw_cksum_native_le": 0xF2DD,
                         "source": "RFC 1071 section 3 numerical example"},
        "crc32c_rfc3720_b4": {
            "note": "standard CRC32C (init 0xffffffff, final xor 0xffffffff); TAS's flow_hash uses the "
                    "same polynomial with init 0 and no final xor",
            "zeros32": "8a9136aa", "ones32": "62a8ab43", "inc32": "46dd794e", "dec32": "113fdb5c",
            "check_123456789": "e3069283",
            "source": "RFC 3720 appendix B.4 (iSCSI CRC32C examples) and the CRC catalogue check value"},
        "ipv4_header_public": {
            "header_hex": "450000730000400040110000c0a80001c0a800c7", "ip_chksum_bytes": "b861",
            "source": "the widely published IPv4 header checksum example (192.168.0.1 -> "
                      "192.168.0.199, UDP, total length 115): checksum field b8 61"},
        "tas_unit_window_update": {
            "frame_hex": bytes(pktgen.kat_frame()).hex(),
            "ip_chksum_bytes": "a3bb", "tcp_chksum_bytes": "cfd7",
            "source": "frame of tests/tas_unit/fastpath.c:187-207 (fast_flows_bump -> "
                      "flow_tx_segment, tas/fast/fast_flows.c:886-928); values hand-derived "
                      "in SURVEY.md section 8c"},
    }
    fl = flow_fixture()
    np.savez_compressed(HERE / "flow_vectors.npz", **fl)
    tx = txseg_fixture()
    np.savez_compressed(HERE / "txseg_vectors.npz", **tx)
    (HERE / "kat.json").write_text(json.dumps(kat, indent=2) + "\n")
    print("raw:", len(raw["lengths"]), "vectors;", "tcp4:", len(tcp["offsets"]), "frames;",
          "txseg:", len(tx["expected"]), "segments;", "flow:", len(fl["expected_fid"]), "frames")


if __name__ == "__main__":
    main()
