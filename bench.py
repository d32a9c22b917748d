"""Benchmark: TAS software TCP/IP checksum path on MI355X (BASELINE.json metric
"TCP/IP checksum GiB/s (device-resident), 1500B MTU batch, 1/2/4/8 GPU").

Headline step = one launch of the TCP4 checksum kernel (tcp_checksums()
flag-off branch: rte_ipv4_cksum + rte_ipv4_udptcp_cksum per frame) over one
batch of 65,536 TAS TX data segments (1514 B frames, ip.len 1500, one per
2048 B mbuf data room: BASELINE.json configs[1] / BASELINE.md), through
tasx_tcp4_cksum_batch_dev_hint with the frame length (the mbuf data_len
tx_send() sets before tx_flush) as the uniform hint.  Inputs are resident in
HBM before the timed region; steps rotate over R distinct batches (R x 134 MB
>> the 256 MiB Infinity Cache) so every step reads HBM, not the MALL.  The K
timed steps are K calls of that C entry point made from C
(tas_amd/benchsrc/bench_loop.c), so no Python runs between launches.

Algorithmic bytes per frame = ip.total_length (1500, the bytes summed) + 4
(results written) -- SURVEY.md section 8d.  value = GiB/s = bytes / s / 2^30.

Multi-GPU (the path shards, no data-path collective):
`python bench.py --gpus N` starts N ranks itself (one process per GPU, before
anything touches a GPU) and refuses when fewer than N GPUs are visible unless
--rehearse (ranks share the visible GPUs, gloo control plane).  Under
torch.distributed.run the ranks come from the launcher (WORLD_SIZE must equal
--gpus).  Each rank pins itself to its GPU's NUMA node, checksums its own
batches on its own stream (weak scaling); the timed region is barrier +
synchronize on both sides, the MAX over ranks is taken, and rank 0 prints one
JSON line with the aggregate and per-rank rates.

Extra legs (all ranks unless noted): the same frames with no hint and a room
(the mbuf data room: the TAS drop-in form) and with neither, the same batches
over two streams, RX verification, a data/ACK flush mix, the RAW payload fold,
the TX segment build, the flow lookup, the one-launch RX pass (verification +
lookup, against the two calls), the end-to-end host-memory rate (one
NUMA-local host thread per GPU), and on rank 0 at N == 1 the CPU oracle
baseline, tx_flush latencies and HBM traffic from rocprofv3 counters (child
runs; --no-pmc skips them).  --workload {shard8m,mixed,tso} measures the other
BASELINE.json configs instead.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from tas_amd import benchloop, pktgen, shard, xsum  # noqa: E402
from tas_amd.benchloop import DEV, HINT, ROOM, VERIFY  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
HBM_ACHIEVABLE_GBS = 6300.0  # the guide's "~6.3 TB/s achievable" (its HBM section)
GIB = float(1 << 30)
METRIC = "TCP/IP checksum GiB/s (device-resident), 1500B MTU batch, 1/2/4/8 GPU"

N_FRAMES = 65536
STRIDE = pktgen.MBUF_ROOM              # 2048, BUFFER_SIZE (tas/fast/internal.h:34)
IP_TOTAL = 1500
FRAME_LEN = pktgen.ETH_LEN + IP_TOTAL  # 1514, the mbuf data_len tx_send() sets
RAW_LEN = 1500
IP_OFF, L4_OFF = pktgen.ETH_LEN, pktgen.ETH_LEN + pktgen.IP_LEN


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=16, help="distinct device batches cycled through")
    ap.add_argument("--workload", default="tcp4", choices=["tcp4", "shard8m", "mixed", "tso"])
    ap.add_argument("--rehearse", action="store_true",
                    help="N ranks may share the visible GPUs (gloo control plane): a rehearsal, not a scaling run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-server-cost", action="store_true", help="skip the resident flush server's price")
    ap.add_argument("--no-raw", action="store_true")
    ap.add_argument("--no-txseg", action="store_true")
    ap.add_argument("--no-flow", action="store_true")
    ap.add_argument("--no-config4", action="store_true", help="skip the BASELINE config 4 leg of the default line")
    ap.add_argument("--no-flushmix", action="store_true")
    ap.add_argument("--no-contexts", action="store_true", help="skip the two-context (two-stream) leg")
    ap.add_argument("--pmc", action="store_true", help=argparse.SUPPRESS)  # default now; kept for old command lines
    ap.add_argument("--no-pmc", action="store_true", help="skip the HBM-traffic rocprofv3 child runs")
    ap.add_argument("--server-cost-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-child", choices=["tcp4", "raw", "txseg", "mixed", "rx", "flushmix", "tso", "shard8m", "readceil"],
                    help=argparse.SUPPRESS)
    ap.add_argument("--control-selftest", action="store_true", help=argparse.SUPPRESS)  # CPU test of the rank plumbing
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# ranks: one process per GPU (control plane only, never data)

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (this
    process never touches a GPU: torch.cuda.device_count() does not initialise
    HIP on this image) and return their combined exit status.  Fewer visible
    GPUs than N is an error unless --rehearse."""
    n = args.gpus
    ndev = 0 if args.control_selftest else torch.cuda.device_count()
    if ndev < n and not (args.rehearse or args.control_selftest):
        print(f"bench.py: --gpus {n} needs {n} GPUs, {ndev} visible "
              f"(--rehearse runs {n} ranks sharing the visible GPUs over gloo: not a scaling measurement)",
              file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))
    # a rank that fails leaves the others waiting in a barrier: end them
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            time.sleep(5)
            for i, p in enumerate(procs):
                if p.poll() is None:
                    p.terminate()
            for i, p in enumerate(procs):
                rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc]
    return bad[0] if bad else 0


def pci_bus_id(dev: int) -> str:
    """The GPU's PCI address as sysfs spells it (domain:bus:device.function)."""
    pr = torch.cuda.get_device_properties(dev)
    return f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"


def _cpulist(text: str) -> set[int]:
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def numa_pin(bus_id: str) -> dict:
    """Pin this rank to the CPUs of its GPU's NUMA node (intersected with the
    CPUs it may use) before any host buffer is touched, so pinned staging and
    the host thread feeding the GPU are NUMA-local."""
    info = {"pci_bus_id": bus_id, "numa_node": None, "cpus": len(os.sched_getaffinity(0))}
    try:
        node = int(Path(f"/sys/bus/pci/devices/{bus_id}/numa_node").read_text())
        info["numa_node"] = node
        if node >= 0:
            local = _cpulist(Path(f"/sys/devices/system/node/node{node}/cpulist").read_text())
            use = local & os.sched_getaffinity(0)
            if use:
                os.sched_setaffinity(0, use)
                info["cpus"] = len(use)
    except (OSError, ValueError):
        pass
    return info


def host_spin_wait(dev: int) -> str:
    """Completion waits by spinning (hipDeviceScheduleSpin) on this rank's GPU,
    set on the HIP runtime torch loaded before its context exists: the
    timed region ends in a synchronize, and a waiting host thread that yields
    adds its wake-up to every K-step interval.  TASX_BENCH_SCHED=auto keeps
    the runtime's default."""
    if os.environ.get("TASX_BENCH_SCHED", "spin") != "spin":
        return "auto"
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so", mode=os.RTLD_NOLOAD)
    except OSError:
        return "auto (HIP runtime not loaded by name)"
    if hip.hipSetDevice(dev) != 0:
        return "auto (hipSetDevice failed)"
    rc = hip.hipSetDeviceFlags(1)  # hipDeviceScheduleSpin
    return "spin" if rc == 0 else f"auto (hipSetDeviceFlags rc {rc})"


def dist_setup(args):
    """Rank setup.  WORLD_SIZE (from the launcher or spawn_ranks) must equal
    --gpus; each rank takes GPU LOCAL_RANK (distinct devices are checked), or
    shares the visible GPUs under --rehearse (gloo)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
    rehearse = args.rehearse or os.environ.get("TASX_DIST_BACKEND") == "gloo"
    info = {}
    if args.control_selftest:
        dev = None
    else:
        ndev = torch.cuda.device_count()
        if not rehearse and local >= ndev:
            raise SystemExit(f"bench.py: rank {rank} needs GPU {local}, {ndev} visible (--rehearse to share)")
        dev = local % max(1, ndev)
        sched = host_spin_wait(dev)
        torch.cuda.set_device(dev)
        info = numa_pin(pci_bus_id(dev))
        info["host_wait"] = sched
    if ws > 1:
        if rehearse or args.control_selftest:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        ids = [None] * ws
        dist.all_gather_object(ids, info.get("pci_bus_id", f"cpu{rank}"))
        if not rehearse and not args.control_selftest and len(set(ids)) != ws:
            raise SystemExit(f"bench.py: ranks share GPUs {ids}; one GPU per rank is required (or --rehearse)")
        info["all_bus_ids"] = ids
    info["rehearse"] = bool(rehearse)
    return ws, rank, local, info


def _red_device():
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def barrier(ws):
    if ws > 1:
        dist.barrier()


def max_over_ranks(x: float, ws: int) -> float:
    if ws == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_red_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, ws: int) -> float:
    if ws == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_red_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_over_ranks(x: float, ws: int) -> list[float]:
    if ws == 1:
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=_red_device())
    out = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


# ---------------------------------------------------------------------------
# workloads: device-resident batches + C launch loops

def _stream_ptrs(streams):
    return [s.cuda_stream for s in streams] if streams else [torch.cuda.current_stream().cuda_stream]


def device_random(nbytes: int, seed: int) -> torch.Tensor:
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)


def device_tcp4_frames(n: int, stride: int, ip_total: int, seed: int) -> torch.Tensor:
    """Random frame bytes generated on the device, then the 66-byte TAS headers
    (pktgen.tcp4_frames layout, ip.len = ip_total) written over each frame."""
    buf = device_random(n * stride, seed)
    hdr = pktgen.tcp4_frames(n, payload=0, stride=128, seed=seed).reshape(n, 128)[:, :pktgen.HDRS_LEN].copy()
    hdr[:, 16] = (ip_total >> 8) & 0xFF
    hdr[:, 17] = ip_total & 0xFF
    buf.view(n, stride)[:, :pktgen.HDRS_LEN] = torch.from_numpy(hdr).cuda()
    return buf


class Tcp4Workload:
    desc = (f"{N_FRAMES} TAS TX segments (1514 B frames, ip.len {IP_TOTAL}, {STRIDE} B mbuf stride), "
            "tcp_checksums() flag-off per frame, frame length (mbuf data_len) as the uniform hint "
            "(tasx_tcp4_cksum_batch_dev_hint)")

    def __init__(self, rotate: int, seed: int, n: int = N_FRAMES, stride: int = STRIDE,
                 ip_total: int = IP_TOTAL, hint: int | None = None, host: bool = True):
        self.n, self.stride, self.ip_total = n, stride, ip_total
        self.hint = pktgen.ETH_LEN + ip_total if hint is None else hint
        if host:
            self.host = pktgen.tcp4_frames(n, payload=ip_total - 52, stride=stride, seed=seed)
            first = torch.from_numpy(self.host).cuda()
        else:
            self.host = None
            first = device_tcp4_frames(n, stride, ip_total, seed)
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.outs = [torch.empty(2 * n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        self.bytes_per_step = n * (ip_total + 4)

    def loop(self, which: int = HINT, *, flen0: int | None = None, room: int = 0, streams=None,
             outs=None, inplace: bool = False) -> benchloop.Loop:
        """The timed call: `which` entry point (HINT: the uniform hint flen0,
        default the frame length; ROOM: no hint, `room` bytes readable per frame;
        DEV: frames only; VERIFY: RX flags into `outs`)."""
        flen0 = self.hint if flen0 is None else flen0
        outs = self.outs if outs is None else outs
        args = [benchloop.Tcp4Args(b.data_ptr(), None, self.stride, None, flen0, room, self.n, IP_OFF, L4_OFF,
                                   xsum.TASX_F_INPLACE if inplace else 0, o.data_ptr())
                for b, o in zip(self.bufs, outs)]
        return benchloop.Loop("tcp4", args, _stream_ptrs(streams), which, "tcp4 batch")


class FlushMixWorkload:
    """A tx_flush-shaped TCP4 batch: flow_tx_segment data frames (1514 B) and
    flow_tx_ack frames (66 B, ip.len 52; fast_flows.c:877-1030) half and half in
    random order, 2048 B mbuf rooms, each frame's length (mbuf data_len) as its
    hint and the mbuf data room as the room (tasx_tcp4_cksum_batch_dev_room)."""
    desc = (f"{N_FRAMES} TAS TX frames in {STRIDE} B rooms, 50% data segments (ip.len {IP_TOTAL}) and 50% "
            "pure ACKs (ip.len 52) in random order, per-frame hints (mbuf data_len), room = the mbuf data room")

    def __init__(self, rotate: int, seed: int, n: int = N_FRAMES, stride: int = STRIDE):
        rng = np.random.default_rng(seed)
        pay = np.where(rng.random(n) < 0.5, 0, IP_TOTAL - 52).astype(np.int64)
        self.n, self.stride = n, stride
        self.host = pktgen.tcp4_frames(n, payload=pay, stride=stride, seed=seed)
        first = torch.from_numpy(self.host).cuda()
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.flen = torch.from_numpy((pktgen.ETH_LEN + 52 + pay).astype(np.int32)).cuda()
        self.outs = [torch.empty(2 * n, dtype=torch.int16, device="cuda") for _ in range(rotate)]
        self.bytes_per_step = int((52 + pay + 4).sum())

    def loop(self, room: int = STRIDE, streams=None) -> benchloop.Loop:
        args = [benchloop.Tcp4Args(b.data_ptr(), None, self.stride, self.flen.data_ptr(), 0, room, self.n, IP_OFF,
                                   L4_OFF, 0, o.data_ptr()) for b, o in zip(self.bufs, self.outs)]
        return benchloop.Loop("tcp4", args, _stream_ptrs(streams), ROOM, "tasx_tcp4_cksum_batch_dev_room")


class RxVerifyWorkload:
    """Receive-side verification over a Tcp4Workload's (checksummed) frames,
    the received frame length as the uniform hint (the read bound)."""

    def __init__(self, wl: Tcp4Workload):
        self.wl = wl
        wl.rx_flags = [torch.empty(wl.n, dtype=torch.uint8, device="cuda") for _ in wl.bufs]
        self.bytes_per_step = wl.n * (wl.ip_total + 1)

    def loop(self, streams=None) -> benchloop.Loop:
        wl = self.wl
        args = [benchloop.Tcp4Args(b.data_ptr(), None, wl.stride, None, wl.hint, 0, wl.n, IP_OFF, L4_OFF, 0,
                                   f.data_ptr()) for b, f in zip(wl.bufs, wl.rx_flags)]
        return benchloop.Loop("tcp4", args, _stream_ptrs(streams), VERIFY, "tasx_tcp4_verify_batch_dev_room")


class RxMixWorkload:
    """Receive-side verification of a FlushMixWorkload's frames after their TX
    checksums (an RX burst of data segments and pure ACKs), each frame's
    received length (the mbuf data_len) as its per-frame hint and read bound."""
    desc = (f"{N_FRAMES} received TAS frames in {STRIDE} B rooms, 50% data segments and 50% pure ACKs, "
            "per-frame received lengths (tasx_tcp4_verify_batch_dev_hint)")

    def __init__(self, mw: "FlushMixWorkload"):
        self.mw = mw
        for b in mw.bufs:  # TX checksums in place: the frames as a receiver gets them
            xsum.tcp4_cksum_batch(b, mw.n, stride=mw.stride, frame_len=mw.flen, room=mw.stride, inplace=True,
                                  want_out=False)
        self.flags = [torch.empty(mw.n, dtype=torch.uint8, device="cuda") for _ in mw.bufs]
        self.bytes_per_step = mw.bytes_per_step - 3 * mw.n  # total_length read + 1 B of flags per frame

    def loop(self, streams=None) -> benchloop.Loop:
        mw = self.mw
        args = [benchloop.Tcp4Args(b.data_ptr(), None, mw.stride, mw.flen.data_ptr(), 0, 0, mw.n, IP_OFF, L4_OFF, 0,
                                   f.data_ptr()) for b, f in zip(mw.bufs, self.flags)]
        return benchloop.Loop("tcp4", args, _stream_ptrs(streams), VERIFY, "tasx_tcp4_verify_batch_dev_hint")


class RawWorkload:
    desc = f"{N_FRAMES} x {RAW_LEN} B packed payloads, rte_raw_cksum per packet"

    def __init__(self, rotate: int, seed: int, n: int = N_FRAMES, length: int = RAW_LEN,
                 offsets=None, lengths=None, total_bytes: int | None = None):
        self.n = n
        self.len0 = length
        if offsets is None:
            first = device_random(n * length, seed)
            self.off = self.lens = None
            self.bytes_per_step = n * (length + 2)
        else:
            first = device_random(total_bytes, seed)
            self.off = torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).cuda()
            self.lens = torch.from_numpy(np.ascontiguousarray(lengths, np.int32)).cuda()
            self.bytes_per_step = int(np.asarray(lengths, np.int64).sum()) + 2 * n
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.outs = [torch.empty(n, dtype=torch.int16, device="cuda") for _ in range(rotate)]

    def loop(self, streams=None) -> benchloop.Loop:
        op = self.off.data_ptr() if self.off is not None else None
        lp = self.lens.data_ptr() if self.lens is not None else None
        args = [benchloop.RawArgs(b.data_ptr(), op, self.len0 if op is None else 0, lp, self.len0, self.n,
                                  o.data_ptr()) for b, o in zip(self.bufs, self.outs)]
        return benchloop.Loop("raw", args, _stream_ptrs(streams), what="tasx_raw_cksum_batch_dev")


class TxSegWorkload:
    """Fused TX segment build: per segment, the
    payload read from the flow's circular TX buffer in shm, written into the
    frame, and both checksums stored (flow_tx_read + tcp_checksums,
    tas/fast/fast_flows.c:930-936).  Headers are pre-filled; shm and frames are
    device-resident.  Algorithmic bytes per segment: payload read + payload
    written + the 20 B IP header and hdrs_len - l4_off L4 header bytes read +
    4 B of checksums written."""
    desc = (f"{N_FRAMES} TAS TX segments of {pktgen.TCP_MSS} B payload from 8192 flows' 16 KiB circular TX "
            f"buffers (wraps included) into 1514 B frames at {STRIDE} B stride (descriptor room = the {STRIDE} B "
            "mbuf data room, scratch past the frame), checksums in place")

    def __init__(self, rotate: int, seed: int, n: int = N_FRAMES):
        self.n = n
        # room = the mbuf data room (TAS: BUFFER_SIZE, tas/fast/internal.h:34),
        # scratch past the frame (an mbuf carries nothing past data_len)
        _, _, segs, shm_len = pktgen.tx_segments(n, seed=seed, nflows=8192, tx_len=16384, make_shm=False,
                                                 room=STRIDE)
        segs["room"] = np.uint32(STRIDE | xsum.TXSEG_SCRATCH)
        self.segs_np, self.shm_len = segs, shm_len
        self.segs = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
        self.shms = [device_random(shm_len, seed + 7 + r) for r in range(rotate)]
        first = device_tcp4_frames(n, STRIDE, IP_TOTAL, seed)
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(rotate)]
        hdr = pktgen.HDRS_LEN - pktgen.ETH_LEN - pktgen.IP_LEN
        self.bytes_per_seg = 2 * pktgen.TCP_MSS + pktgen.IP_LEN + hdr + 4
        self.bytes_per_step = n * self.bytes_per_seg
        self.block_floor = txseg_block_floor(segs)

    def loop(self, streams=None) -> benchloop.Loop:
        args = [benchloop.TxSegArgs(sh.data_ptr(), self.shm_len, b.data_ptr(), self.segs.data_ptr(), self.n, IP_OFF,
                                    L4_OFF, o.data_ptr()) for sh, b, o in zip(self.shms, self.bufs, self.outs)]
        return benchloop.Loop("txseg", args, _stream_ptrs(streams), what="tasx_tx_segment_batch_dev")

    def cpu_check(self, budget_s: float) -> dict:
        """The oracle's copy + tcp_checksums per segment on this box's cores, on
        rotation 0's inputs, and a bit-exact comparison of the built frames."""
        from oracle import oracle_lib
        orc = oracle_lib.Oracle()
        torch.cuda.synchronize()
        shm = self.shms[0].cpu().numpy()
        gpu_frames = self.bufs[0].cpu().numpy()
        frames = gpu_frames.copy()
        # un-build: the oracle must produce the built frames from scratch
        f2 = frames.reshape(self.n, STRIDE)
        f2[:, pktgen.HDRS_LEN:FRAME_LEN] ^= 0x5A
        f2[:, 24:26] = 0
        f2[:, 50:52] = 0
        threads = min(16, len(os.sched_getaffinity(0)))
        t = orc.bench_tx_segment(shm, self.shm_len, frames, self.segs_np, threads=threads, reps=1)
        reps = max(3, min(500, int(budget_s / max(t, 1e-6))))
        t = orc.bench_tx_segment(shm, self.shm_len, frames, self.segs_np, threads=threads, reps=reps)
        # one core (what a TAS fast-path core pays per segment: the copy and the checksums)
        t1 = orc.bench_tx_segment(shm, self.shm_len, frames, self.segs_np, threads=1, reps=3)
        return {"value": self.bytes_per_step / t / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": f"rotation 0's {self.n} segments, oracle flow_tx_read + tcp_checksums per segment, "
                          f"median of {reps} passes",
                "single_core_us_per_segment": round(t1 / self.n * 1e6, 4),
                "parity_vs_gpu": "bit-exact" if np.array_equal(frames, gpu_frames) else "MISMATCH"}


def txseg_pattern_ceiling(tw: "TxSegWorkload", avg_us: float, launches: int = 100) -> dict:
    """The TX segment build's access pattern alone, timed live over the same
    rotation: tasx_ab_tx_segment_form(40) of the comparison build -- the
    product's descriptor, header and aligned source loads and its frame
    stores, the loaded chunks stored as they are (no LDS realignment, no
    splice)."""
    ab = xsum._load(xsum.AB_LIB_PATH)
    s = torch.cuda.current_stream().cuda_stream
    R = len(tw.shms)

    # the same rotation of shm regions and frame buffers as the leg (the
    # pattern stores unrealigned bytes: the leg's frames are not checked after it)
    def pat(k):
        rc = ab.tasx_ab_tx_segment_form(40, tw.shms[k % R].data_ptr(), tw.shm_len, tw.bufs[k % R].data_ptr(),
                                        tw.segs.data_ptr(), tw.n, IP_OFF, L4_OFF, tw.outs[k % R].data_ptr(), s)
        if rc:
            raise xsum.TasxError(rc, "tasx_ab_tx_segment_form(40)")
    for k in range(10):
        pat(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(launches):
        pat(k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / launches
    return {"bound": "the access pattern", "us": round(us, 3), "frac": round(us / avg_us, 4),
            "kernel": "tx_segment_lds_kernel<pattern> (libtasx_ab.so): the product's loads and stores, "
                      "no realignment through LDS"}


def txseg_block_floor(segs, block: int = 128) -> dict:
    """HBM bytes the TX segment build cannot avoid at the memory side's 128-byte
    request granularity (calibrated: tools/fetch_calib.hip): the blocks each
    payload piece (two at a wrap) occupies in shm, the frame's header block,
    the 32-byte descriptor; writes of the frame's whole blocks (scratch room)."""
    base = segs["tx_base"].astype(np.int64)
    pos = segs["pos"].astype(np.int64)
    pay = segs["payload"].astype(np.int64)
    tlen = segs["tx_len"].astype(np.int64)
    p1 = np.minimum(pay, tlen - pos)
    a1, b1 = base + pos, base + pos + p1
    blocks = np.where(p1 > 0, (b1 + block - 1) // block - a1 // block, 0)
    p2 = pay - p1
    blocks += np.where(p2 > 0, (base + p2 + block - 1) // block - base // block, 0)
    off = segs["frame_off"].astype(np.int64)
    fend = off + segs["hdrs_len"].astype(np.int64) + pay
    reads = int(blocks.sum()) * block + len(segs) * (block + 32)
    writes = int(((fend + block - 1) // block - off // block).sum()) * block
    return {"read_bytes": reads, "write_bytes": writes, "bytes": reads + writes, "block": block}


class FlowLookupWorkload:
    """RX flow lookup (fast_flows_packet_fss,
    tas/fast/fast_flows.c:1084-1163): per received frame the CRC32C flow hash,
    the 4-entry bucket probe and the flow-state key check.  TAS-sized table:
    FLEXNIC_PL_FLOWST_NUM = 131072 flows, 2x hash entries; 90% of the frames
    hit a random flow, 10% carry unknown keys.  Frames one per 2 KiB mbuf.
    Bytes per frame: 12 key + 32 bucket + 12 flow key read, 8 written."""
    NFLOWS, ENTRIES, N = 131072, 262144, 262144
    desc = (f"{N} RX frames (2 KiB mbufs) looked up in a {NFLOWS}-flow / {ENTRIES}-entry flow table "
            "(CRC32C hash, 4-entry bucket, flow-state key check), 10% unknown keys")

    def __init__(self, rotate: int, seed: int):
        keys = pktgen.flow_keys(self.NFLOWS, seed=seed)
        self.keys = keys
        self.fs_np = pktgen.flow_state(keys, seed=seed)
        self.fs = torch.from_numpy(self.fs_np).cuda()
        # hashes of the flows' own keys through the kernel (one-entry dummy table)
        fr = torch.from_numpy(pktgen.rx_frames(keys, stride=128, seed=seed)).cuda()
        dummy = torch.zeros(2, dtype=torch.int32, device="cuda")
        h, _ = xsum.flow_lookup_batch(fr, self.NFLOWS, dummy, self.fs, self.NFLOWS, stride=128)
        ht, ok = pktgen.flow_table(h.cpu().numpy().view(np.uint32), self.ENTRIES)
        self.ht_np = ht
        self.ht = torch.from_numpy(ht).cuda()
        rng = np.random.default_rng(seed)
        fkeys = keys[rng.integers(0, self.NFLOWS, self.N)].copy()
        miss = rng.random(self.N) < 0.1
        fkeys[miss, 4] ^= 0x5A
        self.frames_np = pktgen.rx_frames(fkeys, stride=STRIDE, seed=seed + 1)
        first = torch.from_numpy(self.frames_np).cuda()
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.fids = [torch.empty(self.N, dtype=torch.int32, device="cuda") for _ in range(rotate)]
        self.hashes = [torch.empty(self.N, dtype=torch.int32, device="cuda") for _ in range(rotate)]
        self.n = self.N
        self.bytes_per_step = self.N * (12 + 32 + 12 + 8)
        self.inserted = float(ok.mean())

    def loop(self, streams=None) -> benchloop.Loop:
        args = [benchloop.FlowArgs(b.data_ptr(), None, STRIDE, self.N, IP_OFF, L4_OFF, self.ht.data_ptr(),
                                   self.ENTRIES, self.fs.data_ptr(), self.NFLOWS, pktgen.FLOWST_SIZE,
                                   pktgen.FLOWST_KEY_OFF, h.data_ptr(), f.data_ptr())
                for b, h, f in zip(self.bufs, self.hashes, self.fids)]
        return benchloop.Loop("flow", args, _stream_ptrs(streams), what="tasx_flow_lookup_batch_dev")

    def cpu_check(self, budget_s: float) -> dict:
        from oracle import oracle_lib
        orc = oracle_lib.Oracle()
        torch.cuda.synchronize()
        gpu_fid = self.fids[0].cpu().numpy().view(np.uint32)
        _, exp = orc.flow_lookup_batch(self.frames_np, self.N, self.ht_np, self.fs_np, fs_num=self.NFLOWS,
                                       stride=STRIDE)
        threads = min(16, len(os.sched_getaffinity(0)))
        kw = dict(fs_num=self.NFLOWS, stride=STRIDE)
        t = orc.bench_flow_lookup(self.frames_np, self.N, self.ht_np, self.fs_np, threads=threads, reps=1, **kw)
        reps = max(3, min(500, int(budget_s / max(t, 1e-6))))
        t = orc.bench_flow_lookup(self.frames_np, self.N, self.ht_np, self.fs_np, threads=threads, reps=reps, **kw)
        return {"value": self.N / t / 1e6, "unit": "Mpps", "cores": threads, "kind": "port",
                "sample": f"rotation 0's {self.N} frames, oracle fast_flows_packet_fss restatement, "
                          f"median of {reps} passes",
                "parity_vs_gpu": "bit-exact" if np.array_equal(exp, gpu_fid) else "MISMATCH"}


class RxPassWorkload:
    """One RX pass (tasx_rx_batch_dev): checksum verification and the flow
    lookup of the same received frames in one kernel (SURVEY.md section 8f rows
    3 + 4; fast_flows_packet_fss, tas/fast/fast_flows.c:1084-1163).  An RX burst
    of 50% data segments and 50% pure ACKs in 2048 B mbufs, each frame's
    received length as its hint and read bound, flow keys drawn from the
    TAS-sized flow table of FlowLookupWorkload (10% unknown).  Algorithmic bytes
    per frame: ip.total_length + 2 B total_length read + 1 B flags (verify), 32
    B bucket + 12 B flow key read + 8 B hash and flow id written (lookup; the
    frame's key is inside the header verify reads)."""
    desc = (f"{N_FRAMES} received TAS frames in {STRIDE} B rooms, 50% data segments and 50% pure ACKs, per-frame "
            f"received lengths, looked up in a {FlowLookupWorkload.NFLOWS}-flow / {FlowLookupWorkload.ENTRIES}-"
            "entry flow table (10% unknown keys): tasx_rx_batch_dev")

    def __init__(self, fw: "FlowLookupWorkload", rotate: int, seed: int, n: int = N_FRAMES, ack_frac: float = 0.5):
        rng = np.random.default_rng(seed)
        pay = np.where(rng.random(n) < ack_frac, 0, IP_TOTAL - 52).astype(np.int64)
        keys = fw.keys[rng.integers(0, fw.NFLOWS, n)].copy()
        keys[rng.random(n) < 0.1, 4] ^= 0x5A
        host = pktgen.tcp4_frames(n, payload=pay, stride=STRIDE, seed=seed)
        pktgen.set_flow_keys(host, keys, STRIDE)
        self.n, self.fw = n, fw
        first = torch.from_numpy(host).cuda()
        self.flen = torch.from_numpy((pktgen.ETH_LEN + 52 + pay).astype(np.int32)).cuda()
        xsum.tcp4_cksum_batch(first, n, stride=STRIDE, frame_len=self.flen, room=STRIDE, inplace=True,
                              want_out=False)
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.flags = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in self.bufs]
        self.fids = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in self.bufs]
        self.hashes = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in self.bufs]
        self.bytes_per_step = int((52 + pay + 3).sum()) + n * (32 + 12 + 8)

    def loop(self, which: int = benchloop.RX_FUSED, streams=None, uniform: bool = False) -> benchloop.Loop:
        """uniform: the received length as one uniform hint (all-data bursts)."""
        fw = self.fw
        flen, flen0 = (None, FRAME_LEN) if uniform else (self.flen.data_ptr(), 0)
        args = [benchloop.RxArgs(
            benchloop.Tcp4Args(b.data_ptr(), None, STRIDE, flen, flen0, 0, self.n, IP_OFF, L4_OFF, 0,
                               fl.data_ptr()),
            benchloop.FlowArgs(b.data_ptr(), None, STRIDE, self.n, IP_OFF, L4_OFF, fw.ht.data_ptr(), fw.ENTRIES,
                               fw.fs.data_ptr(), fw.NFLOWS, pktgen.FLOWST_SIZE, pktgen.FLOWST_KEY_OFF,
                               h.data_ptr(), f.data_ptr()))
            for b, fl, h, f in zip(self.bufs, self.flags, self.hashes, self.fids)]
        what = "tasx_rx_batch_dev" if which == benchloop.RX_FUSED else "verify + flow lookup"
        return benchloop.Loop("rx", args, _stream_ptrs(streams), which, what)


# Flow lookup bounds.  The lookup is a dependent chain
# per frame: the frame's key (HBM), its 4-entry bucket (flowht, 2 MB), the
# candidate flows' keys (flowst, 16 MB; both MALL-resident).  Each random
# access costs a whole 128-byte L2 line, so the HBM roofline counts 128 B per
# frame header (+ 8 B written), and the ceiling of the chain itself is
# measured live: the same access pattern with no hashing or key logic
# (tasx_ab_flow_pattern, the A/B build; tools/flow_ceiling.hip).
L2_LINE = 128


def flow_bounds(fw: "FlowLookupWorkload", avg_us: float, launches: int = 100) -> dict:
    ab = xsum._load(xsum.AB_LIB_PATH)
    out = torch.empty(fw.N, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    R = len(fw.bufs)

    def pat(k):
        rc = ab.tasx_ab_flow_pattern(fw.bufs[k % R].data_ptr(), STRIDE, fw.N, IP_OFF, fw.ht.data_ptr(), fw.ENTRIES,
                                     fw.fs.data_ptr(), fw.NFLOWS, pktgen.FLOWST_SIZE, pktgen.FLOWST_KEY_OFF,
                                     out.data_ptr(), s)
        if rc:
            raise xsum.TasxError(rc, "tasx_ab_flow_pattern")
    for k in range(20):
        pat(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(launches):
        pat(k)
    e1.record()
    torch.cuda.synchronize()
    ceil_us = e0.elapsed_time(e1) * 1e3 / launches
    line_bytes = fw.N * (L2_LINE + 8)
    return {
        "line_roofline": {"bound": "hbm", "bytes_per_frame": L2_LINE + 8,
                          "achieved": round(line_bytes / avg_us / 1e3, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(line_bytes / avg_us / 1e3 / HBM_PEAK_GBS, 4),
                          "achievable_peak": HBM_ACHIEVABLE_GBS,
                          "frac_of_achievable": round(line_bytes / avg_us / 1e3 / HBM_ACHIEVABLE_GBS, 4),
                          "note": "one 128-byte L2 line per frame header (the key's 12 bytes cost a whole line); "
                                  "achievable_peak: MI355X_MICROARCH.md's ~6.3 TB/s"},
        "pattern_ceiling": {"bound": "dependent access chain", "us": round(ceil_us, 3),
                            "frac": round(ceil_us / avg_us, 4),
                            "chain": "frame key (HBM) -> 4-entry bucket (flowht) -> candidate keys (flowst)",
                            "kernel": "flow_pattern_kernel (libtasx_ab.so): the same loads, no CRC or compares"},
    }


def tcp4_pattern_ceiling(wl: "Tcp4Workload", avg_us: float, launches: int = 200) -> dict:
    """The headline's access pattern with no checksum logic
    (tasx_ab_tcp4_pattern, the A/B build), timed over the same rotation."""
    ab = xsum._load(xsum.AB_LIB_PATH)
    s = torch.cuda.current_stream().cuda_stream
    R = len(wl.bufs)
    outs = [torch.empty(wl.n, dtype=torch.int32, device="cuda") for _ in range(2)]  # not the checked results

    def pat(k):
        rc = ab.tasx_ab_tcp4_pattern(wl.bufs[k % R].data_ptr(), wl.stride, wl.n, wl.hint, IP_OFF,
                                     outs[k % 2].data_ptr(), s)
        if rc:
            raise xsum.TasxError(rc, "tasx_ab_tcp4_pattern")
    for k in range(20):
        pat(k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(launches):
        pat(k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / launches
    return {"bound": "the access pattern", "us": round(us, 3), "frac": round(us / avg_us, 4),
            "kernel": "tcp4_pattern_kernel (libtasx_ab.so): the headline's rows, loads, result stores and "
                      "residency, words xor-folded instead of summed"}


# tasx_ab_stream_read paths: 0 register loads in grid order, 2 + k register
# loads with the blocks in XCD runs of 2^k (round 5, xcd_run: runs of 64 read
# config 4's 12.6 GB fastest, profiles/r05/INDEX.md r05b).  LDS-DMA (path 1)
# was slower at every size (profiles/r04/INDEX.md r04a) and left the line in
# round 6 with the other inline-asm M0 code.
READ_PATHS = {"register": 0, "register_xcd64": 8, "register_xcd256": 10}


def read_ceiling(wl, avg_us: float, launches: int = 200) -> dict:
    """A pure streaming read of a leg's algorithmic bytes per launch, over the
    same buffer rotation (wl.bufs), by tasx_ab_stream_read of the comparison
    build: register loads in grid order and in XCD runs.  The fastest is the
    read ceiling.  Launch counts shrink with the size (about 0.1 s of reads per
    path)."""
    ab = xsum._load(xsum.AB_LIB_PATH)
    s = torch.cuda.current_stream().cuda_stream
    R = len(wl.bufs)
    nbytes = min(wl.bytes_per_step, min(b.numel() for b in wl.bufs)) // 1024 * 1024
    launches = max(10, min(launches, int(0.1 / (nbytes / 7e12))))
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")

    def timed(path: int) -> float:
        def rd(k):
            rc = ab.tasx_ab_stream_read(wl.bufs[k % R].data_ptr(), nbytes, path, sink.data_ptr(), s)
            if rc:
                raise xsum.TasxError(rc, "tasx_ab_stream_read")
        for k in range(min(20, launches)):
            rd(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(launches):
            rd(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / launches
    per = {name: timed(path) for name, path in READ_PATHS.items()}
    best = min(per, key=per.get)
    us = per[best]
    return {"bound": "a pure streaming read of the same bytes", "bytes": nbytes, "launches": launches,
            **{f"{k}_us": round(v, 3) for k, v in per.items()}, "us": round(us, 3), "path": best,
            "frac": round(us / avg_us, 4), "achieved_gbs": round(nbytes / us / 1e3, 1),
            "kernels": "stream_read_reg_kernel in grid order / XCD runs (libtasx_ab.so)"}


def mix_bounds(mw: "FlushMixWorkload", launches: int = 200) -> dict:
    """The data/ACK mix's latency roofline, measured live
    with the A/B build's tasx_ab_tcp4_mix_pattern over the flush_mix frames:
    `chain_us` -- each row's dependent chain alone (hint -> the chunk holding
    the frame's end -> result store, 8 waves per SIMD as the product: almost no
    bytes), `pattern_us` -- the product's exact loads and stores with the words
    xor-folded.  The roofline is the larger of the chain and the HBM time of
    the algorithmic bytes at 8 TB/s; the chain over its generations of
    resident rows gives the loaded latency per dependent load."""
    ab = xsum._load(xsum.AB_LIB_PATH)
    s = torch.cuda.current_stream().cuda_stream
    R = len(mw.bufs)
    outs = [torch.empty(mw.n, dtype=torch.int32, device="cuda") for _ in range(2)]  # not the checked results

    def timed(chain: int) -> float:
        def pat(k):
            rc = ab.tasx_ab_tcp4_mix_pattern(mw.bufs[k % R].data_ptr(), mw.stride, mw.n, mw.flen.data_ptr(), IP_OFF,
                                             chain, outs[k % 2].data_ptr(), s)
            if rc:
                raise xsum.TasxError(rc, "tasx_ab_tcp4_mix_pattern")
        for k in range(20):
            pat(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(launches):
            pat(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / launches

    # medians of 3 interleaved runs each: one chain run slowed by anything
    # else on the device (a profiler, another process) would otherwise set the bound
    runs = [(timed(0), timed(1)) for _ in range(MIX_BOUND_RUNS)]
    pattern_runs, chain_runs = sorted(r[0] for r in runs), sorted(r[1] for r in runs)
    pattern_us, chain_us = pattern_runs[len(runs) // 2], chain_runs[len(runs) // 2]
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    rows_in_flight = cus * 4 * 8 * 4  # CUs x SIMDs x 8 waves x 4 rows of 16 lanes
    gens = -(-mw.n // rows_in_flight)
    return {"pattern_us": round(pattern_us, 3), "chain_us": round(chain_us, 3),
            "pattern_runs_us": [round(x, 3) for x in pattern_runs], "chain_runs_us": [round(x, 3) for x in chain_runs],
            "rows": mw.n, "rows_in_flight": rows_in_flight, "generations": gens, "dependent_loads_per_row": 2,
            "loaded_latency_us": round(chain_us / (gens * 2), 3),
            "kernel": "tcp4_mix_pattern_kernel<chain> / tcp4_mix_pattern_kernel (libtasx_ab.so)"}


MIX_BOUND_RUNS = 3


def price_mix(leg_: dict, mb: dict, alg_bytes: int) -> None:
    """Attach the latency roofline (mix_bounds) to a data/ACK mix leg's roofline.
    The chain kernel does a subset of the product's work, so a chain that
    times slower than the product's own access pattern is a disturbed
    measurement (round 3: 10.1 us under rocprofv3 against 5.1 us alone), and
    then no fraction is claimed (frac null)."""
    avg = leg_["roofline"]["launch_avg_us"]
    hbm_us = alg_bytes / HBM_PEAK_GBS / 1e3
    bound_us = max(mb["chain_us"], hbm_us)
    sane = mb["chain_us"] <= mb["pattern_us"]
    leg_["roofline"]["latency"] = dict(mb, **{
        "bound": "max(dependent chain, HBM)", "hbm_us": round(hbm_us, 3), "bound_us": round(bound_us, 3),
        "frac": round(bound_us / avg, 4) if sane else None, "frac_of_pattern": round(mb["pattern_us"] / avg, 4),
        "model": "chain_us = generations x dependent_loads_per_row x loaded_latency_us; "
                 "frac = max(chain_us, bytes / 8 TB/s) / launch",
        **({} if sane else {"note": "chain slower than the product's access pattern: disturbed run, no frac"})})


def copy_ceiling(nbytes: int, copies: int = 50, rotate: int = 4) -> dict:
    """The device's read+write streaming rate, measured live: a grid-stride
    copy kernel (one non-temporal 16-byte load and store per lane;
    tasx_ab_stream_copy, the A/B build) of `nbytes` between rotating buffer
    pairs (4 pairs: more than the MALL holds), events around `copies` copies --
    faster than the runtime's hipMemcpyAsync D2D, which is timed beside it.
    The TX segment build moves about as many bytes each way."""
    nbytes = nbytes // 16 * 16
    ab = xsum._load(xsum.AB_LIB_PATH)
    st = torch.cuda.current_stream().cuda_stream
    src = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(rotate)]
    dst = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(rotate)]

    def kern(k):
        rc = ab.tasx_ab_stream_copy(src[k % rotate].data_ptr(), dst[k % rotate].data_ptr(), nbytes, st)
        if rc:
            raise xsum.TasxError(rc, "tasx_ab_stream_copy")

    def runtime(k):
        dst[k % rotate].copy_(src[k % rotate])

    def timed(fn):
        for k in range(8):
            fn(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(copies):
            fn(k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / copies
    us, us_rt = timed(kern), timed(runtime)
    del src, dst
    torch.cuda.empty_cache()
    return {"bytes_each_way": nbytes, "us": round(us, 3), "GBps": round(2 * nbytes / us / 1e3, 1),
            "frac_of_spec": round(2 * nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "how": "stream_copy_kernel (libtasx_ab.so): grid-stride, one non-temporal 16-byte load and store per "
                   "lane, 4 rotating buffer pairs, HIP events around 50 copies",
            "hipmemcpy_us": round(us_rt, 3), "hipmemcpy_GBps": round(2 * nbytes / us_rt / 1e3, 1)}


def prewarm(run, seconds: float = 0.25):
    """Bring the GPU out of idle clocks before any measured step (not part of
    W or K)."""
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        run(k, 32)
        k += 32
        torch.cuda.synchronize()


CTX2_MIN_STEPS = 200  # the two-context leg's minimum step count


def timed_run(run, steps: int, warmup: int, ws: int, streams=None, spans: dict | None = None):
    """W untimed steps, then exactly K timed steps between barrier+sync pairs,
    issued by one C loop.  HIP events on the launch stream give the average
    launch duration (no per-launch events, which would add gaps of their
    own): on one stream, from an event behind the FIRST timed launch to one
    behind the last, over launches 2..K -- the first launch after the
    synchronize also carries an idle GPU's dispatch of it (~6 us, which at the
    driver's K = 20 read as 0.3 us on every launch against rocprofv3's own
    kernel durations, profiles/r05 r05t); the start event sits before the
    first launch all the same, and e0 -> e1 / K is returned in `spans`.  The
    middle event costs the host a few us while the GPU runs launch 1, so the
    timed region (GPU-bound) is unchanged.  With several streams one event
    pair brackets all of them (they wait on the start event; the current
    stream waits on each one's end)."""
    prewarm(run)
    run(0, warmup)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    em = torch.cuda.Event(enable_timing=True)
    mid = not streams and steps > 1
    # torch creates an event's HIP handle on its first record(): do that here,
    # not inside the timed region (10-44 us per event, profiles/r02/r02aw)
    e0.record(cur)
    em.record(cur)
    e1.record(cur)
    torch.cuda.synchronize()
    barrier(ws)
    torch.cuda.synchronize()
    # the start event goes in just before t0: it brackets the launches (the
    # roofline's kernel time) without its host cost inside the timed region
    e0.record(cur)
    for s in streams or []:
        s.wait_event(e0)
    t0 = time.perf_counter()
    ta = time.perf_counter()
    if mid:
        run(warmup, 1)
        em.record(cur)
        run(warmup + 1, steps - 1)
    else:
        run(warmup, steps)
    tb = time.perf_counter()
    for s in streams or []:
        cur.wait_stream(s)
    e1.record(cur)
    tc = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    # the closing barrier aligns the ranks for what follows; it stays out of
    # each rank's interval (an RCCL round trip at N > 1), and the MAX over
    # ranks taken by the caller is the slowest rank's K steps
    barrier(ws)
    if os.environ.get("TASX_BENCH_TRACE"):
        print(json.dumps({"K": steps, "rec0_us": round((ta - t0) * 1e6, 2), "issue_us": round((tb - ta) * 1e6, 2),
                          "rec1_us": round((tc - tb) * 1e6, 2), "sync_us": round((t1 - tc) * 1e6, 2),
                          "host_us": round((t1 - t0) * 1e6, 2),
                          "event_us": round(e0.elapsed_time(e1) * 1e3, 2)}), file=sys.stderr)
    span = e0.elapsed_time(e1) / steps
    if spans is not None:
        spans["span_avg_us"] = round(span * 1e3, 3)
    return t1 - t0, em.elapsed_time(e1) / (steps - 1) if mid else span


def drop_rehearsal_fractions(obj):
    """--rehearse: ranks share one GPU, so no fraction of a roofline, a ceiling
    or N x HBM is a claim; any such fraction above 1 is dropped (None)."""
    if isinstance(obj, dict):
        return {k: (None if "frac" in k and isinstance(v, (int, float)) and v > 1 else drop_rehearsal_fractions(v))
                for k, v in obj.items()}
    if isinstance(obj, list):
        return [drop_rehearsal_fractions(v) for v in obj]
    return obj


def roofline(bytes_per_launch: int, avg_ms: float, traffic):
    avg_s = avg_ms / 1e3
    achieved = bytes_per_launch / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "launch_avg_us": round(avg_s * 1e6, 3), "algorithmic_bytes_per_launch": bytes_per_launch}


def leg(run, bytes_per_step: int, args, ws, desc, kernel: str = "", streams=None):
    spans = {}
    dt, avg_ms = timed_run(run, args.steps, args.warmup, ws, streams, spans)
    per_rank = gather_over_ranks(bytes_per_step * args.steps / dt / GIB, ws)
    dtm = max_over_ranks(dt, ws)
    total = sum_over_ranks(float(bytes_per_step * args.steps), ws)
    r = {"value": total / dtm / GIB, "unit": "GiB/s", "ms_per_step": dtm / args.steps * 1e3,
         "workload": desc, "roofline": roofline(bytes_per_step, avg_ms, None), "seconds": dt}
    r["roofline"]["span_avg_us"] = spans.get("span_avg_us")  # e0 -> e1 over all K launches
    if kernel:
        r["kernel"] = kernel
    if ws > 1:
        r["per_rank_value"] = [round(v, 2) for v in per_rank]
    return r


# ---------------------------------------------------------------------------
# end to end (PCIe-inclusive; never the headline)

def txseg_host_leg(ws: int, rank: int, reps: int) -> dict:
    """The fused TX segment build as TAS would run it: the
    app's TX buffers (tas_shm), the mbuf frames and the descriptors all in
    pinned host memory mapped for the GPU; the kernel gathers each payload and
    writes each frame over PCIe.  The same 64K segments as the device-resident
    tx_segment leg; tests/test_txseg.py::test_gpu_txseg_host_memory checks it."""
    n = N_FRAMES
    _, _, segs, shm_len = pktgen.tx_segments(n, seed=pktgen.SEED + 2000 + rank, nflows=8192, tx_len=16384,
                                             make_shm=False, room=STRIDE)
    pins = []
    try:
        hs = xsum.PinnedBuffer(shm_len)
        pins.append(hs)
        hs.array[:] = device_random(shm_len, pktgen.SEED + 7 + rank).cpu().numpy()
        hf = xsum.PinnedBuffer(n * STRIDE)
        pins.append(hf)
        hf.array[:] = device_tcp4_frames(n, STRIDE, IP_TOTAL, pktgen.SEED + rank).cpu().numpy()
        hd = xsum.PinnedBuffer(segs.nbytes)
        pins.append(hd)
        hd.array[:] = segs.view(np.uint8)
        out = torch.empty(n, dtype=torch.int32, device="cuda")

        def run():
            xsum.tx_segment_batch(hs.dev_addr, hf.dev_addr, hd.dev_addr, n, shm_len=shm_len, out=out)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.25:  # clocks and PCIe out of idle (~3 ms per launch)
            run()
            torch.cuda.current_stream().synchronize()  # (no backlog of queued launches into the timed region)
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        tm = max_over_ranks(t, ws)
        kernel = xsum.last_kernel()
        # the kernel's own time by HIP events, for the link ceiling below
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        kern_us = e0.elapsed_time(e1) * 1e3 / reps
        # its access pattern alone over the same host buffers (as
        # txseg_pattern_ceiling: the loads and stores, no realignment; last,
        # since it stores unrealigned bytes into the frames)
        ab = xsum._load(xsum.AB_LIB_PATH)
        s = torch.cuda.current_stream().cuda_stream

        def pat():
            rc = ab.tasx_ab_tx_segment_form(40, hs.dev_addr, shm_len, hf.dev_addr, hd.dev_addr, n, IP_OFF, L4_OFF,
                                            out.data_ptr(), s)
            if rc:
                raise xsum.TasxError(rc, "tasx_ab_tx_segment_form(40)")
        pat()
        e0.record()
        for _ in range(reps):
            pat()
        e1.record()
        torch.cuda.synchronize()
        pat_us = e0.elapsed_time(e1) * 1e3 / reps
        hdr = pktgen.HDRS_LEN - pktgen.ETH_LEN - pktgen.IP_LEN
        alg = n * (2 * pktgen.TCP_MSS + pktgen.IP_LEN + hdr + 4)
        h2d, d2h = n * (pktgen.TCP_MSS + pktgen.HDRS_LEN + 32), n * (pktgen.HDRS_LEN + pktgen.TCP_MSS)
        res = {"value": sum_over_ranks(alg * reps, ws) / tm / GIB, "unit": "GiB/s (algorithmic, as tx_segment)",
               "ms_per_batch": tm / reps * 1e3, "segments_per_s": sum_over_ranks(n * reps, ws) / tm,
               "kernel_us_events": round(kern_us, 1),
               "pattern_ceiling": {"us": round(pat_us, 1), "frac": round(pat_us / kern_us, 4),
                                   "kernel": "tx_segment_lds_kernel<pattern> (libtasx_ab.so) over the same host "
                                             "buffers: the product's loads and stores, no realignment"},
               "pcie_h2d_bytes_per_rank": h2d, "pcie_d2h_bytes_per_rank": d2h,
               "kernel": kernel,
               "note": "tas_shm, frames and descriptors in pinned host memory; payload read and frame "
                       "written over PCIe in one pass"}
    finally:
        for pb in pins:
            pb.free()
    if rank == 0:
        # is the link the bound?  The same bytes each way moved by a plain
        # streaming copy between two pinned host buffers
        res["link_ceiling"] = host_link_ceiling(max(h2d, d2h))
        lc = res["link_ceiling"]
        lc["build_frac_of_copy"] = round(lc["us"] / res["kernel_us_events"], 4)
        lc["build_frac_of_copy_wall"] = round(lc["us"] / (res["ms_per_batch"] * 1e3), 4)
    return res


def host_link_ceiling(nbytes: int, copies: int = 20) -> dict:
    """The GPU's concurrent read-from and write-to host rate, measured live:
    the grid-stride copy kernel (tasx_ab_stream_copy, the A/B build) from one
    pinned host buffer to another, `nbytes` each way -- what the TX build from
    host memory moves (payloads and headers in, frames out), with none of its
    gather.  Also the read-only and write-only halves (host -> HBM, HBM ->
    host) by the same kernel."""
    nbytes = nbytes // 16 * 16
    ab = xsum._load(xsum.AB_LIB_PATH)
    st = torch.cuda.current_stream().cuda_stream
    pins = []
    try:
        a = xsum.PinnedBuffer(nbytes)
        pins.append(a)
        b = xsum.PinnedBuffer(nbytes)
        pins.append(b)
        a.array[:] = 1
        d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")

        def copy(src, dst):
            rc = ab.tasx_ab_stream_copy(src, dst, nbytes, st)
            if rc:
                raise xsum.TasxError(rc, "tasx_ab_stream_copy")

        def timed(src, dst):
            for _ in range(3):
                copy(src, dst)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(copies):
                copy(src, dst)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / copies
        us = timed(a.dev_addr, b.dev_addr)
        us_rd = timed(a.dev_addr, d.data_ptr())
        us_wr = timed(d.data_ptr(), b.dev_addr)
        del d
        return {"bytes_each_way": nbytes, "us": round(us, 1), "GBps_each_way": round(nbytes / us / 1e3, 1),
                "read_only_GBps": round(nbytes / us_rd / 1e3, 1), "write_only_GBps": round(nbytes / us_wr / 1e3, 1),
                "how": "stream_copy_kernel (libtasx_ab.so) between two pinned host buffers (and host -> HBM, "
                       "HBM -> host), HIP events around 20 copies"}
    finally:
        for pb in pins:
            pb.free()


def timed_host_batch(call, alg: int, reps: int, ws: int, *, pcie_h2d_bytes: int, what: str) -> dict:
    """One warm call, then `reps` timed calls of a host batch (each returns
    after its results are in host memory) between a barrier and the slowest
    rank's time."""
    call()
    barrier(ws)
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    t = time.perf_counter() - t0
    tm = max_over_ranks(t, ws)
    return {"value": sum_over_ranks(alg * reps, ws) / tm / GIB, "unit": "GiB/s (algorithmic)",
            "ms_per_batch": tm / reps * 1e3, "pcie_h2d_bytes_per_rank": pcie_h2d_bytes, "entry_point": what,
            "kernel": xsum.last_kernel()}


def e2e_mixed_leg(ws: int, rank: int, reps: int = 3) -> dict:
    """Config 3 from host memory: the 1M mixed-MTU packets (2.92 GB, this rank's
    byte-balanced shard at N > 1) at their packed offsets in pinned memory,
    through tasx_raw_cksum_batch_host_offs: staged (the CPU gathers each
    packet's bytes into pinned staging, H2D, raw_wave_kernel, D2H) and
    zero-copy (the kernel reads the packets in place over PCIe).  Both results
    are checked against the device-resident kernel on the same packets."""
    wl = mixed_workload(ws, rank)
    n = wl.n
    offs = wl.off.cpu().numpy().astype(np.uint64)
    lens = wl.lens.cpu().numpy().astype(np.uint32)
    total = int(wl.bufs[0].numel())
    alg = int(lens.astype(np.int64).sum()) + 2 * n
    pin = xsum.PinnedBuffer(total + 64)
    res = {"workload": f"config 3 from pinned host memory: {n} packets, {alg / 1e9:.2f} GB algorithmic"}
    try:
        xsum._check(xsum.lib().tasx_memcpy_d2h(pin.addr, wl.bufs[0].data_ptr(), total), "tasx_memcpy_d2h")
        ref = wl.loop()
        ref(0, 1)
        torch.cuda.synchronize()
        exp = wl.outs[0].cpu().numpy().view(np.uint16).copy()
        del wl, ref
        torch.cuda.empty_cache()
        out = np.empty(n, np.uint16)
        xsum.ctx_init(1, torch.cuda.current_device(), 64 << 20)
        try:
            res["staged"] = timed_host_batch(
                lambda: xsum.raw_cksum_batch_host_offs(1, pin.addr, offs, n, lengths=lens, out=out), alg, reps, ws,
                pcie_h2d_bytes=int(((lens.astype(np.int64) + 15) // 16 * 16).sum()) + 12 * n,
                what="tasx_raw_cksum_batch_host_offs (staged gather)")
            res["staged"]["matches_device"] = bool(np.array_equal(out, exp))
            out[:] = 0
            res["zero_copy"] = timed_host_batch(
                lambda: xsum.raw_cksum_batch_host_offs(1, pin.addr, offs, n, lengths=lens, out=out, zerocopy=True),
                alg, reps, ws, pcie_h2d_bytes=alg + 12 * n, what="tasx_raw_cksum_batch_host_offs (zero-copy)")
            res["zero_copy"]["matches_device"] = bool(np.array_equal(out, exp))
        finally:
            xsum.ctx_destroy(1)
    finally:
        pin.free()
    return res


def e2e_tso_leg(ws: int, rank: int, reps: int = 3) -> dict:
    """Config 5 from host memory: 16,384 TSO segments (ip.len 65535) in pinned
    memory at 65,552 B strides, through tasx_tcp4_cksum_batch_host_offs:
    staged (the CPU gathers header + L4 of each segment, H2D, one stride-mode
    launch per chunk, D2H) and zero-copy (frame lengths as hints, the kernel
    reads the segments in place).  Checked against the device-resident kernel."""
    wl = tso_workload(rank)
    n, stride = wl.n, wl.stride
    alg = n * (wl.ip_total + 4)
    pin = xsum.PinnedBuffer(n * stride + 64)
    res = {"workload": f"config 5 from pinned host memory: {n} TSO segments, {alg / 1e9:.2f} GB algorithmic"}
    try:
        xsum._check(xsum.lib().tasx_memcpy_d2h(pin.addr, wl.bufs[0].data_ptr(), n * stride), "tasx_memcpy_d2h")
        wl.loop(HINT)(0, 1)
        torch.cuda.synchronize()
        exp = wl.outs[0].cpu().numpy().view(np.uint16).copy()
        del wl
        torch.cuda.empty_cache()
        offs = np.arange(n, dtype=np.uint64) * np.uint64(stride)
        flen = np.full(n, pktgen.ETH_LEN + 65535, np.uint32)
        out = np.empty(2 * n, np.uint16)
        xsum.ctx_init(1, torch.cuda.current_device(), 64 << 20)
        try:
            res["staged"] = timed_host_batch(
                lambda: xsum.tcp4_cksum_batch_host_offs(1, pin.addr, offs, n, out=out), alg, reps, ws,
                pcie_h2d_bytes=n * 65552, what="tasx_tcp4_cksum_batch_host_offs (staged gather)")
            res["staged"]["matches_device"] = bool(np.array_equal(out, exp))
            out[:] = 0
            res["zero_copy"] = timed_host_batch(
                lambda: xsum.tcp4_cksum_batch_host_offs(1, pin.addr, offs, n, out=out, frame_len=flen, zerocopy=True),
                alg, reps, ws, pcie_h2d_bytes=n * 65536 + 12 * n, what="tasx_tcp4_cksum_batch_host_offs (zero-copy)")
            res["zero_copy"]["matches_device"] = bool(np.array_equal(out, exp))
        finally:
            xsum.ctx_destroy(1)
    finally:
        pin.free()
    return res


def fastpath_mt_leg(flushes: int = 3000) -> dict:
    """tx_flush at TAS's batch size from several fast-path threads
    (tas/fast/fastemu.c:544-566: at most TXBUF_SIZE = 32 frames per core per
    loop), issued from C (tasxb_fastpath_mt; INTEGRATION.md section 4b loop):
    each thread on its own context over a pinned mempool of 32-frame slots,
    half 1514-B data segments and half 66-B ACKs, with up to `in flight`
    batches out.  Per-context launches, the shared feeder and the persistent
    flush server at 1 thread x 1 in flight (latency), 8 x 3 and 8 x 7
    (throughput); then the fused TX segment build through the server
    (tasx_server_tx_segments: 32 segments of 1448 B per flush, payload gathered
    from pinned TX buffers), the same shapes.  The server's in-place fields of
    thread 0's last batches are compared with the device-resident batch kernel
    on the same frames."""
    dev = torch.cuda.current_device()
    res = {"unit": "frames/s, us", "frames_per_flush": 32,
           "note": "latency_us from the submit call's return, latency_from_submit_us from its start (a "
                   "per-context launch is paid inside the call); core_us_per_flush = record 32 frames + "
                   "submit + polls on the fast-path core; tools/feeder_bench.c adds 2 and 4 threads and the "
                   "CPU's own per-frame cost"}
    keep = None
    for mode in ("per_context", "feeder", "server"):
        for th, q in ((1, 1), (8, 3), (8, 7)):
            kp = np.zeros((q + 1) * 32 * STRIDE, np.uint8) if (mode == "server" and th == 8 and q == 7) else None
            r = benchloop.fastpath_mt(dev, 8, th, q, flushes, mode, kp)
            r["frames_per_s"] = round(r["frames_per_s"])
            res[f"{mode}_{th}x{q}"] = r
            if kp is not None:
                keep = kp
    # the fused TX segment build (payload copy + checksums) handed to the server
    for th, q in ((1, 1), (8, 3), (8, 7)):
        res[f"txseg_server_{th}x{q}"] = benchloop.txseg_server_mt(dev, 8, th, q, flushes)
    res["txseg_note"] = ("a 32-segment flush is ONE TX segment slot (41 segments a slot since round 5; round 4's "
                         "20-segment slots took two), so 7 in flight fit a ring's 8 slots and 8x7's "
                         "core_us_per_flush holds no wait for a free slot; segments_per_s over all threads")
    n = len(keep) // STRIDE
    dres = xsum.tcp4_cksum_batch(torch.from_numpy(keep.copy()).cuda(), n, stride=STRIDE)
    torch.cuda.synchronize()
    fv = keep.reshape(n, STRIDE)
    got = np.stack([fv[:, 24:26].copy().view(np.uint16)[:, 0], fv[:, 50:52].copy().view(np.uint16)[:, 0]], 1)
    res["server_matches_device"] = bool(np.array_equal(got.reshape(-1), dres.cpu().numpy().view(np.uint16)))
    return res


def server_cost_leg(rank: int, rot: int, flushes: int = 300000) -> dict:
    """What the resident flush server costs the device-resident work on the
    same GPU: the headline batch (2,000 launches) and the
    TX segment build (800) timed with the server stopped, started but idle (its
    32 workgroups of 1,024 threads resident, rings polled by their headers), and
    started with 8 fast-path threads flushing through it meanwhile (32-frame
    batches, 3 in flight each: tasxb_fastpath_mt in a second thread; the
    flush rate of that run, which also spans the parts without device work, is
    reported beside it; it is sized to outlast the timed launches, and
    busy_overlap_complete says whether it did).  Event-timed launches, each
    state's median of 3; "stopped" is measured before and after the other
    states and the lower taken (the first pass can still meet clocks ramping)."""
    import threading
    dev = torch.cuda.current_device()
    wl = Tcp4Workload(rot, pktgen.SEED + 7000 + rank, host=False)
    tw = TxSegWorkload(rot, pktgen.SEED + 7100 + rank)
    legs = {"headline": (wl.loop(HINT), wl.bytes_per_step, 2000), "tx_segment": (tw.loop(), tw.bytes_per_step, 800)}
    for run, _, _ in legs.values():
        prewarm(run)
    torch.cuda.synchronize()

    walls = []  # host seconds per timed() phase: warm launches, their wait, timed launches, their wait

    def timed(run, k):
        # stream-level waits only: a device-wide synchronize would wait for the
        # resident server kernel itself
        cur = torch.cuda.current_stream()
        w0 = time.perf_counter()
        run(0, 20)
        w1 = time.perf_counter()
        cur.synchronize()
        w2 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        run(20, k)
        w3 = time.perf_counter()
        e1.record(cur)
        e1.synchronize()
        w4 = time.perf_counter()
        walls.append([round(w1 - w0, 4), round(w2 - w1, 4), round(w3 - w2, 4), round(w4 - w3, 4)])
        return e0.elapsed_time(e1) * 1e3 / k

    def measure():
        return {name: float(np.median([timed(run, k) for _ in range(3)])) for name, (run, _, k) in legs.items()}
    res = {"unit": "us per launch", "states": {}}
    res["states"]["stopped"] = measure()
    xsum.server_start(dev)
    try:
        res["states"]["idle"] = measure()
    finally:
        xsum.server_stop(dev)

    def busy_pass(nflush):
        """the timed launches while a flush run of nflush flushes per thread
        goes through the server; (times, flush run, overlapped, seconds the
        run took to start flushing, seconds the timed launches took)"""
        flush, err = {}, []

        def body():
            try:
                flush.update(benchloop.fastpath_mt(dev, 8, 8, 3, nflush, "server"))
            except Exception as e:  # reported, and the pass counts as not overlapped
                err.append(repr(e))
        th = threading.Thread(target=body)
        th.start()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 10.0 and th.is_alive():  # started its server, its threads flushing
            try:
                if xsum.server_stats(dev)[0] > 2000:
                    break
            except xsum.TasxError:
                pass
            time.sleep(0.001)
        def batches():
            try:
                return xsum.server_stats(dev)[0]
            except xsum.TasxError:
                return None
        b1, t1 = batches(), time.perf_counter()
        walls.clear()
        times = measure()
        flush["host_walls_s"] = list(walls)
        b2, t2 = batches(), time.perf_counter()
        overlapped = th.is_alive() and b2 is not None  # the run outlasted the timed launches
        th.join()
        if err:
            flush["error"] = err[0]
        # the flush run's own rate while the timed launches ran
        flush["frames_per_s_meanwhile"] = round((b2 - b1) * 32 / (t2 - t1)) if b1 is not None and b2 else None
        return times, flush, overlapped and not err, round(t1 - t0, 3), round(t2 - t1, 3)
    busy, flush, overlapped, t_start, t_meas = busy_pass(flushes)
    if not overlapped:  # once more, with a run four times as long
        busy, flush, overlapped, t_start, t_meas = busy_pass(4 * flushes)
    batches_after = overlapped
    after = measure()
    res["states"]["stopped"] = {k: min(v, after[k]) for k, v in res["states"]["stopped"].items()}
    res["states"]["busy_8x3"] = busy
    res["busy_flush_run"] = flush
    res["busy_overlap_complete"] = bool(batches_after)
    res["busy_seconds"] = {"run_start": t_start, "timed_launches": t_meas}
    for name, (_, nbytes, _) in legs.items():
        st = {k: v[name] for k, v in res["states"].items()}
        res[name] = {"us": {k: round(v, 3) for k, v in st.items()},
                     "slowdown_idle": round(st["idle"] / st["stopped"], 4),
                     "slowdown_busy": round(st["busy_8x3"] / st["stopped"], 4),
                     "frac_busy": round(nbytes / st["busy_8x3"] / 1e3 / HBM_PEAK_GBS, 4)}
    del res["states"]
    return res


def server_cost_child_leg(rot: int) -> dict:
    """server_cost_leg in a fresh child process (bench.py --server-cost-child):
    run inside the full bench process after the two-context and flush-mix
    legs, the busy pass's first synchronize blocked until the flush run had
    ended (profiles/r05 r05q), so that process measured nothing busy; a fresh
    process measures the leg alone."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--server-cost-child", "--rotate", str(rot)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "server_cost child: no answer within 240 s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"server_cost child rc={r.returncode}: {r.stderr[-400:]}"}
    res = json.loads(lines[-1])
    res["process"] = "a child process of its own (bench.py --server-cost-child)"
    return res


def e2e_leg(ws: int, rank: int, reps: int = 5) -> dict:
    """Every rank at once, each from its own NUMA-local host thread (this
    process, pinned by numa_pin before these buffers were touched):
    * staged: host frames -> chunked pinned H2D of whole mbuf rooms -> kernel ->
      D2H of the results (tasx_tcp4_cksum_batch_host);
    * zero-copy: the kernel reads the frames from pinned host memory over PCIe
      (only the bytes it sums) and writes the results to device memory;
    * (rank 0) tx_flush at TAS's batch size (32 frames): deferred tcp_checksums()
      calls + tasx_flush, staged and zero-copy (frames in a registered region)."""
    n = N_FRAMES
    frames = pktgen.tcp4_frames(n, payload=IP_TOTAL - 52, stride=STRIDE, seed=41 + rank)
    pin = xsum.PinnedBuffer(frames.size)
    pin.array[:] = frames
    out = np.empty(2 * n, np.uint16)
    dout = torch.empty(2 * n, dtype=torch.int16, device="cuda")
    alg = n * (IP_TOTAL + 4)
    res = {}
    xsum.ctx_init(0, torch.cuda.current_device(), 32 << 20)
    try:
        xsum.tcp4_cksum_batch_host(0, pin.addr, STRIDE, n, out.ctypes.data)  # warm
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(reps):
            xsum.tcp4_cksum_batch_host(0, pin.addr, STRIDE, n, out.ctypes.data)
        t = time.perf_counter() - t0
        tm = max_over_ranks(t, ws)
        res["staged"] = {"value": sum_over_ranks(alg * reps, ws) / tm / GIB, "unit": "GiB/s",
                         "ms_per_batch": tm / reps * 1e3, "pcie_h2d_bytes_per_rank": n * STRIDE,
                         "pcie_d2h_bytes_per_rank": n * 4}
        xsum.tcp4_cksum_batch(pin.dev_addr, n, stride=STRIDE, out=dout, frame_len=FRAME_LEN)
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
        for _ in range(reps):
            xsum.tcp4_cksum_batch(pin.dev_addr, n, stride=STRIDE, out=dout, frame_len=FRAME_LEN)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        tm = max_over_ranks(t, ws)
        res["zero_copy"] = {"value": sum_over_ranks(alg * reps, ws) / tm / GIB, "unit": "GiB/s",
                            "ms_per_batch": tm / reps * 1e3,
                            "note": "frames stay in pinned host memory; results land in HBM"}
        if rank == 0:
            # tx_flush at TXBUF_SIZE = 32 frames (tas/include/fastpath.h:38)
            f32 = xsum.PinnedBuffer(32 * STRIDE)
            f32.array[:] = pktgen.tcp4_frames(32, payload=IP_TOTAL - 52, stride=STRIDE, seed=42)
            plain = pktgen.tcp4_frames(32, payload=IP_TOTAL - 52, stride=STRIDE, seed=42)

            def flush_lat(base):  # from C: the fast-path core's record + submit + wait
                return round(float(np.median(benchloop.flush_loop(0, base, STRIDE, 32, 400)[50:])), 3)
            res["flush32_staged_us"] = flush_lat(plain.ctypes.data)
            xsum.register_frames(0, f32.addr, f32.nbytes)
            res["flush32_zero_copy_us"] = flush_lat(f32.addr)
            # the same flushes through the persistent flush server (no launch per flush)
            xsum.server_start(torch.cuda.current_device())
            try:
                xsum.use_server(0)
                res["flush32_server_us"] = flush_lat(f32.addr)
                xsum.use_server(0, False)
            finally:
                xsum.server_stop(torch.cuda.current_device())
            # the server's in-place fields against the device-resident batch kernel on the same frames
            dres = xsum.tcp4_cksum_batch(torch.from_numpy(plain.copy()).cuda(), 32, stride=STRIDE)
            torch.cuda.synchronize()
            fv = f32.array.reshape(32, STRIDE)
            got = np.stack([fv[:, 24:26].copy().view(np.uint16)[:, 0], fv[:, 50:52].copy().view(np.uint16)[:, 0]], 1)
            res["flush32_server_matches_device"] = bool(np.array_equal(got.reshape(-1), dres.cpu().numpy().view(np.uint16)))
            res["flush32_note"] = ("32 x tasx_defer_tcp4 + tasx_flush_submit + tasx_flush_wait, issued from C "
                                   "(tasxb_flush_loop), median us per flush: staged, zero-copy per-context launches, "
                                   "and the persistent flush server; tools/feeder_bench.c has the multi-thread numbers")
            f32.free()
            try:  # a failure here must not cost the bench line its other numbers
                res["fastpath_mt"] = fastpath_mt_leg()
            except xsum.TasxError as e:
                res["fastpath_mt"] = {"error": str(e)}
                try:  # never leave a server running under the legs that follow (HIP frees wait for it)
                    xsum.server_stop(torch.cuda.current_device())
                except xsum.TasxError:
                    pass
        # the same frames as scattered mbufs: the CPU gathers only the summed
        # bytes (tasx_tcp4_cksum_batch_host_offs, staged)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(STRIDE)
        res["staged_gather"] = timed_host_batch(
            lambda: xsum.tcp4_cksum_batch_host_offs(0, pin.addr, offs, n, out=out), alg, reps, ws,
            pcie_h2d_bytes=n * 1536 + 12 * n, what="tasx_tcp4_cksum_batch_host_offs (staged gather)")
        res["tx_segment_host"] = txseg_host_leg(ws, rank, 20)
    finally:
        xsum.ctx_destroy(0)
        pin.free()
    res["mixed"] = e2e_mixed_leg(ws, rank)
    res["tso"] = e2e_tso_leg(ws, rank)
    res["value"] = res["staged"]["value"]
    res["unit"] = "GiB/s"
    res["host_threads"] = f"one per GPU ({ws}), each pinned to its GPU's NUMA node"
    return res


# ---------------------------------------------------------------------------
# CPU baseline (rank 0, N == 1)

def host_oracle():
    """The C oracle built with the reference's own flags (-O3 -march=native) for
    THIS host, in a temp dir the caller removes; the prebuilt one otherwise."""
    from oracle import oracle_lib
    tmp = Path(tempfile.mkdtemp(prefix="tasx_oracle_"))
    try:
        lib_path = oracle_lib.build(out_dir=tmp, march="native")
        kind_note = "-O3 -march=native (built on this host)"
    except Exception:
        lib_path = None
        kind_note = "-O3 -march=x86-64-v3 (prebuilt)"
    return oracle_lib.Oracle(lib_path), kind_note, tmp


def cpu_model() -> str:
    try:
        return [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:
        return "unknown"


# The box's CPU share for one GPU: worker pools stay within it (the machine's
# other cores serve the other GPUs' jobs; OMP_NUM_THREADS is 16 there)
CPU_SHARE = 16
CPU_SWEEP = (1, 2, 4, 8, 16)


def cpu_sweep(bench_fn, alg_bytes: int, budget_s: float) -> tuple[dict, dict]:
    """The oracle over the WHOLE batch at 1, 2, 4, 8 and 16 pinned threads (the
    ones this rank may use, up to the GPU's CPU share); bench_fn(threads, reps)
    returns the median seconds per pass.  Returns ({threads: GiB/s}, {threads:
    passes})."""
    allowed = len(os.sched_getaffinity(0))
    ths = [t for t in CPU_SWEEP if t <= min(CPU_SHARE, allowed)] or [1]
    rate, reps_used = {}, {}
    for t in ths:
        t1 = bench_fn(t, 1)
        reps = max(3, min(2000, int(budget_s / len(ths) / max(t1, 1e-6))))
        rate[t] = alg_bytes / bench_fn(t, reps) / GIB
        reps_used[t] = reps
    return rate, reps_used


def cpu_record(rate: dict, reps: dict, sample: str, kind_note: str, parity: bool) -> dict:
    top = max(rate)
    allowed = len(os.sched_getaffinity(0))
    return {
        "value": rate[top], "unit": "GiB/s", "cores": top, "kind": "port",
        "sample": f"{sample}; median of {reps[top]} passes on {top} pinned threads; {kind_note}; CPU {cpu_model()}",
        "single_core_value": rate[min(rate)],
        "thread_sweep": {str(t): round(v, 3) for t, v in rate.items()},
        "sweep_passes": {str(t): v for t, v in reps.items()},
        "host_cpus": os.cpu_count(), "cpus_this_rank": allowed, "cpu_model": cpu_model(),
        "cores_note": (f"measured at 1..{top} threads over the whole batch; {CPU_SHARE} is the box's CPU share for "
                       f"one GPU (worker pools stay within it: the host's other {(os.cpu_count() or 0) - CPU_SHARE} "
                       "CPUs serve the other GPUs' jobs), so no run uses more"),
        "parity_vs_gpu": "bit-exact" if parity else "MISMATCH",
    }


def cpu_baseline_leg(wl: Tcp4Workload, gpu_out: np.ndarray, budget_s: float) -> dict:
    """The oracle (C restatement of the reference path, per-frame calls) timed on
    this box's host cores over the whole headline batch, at 1..16 threads
    (threads pinned to the cores this rank may use)."""
    orc, kind_note, tmp = host_oracle()
    frames = wl.host.copy()
    n = wl.n
    exp = orc.tcp4_batch(frames.copy(), n, stride=STRIDE)
    parity = bool(np.array_equal(exp, gpu_out))
    alg = n * (IP_TOTAL + 4)
    rate, reps = cpu_sweep(lambda t, r: orc.bench(1, frames, n, stride=STRIDE, threads=t, reps=r), alg, budget_s)
    shutil.rmtree(tmp, ignore_errors=True)
    return cpu_record(rate, reps, "the whole 64K-frame TCP4 batch (98.6 MB algorithmic), per-frame "
                      "oracle_tcp_checksums (DPDK 19.11 restatement)", kind_note, parity)


def pmc_leg(mode: str, kernel_name: str, launches: int) -> dict | None:
    """HBM bytes per launch from rocprofv3 PMC counters, one counter per pass
    (MI355X_MICROARCH.md HBM: FETCH_SIZE reads 1/2 of a wide streaming read on
    gfx950 -> x2; WRITE_SIZE exact for wide stores; both in KiB)."""
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(rocprof).exists():
        return None
    res = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        outdir = Path(tempfile.mkdtemp(prefix=f"pmc_{ctr}_"))
        cmd = [rocprof, "--pmc", ctr, "--output-format", "csv", "-d", str(outdir), "-o", "run", "--",
               sys.executable, str(ROOT / "bench.py"), "--pmc-child", mode, "--steps", str(launches)]
        env = dict(os.environ)
        for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
            env.pop(k, None)
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        if r.returncode != 0:
            return {"error": f"rocprofv3 {ctr} rc={r.returncode}: {r.stderr[-400:]}"}
        vals = []
        for csvf in outdir.rglob("*counter_collection.csv"):
            with open(csvf) as fh:
                for row in csv.DictReader(fh):
                    if kernel_name in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                        vals.append(float(row["Counter_Value"]))
        shutil.rmtree(outdir, ignore_errors=True)
        if not vals:
            return {"error": f"no {ctr} rows for {kernel_name}"}
        res[ctr] = float(np.median(vals))
    fetch = res["FETCH_SIZE"] * 1024 * 2
    write = res["WRITE_SIZE"] * 1024
    return {"FETCH_SIZE_kib": res["FETCH_SIZE"], "WRITE_SIZE_kib": res["WRITE_SIZE"],
            "hbm_bytes_per_launch": fetch + write,
            "method": "median over launches; FETCH_SIZE x 2 (gfx950 wide-read correction) + WRITE_SIZE, KiB x 1024"}


def pmc_child(mode: str, steps: int):
    torch.cuda.set_device(0)
    xsum.lib()
    if mode == "tcp4":
        run = Tcp4Workload(16, pktgen.SEED).loop(HINT)
    elif mode == "raw":
        run = RawWorkload(16, pktgen.SEED).loop()
    elif mode == "txseg":
        run = TxSegWorkload(16, pktgen.SEED + 2000).loop()
    elif mode == "rx":
        run = RxPassWorkload(FlowLookupWorkload(1, pktgen.SEED + 3000), 12, pktgen.SEED + 4000).loop()
    elif mode == "flushmix":
        run = FlushMixWorkload(12, pktgen.SEED + 500).loop()
    elif mode == "tso":
        run = tso_workload(0).loop(HINT)
    elif mode == "shard8m":
        run = shard8m_workload(1, 0).loop()
    elif mode == "readceil":
        # the headline's read ceiling (read_ceiling): a streaming read of the
        # headline's algorithmic bytes over the same 16 buffers, by the
        # tasx_ab_stream_read path TASX_READ_PATH (default 0: grid order) --
        # the counter comparison of tools/pmc_read_compare.sh
        wl = Tcp4Workload(16, pktgen.SEED)
        ab = xsum._load(xsum.AB_LIB_PATH)
        path = int(os.environ.get("TASX_READ_PATH", "0"))
        nbytes = wl.bytes_per_step // 1024 * 1024
        sink = torch.zeros(1, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def run(_, k):
            for j in range(k):
                rc = ab.tasx_ab_stream_read(wl.bufs[j % 16].data_ptr(), nbytes, path, sink.data_ptr(), st)
                if rc:
                    raise xsum.TasxError(rc, "tasx_ab_stream_read")
    else:
        run = mixed_workload().loop()
    run(0, steps)
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------
# other BASELINE.json configs (--workload)

MIXED_N = 1 << 20


def mixed_workload(ws: int = 1, rank: int = 0) -> RawWorkload:
    """Config 3: 1,048,576 RAW packets, sizes uniform over {64,576,1500,9000} B in
    random order, packed at 16-byte aligned offsets.  Over N ranks the one batch
    is split into contiguous byte-balanced shards (tas_amd/shard.py); rank r
    holds its shard's packets (random bytes of its own)."""
    lens_all = pktgen.mixed_lengths(MIXED_N, seed=pktgen.SEED).astype(np.int64)
    a, b = shard.shard_ranges(lens_all, ws)[rank]
    lens = lens_all[a:b]
    slot = (lens + 15) // 16 * 16
    offs = np.zeros(len(lens), np.int64)
    np.cumsum(slot[:-1], out=offs[1:])
    wl = RawWorkload(1, pktgen.SEED + rank, n=len(lens), offsets=offs, lengths=lens,
                     total_bytes=int(offs[-1] + slot[-1]))
    wl.shard = (a, b)
    return wl


SHARD8M_N = 8 * (1 << 20)


def shard8m_workload(ws: int, rank: int) -> RawWorkload:
    """Config 4: 8,388,608 x 1500 B split over the ranks (1,048,576 per GPU at 8)."""
    a, b = shard.shard_ranges(SHARD8M_N, ws)[rank]
    wl = RawWorkload(1, pktgen.SEED + rank, n=b - a, length=RAW_LEN)
    wl.shard = (a, b)
    return wl


def tso_workload(rank: int) -> Tcp4Workload:
    """Config 5: 16,384 TSO segments per GPU (ip.len 65535, L4 65,515 B) in
    65,552 B rooms, the frame length as the uniform hint."""
    return Tcp4Workload(2, pktgen.SEED + rank, n=16384, stride=65552, ip_total=65535, host=False)


def other_workload(args, ws, rank, info):
    name = args.workload
    if name == "shard8m":
        wl = shard8m_workload(ws, rank)
        run, kernel = wl.loop(), "raw_sad_kernel<s32>"
        desc = f"8,388,608 x 1500 B payloads sharded over {ws} GPU(s): {wl.n} packets on this rank"
        scaling = "strong"
    elif name == "mixed":
        wl = mixed_workload(ws, rank)
        run, kernel = wl.loop(), "raw_wave_kernel"
        desc = (f"1,048,576 RAW packets, sizes uniform over {{64,576,1500,9000}} B in random order, split by bytes "
                f"over {ws} GPU(s): {wl.n} packets on this rank")
        scaling = "strong"
    else:  # tso
        wl = tso_workload(rank)
        run, kernel = wl.loop(HINT), "tcp4_tas_kernel"
        desc = "16,384 TSO segments per GPU (ip.len 65535, L4 65,515 B), tcp_checksums() flag-off, hinted"
        scaling = "weak"
    r = leg(run, wl.bytes_per_step, args, ws, desc, kernel)
    # the leg's own live read ceiling (configs 3-5 carry one too)
    if rank == 0 and not info.get("rehearse"):
        torch.cuda.synchronize()
        r["roofline"]["read_ceiling"] = read_ceiling(wl, r["roofline"]["launch_avg_us"])
    # per-rank accounting: packets, algorithmic bytes, seconds for the K steps
    shards = {"packets": [int(v) for v in gather_over_ranks(float(wl.n), ws)],
              "bytes_per_step": [int(v) for v in gather_over_ranks(float(wl.bytes_per_step), ws)],
              "first_packet": [int(v) for v in gather_over_ranks(float(getattr(wl, "shard", (0, 0))[0]), ws)],
              "seconds": gather_over_ranks(r["seconds"], ws)}
    rehearse = bool(info.get("rehearse"))
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        torch.cuda.synchronize()
        cpu = other_cpu_baseline(name, wl, args.cpu_seconds / 2)
    pmc = None
    if rank == 0 and ws == 1 and not args.no_pmc:
        # rocprofv3's kernel names (the template, not tasx_last_kernel's label)
        pmc = pmc_leg(name, {"mixed": "raw_wave_kernel", "shard8m": "raw_sad_kernel", "tso": "tcp4_tas_kernel<"}[name],
                      4 if name == "shard8m" else 8)
        if pmc and "hbm_bytes_per_launch" in pmc:
            r["roofline"]["traffic"] = int(pmc["hbm_bytes_per_launch"])
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(r["value"], 2), "unit": "GiB/s", "n_gpus": ws,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
                          "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
                          "data": "synthetic (device-generated random bytes)",
                          "config": {"workload": desc, "parallelism": f"shard{ws}"},
                          "roofline": r["roofline"], "kernel": kernel,
                          # ranks sharing one GPU (--rehearse) make no HBM-fraction claim
                          "frac_of_n_hbm": None if rehearse else round(r["value"] * GIB / 1e9 / (ws * HBM_PEAK_GBS), 4),
                          **({"per_rank_value": r["per_rank_value"]} if "per_rank_value" in r else {}),
                          "shards": shards,
                          "ranks": {"bus_ids": info.get("all_bus_ids", [info.get("pci_bus_id")]), "rehearse": rehearse},
                          "cpu_baseline": cpu, **({"pmc": pmc} if pmc else {})}), flush=True)


def other_cpu_baseline(name: str, wl, budget_s: float) -> dict:
    """The oracle over the WHOLE batch of the other configs (BASELINE.md's CPU
    plan: the same generator, per-packet calls), at 1..16 threads, checked
    against the GPU's results for the same packets."""
    orc, kind_note, tmp = host_oracle()
    m = wl.n
    if name == "tso":
        stride = wl.stride
        host = wl.bufs[0].cpu().numpy().copy()
        gpu = wl.outs[0][:2 * m].cpu().numpy().view(np.uint16)
        parity = np.array_equal(orc.tcp4_batch(host.copy(), m, stride=stride), gpu)
        kw = dict(stride=stride)
        mode, alg = 1, m * (wl.ip_total + 4)
        sample = f"all {m} TSO segments (ip.len {wl.ip_total}), per-segment oracle_tcp_checksums"
    else:
        gpu = wl.outs[0][:m].cpu().numpy().view(np.uint16)
        host = wl.bufs[0].cpu().numpy()
        if wl.off is None:
            kw = dict(stride=wl.len0, len0=wl.len0)
            alg = m * (wl.len0 + 2)
        else:
            kw = dict(offsets=wl.off.cpu().numpy().astype(np.uint64), lengths=wl.lens.cpu().numpy().astype(np.uint32))
            alg = int(kw["lengths"].astype(np.int64).sum()) + 2 * m
        parity = np.array_equal(orc.raw_batch(host, m, **kw), gpu)
        mode = 0
        sample = f"all {m} packets of this rank's batch, per-packet oracle_raw_cksum (rte_raw_cksum restatement)"
    rate, reps = cpu_sweep(lambda t, r: orc.bench(mode, host, m, threads=t, reps=r, **kw), alg, budget_s)
    shutil.rmtree(tmp, ignore_errors=True)
    return cpu_record(rate, reps, f"{sample} ({alg / 1e6:.1f} MB algorithmic)", kind_note, parity)


# ---------------------------------------------------------------------------

def control_selftest(ws: int, rank: int, info: dict) -> None:
    """--control-selftest: the rank plumbing without a GPU (gloo): barrier,
    MAX / SUM / gather over ranks; rank 0 prints what a run would aggregate."""
    barrier(ws)
    per = gather_over_ranks(float(rank + 1), ws)
    tot = sum_over_ranks(float(rank + 1), ws)
    mx = max_over_ranks(float(rank + 1), ws)
    barrier(ws)
    if rank == 0:
        print(json.dumps({"n_gpus": ws, "per_rank_value": per, "sum": tot, "max": mx,
                          "ranks": info.get("all_bus_ids")}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.server_cost_child:
        torch.cuda.set_device(0)
        xsum.lib()
        print(json.dumps(server_cost_leg(0, args.rotate)), flush=True)
        return 0
    if args.pmc_child:
        pmc_child(args.pmc_child, args.steps)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, argv)
    ws, rank, local, info = dist_setup(args)
    try:
        if args.control_selftest:
            control_selftest(ws, rank, info)
            return 0
        xsum.lib()
        if args.workload != "tcp4":
            other_workload(args, ws, rank, info)
        else:
            run_tcp4(args, ws, rank, info)
        return 0
    finally:
        if ws > 1:
            dist.destroy_process_group()


def rx_pass_leg(fw: FlowLookupWorkload, rot: int, args, ws: int, rank: int) -> dict:
    """The fused RX pass against the two calls it replaces, timed the same way
    on the same frames and outputs (tests/test_rx_fused.py checks both)."""
    rp = RxPassWorkload(fw, min(rot, 12), pktgen.SEED + 4000 + rank)
    r = leg(rp.loop(benchloop.RX_FUSED), rp.bytes_per_step, args, ws, RxPassWorkload.desc,
            "tcp4_tas14_kernel<hints,verify,flow>")
    sep = leg(rp.loop(benchloop.RX_SEPARATE), rp.bytes_per_step, args, ws,
              "same frames: tasx_tcp4_verify_batch_dev_room, then tasx_flow_lookup_batch_dev")
    # verification alone on the same frames: the floor any pass that also looks up can reach
    vloop = benchloop.Loop("tcp4", [a.v for a in rp.loop(benchloop.RX_FUSED).arr], _stream_ptrs(None), VERIFY,
                           "tasx_tcp4_verify_batch_dev_room")
    # the median of three runs: a single run of this short leg has read 16 % high on one box (round_b)
    v_runs = sorted(timed_run(vloop, args.steps, args.warmup, ws)[1] for _ in range(3))
    v_ms = v_runs[1]
    torch.cuda.synchronize()
    r["verify_only_us"] = round(v_ms * 1e3, 3)
    r["verify_only_runs_us"] = [round(x * 1e3, 3) for x in v_runs]
    r["lookup_cost_us"] = round(r["roofline"]["launch_avg_us"] - v_ms * 1e3, 3)
    r["separate"] = {"ms_per_step": sep["ms_per_step"], "launch_pair_avg_us": sep["roofline"]["launch_avg_us"],
                     "kernels": "tcp4_tas14_kernel<hints,verify> + flow_lookup_kernel"}
    r["speedup_vs_separate"] = round(sep["roofline"]["launch_avg_us"] / r["roofline"]["launch_avg_us"], 3)
    r["all_frames_verified"] = bool(all((f == 3).all().item() for f in rp.flags))
    r["found_frac"] = round(float((rp.fids[0] != -1).float().mean().item()), 4)
    r["parity"] = "tests/test_rx_fused.py::test_rx_fused_forms[hints]"
    del rp
    torch.cuda.empty_cache()
    return r


def config4_leg(args, ws: int, rank: int, info: dict) -> dict:
    """BASELINE config 4 inside the default line: the
    8,388,608 x 1500 B batch split over the ranks -- all of it on one GPU at
    N = 1 (12.6 GB a step), 1,048,576 packets per GPU at N = 8 -- through the
    same raw_sad_kernel<s32> call as `--workload shard8m`, with its live read
    ceiling and (N = 1) its PMC traffic.  Parity: the whole batch on one GPU
    through this call, tests/test_bench_configs.py::test_bench_config4_whole_on_one_gpu."""
    wl = shard8m_workload(ws, rank)
    r = leg(wl.loop(), wl.bytes_per_step, args, ws,
            f"BASELINE config 4: 8,388,608 x 1500 B payloads split over {ws} GPU(s), {wl.n} packets on this "
            "rank, rte_raw_cksum per packet, one launch a step", "raw_sad_kernel<s32>")
    rehearse = bool(info.get("rehearse"))
    r["packets_per_rank"] = [int(v) for v in gather_over_ranks(float(wl.n), ws)]
    r["frac_of_n_hbm"] = None if rehearse else round(r["value"] * GIB / 1e9 / (ws * HBM_PEAK_GBS), 4)
    r["parity"] = "tests/test_bench_configs.py::test_bench_config4_whole_on_one_gpu"
    if rank == 0 and not rehearse:
        torch.cuda.synchronize()
        r["roofline"]["read_ceiling"] = read_ceiling(wl, r["roofline"]["launch_avg_us"], launches=40)
    del wl
    torch.cuda.empty_cache()
    if rank == 0 and ws == 1 and not args.no_pmc:
        p = pmc_leg("shard8m", "raw_sad_kernel", 4)
        if p and "hbm_bytes_per_launch" in p:
            r["roofline"]["traffic"] = int(p["hbm_bytes_per_launch"])
        r["pmc"] = p
    return r


def run_tcp4(args, ws: int, rank: int, info: dict) -> None:
    rot = max(1, args.rotate)
    wl = Tcp4Workload(rot, pktgen.SEED + rank)
    head = leg(wl.loop(HINT), wl.bytes_per_step, args, ws, Tcp4Workload.desc, "tcp4_tas14_kernel<hint>")
    rehearse = bool(info.get("rehearse"))
    if rehearse:  # ranks share the GPU: another rank's launches overlap this one's
        head["roofline"]["pattern_ceiling"] = None
        head["roofline"]["read_ceiling"] = None
    else:
        head["roofline"]["pattern_ceiling"] = tcp4_pattern_ceiling(wl, head["roofline"]["launch_avg_us"])
        head["roofline"]["read_ceiling"] = read_ceiling(wl, head["roofline"]["launch_avg_us"])
    ctx2 = None
    if not args.no_contexts:
        streams = [torch.cuda.Stream() for _ in range(2)]
        # its own step count: the cross-stream event waits around the timed
        # launches cost ~40 us per run, which K = 20 cannot amortise (the
        # interval reads 17.2 us at K = 20 against 15.3 at K = 200, round_c)
        k2 = max(args.steps, CTX2_MIN_STEPS)
        dt2, avg2 = timed_run(wl.loop(HINT, streams=streams), k2, args.warmup, ws, streams)
        dt2 = max_over_ranks(dt2, ws)
        total = sum_over_ranks(float(wl.bytes_per_step * k2), ws)
        ctx2 = {"value": total / dt2 / GIB, "unit": "GiB/s", "ms_per_step": dt2 / k2 * 1e3, "steps": k2,
                "workload": "the headline batches alternating over 2 streams (two fast-path contexts, "
                            "independent batches): one batch's ramp-up overlaps the other's drain",
                "batch_interval_us": round(avg2 * 1e3, 3),
                "alg_GBps_per_interval": round(wl.bytes_per_step / (avg2 * 1e-3) / 1e9, 1),
                "note": "kernels overlap, so a kernel's own duration is longer than the interval; "
                        "the headline roofline uses the single-stream launch"}
    # the drop-in forms: no hint with the mbuf data room (what TAS would pass),
    # and frames only
    nohint = leg(wl.loop(ROOM, flen0=0, room=STRIDE), wl.bytes_per_step, args, ws,
                 "same frames, tasx_tcp4_cksum_batch_dev_room (no hint, room = the 2048 B mbuf data room)",
                 "tcp4_tas14_kernel<room>")
    frames_only = leg(wl.loop(DEV, flen0=0), wl.bytes_per_step, args, ws,
                      "same frames, tasx_tcp4_cksum_batch_dev (frames only: no hint, no room)",
                      "tcp4_tas14_kernel<tl_first>")
    # receive-side verification of the same frames (after in-place TX checksums)
    xsum.tcp4_cksum_batch(wl.bufs[0], wl.n, stride=wl.stride, inplace=True, want_out=False)
    for b in wl.bufs[1:]:
        b.copy_(wl.bufs[0])
    rv = RxVerifyWorkload(wl)
    rx = leg(rv.loop(), rv.bytes_per_step, args, ws,
             "same frames after TX checksums, tasx_tcp4_verify_batch_dev_room (received frame length as the "
             "uniform hint)", "tcp4_tas14_kernel<hint,verify>")
    torch.cuda.synchronize()
    rx["all_frames_verified"] = bool((wl.rx_flags[0] == 3).all().item())
    src = torch.from_numpy(wl.host).cuda()
    for b in wl.bufs:  # restore the un-checksummed frames for the legs below
        b.copy_(src)
    del src
    mix = rx_mix = None
    if not args.no_flushmix:
        mw = FlushMixWorkload(min(rot, 12), pktgen.SEED + 500 + rank)
        mix = leg(mw.loop(), mw.bytes_per_step, args, ws, FlushMixWorkload.desc, "tcp4_tas14_kernel<hints>")
        mix["parity"] = "tests/test_bench_configs.py::test_bench_flush_mix"
        mb = None if rehearse else mix_bounds(mw)  # before the RX form checksums the frames in place
        if mb is not None:
            price_mix(mix, mb, mw.bytes_per_step)
        rm = RxMixWorkload(mw)
        rx_mix = leg(rm.loop(), rm.bytes_per_step, args, ws, RxMixWorkload.desc, "tcp4_tas14_kernel<hints,verify>")
        torch.cuda.synchronize()
        rx_mix["all_frames_verified"] = bool(all((f == 3).all().item() for f in rm.flags))
        rx_mix["parity"] = "tests/test_bench_configs.py::test_bench_rx_mix"
        if mb is not None:  # the same frames and rows: the same chain and pattern
            price_mix(rx_mix, mb, rm.bytes_per_step)
        del mw, rm
        torch.cuda.empty_cache()
    raw = None
    if not args.no_raw:
        rw = RawWorkload(rot, pktgen.SEED + 1000 + rank)
        raw = leg(rw.loop(), rw.bytes_per_step, args, ws, RawWorkload.desc, "raw_sad_kernel<s32>")
        raw["algorithmic_bytes_per_packet"] = RAW_LEN + 2
        del rw
        torch.cuda.empty_cache()

    txseg = None
    if not args.no_txseg:
        del wl.bufs[1:], wl.outs[1:]
        torch.cuda.empty_cache()
        tw = TxSegWorkload(rot, pktgen.SEED + 2000 + rank)
        txseg = leg(tw.loop(), tw.bytes_per_step, args, ws, TxSegWorkload.desc, "tx_segment_lds_kernel")
        txseg["algorithmic_bytes_per_segment"] = tw.bytes_per_seg
        txseg["block_floor"] = dict(tw.block_floor)
        # bytes each way of the 128-byte block floor (the kernel's reads and writes)
        cc = copy_ceiling(int(tw.block_floor["bytes"]) // 2)
        cc["alg_frac_of_copy"] = round(txseg["roofline"]["achieved"] / cc["GBps"], 4)
        txseg["copy_ceiling"] = cc
        if rank == 0 and ws == 1 and not args.no_cpu_baseline:
            txseg["cpu_baseline"] = tw.cpu_check(3.0)
        if not rehearse:  # last: it overwrites the leg's frames
            txseg["pattern_ceiling"] = txseg_pattern_ceiling(tw, txseg["roofline"]["launch_avg_us"])
        del tw
        torch.cuda.empty_cache()

    flow = rx_pass = None
    if not args.no_flow:
        fw = FlowLookupWorkload(min(rot, 4), pktgen.SEED + 3000 + rank)
        flow = leg(fw.loop(), fw.bytes_per_step, args, ws, FlowLookupWorkload.desc, "flow_lookup_kernel")
        flow["mpps"] = fw.N / (flow["roofline"]["launch_avg_us"] * 1e-6) / 1e6
        flow["flows_inserted_frac"] = fw.inserted
        flow["bytes_per_frame"] = 64
        flow.update(flow_bounds(fw, flow["roofline"]["launch_avg_us"]))
        # the leg's bound is its dependent access chain, not HBM bandwidth
        # (DESIGN.md section 5.4): priced in lookups per second against the
        # same chain with no hashing or compares, measured live; the HBM view
        # stays beside it
        pc, hbm = flow["pattern_ceiling"], flow["roofline"]
        flow["roofline"] = {"bound": "dependent access chain", "achieved": round(flow["mpps"] / 1e3, 3),
                            "peak": round(fw.N / pc["us"] / 1e3, 3), "unit": "G lookups/s", "frac": pc["frac"],
                            "traffic": None, "launch_avg_us": hbm["launch_avg_us"],
                            "algorithmic_bytes_per_launch": hbm["algorithmic_bytes_per_launch"], "hbm": hbm}
        if rank == 0 and ws == 1 and not args.no_cpu_baseline:
            flow["cpu_baseline"] = fw.cpu_check(3.0)
        rx_pass = rx_pass_leg(fw, rot, args, ws, rank)
        del fw
        torch.cuda.empty_cache()

    config4 = None
    if not args.no_config4:
        config4 = config4_leg(args, ws, rank, info)

    extra = {}
    if not args.no_server_cost and rank == 0 and ws == 1:
        extra["server_cost"] = server_cost_child_leg(rot)
        torch.cuda.empty_cache()
    if not args.no_e2e:
        extra["e2e"] = e2e_leg(ws, rank)
    if rank == 0 and ws == 1:
        torch.cuda.synchronize()
        gpu_out = wl.outs[0].cpu().numpy().view(np.uint16).copy()
        if not args.no_cpu_baseline:
            extra["cpu_baseline"] = cpu_baseline_leg(wl, gpu_out, args.cpu_seconds)
        if not args.no_pmc:
            del wl
            torch.cuda.empty_cache()
            p = pmc_leg("tcp4", "tcp4", 64)
            extra["pmc"] = p
            if p and "hbm_bytes_per_launch" in p:
                head["roofline"]["traffic"] = int(p["hbm_bytes_per_launch"])
            if raw is not None:
                pr = pmc_leg("raw", "_raw_", 64)
                if pr and "hbm_bytes_per_launch" in pr:
                    raw["roofline"]["traffic"] = int(pr["hbm_bytes_per_launch"])
                raw["pmc"] = pr
            if txseg is not None:
                pt = pmc_leg("txseg", "tx_segment", 32)
                if pt and "hbm_bytes_per_launch" in pt:
                    txseg["roofline"]["traffic"] = int(pt["hbm_bytes_per_launch"])
                    fl = txseg.get("block_floor")
                    if fl:
                        fl["traffic_over_floor"] = round(pt["hbm_bytes_per_launch"] / fl["bytes"], 4)
                    cc = txseg.get("copy_ceiling")
                    if cc:  # the kernel's own HBM traffic rate against the copy's
                        rate = pt["hbm_bytes_per_launch"] / txseg["roofline"]["launch_avg_us"] / 1e3
                        cc["traffic_GBps"] = round(rate, 1)
                        cc["traffic_frac_of_copy"] = round(rate / cc["GBps"], 4)
                txseg["pmc"] = pt
            if mix is not None:  # tcp4_tas14_kernel<hints>: MODE kHintArr = 5, TX, 8 waves per SIMD, stride mode
                pm = pmc_leg("flushmix", "<6, 5, false, 8, false, 0>", 48)
                if pm and "hbm_bytes_per_launch" in pm:
                    mix["roofline"]["traffic"] = int(pm["hbm_bytes_per_launch"])
                mix["pmc"] = pm
            if rx_pass is not None:  # the one-pass RX kernel (per-frame lengths: tcp4_tas14_kernel<..., kFlowSplitX = 5>)
                prx = pmc_leg("rx", "<6, 5, true, 8, false, 5>", 48)
                if prx and "hbm_bytes_per_launch" in prx:
                    rx_pass["roofline"]["traffic"] = int(prx["hbm_bytes_per_launch"])
                rx_pass["pmc"] = prx

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(head["value"], 2), "unit": "GiB/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64-seeded frames, tas_amd/pktgen.py)",
            "config": {"workload": Tcp4Workload.desc, "frames_per_gpu_step": N_FRAMES,
                       "algorithmic_bytes_per_frame": IP_TOTAL + 4, "rotation_batches": rot,
                       "parallelism": f"shard{ws} (independent per-GPU batches, no collective)"},
            "roofline": head["roofline"],
            "kernel": head["kernel"],
            "frac_of_n_hbm": None if rehearse else round(head["value"] * GIB / 1e9 / (ws * HBM_PEAK_GBS), 4),
            "per_rank_value": head.get("per_rank_value", [round(head["value"], 2)]),
            "ranks": {"bus_ids": info.get("all_bus_ids", [info.get("pci_bus_id")]),
                      "numa_node_rank0": info.get("numa_node"), "rehearse": info.get("rehearse"),
                      "host_wait": info.get("host_wait")},
            "cpu_baseline": extra.get("cpu_baseline"),
            "tcp4_nohint": nohint,
            "tcp4_frames_only": frames_only,
            "two_contexts": ctx2,
            "rx_verify": rx,
            "rx_verify_mix": rx_mix,
            "flush_mix": mix,
        }
        if raw is not None:
            line["raw"] = raw
        if txseg is not None:
            line["tx_segment"] = txseg
        if flow is not None:
            line["flow_lookup"] = flow
        if rx_pass is not None:
            line["rx_pass"] = rx_pass
        if config4 is not None:
            line["config4"] = config4
        if "server_cost" in extra:
            line["server_cost"] = extra["server_cost"]
        if "e2e" in extra:
            line["e2e"] = extra["e2e"]
        if "pmc" in extra:
            line["pmc"] = extra["pmc"]
        if rehearse:
            line = drop_rehearsal_fractions(line)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.exit(main())
