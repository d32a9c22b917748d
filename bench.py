"""Benchmark: TAS software TCP/IP checksum path on MI355X (BASELINE.json metric
"TCP/IP checksum GiB/s (device-resident), 1500B MTU batch, 1/2/4/8 GPU").

Headline step = one launch of the TCP4 checksum kernel (tcp_checksums()
flag-off branch: rte_ipv4_cksum + rte_ipv4_udptcp_cksum per frame) over one
batch of 65,536 TAS TX data segments (1514 B frames, ip.len 1500, one per
2048 B mbuf data room: BASELINE.json configs[1] / BASELINE.md), with the frame
length (the mbuf data_len tx_send() sets before tx_flush) as the prefetch hint.
Inputs are resident in HBM before the timed region; steps rotate over R
distinct batches (R x 134 MB >> the 256 MiB Infinity Cache) so every step
reads HBM, not the MALL.

Algorithmic bytes per frame = ip.total_length (1500, the bytes summed) + 4
(results written) -- SURVEY.md section 8d.  value = GiB/s = bytes / s / 2^30.

Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
One process per GPU, each with its own batches and stream (weak scaling, no
data-path collective: the path shards); the timed region is
barrier + synchronize on both sides and the MAX over ranks is taken.  Rank 0
prints one JSON line.

Extra legs (rank 0, N == 1): the same frames without the hint, the same
batches over two streams (two fast-path contexts), RX verification, the RAW
payload fold (rte_raw_cksum over 64K x 1500 B), the TX segment build, the flow
lookup, the end-to-end host-memory rate through pinned memory, the CPU oracle
baseline, and HBM traffic from rocprofv3 counters (two short child runs;
--no-pmc skips them).  --workload {shard8m,mixed,tso} measures the other
BASELINE.json configs instead (one JSON line each, with the oracle timed on a
bounded sample of the same packets at N == 1).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
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

from tas_amd import pktgen, shard, xsum  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)
METRIC = "TCP/IP checksum GiB/s (device-resident), 1500B MTU batch, 1/2/4/8 GPU"

N_FRAMES = 65536
STRIDE = pktgen.MBUF_ROOM              # 2048
IP_TOTAL = 1500
FRAME_LEN = pktgen.ETH_LEN + IP_TOTAL  # 1514, the mbuf data_len tx_send() sets
RAW_LEN = 1500


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=16, help="distinct device batches cycled through")
    ap.add_argument("--workload", default="tcp4", choices=["tcp4", "shard8m", "mixed", "tso"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-raw", action="store_true")
    ap.add_argument("--no-txseg", action="store_true")
    ap.add_argument("--no-flow", action="store_true")
    ap.add_argument("--no-flushmix", action="store_true")
    ap.add_argument("--no-contexts", action="store_true", help="skip the two-context (two-stream) leg")
    ap.add_argument("--pmc", action="store_true", help=argparse.SUPPRESS)  # default now; kept for old command lines
    ap.add_argument("--no-pmc", action="store_true", help="skip the HBM-traffic rocprofv3 child runs")
    ap.add_argument("--pmc-child", choices=["tcp4", "raw", "txseg", "mixed"], help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# distributed plumbing (one process per GPU; control only, never data)

def dist_setup():
    """One process per GPU.  The process group carries only the barrier and two
    scalar reductions (RCCL as "nccl"; TASX_DIST_BACKEND=gloo runs the same
    control plane on the CPU, e.g. to rehearse N ranks on a one-GPU box)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        backend = os.environ.get("TASX_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return ws, rank, local


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


# ---------------------------------------------------------------------------
# workloads: device-resident batches + a zero-overhead launcher

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
            "tcp_checksums() flag-off per frame, frame length (mbuf data_len) as the prefetch hint")

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

    def launcher(self, streams=None):
        """streams: launch batch k on streams[k % S] (independent batches of S
        fast-path contexts, each with its own stream); default: the current stream."""
        fn = xsum.lib().tasx_tcp4_cksum_batch_dev_hint
        ss = [s.cuda_stream for s in streams] if streams else [torch.cuda.current_stream().cuda_stream]
        S = len(ss)
        args = [(b.data_ptr(), None, self.stride, None, self.hint, self.n, pktgen.ETH_LEN,
                 pktgen.ETH_LEN + pktgen.IP_LEN, o.data_ptr(), 0) for b, o in zip(self.bufs, self.outs)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R], ss[k % S])
            if rc:
                raise xsum.TasxError(rc, "tasx_tcp4_cksum_batch_dev_hint")
        return launch


class FlushMixWorkload:
    """A tx_flush-shaped TCP4 batch: flow_tx_segment data frames (1514 B) and
    flow_tx_ack frames (66 B, ip.len 52; fast_flows.c:877-1030) half and half in
    random order, 2048 B mbuf rooms, each frame's length (mbuf data_len) as its
    hint; automatic kernel selection."""
    desc = (f"{N_FRAMES} TAS TX frames in {STRIDE} B rooms, 50% data segments (ip.len {IP_TOTAL}) and 50% "
            "pure ACKs (ip.len 52) in random order, per-frame hints (mbuf data_len)")

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

    def launcher(self):
        fn = xsum.lib().tasx_tcp4_cksum_batch_dev_hint
        s = torch.cuda.current_stream().cuda_stream
        args = [(b.data_ptr(), None, self.stride, self.flen.data_ptr(), 0, self.n, pktgen.ETH_LEN,
                 pktgen.ETH_LEN + pktgen.IP_LEN, o.data_ptr(), 0, s) for b, o in zip(self.bufs, self.outs)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R])
            if rc:
                raise xsum.TasxError(rc, "tasx_tcp4_cksum_batch_dev_hint")
        return launch


class RxVerifyWorkload:
    """Receive-side verification over a Tcp4Workload's (checksummed) frames."""

    def __init__(self, wl: Tcp4Workload):
        self.wl = wl
        wl.rx_flags = [torch.empty(wl.n, dtype=torch.uint8, device="cuda") for _ in wl.bufs]
        self.bytes_per_step = wl.n * (wl.ip_total + 1)

    def launcher(self):
        # the received frames' length (mbuf data_len) as the prefetch hint
        fn = xsum.lib().tasx_tcp4_verify_batch_dev_hint
        stream = torch.cuda.current_stream().cuda_stream
        wl = self.wl
        args = [(b.data_ptr(), None, wl.stride, None, wl.hint, wl.n, pktgen.ETH_LEN,
                 pktgen.ETH_LEN + pktgen.IP_LEN, f.data_ptr(), stream) for b, f in zip(wl.bufs, wl.rx_flags)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R])
            if rc:
                raise xsum.TasxError(rc, "tasx_tcp4_verify_batch_dev_hint")
        return launch


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

    def launcher(self):
        fn = xsum.lib().tasx_raw_cksum_batch_dev
        stream = torch.cuda.current_stream().cuda_stream
        op = self.off.data_ptr() if self.off is not None else None
        lp = self.lens.data_ptr() if self.lens is not None else None
        args = [(b.data_ptr(), op, self.len0 if op is None else 0, lp, self.len0, self.n, o.data_ptr(), stream)
                for b, o in zip(self.bufs, self.outs)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R])
            if rc:
                raise xsum.TasxError(rc, "tasx_raw_cksum_batch_dev")
        return launch


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
            "mbuf data room), checksums in place")

    def __init__(self, rotate: int, seed: int, n: int = N_FRAMES):
        self.n = n
        # room = the mbuf data room (TAS: BUFFER_SIZE, tas/fast/internal.h:34)
        _, _, segs, shm_len = pktgen.tx_segments(n, seed=seed, nflows=8192, tx_len=16384, make_shm=False,
                                                 room=STRIDE)
        self.segs_np, self.shm_len = segs, shm_len
        self.segs = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
        self.shms = [device_random(shm_len, seed + 7 + r) for r in range(rotate)]
        first = device_tcp4_frames(n, STRIDE, IP_TOTAL, seed)
        self.bufs = [first] + [first.clone() for _ in range(rotate - 1)]
        self.outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(rotate)]
        hdr = pktgen.HDRS_LEN - pktgen.ETH_LEN - pktgen.IP_LEN
        self.bytes_per_seg = 2 * pktgen.TCP_MSS + pktgen.IP_LEN + hdr + 4
        self.bytes_per_step = n * self.bytes_per_seg

    def launcher(self):
        fn = xsum.lib().tasx_tx_segment_batch_dev
        stream = torch.cuda.current_stream().cuda_stream
        args = [(sh.data_ptr(), self.shm_len, b.data_ptr(), self.segs.data_ptr(), self.n, pktgen.ETH_LEN,
                 pktgen.ETH_LEN + pktgen.IP_LEN, o.data_ptr(), stream)
                for sh, b, o in zip(self.shms, self.bufs, self.outs)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R])
            if rc:
                raise xsum.TasxError(rc, "tasx_tx_segment_batch_dev")
        return launch

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
        return {"value": self.bytes_per_step / t / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": f"rotation 0's {self.n} segments, oracle flow_tx_read + tcp_checksums per segment, "
                          f"median of {reps} passes",
                "parity_vs_gpu": "bit-exact" if np.array_equal(frames, gpu_frames) else "MISMATCH"}


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

    def launcher(self):
        fn = xsum.lib().tasx_flow_lookup_batch_dev
        stream = torch.cuda.current_stream().cuda_stream
        args = [(b.data_ptr(), None, STRIDE, self.N, pktgen.ETH_LEN, pktgen.ETH_LEN + pktgen.IP_LEN,
                 self.ht.data_ptr(), self.ENTRIES, self.fs.data_ptr(), self.NFLOWS, pktgen.FLOWST_SIZE,
                 pktgen.FLOWST_KEY_OFF, h.data_ptr(), f.data_ptr(), stream)
                for b, h, f in zip(self.bufs, self.hashes, self.fids)]
        R = len(args)

        def launch(k):
            rc = fn(*args[k % R])
            if rc:
                raise xsum.TasxError(rc, "tasx_flow_lookup_batch_dev")
        return launch

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


def prewarm(launch, seconds: float = 0.25):
    """Bring the GPU out of idle clocks before any measured step (not part of
    W or K)."""
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(32):
            launch(k)
            k += 1
        torch.cuda.synchronize()


def timed_run(wl, steps: int, warmup: int, ws: int):
    """W untimed steps, then exactly K timed steps between barrier+sync pairs.
    A HIP event pair on the launch stream around the K back-to-back launches
    gives the average launch duration (no per-launch events, which would add
    gaps of their own)."""
    launch = wl.launcher()
    prewarm(launch)
    for k in range(warmup):
        launch(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for k in range(steps):
        launch(warmup + k)
    e1.record()
    torch.cuda.synchronize()
    barrier(ws)
    t1 = time.perf_counter()
    return t1 - t0, e0.elapsed_time(e1) / steps


def timed_run_contexts(wl, steps: int, warmup: int, ws: int, n_ctx: int):
    """As timed_run, with batch k launched on stream k % n_ctx: n_ctx fast-path
    contexts submitting independent batches, so one batch's ramp-up overlaps
    another's drain.  The event pair brackets all streams (they wait on the
    start event; the current stream waits on each one's end)."""
    streams = [torch.cuda.Stream() for _ in range(n_ctx)]
    launch = wl.launcher(streams)
    prewarm(launch)
    for k in range(warmup):
        launch(k)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(cur)
    for s in streams:
        s.wait_event(e0)
    for k in range(steps):
        launch(warmup + k)
    for s in streams:
        cur.wait_stream(s)
    e1.record(cur)
    torch.cuda.synchronize()
    barrier(ws)
    t1 = time.perf_counter()
    return t1 - t0, e0.elapsed_time(e1) / steps


def roofline(bytes_per_launch: int, avg_ms: float, traffic):
    avg_s = avg_ms / 1e3
    achieved = bytes_per_launch / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "launch_avg_us": round(avg_s * 1e6, 3), "algorithmic_bytes_per_launch": bytes_per_launch}


def leg(wl, args, ws, desc):
    dt, avg_ms = timed_run(wl, args.steps, args.warmup, ws)
    dt = max_over_ranks(dt, ws)
    total = sum_over_ranks(float(wl.bytes_per_step * args.steps), ws)
    return {"value": total / dt / GIB, "unit": "GiB/s", "ms_per_step": dt / args.steps * 1e3,
            "workload": desc, "roofline": roofline(wl.bytes_per_step, avg_ms, None)}


# ---------------------------------------------------------------------------
# rank-0 extra legs

def e2e_leg(reps: int = 5) -> dict:
    """PCIe-inclusive rates (never the headline):
    * staged: host frames -> chunked pinned H2D of whole mbuf rooms -> kernel ->
      D2H of the results (tasx_tcp4_cksum_batch_host);
    * zero-copy: the kernel reads the frames from pinned host memory over PCIe
      (only the bytes it sums) and writes the results to device memory;
    * tx_flush at TAS's batch size (32 frames): deferred tcp_checksums() calls +
      tasx_flush, staged and zero-copy (frames in a registered region)."""
    n = N_FRAMES
    frames = pktgen.tcp4_frames(n, payload=IP_TOTAL - 52, stride=STRIDE, seed=41)
    pin = xsum.PinnedBuffer(frames.size)
    pin.array[:] = frames
    out = np.empty(2 * n, np.uint16)
    dout = torch.empty(2 * n, dtype=torch.int16, device="cuda")
    alg = n * (IP_TOTAL + 4)
    res = {}
    xsum.ctx_init(0, torch.cuda.current_device(), 32 << 20)
    try:
        xsum.tcp4_cksum_batch_host(0, pin.addr, STRIDE, n, out.ctypes.data)  # warm
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            xsum.tcp4_cksum_batch_host(0, pin.addr, STRIDE, n, out.ctypes.data)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        res["staged"] = {"value": alg / t / GIB, "unit": "GiB/s", "ms_per_batch": t * 1e3,
                         "pcie_h2d_bytes": n * STRIDE, "pcie_d2h_bytes": n * 4}
        zc = []
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            xsum.tcp4_cksum_batch(pin.dev_addr, n, stride=STRIDE, out=dout, frame_len=FRAME_LEN)
            torch.cuda.synchronize()
            if r:
                zc.append(time.perf_counter() - t0)
        t = float(np.median(zc))
        res["zero_copy"] = {"value": alg / t / GIB, "unit": "GiB/s", "ms_per_batch": t * 1e3,
                            "note": "frames stay in pinned host memory; results land in HBM"}
        # tx_flush at TXBUF_SIZE = 32 frames (tas/include/fastpath.h:38)
        f32 = xsum.PinnedBuffer(32 * STRIDE)
        f32.array[:] = pktgen.tcp4_frames(32, payload=IP_TOTAL - 52, stride=STRIDE, seed=42)
        plain = pktgen.tcp4_frames(32, payload=IP_TOTAL - 52, stride=STRIDE, seed=42)

        def flush_lat(base):
            lat = []
            for _ in range(60):
                t0 = time.perf_counter()
                for i in range(32):
                    xsum.defer_tcp4(0, base + i * STRIDE)
                xsum.tx_flush(0)
                lat.append(time.perf_counter() - t0)
            return float(np.median(lat[10:])) * 1e6
        res["flush32_staged_us"] = flush_lat(plain.ctypes.data)
        xsum.register_frames(0, f32.addr, f32.nbytes)
        res["flush32_zero_copy_us"] = flush_lat(f32.addr)
        res["flush32_note"] = ("32 x tasx_defer_tcp4 + tasx_flush via ctypes (Python call overhead "
                               "included); the CPU oracle needs ~7.5 us for the same 32 frames on one core")
        f32.free()
    finally:
        xsum.ctx_destroy(0)
        pin.free()
    res["value"] = res["staged"]["value"]
    res["unit"] = "GiB/s"
    return res


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


def cpu_baseline_leg(wl: Tcp4Workload, gpu_out: np.ndarray, budget_s: float) -> dict:
    """The oracle (C restatement of the reference path, per-frame calls) timed on
    this box's host cores, on a bounded sample of the same workload."""
    orc, kind_note, tmp = host_oracle()
    frames = wl.host.copy()
    n = wl.n
    exp = orc.tcp4_batch(frames.copy(), n, stride=STRIDE)
    parity = bool(np.array_equal(exp, gpu_out))
    ncpu = len(os.sched_getaffinity(0))
    threads = min(16, ncpu)  # the box's CPU share for one GPU
    t1 = orc.bench(1, frames, n, stride=STRIDE, threads=1, reps=1)
    reps1 = max(3, min(200, int(budget_s * 0.4 / max(t1, 1e-6))))
    t1 = orc.bench(1, frames, n, stride=STRIDE, threads=1, reps=reps1)
    tn = orc.bench(1, frames, n, stride=STRIDE, threads=threads, reps=1)
    repsn = max(3, min(2000, int(budget_s * 0.4 / max(tn, 1e-6))))
    tn = orc.bench(1, frames, n, stride=STRIDE, threads=threads, reps=repsn)
    alg = n * (IP_TOTAL + 4)
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    shutil.rmtree(tmp, ignore_errors=True)
    return {
        "value": alg / tn / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"the 64K-frame TCP4 batch (98.6 MB algorithmic), per-frame oracle_tcp_checksums "
                  f"(DPDK 19.11 restatement), median of {repsn} passes on {threads} pinned threads; "
                  f"1 thread: {alg / t1 / GIB:.2f} GiB/s (median of {reps1}); {kind_note}; CPU {model}, "
                  f"{ncpu} cpus visible",
        "single_core_value": alg / t1 / GIB,
        "parity_vs_gpu": "bit-exact" if parity else "MISMATCH",
    }


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
        wl = Tcp4Workload(16, pktgen.SEED)
    elif mode == "raw":
        wl = RawWorkload(16, pktgen.SEED)
    elif mode == "txseg":
        wl = TxSegWorkload(16, pktgen.SEED + 2000)
    else:
        wl = mixed_workload(0)
    launch = wl.launcher()
    for k in range(steps):
        launch(k)
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------
# other BASELINE.json configs (--workload)

def mixed_workload(rank: int) -> "RawWorkload":
    """Config 3: 1,048,576 RAW packets, sizes uniform over {64,576,1500,9000} B in
    random order, packed at 16-byte aligned offsets."""
    n = 1 << 20
    lens = pktgen.mixed_lengths(n, seed=pktgen.SEED + rank).astype(np.int64)
    slot = (lens + 15) // 16 * 16
    offs = np.zeros(n, np.int64)
    np.cumsum(slot[:-1], out=offs[1:])
    return RawWorkload(1, pktgen.SEED + rank, n=n, offsets=offs, lengths=lens,
                       total_bytes=int(offs[-1] + slot[-1]))


def other_workload(args, ws, rank):
    name = args.workload
    if name == "shard8m":
        total = 8 * (1 << 20)
        a, b = shard.shard_ranges(total, ws)[rank]
        wl = RawWorkload(1, pktgen.SEED + rank, n=b - a, length=RAW_LEN)
        desc = f"8,388,608 x 1500 B payloads sharded over {ws} GPU(s): {b - a} packets on this rank"
        scaling = "strong"
    elif name == "mixed":
        wl = mixed_workload(rank)
        desc = "1,048,576 RAW packets per GPU, sizes uniform over {64,576,1500,9000} B in random order"
        scaling = "weak"
    else:  # tso
        wl = Tcp4Workload(2, pktgen.SEED + rank, n=16384, stride=65552, ip_total=65535, host=False)
        desc = "16,384 TSO segments per GPU (ip.len 65535, L4 65,515 B), tcp_checksums() flag-off, hinted"
        scaling = "weak"
    r = leg(wl, args, ws, desc)
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline:
        torch.cuda.synchronize()
        cpu = other_cpu_baseline(name, wl, args.cpu_seconds / 2)
    pmc = None
    if rank == 0 and ws == 1 and not args.no_pmc and name == "mixed":
        pmc = pmc_leg("mixed", "raw_wave_kernel", 8)
        if pmc and "hbm_bytes_per_launch" in pmc:
            r["roofline"]["traffic"] = int(pmc["hbm_bytes_per_launch"])
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(r["value"], 2), "unit": "GiB/s", "n_gpus": ws,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
                          "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
                          "data": "synthetic (device-generated random bytes)",
                          "config": {"workload": desc, "parallelism": f"shard{ws}"},
                          "roofline": r["roofline"], "cpu_baseline": cpu,
                          **({"pmc": pmc} if pmc else {})}), flush=True)


def other_cpu_baseline(name: str, wl, budget_s: float) -> dict:
    """The oracle on a bounded sample of the other configs (BASELINE.md's CPU
    plan: the same generator, per-packet calls, 1 and 16 host threads), checked
    against the GPU's results for the same packets."""
    orc, kind_note, tmp = host_oracle()
    threads = min(16, len(os.sched_getaffinity(0)))
    if name == "tso":
        m, stride = 4096, wl.stride  # 268 MB: beyond the 16 threads' share of L3
        host = wl.bufs[0][:m * stride].cpu().numpy().copy()
        gpu = wl.outs[0][:2 * m].cpu().numpy().view(np.uint16)
        parity = np.array_equal(orc.tcp4_batch(host.copy(), m, stride=stride), gpu)
        kw = dict(stride=stride)
        mode, alg = 1, m * (wl.ip_total + 4)
        sample = f"the first {m} TSO segments (ip.len {wl.ip_total}), per-segment oracle_tcp_checksums in place"
    else:
        m = 65536 if wl.off is not None else 262144  # 182 / 393 MB: streamed, not L3-resident
        gpu = wl.outs[0][:m].cpu().numpy().view(np.uint16)
        if wl.off is None:
            host = wl.bufs[0][:m * wl.len0].cpu().numpy()
            kw = dict(stride=wl.len0, len0=wl.len0)
            alg = m * (wl.len0 + 2)
        else:
            offs = wl.off[:m].cpu().numpy().astype(np.uint64)
            lens = wl.lens[:m].cpu().numpy().astype(np.uint32)
            host = wl.bufs[0][:int(offs[-1]) + int(lens[-1])].cpu().numpy()
            kw = dict(offsets=offs, lengths=lens)
            alg = int(lens.astype(np.int64).sum()) + 2 * m
        parity = np.array_equal(orc.raw_batch(host, m, **kw), gpu)
        mode = 0
        sample = f"the first {m} packets of the batch, per-packet oracle_raw_cksum (rte_raw_cksum restatement)"
    t1 = orc.bench(mode, host, m, threads=1, reps=1, **kw)
    reps1 = max(3, min(200, int(budget_s * 0.4 / max(t1, 1e-6))))
    t1 = orc.bench(mode, host, m, threads=1, reps=reps1, **kw)
    tn = orc.bench(mode, host, m, threads=threads, reps=1, **kw)
    repsn = max(3, min(2000, int(budget_s * 0.4 / max(tn, 1e-6))))
    tn = orc.bench(mode, host, m, threads=threads, reps=repsn, **kw)
    shutil.rmtree(tmp, ignore_errors=True)
    return {"value": alg / tn / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{sample} ({alg / 1e6:.1f} MB algorithmic), median of {repsn} passes on {threads} "
                      f"pinned threads; 1 thread: {alg / t1 / GIB:.2f} GiB/s (median of {reps1}); {kind_note}",
            "single_core_value": alg / t1 / GIB,
            "parity_vs_gpu": "bit-exact" if parity else "MISMATCH"}


def main():
    args = parse()
    if args.pmc_child:
        pmc_child(args.pmc_child, args.steps)
        return
    ws, rank, local = dist_setup()
    xsum.lib()
    if args.workload != "tcp4":
        other_workload(args, ws, rank)
        if ws > 1:
            dist.destroy_process_group()
        return
    rot = max(1, args.rotate)

    wl = Tcp4Workload(rot, pktgen.SEED + rank)
    head = leg(wl, args, ws, Tcp4Workload.desc)
    ctx2 = None
    if not args.no_contexts:
        dt2, avg2 = timed_run_contexts(wl, args.steps, args.warmup, ws, 2)
        dt2 = max_over_ranks(dt2, ws)
        total = sum_over_ranks(float(wl.bytes_per_step * args.steps), ws)
        ctx2 = {"value": total / dt2 / GIB, "unit": "GiB/s", "ms_per_step": dt2 / args.steps * 1e3,
                "workload": "the headline batches alternating over 2 streams (two fast-path contexts, "
                            "independent batches): one batch's ramp-up overlaps the other's drain",
                "batch_interval_us": round(avg2 * 1e3, 3),
                "alg_GBps_per_interval": round(wl.bytes_per_step / (avg2 * 1e-3) / 1e9, 1),
                "note": "kernels overlap, so a kernel's own duration is longer than the interval; "
                        "the headline roofline uses the single-stream launch"}
    wl.hint = 0
    nohint = leg(wl, args, ws, "same frames, tasx_tcp4_cksum_batch_dev (frames only, no hint)")
    wl.hint = FRAME_LEN
    # receive-side verification of the same frames (after in-place TX checksums)
    xsum.tcp4_cksum_batch(wl.bufs[0], wl.n, stride=wl.stride, inplace=True, want_out=False)
    for b in wl.bufs[1:]:
        b.copy_(wl.bufs[0])
    rx = leg(RxVerifyWorkload(wl), args, ws, "same frames after TX checksums, tasx_tcp4_verify_batch_dev_hint "
             "(received frame length as the hint)")
    torch.cuda.synchronize()
    rx["all_frames_verified"] = bool((wl.rx_flags[0] == 3).all().item())
    src = torch.from_numpy(wl.host).cuda()
    for b in wl.bufs:  # restore the un-checksummed frames for the legs below
        b.copy_(src)
    del src
    mix = None
    if not args.no_flushmix:
        mw = FlushMixWorkload(min(rot, 12), pktgen.SEED + 500 + rank)
        mix = leg(mw, args, ws, FlushMixWorkload.desc)
        mix["parity"] = "tests/test_gpu_parity.py::test_tcp4_flush_mix_per_frame_hints"
        del mw
        torch.cuda.empty_cache()
    raw = None
    if not args.no_raw:
        rw = RawWorkload(rot, pktgen.SEED + 1000 + rank)
        raw = leg(rw, args, ws, RawWorkload.desc)
        raw["algorithmic_bytes_per_packet"] = RAW_LEN + 2
        del rw
        torch.cuda.empty_cache()

    txseg = None
    if not args.no_txseg:
        del wl.bufs[1:], wl.outs[1:]
        torch.cuda.empty_cache()
        tw = TxSegWorkload(rot, pktgen.SEED + 2000 + rank)
        txseg = leg(tw, args, ws, TxSegWorkload.desc)
        txseg["algorithmic_bytes_per_segment"] = tw.bytes_per_seg
        if rank == 0 and ws == 1 and not args.no_cpu_baseline:
            txseg["cpu_baseline"] = tw.cpu_check(3.0)
        del tw
        torch.cuda.empty_cache()

    flow = None
    if not args.no_flow:
        fw = FlowLookupWorkload(min(rot, 4), pktgen.SEED + 3000 + rank)
        flow = leg(fw, args, ws, FlowLookupWorkload.desc)
        flow["mpps"] = fw.N * args.steps / (flow["ms_per_step"] * 1e-3 * args.steps) / 1e6
        flow["flows_inserted_frac"] = fw.inserted
        flow["bytes_per_frame"] = 64
        if rank == 0 and ws == 1 and not args.no_cpu_baseline:
            flow["cpu_baseline"] = fw.cpu_check(3.0)
        del fw
        torch.cuda.empty_cache()

    extra = {}
    if rank == 0 and ws == 1:
        torch.cuda.synchronize()
        gpu_out = wl.outs[0].cpu().numpy().view(np.uint16).copy()
        if not args.no_cpu_baseline:
            extra["cpu_baseline"] = cpu_baseline_leg(wl, gpu_out, args.cpu_seconds)
        if not args.no_e2e:
            extra["e2e"] = e2e_leg()
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
                txseg["pmc"] = pt

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
            "cpu_baseline": extra.get("cpu_baseline"),
            "tcp4_nohint": nohint,
            "two_contexts": ctx2,
            "rx_verify": rx,
            "flush_mix": mix,
        }
        if raw is not None:
            line["raw"] = raw
        if txseg is not None:
            line["tx_segment"] = txseg
        if flow is not None:
            line["flow_lookup"] = flow
        if "e2e" in extra:
            line["e2e"] = extra["e2e"]
        if "pmc" in extra:
            line["pmc"] = extra["pmc"]
        print(json.dumps(line), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
