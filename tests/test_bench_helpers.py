"""bench.py's pricing helpers on the CPU: the roofline record, the data/ACK
mixes' latency roofline (price_mix), the TX segment build's 128-byte block
floor, the rehearsal filter that drops any fraction above 1 when ranks
share one GPU, the price leg's child process failing softly, and the host
wait setting.  No GPU work."""
import numpy as np

import bench
from tas_amd import pktgen


def test_roofline_record():
    r = bench.roofline(98_566_144, 15.8e-3, None)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - 98_566_144 / 15.8e-6 / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-4
    assert r["launch_avg_us"] == 15.8


def test_price_mix_bound_is_the_larger_of_chain_and_hbm():
    mb = {"pattern_us": 10.0, "chain_us": 5.0, "rows": 65536, "rows_in_flight": 32768, "generations": 2,
          "dependent_loads_per_row": 2, "loaded_latency_us": 1.25, "kernel": "k"}
    leg = {"roofline": bench.roofline(51_190_000, 10.1e-3, None)}
    bench.price_mix(leg, mb, 51_190_000)
    lat = leg["roofline"]["latency"]
    hbm_us = 51_190_000 / bench.HBM_PEAK_GBS / 1e3
    assert abs(lat["hbm_us"] - hbm_us) < 1e-3
    assert lat["bound_us"] == round(max(5.0, hbm_us), 3)
    assert abs(lat["frac"] - lat["bound_us"] / 10.1) < 1e-3
    assert abs(lat["frac_of_pattern"] - 10.0 / 10.1) < 1e-3
    # chain-bound case: a chain longer than the HBM time sets the bound
    leg2 = {"roofline": bench.roofline(1_000_000, 9.0e-3, None)}
    bench.price_mix(leg2, dict(mb, chain_us=7.5), 1_000_000)
    assert leg2["roofline"]["latency"]["bound_us"] == 7.5


def test_price_mix_disturbed_chain_claims_no_fraction():
    """A chain kernel slower than the product's own access pattern (round 3's
    rocprofv3 run: 10.10 us against a 10.17 us pattern would read frac 0.98)
    is a disturbed measurement: frac is null, the raw numbers stay."""
    mb = {"pattern_us": 10.0, "chain_us": 10.1, "rows": 65536, "rows_in_flight": 32768, "generations": 2,
          "dependent_loads_per_row": 2, "loaded_latency_us": 2.5, "kernel": "k"}
    leg = {"roofline": bench.roofline(51_190_000, 10.3e-3, None)}
    bench.price_mix(leg, mb, 51_190_000)
    lat = leg["roofline"]["latency"]
    assert lat["frac"] is None and "note" in lat
    assert lat["chain_us"] == 10.1 and abs(lat["frac_of_pattern"] - 10.0 / 10.3) < 1e-3
    assert bench.MIX_BOUND_RUNS >= 3


def test_txseg_block_floor_counts_lines():
    _, _, segs, _ = pktgen.tx_segments(64, seed=3, nflows=8, tx_len=4096, make_shm=False, room=2048)
    fl = bench.txseg_block_floor(segs)
    # reads: the 128-byte blocks each payload piece spans, the header block and the 32-byte descriptor
    exp_r = 0
    for s in segs:
        base, pos, pay, tlen = int(s["tx_base"]), int(s["pos"]), int(s["payload"]), int(s["tx_len"])
        p1 = min(pay, tlen - pos)
        if p1 > 0:
            exp_r += (base + pos + p1 + 127) // 128 - (base + pos) // 128
        if pay - p1 > 0:
            exp_r += (base + pay - p1 + 127) // 128 - base // 128
    exp_r = exp_r * 128 + len(segs) * (128 + 32)
    off = segs["frame_off"].astype(np.int64)
    fend = off + segs["hdrs_len"].astype(np.int64) + segs["payload"].astype(np.int64)
    exp_w = int((((fend + 127) // 128) - off // 128).sum()) * 128
    assert fl == {"read_bytes": exp_r, "write_bytes": exp_w, "bytes": exp_r + exp_w, "block": 128}


def test_rehearsal_drops_fractions_above_one():
    line = {"frac_of_n_hbm": 1.2, "roofline": {"frac": 0.7, "pattern_ceiling": {"frac": 1.05, "us": 15.0}},
            "legs": [{"frac": 1.5}, {"frac": 0.5}], "value": 6000.0}
    out = bench.drop_rehearsal_fractions(line)
    assert out["frac_of_n_hbm"] is None and out["roofline"]["frac"] == 0.7
    assert out["roofline"]["pattern_ceiling"] == {"frac": None, "us": 15.0}
    assert out["legs"] == [{"frac": None}, {"frac": 0.5}] and out["value"] == 6000.0


def test_fastpath_mt_refuses_bad_shapes_before_any_gpu_call():
    """tasxb_fastpath_mt (bench.py's fastpath_mt line) checks its arguments
    before it touches HIP: thread counts, in-flight depth (the 8-slot queue),
    mode and the context-id range."""
    import errno
    from tas_amd import benchloop, xsum
    bad = [(0, 1, 100, "server", 8), (17, 1, 100, "server", 0), (1, 0, 100, "feeder", 8),
           (1, 8, 100, "feeder", 8), (1, 1, 0, "per_context", 8), (9, 1, 100, "server", 8)]
    for th, q, fl, mode, ctx0 in bad:
        try:
            benchloop.fastpath_mt(0, ctx0, th, q, fl, mode)
        except xsum.TasxError as e:
            assert e.code == -errno.EINVAL, (th, q, fl, mode, ctx0, e.code)
        else:
            raise AssertionError((th, q, fl, mode, ctx0))


def test_server_cost_child_failure_is_reported_not_raised():
    """The price leg runs in a child process (bench.py --server-cost-child); a
    child that fails (here: no GPU) leaves an error record in the bench line
    instead of ending the bench."""
    import torch
    if torch.cuda.is_available():
        return  # on a GPU box the child runs for real (tests/test_bench_configs.py covers the legs)
    r = bench.server_cost_child_leg(1)
    assert set(r) == {"error"} and "server_cost child" in r["error"]


def test_host_spin_wait_can_be_turned_off(monkeypatch):
    monkeypatch.setenv("TASX_BENCH_SCHED", "auto")
    assert bench.host_spin_wait(0) == "auto"
