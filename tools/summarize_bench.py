"""Print the key numbers of a bench.py JSON line (the last {...} line of a log)."""
import json
import sys

for path in sys.argv[1:]:
    line = [ln for ln in open(path) if ln.startswith("{")][-1]
    d = json.loads(line)
    print(f"== {path}: value {d['value']} GiB/s, ms_per_step {d['ms_per_step'] * 1e3:.3f} us, "
          f"launch_avg {d['roofline']['launch_avg_us']} us, frac {d['roofline']['frac']}, "
          f"traffic {d['roofline'].get('traffic')}, kernel {d.get('kernel')}, "
          f"pattern_ceiling {(d['roofline'].get('pattern_ceiling') or {}).get('us')} us")
    for k in ("tcp4_nohint", "tcp4_frames_only", "rx_verify", "flush_mix", "rx_verify_mix", "raw", "tx_segment", "flow_lookup",
              "rx_pass"):
        v = d.get(k)
        if not v:
            continue
        r = v["roofline"]
        extra = ""
        if k in ("tx_segment", "rx_pass") and r.get("traffic"):
            extra = f" traffic/alg {r['traffic'] / r['algorithmic_bytes_per_launch']:.3f}"
        if k == "tx_segment" and v.get("copy_ceiling"):
            extra += f" copy_ceiling {v['copy_ceiling'].get('us')} us"
        if k == "tx_segment" and v.get("pattern_ceiling"):
            extra += f" pattern_ceiling {v['pattern_ceiling'].get('us')} us"
        if k in ("flush_mix", "rx_verify_mix") and r.get("latency"):
            extra = f" latency-roofline frac {r['latency'].get('frac')} of-pattern {r['latency'].get('frac_of_pattern')}"
        if k == "flow_lookup":
            extra = f" line {v.get('line_roofline', {}).get('frac')} ceiling {v.get('pattern_ceiling')}"
        print(f"  {k:17s} {v['value']:8.1f} GiB/s  step {v['ms_per_step'] * 1e3:7.3f} us  launch {r['launch_avg_us']:7.3f} us"
              f"  frac {r['frac']:.4f}  {v.get('kernel', '')}{extra}")
    if d.get("two_contexts"):
        print(f"  two_contexts interval {d['two_contexts']['batch_interval_us']} us")
    if d.get("cpu_baseline"):
        c = d["cpu_baseline"]
        print(f"  cpu_baseline {c['value']:.1f} GiB/s on {c['cores']} cores, 1 core {c.get('single_core_value', 0):.2f}")
    if d.get("e2e"):
        e = d["e2e"]
        print(f"  e2e staged {e['staged']['value']:.1f} zero-copy {e['zero_copy']['value']:.1f} GiB/s "
              f"flush32 {e.get('flush32_staged_us', 0):.1f} / {e.get('flush32_zero_copy_us', 0):.1f} us")
        if e.get("tx_segment_host"):
            h = e["tx_segment_host"]
            print(f"  e2e tx_segment_host {h['value']:.1f} GiB/s alg, {h['ms_per_batch']:.3f} ms per 64K segments, "
                  f"{h['segments_per_s'] / 1e6:.1f} M segments/s")
