"""bench.py's server_cost leg alone, one JSON line:
what the resident flush server costs the headline batch and the TX segment
build on the same GPU (stopped / idle / 8 fast-path threads flushing 8 x 3).
Usage (GPU box): python3 tools/price_leg.py FORM; with TASX_LIB=libtasx_ab.so
and TASX_SRV_ACQ=1|2 the A/B build's price diagnostics (agent-scope acquire /
none: not a product form)."""
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from tas_amd import xsum  # noqa: E402


def beat():
    while True:
        time.sleep(20)
        print("alive", time.time(), file=sys.stderr, flush=True)


threading.Thread(target=beat, daemon=True).start()
xsum.lib()
print(json.dumps({"form": sys.argv[1] if len(sys.argv) > 1 else "product",
                  "server_cost": bench.server_cost_leg(0, 16)}), flush=True)
