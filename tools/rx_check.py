# quick bit-exactness check of an A/B RX variant against the product on the bench's RX frames
import sys, torch, numpy as np
sys.path.insert(0, '.')
import bench
from tas_amd import xsum, pktgen, benchloop
v = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.N_FRAMES
w = bench.RxPassWorkload(bench.FlowLookupWorkload(1, pktgen.SEED + 3000), 2, pktgen.SEED + 4000, n=n)
w.loop(benchloop.RX_FUSED)(0, 1); torch.cuda.synchronize()
ref = (w.flags[0].clone(), w.fids[0].clone(), w.hashes[0].clone())
for t in (w.flags[0], w.fids[0], w.hashes[0]): t.fill_(0x5a)
with xsum.using_library(xsum.AB_LIB_PATH):
    xsum.set_kernel_variant(v)
    fw = w.fw
    xsum.rx_batch(w.bufs[0], w.n, fw.ht, fw.fs, fw.NFLOWS, stride=bench.STRIDE, frame_len=w.flen,
                  flags=w.flags[0], fid=w.fids[0], h=w.hashes[0])
    torch.cuda.synchronize()
    print('variant', v, 'n', n, xsum.last_kernel(), 'flags', bool((w.flags[0] == ref[0]).all()), 'fid', bool((w.fids[0] == ref[1]).all()),
          'hash', bool((w.hashes[0] == ref[2]).all()))
if not ((w.flags[0] == ref[0]).all() and (w.fids[0] == ref[1]).all() and (w.hashes[0] == ref[2]).all()):
    sys.exit(1)
