// flow_kernels.hip -- RX flow lookup for gfx950:
// the batch part of fast_flows_packet_fss()
// (/root/reference/tas/fast/fast_flows.c:1084-1163): per received frame, the
// CRC32C flow hash of its 4-tuple (flow_hash, :1078-1082) and the probe of
// FLEXNIC_PL_FLOWHT_NBSZ hash-table entries, each candidate confirmed against
// the 4-tuple in its flow state.
//
// Layout: two frames per lane.  The work is latency-bound random access (a
// dependent chain frame header -> bucket -> flow state), not bandwidth: every
// load of a phase is issued before any is used (both frames' keys, then their
// eight bucket entries together, then the candidates' keys together, clamped
// to flow 0 when not a candidate), and the kernel keeps few registers so many
// chains are in flight per CU.  CRC32C is computed bit by bit on the VALU (a
// slice-by-4 form from LDS tables measured the same: the CRC is not on the
// critical path).
#include "flow_device.h"

extern "C" int tasx_launch_flow_lookup(const tasx_flow_params *p, int variant, void *stream)
{
  if (p->n == 0)
    return 0;
  hipStream_t s = (hipStream_t) stream;
  // two frames per lane: 256K lookups 11.85 us against 12.53 with one and
  // 12.98 with four (register pressure; profiles/r02/r02ca); the frame keys
  // non-temporal (round 4, above)
  (void) variant; // one form (tasx_set_kernel_variant selects none here)
  return launch_flow_f<kFlowFramesPerLane>("flow_lookup_kernel", p, s);
}
