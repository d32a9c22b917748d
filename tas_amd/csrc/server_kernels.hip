// server_kernels.hip -- the persistent flush server (round 4): one long-running
// kernel per GPU that takes TAS's tx_flush batches (tas/fast/fastemu.c:544-566,
// at most TXBUF_SIZE = 32 frames per core per loop, tas/include/fastpath.h:38)
// straight from pinned host memory, with no HIP call on the fast-path core.
//
// Every deferred flush so far paid a kernel launch plus a completion round
// trip (~13 us), more than one core's CPU checksums of
// the same 32 frames.  Here the fast-path core writes a descriptor slot into
// its context's ring in coherent pinned memory (frame offsets in its
// registered mbuf region, each with its ip.total_length) and the header last;
// the workgroups of ring r poll its slots, sum the frames in place over PCIe
// and store both checksum fields into them, then post each slot's done word.
// Layout and protocol: tasx_kernels.h (TASX_SRV_*), tasx_host.c
// (server_submit).
//
// Coherence (MI355X_MICROARCH.md, hand-off rules): every word the host writes
// is read with system-scope (sc0 sc1) loads, so no cache level can return an
// older copy.  TAS reuses an mbuf as soon as its frame has left, so a frame
// line an XCD's L2 cached for an earlier batch must never be summed: after
// taking a batch, the polling wave issues one system-scope acquire
// (buffer_inv sc0 sc1: this CU's L1 and the XCD's L2 drop their non-coherent
// lines) and the rows then read the frames with nt buffer loads.  Without the
// acquire, tests/test_server.py::test_server_refilled_mbufs_every_flush
// fails; with system-scope frame loads instead (round 4's first server) the
// server tops out at 14-19 M frames/s from 8 cores, against 24-28 this way
// (profiles/r04/r04g; 42-48 in the bench lines of round 4's last passes).
// The two checksum fields are written by sc0 sc1 stores (write-through to host
// memory).  Each wave waits for its stores (vmcnt(0)), the workgroup meets at
// a barrier, and only then does one lane store the slot's done word, also sc0
// sc1: the host sees the word after the fields.  Descriptor words carry the
// 16-bit tag of their ring position (every entry word of a slot, used or not,
// is rewritten per submit), so a slot read over PCIe while the host was still
// writing it is recognised (a word with an older tag) and read again -- no
// separate doorbell round trip.
//
// TX segment slots (TASX_SRV_SEG, tasx_server_tx_segments): the rows run the
// general TX segment row (txseg_device.h) -- payload gathered from the app's
// TX buffer into the frame, both checksums -- with plain stores, and one lane
// issues a system-scope release (buffer_wbl2 sc0 sc1) before the done word.
//
// Epochs (round 6): one launch serves for P.period_ticks of the GPU's wall
// clock, then every workgroup leaves at its next poll (a batch it is summing
// is finished first), storing its ring position and the time of its last
// batch; the host's epoch thread keeps the next launch queued behind it on the
// same stream, and that launch resumes at those positions.  A HIP call that
// waits for all of the device's work (hipDeviceSynchronize, the frees, a
// synchronous copy) therefore waits for at most the launches queued when it
// was made -- about two periods -- instead of for a kernel that never ends.
// Every wave also leaves at once when the host sets the stop word (stop,
// pause, abort); a process that is gone queues no further epoch.
#include "server_device.h"

extern "C" int tasx_launch_server(const tasx_srv_params *p, void *stream)
{
  if (p->k == 0u || TASX_SRV_RING % p->k != 0u || p->k > TASX_SRV_KMAX)
    return -1;
  hipLaunchKernelGGL(flush_server_kernel, dim3(TASX_MAX_CTX * p->k), dim3(kSrvBlock), 0, (hipStream_t) stream,
                     *p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
