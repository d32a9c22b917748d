/*
 * tasx_host.c -- C host layer of libtasx: argument checking, per-fast-path-core
 * contexts, the deferred tcp_checksums()/tx_flush() surface and the
 * end-to-end (host memory, PCIe) batch pipeline.  Kernels live in
 * xsum_kernels.hip.  See include/tasx_xsum.h for the contract and the
 * reference interfaces each entry point replaces.
 *
 * No CPU checksum code exists in this library: every checksum is computed by
 * the GPU kernels, and a HIP failure is returned to the caller.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "tasx_kernels.h"

/* pipeline slots per context: flush t uses slot t % NSLOT, so NSLOT divides
 * 2^32 and the mapping stays consistent when tickets wrap */
#define NSLOT 4
#define DEFAULT_SLOT_BYTES (64u << 20)
#define DEFER_MAX_FRAME 65536u /* ip_off + 65535-byte datagram */

static __thread char g_err[256];

static int set_err(int code, const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static int hip_err(hipError_t e, const char *what)
{
  return set_err(-EIO, "%s: %s", what, hipGetErrorString(e));
}

#define HIPCHK(call)                                   \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess)                              \
      return hip_err(e_, #call);                       \
  } while (0)

int tasx_abi_version(void) { return TASX_XSUM_ABI; }
const char *tasx_last_error(void) { return g_err; }

int tasx_device_count(void)
{
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess)
    return hip_err(e, "hipGetDeviceCount");
  return n;
}

/* ---------------------------------------------------------------------- */
/* device-resident batches */

/* kernel selection (tasx_set_kernel_variant), per calling thread -- one
 * fast-path core per thread in TAS, so each context selects independently;
 * 0 = automatic */
static __thread int g_variant = 0;

int tasx_set_kernel_variant(int variant)
{
  if (variant < 0 || variant > 7 || variant == 1 || variant == 4 || variant == 5)
    return set_err(-EINVAL, "kernel variant %d does not exist (0, 2, 3, 6, 7)", variant);
  g_variant = variant;
  return 0;
}

int tasx_raw_cksum_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *len, uint32_t len0, uint32_t n,
    uint16_t *out, void *stream)
{
  tasx_raw_params p;
  int r;
  if (n == 0)
    return 0;
  if (!out || (!base && !off))
    return set_err(-EINVAL, "raw batch: NULL out/base");
  if (!len && len0 > TASX_RAW_MAX_LEN)
    return set_err(-EINVAL, "raw batch: len0 %u > %u", len0, TASX_RAW_MAX_LEN);
  p.base = (const uint8_t *) base;
  p.off = off;
  p.len = len;
  p.out = out;
  p.stride = stride;
  p.len0 = len0;
  p.n = n;
  r = tasx_launch_raw(&p, g_variant, stream);
  if (r != 0)
    return hip_err(hipGetLastError(), "raw_cksum_kernel launch");
  return 0;
}

/* RX: a uniform received length beyond the frame's room or stride slot is not
 * trusted for reads (the kernels cap per-frame lengths the same way) */
static uint32_t rx_cap_flen0(uint32_t flen0, uint32_t room, uint64_t stride, const uint64_t *off)
{
  if (room && flen0 > room)
    return room;
  if (!room && !off && stride && flen0 > stride)
    return stride < 0xffffffffull ? (uint32_t) stride : flen0;
  return flen0;
}

/* a room must hold the headers a row always reads and may not reach into the
 * next frame of a stride-mode batch */
static int check_room(uint32_t room, uint64_t stride, const uint64_t *off, uint32_t ip_off,
    uint32_t l4_off, const char *what)
{
  if (room == 0)
    return 0;
  if ((uint64_t) room < (uint64_t) ip_off + 20 || (uint64_t) room < (uint64_t) l4_off + 18)
    return set_err(-EINVAL, "%s: room %u does not hold the headers", what, room);
  if (!off && stride && room > stride)
    return set_err(-EINVAL, "%s: room %u exceeds the stride %llu", what, room,
        (unsigned long long) stride);
  return 0;
}

int tasx_tcp4_cksum_batch_dev_room(void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t room,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out,
    uint32_t flags, void *stream)
{
  tasx_tcp4_params p;
  int r;
  if (n == 0)
    return 0;
  if ((!base && !off) || (!out && !(flags & TASX_F_INPLACE)))
    return set_err(-EINVAL, "tcp4 batch: NULL base/out");
  if (out && ((uintptr_t) out & 3))
    return set_err(-EINVAL, "tcp4 batch: out must be 4-byte aligned");
  if (flags & ~TASX_F_INPLACE)
    return set_err(-EINVAL, "tcp4 batch: unknown flags 0x%x", flags);
  if ((r = check_room(room, stride, off, ip_off, l4_off, "tcp4 batch")) != 0)
    return r;
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.off = off;
  p.out = out;
  p.stride = stride;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  p.flags = flags;
  p.flen = flen;
  p.flen0 = flen0;
  p.room = room;
  r = tasx_launch_tcp4(&p, g_variant, stream);
  if (r != 0)
    return hip_err(hipGetLastError(), "tcp4_cksum_kernel launch");
  return 0;
}

int tasx_tcp4_cksum_batch_dev_hint(void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint16_t *out, uint32_t flags,
    void *stream)
{
  return tasx_tcp4_cksum_batch_dev_room(base, off, stride, flen, flen0, 0, n, ip_off,
      l4_off, out, flags, stream);
}

int tasx_tcp4_cksum_batch_dev(void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint16_t *out, uint32_t flags, void *stream)
{
  return tasx_tcp4_cksum_batch_dev_room(base, off, stride, NULL, 0, 0, n, ip_off,
      l4_off, out, flags, stream);
}

int tasx_tcp4_offload_batch_dev(void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint16_t *out, uint32_t flags, void *stream)
{
  tasx_tcp4_params p;
  if (n == 0)
    return 0;
  if ((!base && !off) || (!out && !(flags & TASX_F_INPLACE)))
    return set_err(-EINVAL, "tcp4 offload batch: NULL base/out");
  if (out && ((uintptr_t) out & 1))
    return set_err(-EINVAL, "tcp4 offload batch: out must be 2-byte aligned");
  if (flags & ~TASX_F_INPLACE)
    return set_err(-EINVAL, "tcp4 offload batch: unknown flags 0x%x", flags);
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.off = off;
  p.out = out;
  p.stride = stride;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  p.flags = flags;
  if (tasx_launch_tcp4_offload(&p, stream) != 0)
    return hip_err(hipGetLastError(), "tcp4_offload_kernel launch");
  return 0;
}

int tasx_tcp4_verify_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint8_t *flags, void *stream)
{
  return tasx_tcp4_verify_batch_dev_room(base, off, stride, NULL, 0, 0, n, ip_off,
      l4_off, flags, stream);
}

int tasx_tcp4_verify_batch_dev_hint(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint8_t *flags, void *stream)
{
  return tasx_tcp4_verify_batch_dev_room(base, off, stride, flen, flen0, 0, n, ip_off,
      l4_off, flags, stream);
}

int tasx_tcp4_verify_batch_dev_room(const void *base, const uint64_t *off,
    uint64_t stride, const uint32_t *flen, uint32_t flen0, uint32_t room,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint8_t *flags, void *stream)
{
  tasx_tcp4_params p;
  int r;
  if (n == 0)
    return 0;
  if ((!base && !off) || !flags)
    return set_err(-EINVAL, "tcp4 verify: NULL base/flags");
  if ((r = check_room(room, stride, off, ip_off, l4_off, "tcp4 verify")) != 0)
    return r;
  flen0 = rx_cap_flen0(flen0, room, stride, off);
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.off = off;
  p.out = (uint16_t *) (void *) flags;
  p.stride = stride;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  p.flen = flen;
  p.flen0 = flen0;
  p.room = room;
  if (tasx_launch_tcp4_verify(&p, g_variant, stream) != 0)
    return hip_err(hipGetLastError(), "tcp4 verify kernel launch");
  return 0;
}

int tasx_tx_segment_batch_dev(const void *shm, uint64_t shm_len, void *frames,
    const tasx_tx_seg *segs, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    uint32_t *out, void *stream)
{
  tasx_txseg_params p;
  if (n == 0)
    return 0;
  if (!shm || !frames || !segs)
    return set_err(-EINVAL, "tx segment: NULL shm/frames/segs");
  if (((uintptr_t) segs & 15u) || ((uintptr_t) out & 3u))
    return set_err(-EINVAL, "tx segment: segs must be 16-byte, out 4-byte aligned");
  if (l4_off < ip_off + 20 || l4_off > 0xffff)
    return set_err(-EINVAL, "tx segment: need ip_off + 20 <= l4_off <= 65535");
  if (shm_len > 0xffffffffull)
    return set_err(-EINVAL, "tx segment: shm_len must be below 4 GiB");
  memset(&p, 0, sizeof(p));
  p.shm = (const uint8_t *) shm;
  p.shm_len = shm_len;
  p.frames = (uint8_t *) frames;
  p.segs = segs;
  p.out = out;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  if (tasx_launch_txseg(&p, stream) != 0)
    return hip_err(hipGetLastError(), "tx segment kernel launch");
  return 0;
}

int tasx_rx_batch_dev(const void *base, const uint64_t *off, uint64_t stride,
    const uint32_t *flen, uint32_t flen0, uint32_t room, uint32_t n,
    uint32_t ip_off, uint32_t l4_off, uint8_t *flags,
    const void *flowht, uint32_t ht_entries, const void *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out, void *stream)
{
  tasx_tcp4_params p;
  int r;
  if (n == 0)
    return 0;
  if ((!base && !off) || !flags)
    return set_err(-EINVAL, "rx batch: NULL base/flags");
  if ((r = check_room(room, stride, off, ip_off, l4_off, "rx batch")) != 0)
    return r;
  flen0 = rx_cap_flen0(flen0, room, stride, off);
  if (!flowht || !flowst || !fid_out)
    return set_err(-EINVAL, "rx batch: NULL flowht/flowst/fid_out");
  if (ht_entries == 0 || fs_num == 0)
    return set_err(-EINVAL, "rx batch: empty flow table");
  if ((fs_stride & 3u) || (fs_key_off & 3u) || ((uintptr_t) flowst & 3u) || ((uintptr_t) flowht & 7u))
    return set_err(-EINVAL, "rx batch: misaligned flow table");
  if (((uintptr_t) fid_out & 3u) || ((uintptr_t) hash_out & 3u))
    return set_err(-EINVAL, "rx batch: outputs must be 4-byte aligned");
  memset(&p, 0, sizeof(p));
  p.base = (uint8_t *) base;
  p.off = off;
  p.out = (uint16_t *) (void *) flags;
  p.stride = stride;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  p.flen = flen;
  p.flen0 = flen0;
  p.room = room;
  p.flowht = (const uint32_t *) flowht;
  p.flowst = (const uint8_t *) flowst;
  p.fid_out = fid_out;
  p.hash_out = hash_out;
  p.ht_entries = ht_entries;
  p.fs_num = fs_num;
  p.fs_stride = fs_stride;
  p.fs_key_off = fs_key_off;
  if (tasx_launch_tcp4_rx(&p, g_variant, stream) != 0)
    return hip_err(hipGetLastError(), "rx kernel launch");
  return 0;
}

int tasx_flow_lookup_batch_dev(const void *base, const uint64_t *off,
    uint64_t stride, uint32_t n, uint32_t ip_off, uint32_t l4_off,
    const void *flowht, uint32_t ht_entries, const void *flowst,
    uint32_t fs_num, uint32_t fs_stride, uint32_t fs_key_off,
    uint32_t *hash_out, uint32_t *fid_out, void *stream)
{
  tasx_flow_params p;
  if (n == 0)
    return 0;
  if ((!base && !off) || !flowht || !flowst || !fid_out)
    return set_err(-EINVAL, "flow lookup: NULL base/flowht/flowst/fid_out");
  if (ht_entries == 0 || fs_num == 0)
    return set_err(-EINVAL, "flow lookup: empty flow table");
  if ((fs_stride & 3u) || (fs_key_off & 3u) || ((uintptr_t) flowst & 3u) || ((uintptr_t) flowht & 7u))
    return set_err(-EINVAL, "flow lookup: misaligned flow table");
  if (((uintptr_t) fid_out & 3u) || ((uintptr_t) hash_out & 3u))
    return set_err(-EINVAL, "flow lookup: outputs must be 4-byte aligned");
  memset(&p, 0, sizeof(p));
  p.base = (const uint8_t *) base;
  p.off = off;
  p.stride = stride;
  p.flowht = (const uint32_t *) flowht;
  p.flowst = (const uint8_t *) flowst;
  p.hash_out = hash_out;
  p.fid_out = fid_out;
  p.n = n;
  p.ip_off = ip_off;
  p.l4_off = l4_off;
  p.ht_entries = ht_entries;
  p.fs_num = fs_num;
  p.fs_stride = fs_stride;
  p.fs_key_off = fs_key_off;
  if (tasx_launch_flow_lookup(&p, g_variant, stream) != 0)
    return hip_err(hipGetLastError(), "flow lookup kernel launch");
  return 0;
}

/* ---------------------------------------------------------------------- */
/* contexts */

/* One submitted flush (tasx_flush_submit): its frames (the staged path copies
 * the results into them when the ticket completes) and the device views of its
 * pinned descriptors.  Flush t uses slot t % NSLOT: the staging, offsets and
 * results buffers of that slot and completion word t % NSLOT. */
struct flush_slot {
  uint32_t ticket; /* the ticket it carries */
  uint32_t n;
  int zerocopy;
  uint8_t **ip, **l4;          /* the batch's frames (slot_frames entries) */
  uint32_t *h_flen, *d_flen;   /* per-frame hints (zero-copy path) */
  uint64_t *d_off;             /* device views of h_off[s], h_stage[s], h_out[s] */
  uint8_t *d_stage;
  uint16_t *d_out;
};

struct tasx_ctx {
  int in_use;
  int device;
  size_t slot_bytes;
  hipStream_t st[NSLOT];
  uint8_t *d_buf[NSLOT];
  uint64_t *d_off[NSLOT];
  uint16_t *d_out[NSLOT];
  uint32_t *d_len[NSLOT]; /* per-packet lengths / hints of a host batch chunk */
  uint8_t *h_stage[NSLOT];
  uint64_t *h_off[NSLOT];
  uint16_t *h_out[NSLOT];
  uint32_t slot_frames; /* offsets / results capacity per slot */
  /* the open batch: frames recorded since the last submit */
  uint8_t **pend_ip;
  uint8_t **pend_l4;
  uint32_t npend;
  /* flushes in flight: tickets done_ticket + 1 .. next_ticket, oldest first,
   * all on stream st[0] in ticket order */
  struct flush_slot fl[NSLOT];
  uint32_t next_ticket, done_ticket;
  /* completion words in coherent pinned memory, one per slot, 64 B apart: a
   * one-lane kernel stores the ticket after the flush's work
   * (tasx_launch_post_done); the caller polls them instead of
   * hipStreamSynchronize (~3.5 us less per flush) */
  uint32_t *h_done, *d_done;
  uint32_t *d_count; /* per slot: blocks finished (flush kernels posting their own word) */
  /* zero-copy frame region (tasx_ctx_register_frames) */
  uint8_t *zc_host;
  uint8_t *zc_dev;
  size_t zc_bytes;
  int zc_registered; /* we called hipHostRegister on it */
  /* the app's shared-memory region (tasx_ctx_register_shm): TX segment
   * payload sources for tasx_server_tx_segments */
  uint8_t *shm_host;
  uint8_t *shm_dev;
  size_t shm_bytes;
  int shm_registered;
  uint32_t n_zerocopy_flushes, n_staged_flushes;
  /* shared feeder (tasx_ctx_use_feeder): zero-copy batches go to the GPU's
   * feeder thread through a single-producer / single-consumer queue */
  struct feeder *fd;
  struct fbatch *fq;  /* FQ batch slots */
  uint32_t fq_head;   /* batches queued (this context's thread, release) */
  uint32_t fq_tail;   /* batches taken (the feeder, release) */
  uint32_t fd_done;   /* the last of its tickets the feeder has completed (release) */
  uint32_t local_last; /* the last ticket this thread launched itself */
  uint32_t n_feeder_flushes;
  /* flush server (tasx_ctx_use_server): batches go to ring (context id) of the
   * GPU's persistent server kernel; no HIP call on submit */
  struct fserver *sv;
  uint32_t sv_pos;      /* next ring position to fill */
  uint32_t sv_done_pos; /* positions the server has finished (as last seen) */
  uint32_t sv_ticket[TASX_SRV_RING]; /* ticket of the batch at each ring position */
  uint32_t n_server_flushes;
  int sv_err; /* the server flagged a frame of this context (sticky until detach) */
  uint64_t sv_batches, sv_frames; /* since attach (this thread's own counters: no shared line per flush) */
  /* frames and TX segments a failed flush left unfinished, handed back by
   * tasx_take_unfinished / _segs (ctx_settle fills them) */
  tasx_frame_ref *unf;
  uint32_t unf_n, unf_cap, unf_pos;
  tasx_tx_seg *unf_seg;
  uint32_t unf_seg_n, unf_seg_cap, unf_seg_pos;
  uint32_t unf_lost; /* frames / segments the store could not hold (no memory): reported, never silent */
};

#define DONE_STRIDE 16u /* uint32 words between completion words (64 B) */

static struct tasx_ctx g_ctx[TASX_MAX_CTX];
/* the calling thread's context (tasx_set_thread_ctx), for TASX_CTX_SELF */
static __thread unsigned t_ctx = TASX_CTX_SELF;

static struct tasx_ctx *get_ctx(unsigned id)
{
  if (id == TASX_CTX_SELF)
    id = t_ctx;
  if (id >= TASX_MAX_CTX || !g_ctx[id].in_use)
    return NULL;
  return &g_ctx[id];
}

int tasx_set_thread_ctx(unsigned ctx_id)
{
  if (ctx_id != TASX_CTX_SELF && ctx_id >= TASX_MAX_CTX)
    return set_err(-EINVAL, "ctx id %u >= %u", ctx_id, TASX_MAX_CTX);
  t_ctx = ctx_id; /* TASX_CTX_SELF unbinds */
  return 0;
}

int tasx_thread_ctx(void)
{
  if (t_ctx == TASX_CTX_SELF)
    return set_err(-EINVAL, "no context bound to this thread");
  return (int) t_ctx;
}

/* ticket order with wrap-around: a at or before b */
static int ticket_le(uint32_t a, uint32_t b)
{
  return (int32_t) (a - b) <= 0;
}

/* Host ranges this library pinned (hipHostRegister) for contexts' frame and
 * shared-memory regions, reference-counted: every core registers the same
 * tas_shm, and the pin must outlive every context that
 * maps it, not only the first registrant's. */
#define MAX_PINS (2u * TASX_MAX_CTX)
static struct pin {
  uint8_t *base;
  size_t bytes;
  uint32_t refs;
} g_pins[MAX_PINS];
static pthread_mutex_t g_pins_mu = PTHREAD_MUTEX_INITIALIZER;

/* The device address of [base, base + bytes): a range inside one this library
 * pinned takes a reference on that pin (*owned = 1); memory pinned elsewhere
 * (tasx_host_alloc, hipHostMalloc) is used as it is (*owned = 0); anything
 * else is pinned here (*owned = 1). */
static int pin_acquire(uint8_t *base, size_t bytes, void **dev, int *owned)
{
  hipError_t e;
  int rc = 0;
  *owned = 0;
  pthread_mutex_lock(&g_pins_mu);
  for (uint32_t k = 0; k < MAX_PINS; k++) {
    struct pin *q = &g_pins[k];
    if (q->refs && base >= q->base && base + bytes <= q->base + q->bytes) {
      if ((e = hipHostGetDevicePointer(dev, base, 0)) != hipSuccess) {
        rc = hip_err(e, "hipHostGetDevicePointer");
      } else {
        q->refs++;
        *owned = 1;
      }
      pthread_mutex_unlock(&g_pins_mu);
      return rc;
    }
    if (q->refs && base < q->base + q->bytes && base + bytes > q->base) {
      /* overlapping a pin of this library without lying inside it: HIP would
       * map the part inside the pin alone (hipHostGetDevicePointer succeeds
       * for its start), and the pin's release would unmap it under this
       * context */
      pthread_mutex_unlock(&g_pins_mu);
      return set_err(-EINVAL, "host range [%p, +%zu) overlaps a region pinned by another context ([%p, +%zu)) "
                     "without lying inside it: register the larger region first", (void *) base, bytes,
                     (void *) q->base, q->bytes);
    }
  }
  if (hipHostGetDevicePointer(dev, base, 0) == hipSuccess) {
    pthread_mutex_unlock(&g_pins_mu);
    return 0;
  }
  (void) hipGetLastError();
  uint32_t k = 0;
  while (k < MAX_PINS && g_pins[k].refs)
    k++;
  if (k == MAX_PINS)
    rc = set_err(-ENOMEM, "more than %u pinned regions", MAX_PINS);
  else if ((e = hipHostRegister(base, bytes, hipHostRegisterMapped)) !=
           hipSuccess)
    rc = hip_err(e, "hipHostRegister");
  else if ((e = hipHostGetDevicePointer(dev, base, 0)) != hipSuccess) {
    hipHostUnregister(base);
    rc = hip_err(e, "hipHostGetDevicePointer");
  } else {
    g_pins[k] = (struct pin){base, bytes, 1u};
    *owned = 1;
  }
  pthread_mutex_unlock(&g_pins_mu);
  return rc;
}

/* drop the reference pin_acquire took for a range starting at base */
static void pin_release(uint8_t *base)
{
  pthread_mutex_lock(&g_pins_mu);
  for (uint32_t k = 0; k < MAX_PINS; k++) {
    struct pin *q = &g_pins[k];
    if (q->refs && base >= q->base && base < q->base + q->bytes) {
      if (--q->refs == 0) {
        hipHostUnregister(q->base);
        q->base = NULL;
        q->bytes = 0;
      }
      break;
    }
  }
  pthread_mutex_unlock(&g_pins_mu);
}

static void ctx_release(struct tasx_ctx *c)
{
  int s;
  for (s = 0; s < NSLOT; s++) {
    if (c->st[s])
      hipStreamDestroy(c->st[s]);
    if (c->d_buf[s])
      hipFree(c->d_buf[s]);
    if (c->d_off[s])
      hipFree(c->d_off[s]);
    if (c->d_out[s])
      hipFree(c->d_out[s]);
    if (c->d_len[s])
      hipFree(c->d_len[s]);
    if (c->h_stage[s])
      hipHostFree(c->h_stage[s]);
    if (c->h_off[s])
      hipHostFree(c->h_off[s]);
    if (c->h_out[s])
      hipHostFree(c->h_out[s]);
    if (c->fl[s].h_flen)
      hipHostFree(c->fl[s].h_flen);
    free(c->fl[s].ip);
    free(c->fl[s].l4);
  }
  if (c->h_done)
    hipHostFree(c->h_done);
  if (c->d_count)
    hipFree(c->d_count);
  if (c->zc_registered)
    pin_release(c->zc_host);
  if (c->shm_registered)
    pin_release(c->shm_host);
  free(c->pend_ip);
  free(c->pend_l4);
  free(c->fq);
  free(c->unf);
  free(c->unf_seg);
  memset(c, 0, sizeof(*c));
}

int tasx_ctx_init(unsigned ctx_id, int device, size_t max_batch_bytes)
{
  struct tasx_ctx *c;
  int s, ndev = 0;
  hipError_t e;

  if (ctx_id == TASX_CTX_SELF)
    ctx_id = t_ctx;
  if (ctx_id >= TASX_MAX_CTX)
    return set_err(-EINVAL, "ctx id %u >= %u", ctx_id, TASX_MAX_CTX);
  c = &g_ctx[ctx_id];
  if (c->in_use)
    return set_err(-EINVAL, "ctx %u already initialised", ctx_id);
  e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess)
    return hip_err(e, "hipGetDeviceCount");
  if (device < 0 || device >= ndev)
    return set_err(-ENODEV, "device %d not present (%d GPUs)", device, ndev);
  memset(c, 0, sizeof(*c));
  c->device = device;
  c->slot_bytes = max_batch_bytes ? max_batch_bytes : DEFAULT_SLOT_BYTES;
  /* one result pair / offset per 64 staged bytes is the densest TAS batch
   * (minimum frame 60 B) */
  c->slot_frames = (uint32_t) (c->slot_bytes / 64 + 1);
  HIPCHK(hipSetDevice(device));
  for (s = 0; s < NSLOT; s++) {
    struct flush_slot *f = &c->fl[s];
    if ((e = hipStreamCreateWithFlags(&c->st[s], hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc((void **) &c->d_buf[s], c->slot_bytes)) != hipSuccess ||
        (e = hipMalloc((void **) &c->d_off[s], (size_t) c->slot_frames * 8)) != hipSuccess ||
        (e = hipMalloc((void **) &c->d_out[s], (size_t) c->slot_frames * 4)) != hipSuccess ||
        (e = hipMalloc((void **) &c->d_len[s], (size_t) c->slot_frames * 4)) != hipSuccess ||
        (e = hipHostMalloc((void **) &c->h_stage[s], c->slot_bytes, 0)) != hipSuccess ||
        (e = hipHostMalloc((void **) &c->h_off[s], (size_t) c->slot_frames * 8, 0)) != hipSuccess ||
        (e = hipHostMalloc((void **) &c->h_out[s], (size_t) c->slot_frames * 4, 0)) != hipSuccess ||
        (e = hipHostMalloc((void **) &f->h_flen, (size_t) c->slot_frames * 4, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &f->d_flen, f->h_flen, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &f->d_off, c->h_off[s], 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &f->d_stage, c->h_stage[s], 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &f->d_out, c->h_out[s], 0)) != hipSuccess) {
      ctx_release(c);
      return hip_err(e, "tasx_ctx_init allocation");
    }
    f->ip = calloc(c->slot_frames, sizeof(*f->ip));
    f->l4 = calloc(c->slot_frames, sizeof(*f->l4));
    if (!f->ip || !f->l4) {
      ctx_release(c);
      return set_err(-ENOMEM, "tasx_ctx_init: out of host memory");
    }
  }
  if ((e = hipHostMalloc((void **) &c->h_done, 4u * DONE_STRIDE * NSLOT, hipHostMallocCoherent)) != hipSuccess ||
      (e = hipHostGetDevicePointer((void **) &c->d_done, c->h_done, 0)) != hipSuccess) {
    ctx_release(c);
    return hip_err(e, "tasx_ctx_init completion words");
  }
  memset(c->h_done, 0, 4u * DONE_STRIDE * NSLOT);
  if ((e = hipMalloc((void **) &c->d_count, 4u * DONE_STRIDE * NSLOT)) != hipSuccess ||
      (e = hipMemset(c->d_count, 0, 4u * DONE_STRIDE * NSLOT)) != hipSuccess) {
    ctx_release(c);
    return hip_err(e, "tasx_ctx_init completion counters");
  }
  c->pend_ip = calloc(c->slot_frames, sizeof(*c->pend_ip));
  c->pend_l4 = calloc(c->slot_frames, sizeof(*c->pend_l4));
  if (!c->pend_ip || !c->pend_l4) {
    ctx_release(c);
    return set_err(-ENOMEM, "tasx_ctx_init: out of host memory");
  }
  c->in_use = 1;
  return 0;
}

static int flush_wait(struct tasx_ctx *c, uint32_t ticket);
static int server_defer_release(struct tasx_ctx *c);
static int free_guard_enter(const char *what);
static void free_guard_exit(void);

int tasx_ctx_destroy(unsigned ctx_id)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  hipSetDevice(c->device);
  if (c->fd)
    (void) tasx_ctx_use_feeder(ctx_id, 0);
  if (c->sv)
    (void) tasx_ctx_use_server(ctx_id, 0);
  (void) flush_wait(c, c->next_ticket);
  for (int s = 0; s < NSLOT; s++)
    hipStreamSynchronize(c->st[s]);
  /* hipFree / hipHostFree / hipHostUnregister wait for every stream of the
   * device, the flush server's too: while one runs, the context's memory is
   * handed to it and released when it stops */
  if (!server_defer_release(c))
    ctx_release(c);
  return 0;
}

/* ---------------------------------------------------------------------- */
/* end-to-end host batches: chunk -> H2D -> kernel -> D2H, NSLOT in flight
 * (they share the slots' pinned buffers with the flushes: in-flight flushes
 * complete first) */

struct chunk_job {
  uint32_t first, cnt;
};

/* An error after the first chunk's launch leaves earlier chunks running on
 * the slot streams, reading and writing the slots' pinned buffers: wait for
 * them all before returning, so no later call (or flush) reuses a buffer a
 * stale chunk still uses.  Returns rc. */
static int host_offs_fail(struct tasx_ctx *c, int rc)
{
  for (int s = 0; s < NSLOT; s++)
    (void) hipStreamSynchronize(c->st[s]);
  (void) hipGetLastError();
  return rc;
}
#define HIPCHK_DRAIN(c, call)                          \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess)                              \
      return host_offs_fail((c), hip_err(e_, #call));  \
  } while (0)


static void finish_tcp4_chunk(struct tasx_ctx *c, int s, const struct chunk_job *j,
    uint8_t *base, uint64_t stride, uint32_t ip_off, uint32_t l4_off,
    uint16_t *out, uint32_t flags)
{
  const uint16_t *r = c->h_out[s];
  if (out)
    memcpy(out + 2 * (size_t) j->first, r, (size_t) j->cnt * 4);
  if (flags & TASX_F_INPLACE) {
    for (uint32_t k = 0; k < j->cnt; k++) {
      uint8_t *f = base + (uint64_t) (j->first + k) * stride;
      memcpy(f + ip_off + 10, &r[2 * k], 2);
      memcpy(f + l4_off + 16, &r[2 * k + 1], 2);
    }
  }
}

int tasx_tcp4_cksum_batch_host(unsigned ctx_id, void *base, uint64_t stride,
    uint32_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out,
    uint32_t flags)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  struct chunk_job jobs[NSLOT];
  uint32_t per, first, k = 0;
  int rc = 0;

  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (n == 0)
    return 0;
  if (!base || stride == 0 || stride > c->slot_bytes || (!out && !(flags & TASX_F_INPLACE)))
    return set_err(-EINVAL, "tcp4 host batch: bad base/stride/out");
  if ((uint64_t) l4_off + 18 > stride || (uint64_t) ip_off + 20 > stride)
    return set_err(-EINVAL, "tcp4 host batch: headers exceed the stride");
  if (flags & ~TASX_F_INPLACE)
    return set_err(-EINVAL, "tcp4 host batch: unknown flags 0x%x", flags);
  HIPCHK(hipSetDevice(c->device));
  if ((rc = flush_wait(c, c->next_ticket)) != 0)
    return rc;
  per = (uint32_t) (c->slot_bytes / stride);
  if (per > c->slot_frames)
    per = c->slot_frames;
  for (first = 0; first < n; first += per, k++) {
    const int s = (int) (k % NSLOT);
    tasx_tcp4_params p;
    if (k >= NSLOT) {
      HIPCHK_DRAIN(c, hipStreamSynchronize(c->st[s]));
      finish_tcp4_chunk(c, s, &jobs[s], (uint8_t *) base, stride, ip_off, l4_off, out, flags);
    }
    jobs[s].first = first;
    jobs[s].cnt = (n - first < per) ? n - first : per;
    HIPCHK_DRAIN(c, hipMemcpyAsync(c->d_buf[s], (uint8_t *) base + (uint64_t) first * stride,
        (size_t) jobs[s].cnt * stride, hipMemcpyHostToDevice, c->st[s]));
    memset(&p, 0, sizeof(p));
    p.base = c->d_buf[s];
    p.off = NULL;
    p.out = c->d_out[s];
    p.stride = stride;
    p.n = jobs[s].cnt;
    p.ip_off = ip_off;
    p.l4_off = l4_off;
    p.flags = 0;
    /* whole mbuf rooms were copied: each frame's stride slot may be read */
    p.room = stride <= 0xffffffffull ? (uint32_t) stride : 0u;

    if (tasx_launch_tcp4(&p, g_variant, c->st[s]) != 0)
      return host_offs_fail(c, hip_err(hipGetLastError(), "tcp4_cksum_kernel launch"));
    HIPCHK_DRAIN(c, hipMemcpyAsync(c->h_out[s], c->d_out[s], (size_t) jobs[s].cnt * 4,
        hipMemcpyDeviceToHost, c->st[s]));
  }
  /* drain: the last min(k, NSLOT) chunks, in submission order */
  for (uint32_t d = (k > NSLOT) ? k - NSLOT : 0; d < k; d++) {
    const int s = (int) (d % NSLOT);
    HIPCHK_DRAIN(c, hipStreamSynchronize(c->st[s]));
    finish_tcp4_chunk(c, s, &jobs[s], (uint8_t *) base, stride, ip_off, l4_off, out, flags);
  }
  return rc;
}

int tasx_raw_cksum_batch_host(unsigned ctx_id, const void *base,
    uint64_t stride, uint32_t len0, uint32_t n, uint16_t *out)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  struct chunk_job jobs[NSLOT];
  uint32_t per, first, k = 0;
  int rc;

  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (n == 0)
    return 0;
  if (!base || !out || len0 > TASX_RAW_MAX_LEN || stride < len0 || stride > c->slot_bytes)
    return set_err(-EINVAL, "raw host batch: bad base/out/stride/len0");
  HIPCHK(hipSetDevice(c->device));
  if ((rc = flush_wait(c, c->next_ticket)) != 0)
    return rc;
  per = (uint32_t) (c->slot_bytes / (stride ? stride : 1));
  if (per > c->slot_frames)
    per = c->slot_frames;
  if (per == 0)
    return set_err(-EINVAL, "raw host batch: stride larger than a slot");
  for (first = 0; first < n; first += per, k++) {
    const int s = (int) (k % NSLOT);
    tasx_raw_params p;
    if (k >= NSLOT) {
      const hipError_t e = hipStreamSynchronize(c->st[s]);
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
      memcpy(out + jobs[s].first, c->h_out[s], (size_t) jobs[s].cnt * 2);
    }
    jobs[s].first = first;
    jobs[s].cnt = (n - first < per) ? n - first : per;
    /* the last packet of a chunk only needs len0 bytes */
    HIPCHK_DRAIN(c, hipMemcpyAsync(c->d_buf[s], (const uint8_t *) base + (uint64_t) first * stride,
        (size_t) (jobs[s].cnt - 1) * stride + len0, hipMemcpyHostToDevice, c->st[s]));
    p.base = c->d_buf[s];
    p.off = NULL;
    p.len = NULL;
    p.out = c->d_out[s];
    p.stride = stride;
    p.len0 = len0;
    p.n = jobs[s].cnt;
    if (tasx_launch_raw(&p, g_variant, c->st[s]) != 0)
      return host_offs_fail(c, hip_err(hipGetLastError(), "raw_cksum_kernel launch"));
    HIPCHK_DRAIN(c, hipMemcpyAsync(c->h_out[s], c->d_out[s], (size_t) jobs[s].cnt * 2,
        hipMemcpyDeviceToHost, c->st[s]));
  }
  for (uint32_t d = (k > NSLOT) ? k - NSLOT : 0; d < k; d++) {
    const int s = (int) (d % NSLOT);
    const hipError_t e = hipStreamSynchronize(c->st[s]);
    if (e != hipSuccess)
      return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
    memcpy(out + jobs[s].first, c->h_out[s], (size_t) jobs[s].cnt * 2);
  }
  return 0;
}

/* ---------------------------------------------------------------------- */
/* end-to-end host batches over scattered packets: (base, off[], len[]) -> u16
 * (TAS's frames are mbufs scattered over a per-core
 * mempool, tas/fast/network.c:320-330).
 *   staged: the CPU gathers only the bytes summed into the slot's pinned
 *     staging (16-byte aligned records), one hipMemcpyAsync H2D of the records
 *     and their descriptors, the kernel from HBM, one D2H of the results;
 *     while the GPU works on chunk k the CPU gathers chunk k + 1.
 *   zero-copy (TASX_F_ZEROCOPY): the packets stay where they are, in pinned or
 *     registered memory; the kernel reads them over PCIe (only the chunks
 *     holding summed bytes) at base's device address + off[i], descriptors and
 *     results through the slot's mapped pinned buffers. */

static uint32_t staged_l4(uint32_t tl);
static size_t staged_rec(uint32_t tl);

static uint8_t *host_pkt(const void *base, const uint64_t *off, uint32_t i)
{
  return (uint8_t *) (base ? (uintptr_t) base + off[i] : (uintptr_t) off[i]);
}

/* the device's address of pinned / registered host memory at base */
static int zc_base(const void *base, uint8_t **dev, const char *what)
{
  void *d = NULL;
  if (!base)
    return set_err(-EINVAL, "%s: zero-copy needs a base in pinned or registered memory", what);
  if (hipHostGetDevicePointer(&d, (void *) base, 0) != hipSuccess) {
    (void) hipGetLastError();
    return set_err(-EINVAL, "%s: base %p is not pinned or registered memory", what, base);
  }
  *dev = (uint8_t *) d;
  return 0;
}

struct host_job {
  uint32_t first, cnt;
};

/* Zero-copy reads stay inside the allocation base lies in (or the
 * context's registered frame region): [base + lo, base + hi) must fit it.
 * Unknown extents (memory the runtime does not describe) are not checked. */
static int zc_extent_ok(const struct tasx_ctx *c, const void *base, uint64_t hi, const char *what)
{
  void *ab = NULL;
  size_t asz = 0;
  const uint8_t *b = (const uint8_t *) base;
  if (hipMemGetAddressRange((hipDeviceptr_t *) &ab, &asz, (hipDeviceptr_t) base) == hipSuccess && ab && asz) {
    if ((const uint8_t *) ab <= b && b + hi <= (const uint8_t *) ab + asz)
      return 0;
    return set_err(-EINVAL, "%s: packets reach %llu bytes past base, beyond its %zu-byte allocation", what,
                   (unsigned long long) hi, asz);
  }
  (void) hipGetLastError();
  if (c->zc_host && b >= c->zc_host && b < c->zc_host + c->zc_bytes && b + hi > c->zc_host + c->zc_bytes)
    return set_err(-EINVAL, "%s: packets reach past the registered frame region", what);
  return 0;
}

/* results of chunk j in slot s: to out (and into the frames, TCP4 in place) */
static void finish_tcp4_offs(struct tasx_ctx *c, int s, const struct host_job *j, void *base,
    const uint64_t *off, uint32_t ip_off, uint32_t l4_off, uint16_t *out, uint32_t flags)
{
  const uint16_t *r = c->h_out[s];
  if (out)
    memcpy(out + 2 * (size_t) j->first, r, (size_t) j->cnt * 4);
  if ((flags & TASX_F_INPLACE) && !(flags & TASX_F_ZEROCOPY)) { /* zero-copy kernels store in place */
    for (uint32_t k = 0; k < j->cnt; k++) {
      uint8_t *f = host_pkt(base, off, j->first + k);
      memcpy(f + ip_off + 10, &r[2 * k], 2);
      memcpy(f + l4_off + 16, &r[2 * k + 1], 2);
    }
  }
}

int tasx_tcp4_cksum_batch_host_offs(unsigned ctx_id, void *base, const uint64_t *off,
    const uint32_t *flen, uint32_t n, uint32_t ip_off, uint32_t l4_off, uint16_t *out,
    uint32_t flags)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  struct host_job jobs[NSLOT];
  const int zc = (flags & TASX_F_ZEROCOPY) != 0;
  uint8_t *dbase = NULL;
  uint32_t first = 0, k = 0;
  int rc;

  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (n == 0)
    return 0;
  if (!off || (!out && !(flags & TASX_F_INPLACE)) || ((uintptr_t) out & 3u))
    return set_err(-EINVAL, "tcp4 host offs batch: NULL off/out, or out not 4-byte aligned");
  if (flags & ~(TASX_F_INPLACE | TASX_F_ZEROCOPY))
    return set_err(-EINVAL, "tcp4 host offs batch: unknown flags 0x%x", flags);
  if (l4_off < ip_off + 20u || l4_off > 0xffffu)
    return set_err(-EINVAL, "tcp4 host offs batch: need ip_off + 20 <= l4_off <= 65535");
  HIPCHK(hipSetDevice(c->device));
  if (zc && (rc = zc_base(base, &dbase, "tcp4 host offs batch")) != 0)
    return rc;
  if (zc) {
    /* the kernels read a frame's whole 16-byte chunks up to its hint (or its
     * header when no hint is given; TX frames' total_length is trusted, as
     * in the _dev forms) */
    uint64_t hi = 0;
    for (uint32_t i = 0; i < n; i++) {
      const uint64_t e = off[i] + (flen && flen[i] > ip_off + 20u ? flen[i] : ip_off + 20u) + 15u;
      hi = e > hi ? e : hi;
    }
    if ((rc = zc_extent_ok(c, base, hi, "tcp4 host offs batch")) != 0)
      return rc;
  } else {
    /* before anything is launched: every record fits a slot, and with frame
     * lengths given, every datagram lies inside its frame (the gather copies
     * ip_off + total_length bytes) */
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t *ip = host_pkt(base, off, i) + ip_off;
      const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
      if (staged_rec(tl) > c->slot_bytes)
        return set_err(-EINVAL, "tcp4 host offs batch: frame %u does not fit a %zu-byte slot", i, c->slot_bytes);
      if (flen && (uint64_t) ip_off + (tl > 20u ? tl : 20u) > flen[i])
        return set_err(-EINVAL, "tcp4 host offs batch: frame %u: ip_off + total_length %u exceeds its length %u", i,
                       tl, flen[i]);
    }
  }
  if ((rc = flush_wait(c, c->next_ticket)) != 0)
    return rc;
  while (first < n) {
    const int s = (int) (k % NSLOT);
    struct flush_slot *f = &c->fl[s];
    tasx_tcp4_params p;
    uint32_t cnt = 0;
    if (k >= NSLOT) {
      const hipError_t e = hipStreamSynchronize(c->st[s]);
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
      finish_tcp4_offs(c, s, &jobs[s], base, off, ip_off, l4_off, out, flags);
    }
    memset(&p, 0, sizeof(p));
    p.l4_off = l4_off;
    if (zc) {
      /* descriptors into the slot's mapped pinned memory; the kernel reads
       * the frames where they are and writes the results to h_out */
      cnt = n - first < c->slot_frames ? n - first : c->slot_frames;
      memcpy(c->h_off[s], off + first, (size_t) cnt * 8);
      if (flen)
        memcpy(f->h_flen, flen + first, (size_t) cnt * 4);
      p.base = dbase;
      p.off = f->d_off;
      p.flen = flen ? f->d_flen : NULL;
      p.out = f->d_out;
      p.ip_off = ip_off;
      p.flags = flags & TASX_F_INPLACE;
    } else {
      /* TAS-layout records as the staged flush builds them: 14 unread lead
       * bytes, the 20-byte IPv4 header at 14 mod 16, the L4 segment after it
       * (the sums are relative to the header / segment start) */
      size_t pos = 0;
      uint32_t rec0 = 0, tl0 = 0, uniform = 1;
      while (first + cnt < n && cnt < c->slot_frames) {
        const uint8_t *fr = host_pkt(base, off, first + cnt);
        const uint8_t *ip = fr + ip_off;
        const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
        const size_t rec = staged_rec(tl);
        if (pos + rec > c->slot_bytes)
          break;
        memcpy(c->h_stage[s] + pos + TASX_TAS_IP_OFF, ip, 20);
        memcpy(c->h_stage[s] + pos + TASX_TAS_IP_OFF + 20, fr + l4_off, staged_l4(tl));
        c->h_off[s][cnt] = pos;
        f->h_flen[cnt] = TASX_TAS_IP_OFF + (tl < 20 ? 20 : tl);
        if (cnt == 0) {
          rec0 = (uint32_t) rec;
          tl0 = tl;
        } else if (rec != rec0 || tl != tl0) {
          uniform = 0;
        }
        pos += rec;
        cnt++;
      }
      if (cnt == 0) /* checked up front; kept as a guard */
        return host_offs_fail(c, set_err(-EINVAL, "tcp4 host offs batch: frame %u does not fit a %zu-byte slot",
                                         first, c->slot_bytes));
      hipError_t e = hipMemcpyAsync(c->d_buf[s], c->h_stage[s], pos, hipMemcpyHostToDevice, c->st[s]);
      p.base = c->d_buf[s];
      if (uniform && tl0 >= 20) {
        /* one record size: stride mode with a uniform hint (the headline and
         * TSO kernels) */
        p.stride = rec0;
        p.flen0 = f->h_flen[0];
      } else {
        if (e == hipSuccess)
          e = hipMemcpyAsync(c->d_off[s], c->h_off[s], (size_t) cnt * 8, hipMemcpyHostToDevice, c->st[s]);
        if (e == hipSuccess)
          e = hipMemcpyAsync(c->d_len[s], f->h_flen, (size_t) cnt * 4, hipMemcpyHostToDevice, c->st[s]);
        p.off = c->d_off[s];
        p.flen = c->d_len[s];
      }
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipMemcpyAsync"));
      p.out = c->d_out[s];
      p.ip_off = TASX_TAS_IP_OFF;
      p.l4_off = TASX_TAS_L4_OFF;
    }
    p.n = cnt;
    if (tasx_launch_tcp4(&p, g_variant, c->st[s]) != 0)
      return host_offs_fail(c, hip_err(hipGetLastError(), "tcp4_cksum_kernel launch"));
    if (!zc) {
      const hipError_t e = hipMemcpyAsync(c->h_out[s], c->d_out[s], (size_t) cnt * 4, hipMemcpyDeviceToHost, c->st[s]);
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipMemcpyAsync"));
    }
    jobs[s].first = first;
    jobs[s].cnt = cnt;
    first += cnt;
    k++;
  }
  for (uint32_t d = (k > NSLOT) ? k - NSLOT : 0; d < k; d++) {
    const int s = (int) (d % NSLOT);
    const hipError_t e = hipStreamSynchronize(c->st[s]);
    if (e != hipSuccess)
      return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
    finish_tcp4_offs(c, s, &jobs[s], base, off, ip_off, l4_off, out, flags);
  }
  return 0;
}

int tasx_raw_cksum_batch_host_offs(unsigned ctx_id, const void *base, const uint64_t *off,
    const uint32_t *len, uint32_t len0, uint32_t n, uint16_t *out, uint32_t flags)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  struct host_job jobs[NSLOT];
  const int zc = (flags & TASX_F_ZEROCOPY) != 0;
  uint8_t *dbase = NULL;
  uint32_t first = 0, k = 0;
  int rc;

  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (n == 0)
    return 0;
  if (!off || !out)
    return set_err(-EINVAL, "raw host offs batch: NULL off/out");
  if (flags & ~TASX_F_ZEROCOPY)
    return set_err(-EINVAL, "raw host offs batch: unknown flags 0x%x", flags);
  if (!len && len0 > TASX_RAW_MAX_LEN)
    return set_err(-EINVAL, "raw host offs batch: len0 %u > %u", len0, TASX_RAW_MAX_LEN);
  for (uint32_t i = 0; len && i < n; i++)
    if (len[i] > TASX_RAW_MAX_LEN)
      return set_err(-EINVAL, "raw host offs batch: len[%u] = %u > %u", i, len[i], TASX_RAW_MAX_LEN);
  HIPCHK(hipSetDevice(c->device));
  if (zc && (rc = zc_base(base, &dbase, "raw host offs batch")) != 0)
    return rc;
  {
    /* before anything is launched: every record fits a slot (staged), every
     * packet's chunks inside base's allocation (zero-copy) */
    uint64_t hi = 0;
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t l = len ? len[i] : len0;
      if (!zc && (((size_t) l + 15) & ~(size_t) 15) > c->slot_bytes)
        return set_err(-EINVAL, "raw host offs batch: packet %u does not fit a %zu-byte slot", i, c->slot_bytes);
      const uint64_t e = off[i] + l + 15u;
      hi = e > hi ? e : hi;
    }
    if (zc && (rc = zc_extent_ok(c, base, hi, "raw host offs batch")) != 0)
      return rc;
  }
  if ((rc = flush_wait(c, c->next_ticket)) != 0)
    return rc;
  while (first < n) {
    const int s = (int) (k % NSLOT);
    struct flush_slot *f = &c->fl[s];
    tasx_raw_params p;
    uint32_t cnt = 0;
    if (k >= NSLOT) {
      const hipError_t e = hipStreamSynchronize(c->st[s]);
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
      memcpy(out + jobs[s].first, c->h_out[s], (size_t) jobs[s].cnt * 2);
    }
    memset(&p, 0, sizeof(p));
    if (zc) {
      cnt = n - first < c->slot_frames ? n - first : c->slot_frames;
      memcpy(c->h_off[s], off + first, (size_t) cnt * 8);
      if (len)
        memcpy(f->h_flen, len + first, (size_t) cnt * 4);
      p.base = dbase;
      p.off = f->d_off;
      p.len = len ? f->d_flen : NULL;
      p.len0 = len0;
      p.out = f->d_out;
    } else {
      /* only the summed bytes, each packet at a 16-byte aligned record (the
       * sum of a buffer does not depend on its address) */
      size_t pos = 0;
      while (first + cnt < n && cnt < c->slot_frames) {
        const uint32_t l = len ? len[first + cnt] : len0;
        const size_t rec = ((size_t) l + 15) & ~(size_t) 15;
        if (pos + rec > c->slot_bytes)
          break;
        memcpy(c->h_stage[s] + pos, host_pkt(base, off, first + cnt), l);
        c->h_off[s][cnt] = pos;
        f->h_flen[cnt] = l;
        pos += rec;
        cnt++;
      }
      if (cnt == 0) /* checked up front; kept as a guard */
        return host_offs_fail(c, set_err(-EINVAL, "raw host offs batch: packet %u does not fit a %zu-byte slot",
                                         first, c->slot_bytes));
      hipError_t e = hipSuccess;
      if (pos)
        e = hipMemcpyAsync(c->d_buf[s], c->h_stage[s], pos, hipMemcpyHostToDevice, c->st[s]);
      p.base = c->d_buf[s];
      if (len) {
        if (e == hipSuccess)
          e = hipMemcpyAsync(c->d_off[s], c->h_off[s], (size_t) cnt * 8, hipMemcpyHostToDevice, c->st[s]);
        if (e == hipSuccess)
          e = hipMemcpyAsync(c->d_len[s], f->h_flen, (size_t) cnt * 4, hipMemcpyHostToDevice, c->st[s]);
        p.off = c->d_off[s];
        p.len = c->d_len[s];
      } else { /* uniform length: stride mode over the records */
        p.stride = len0 ? ((uint64_t) len0 + 15) & ~(uint64_t) 15 : 16;
        p.len0 = len0;
      }
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipMemcpyAsync"));
      p.out = c->d_out[s];
    }
    p.n = cnt;
    if (tasx_launch_raw(&p, g_variant, c->st[s]) != 0)
      return host_offs_fail(c, hip_err(hipGetLastError(), "raw_cksum_kernel launch"));
    if (!zc) {
      const hipError_t e = hipMemcpyAsync(c->h_out[s], c->d_out[s], (size_t) cnt * 2, hipMemcpyDeviceToHost, c->st[s]);
      if (e != hipSuccess)
        return host_offs_fail(c, hip_err(e, "hipMemcpyAsync"));
    }
    jobs[s].first = first;
    jobs[s].cnt = cnt;
    first += cnt;
    k++;
  }
  for (uint32_t d = (k > NSLOT) ? k - NSLOT : 0; d < k; d++) {
    const int s = (int) (d % NSLOT);
    const hipError_t e = hipStreamSynchronize(c->st[s]);
    if (e != hipSuccess)
      return host_offs_fail(c, hip_err(e, "hipStreamSynchronize"));
    memcpy(out + jobs[s].first, c->h_out[s], (size_t) jobs[s].cnt * 2);
  }
  return 0;
}

/* ---------------------------------------------------------------------- */
/* deferred per-frame surface */

int tasx_defer_tcp4(unsigned ctx_id, void *frame, uint16_t ip_off, uint16_t l4_off)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!frame || l4_off < ip_off + 20u)
    return set_err(-EINVAL, "defer: NULL frame or l4_off < ip_off + 20");
  if (c->npend >= c->slot_frames)
    return set_err(-ENOSPC, "defer: %u frames pending", c->npend);
  c->pend_ip[c->npend] = (uint8_t *) frame + ip_off;
  c->pend_l4[c->npend] = (uint8_t *) frame + l4_off;
  c->npend++;
  return 0;
}

int tasx_tcp_checksums(unsigned ctx_id, void *nbh, void *p, uint32_t ip_s,
    uint32_t ip_d, uint16_t l3_paylen)
{
  /* the flag-off branch uses only the frame; ip_s/ip_d/l3_paylen feed the
   * offload branch (fast_flows.c:1062-1063), which stays in TAS */
  (void) nbh;
  (void) ip_s;
  (void) ip_d;
  (void) l3_paylen;
  return tasx_defer_tcp4(ctx_id, p, TASX_TAS_IP_OFF, TASX_TAS_L4_OFF);
}

int tasx_fast_flows_kernelxsums(unsigned ctx_id, void *nbh, void *p)
{
  (void) nbh;
  return tasx_defer_tcp4(ctx_id, p, TASX_TAS_IP_OFF, TASX_TAS_L4_OFF);
}

int tasx_pending(unsigned ctx_id)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  return (int) c->npend;
}

int tasx_ctx_register_frames(unsigned ctx_id, void *base, size_t bytes)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  void *dev = NULL;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!base || bytes == 0)
    return set_err(-EINVAL, "register_frames: empty region");
  if (c->zc_host)
    return set_err(-EINVAL, "ctx %u already has a frame region", ctx_id);
  HIPCHK(hipSetDevice(c->device));
  /* already pinned (tasx_host_alloc / hipHostMalloc, or by another context)?  else pin it */
  int rc = pin_acquire((uint8_t *) base, bytes, &dev, &c->zc_registered);
  if (rc)
    return rc;
  c->zc_host = (uint8_t *) base;
  c->zc_dev = (uint8_t *) dev;
  c->zc_bytes = bytes;
  return 0;
}

int tasx_ctx_register_shm(unsigned ctx_id, void *shm, size_t bytes)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  void *dev = NULL;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!shm || bytes == 0 || bytes >= (1ull << 32))
    return set_err(-EINVAL, "register_shm: empty region or not below 4 GiB");
  if (c->shm_host)
    return set_err(-EINVAL, "ctx %u already has a shared-memory region", ctx_id);
  HIPCHK(hipSetDevice(c->device));
  /* every core registers the same tas_shm: one pin, counted (pin_acquire) */
  int rc = pin_acquire((uint8_t *) shm, bytes, &dev, &c->shm_registered);
  if (rc)
    return rc;
  if ((uint64_t) (uintptr_t) dev + bytes >= (1ull << 48)) {
    if (c->shm_registered)
      pin_release((uint8_t *) shm);
    c->shm_registered = 0;
    return set_err(-EINVAL, "register_shm: device address beyond 48 bits");
  }
  c->shm_host = (uint8_t *) shm;
  c->shm_dev = (uint8_t *) dev;
  c->shm_bytes = bytes;
  return 0;
}

int tasx_ctx_stats(unsigned ctx_id, uint32_t *zerocopy_flushes, uint32_t *staged_flushes)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (zerocopy_flushes)
    *zerocopy_flushes = c->n_zerocopy_flushes;
  if (staged_flushes)
    *staged_flushes = c->n_staged_flushes;
  return 0;
}

/* Test support (libtasx_ab.so exports it as tasx_ab_ctx_set_tickets):
 * restart the context's tickets at `start` (nothing in flight), so a test can
 * run flushes across the 2^32 wrap.  Every completion word holds `start`,
 * which no upcoming ticket equals (as 0 does after tasx_ctx_init). */
int tasx_ctx_set_tickets_internal(unsigned ctx_id, uint32_t start)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (c->npend || c->fd || !ticket_le(c->next_ticket, c->done_ticket))
    return set_err(-EBUSY, "ctx %u has frames pending, flushes in flight or a feeder", ctx_id);
  for (int s = 0; s < NSLOT; s++)
    __atomic_store_n(c->h_done + DONE_STRIDE * (uint32_t) s, start, __ATOMIC_RELEASE);
  c->next_ticket = c->done_ticket = c->local_last = c->fd_done = start;
  return 0;
}

/* Complete every flush up to `upto` whose completion word has arrived, oldest
 * first (the staged path copies its results into the frames); returns 1 when
 * `upto` is complete, 0 if not yet. */
static void server_reap(struct tasx_ctx *c);

static int flush_reap(struct tasx_ctx *c, uint32_t upto)
{
  if (c->sv)
    server_reap(c);
  if (c->fd) { /* tickets the feeder completed (all of its tickets before them too) */
    const uint32_t fdone = __atomic_load_n(&c->fd_done, __ATOMIC_ACQUIRE);
    if (!ticket_le(fdone, c->done_ticket))
      c->done_ticket = fdone;
  }
  while (!ticket_le(upto, c->done_ticket)) {
    const uint32_t t = c->done_ticket + 1;
    struct flush_slot *f = &c->fl[t % NSLOT];
    volatile uint32_t *w = c->h_done + DONE_STRIDE * (t % NSLOT);
    if (*w != t)
      return 0;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (!f->zerocopy) {
      const uint16_t *r = c->h_out[t % NSLOT];
      for (uint32_t i = 0; i < f->n; i++) {
        memcpy(f->ip[i] + 10, &r[2 * i], 2);
        memcpy(f->l4[i] + 16, &r[2 * i + 1], 2);
      }
    }
    c->done_ticket = t;
  }
  return 1;
}

/* Spin until flush `ticket` (and every earlier one) is complete.  Every 4096
 * polls (a few microseconds) the stream is queried, so an error or a lost word
 * ends the wait instead of spinning on. */
static int feeder_error(const struct tasx_ctx *c);
static int server_health(const struct tasx_ctx *c);
static int server_err(const struct tasx_ctx *c);
static int server_alive(const struct tasx_ctx *c);

static int flush_wait(struct tasx_ctx *c, uint32_t ticket)
{
  uint32_t k = 0;
  int rc;
  while (!flush_reap(c, ticket)) {
    if (c->sv && c->sv_err)
      return server_err(c);
    if ((++k & 4095u) == 0 && c->fd && feeder_error(c))
      return set_err(-EIO, "flush: the feeder thread failed");
    if ((k & 4095u) == 0 && c->sv && (rc = server_health(c)) != 0)
      return rc;
    /* only server tickets outstanding: this context's stream has nothing to do */
    if ((k & 4095u) == 0 && c->sv && ticket_le(c->local_last, c->done_ticket))
      continue;
    /* only feeder tickets outstanding: this context's stream has nothing to do */
    if ((k & 4095u) == 0 && c->fd && ticket_le(c->local_last, c->done_ticket))
      continue;
    if ((k & 4095u) == 0) {
      hipError_t e = hipStreamQuery(c->st[0]);
      if (e == hipSuccess && !flush_reap(c, ticket))
        return set_err(-EIO, "flush: stream idle but flush %u not complete", c->done_ticket + 1);
      if (e != hipSuccess && e != hipErrorNotReady)
        return hip_err(e, "flush: hipStreamQuery");
    }
  }
  return c->sv && c->sv_err ? server_err(c) : 0;
}

static int zerocopy_ok(const struct tasx_ctx *c, uint32_t n)
{
  uint32_t i;
  if (!c->zc_host)
    return 0;
  for (i = 0; i < n; i++) {
    const uint8_t *ip = c->pend_ip[i];
    uint32_t tl;
    if (c->pend_l4[i] != ip + 20 || ip < c->zc_host || ip + 20 > c->zc_host + c->zc_bytes)
      return 0;
    tl = ((uint32_t) ip[2] << 8) | ip[3];
    /* rows read whole 16-byte chunks: up to 15 bytes past the datagram */
    if (ip + (tl < 38 ? 38 : tl) + 16 > c->zc_host + c->zc_bytes)
      return 0;
  }
  return 1;
}

/* staged record of a frame with ip.total_length tl: the L4 bytes copied (the
 * kernel reads the checksum field of short segments too) and the record size
 * (14-byte lead + IPv4 header + L4, 16-byte multiple) */
static uint32_t staged_l4(uint32_t tl)
{
  const uint32_t l4len = tl > 20 ? tl - 20 : 0;
  return l4len < 18 ? 18 : l4len;
}
static size_t staged_rec(uint32_t tl)
{
  return ((size_t) TASX_TAS_IP_OFF + 20 + staged_l4(tl) + 15) & ~(size_t) 15;
}

/* Post a completion word after the stream's earlier work (the one-lane
 * kernel; the command processor's hipStreamWriteValue32 measured no faster,
 * profiles/r02/INDEX.md) */
static int post_done(uint32_t *word, uint32_t seq, hipStream_t st)
{
  return tasx_launch_post_done(word, seq, st);
}

/* Submit the first `cnt` pending frames as flush `t` into slot t % NSLOT
 * (whose previous flush the caller has completed), and drop them from the
 * open batch.
 *   zero-copy: every frame in the registered region, TAS layout: the kernel
 *     reads the frames over PCIe (only the bytes it sums) and stores both
 *     fields in place; descriptors (frame-start offset, frame-length hint)
 *     from pinned memory.
 *   staged: [14-byte lead | 20-byte IPv4 header | L4 segment] of each frame
 *     gathered into the slot's pinned staging (16-byte aligned records, TAS's
 *     frame layout: the sums are relative to the header / segment start, so
 *     where a record sits does not change them); the kernel reads the records and writes the results to pinned
 *     memory directly (no copy-engine work), and the completion copies them
 *     into the frames. */
static int flush_launch(struct tasx_ctx *c, uint32_t t, uint32_t cnt, int zc)
{
  const int s = (int) (t % NSLOT);
  struct flush_slot *f = &c->fl[s];
  tasx_tcp4_params p;
  uint32_t i, lead = TASX_TAS_IP_OFF;
  memset(&p, 0, sizeof(p));
  p.n = cnt;
  p.off = f->d_off;
  p.flen = f->d_flen;
  if (zc) {
    /* frame starts (ip - 14) where the region holds them: the TAS-layout
     * kernels (tcp4_tas14_kernel<hints,offs>); else records at the header */
    for (i = 0; i < cnt && lead; i++)
      if (c->pend_ip[i] < c->zc_host + TASX_TAS_IP_OFF)
        lead = 0;
    for (i = 0; i < cnt; i++) {
      const uint8_t *ip = c->pend_ip[i];
      const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
      c->h_off[s][i] = (uint64_t) (ip - lead - c->zc_host);
      f->h_flen[i] = lead + (tl < 20 ? 20 : tl);
    }
    p.base = c->zc_dev;
    p.flags = TASX_F_INPLACE;
    c->n_zerocopy_flushes++;
  } else {
    size_t pos = 0;
    for (i = 0; i < cnt; i++) {
      const uint8_t *ip = c->pend_ip[i];
      const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
      /* TAS's frame layout in the slot: 14 bytes of (unread) lead, the IPv4
       * header at 14 mod 16, the L4 segment right after it */
      memcpy(c->h_stage[s] + pos + lead, ip, 20);
      memcpy(c->h_stage[s] + pos + lead + 20, c->pend_l4[i], staged_l4(tl));
      c->h_off[s][i] = pos;
      f->h_flen[i] = lead + (tl < 20 ? 20 : tl);
      pos += staged_rec(tl);
    }
    p.base = f->d_stage;
    p.out = f->d_out;
    c->n_staged_flushes++;
  }
  p.ip_off = lead;
  p.l4_off = lead + 20;
  memcpy(f->ip, c->pend_ip, (size_t) cnt * sizeof(*f->ip));
  memcpy(f->l4, c->pend_l4, (size_t) cnt * sizeof(*f->l4));
  f->n = cnt;
  f->zerocopy = zc;
  f->ticket = t;
  /* a failed launch leaves the frames pending (ctx_settle hands them back) */
  if (tasx_launch_tcp4(&p, g_variant, c->st[0]) != 0)
    return hip_err(hipGetLastError(), "tcp4_cksum_kernel launch");
  if (post_done(c->d_done + DONE_STRIDE * (uint32_t) s, t, c->st[0]) != 0)
    return hip_err(hipGetLastError(), "completion-word launch");
  c->local_last = t;
  c->next_ticket = t;
  if (cnt < c->npend) {
    memmove(c->pend_ip, c->pend_ip + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_ip));
    memmove(c->pend_l4, c->pend_l4 + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_l4));
  }
  c->npend -= cnt;
  return 0;
}

/* frames of the open batch whose staged records fit one slot */
static uint32_t staged_fit(const struct tasx_ctx *c, size_t *need)
{
  size_t pos = 0;
  uint32_t i;
  for (i = 0; i < c->npend; i++) {
    const uint8_t *ip = c->pend_ip[i];
    const size_t rec = staged_rec(((uint32_t) ip[2] << 8) | ip[3]);
    if (pos + rec > c->slot_bytes) {
      *need = rec;
      break;
    }
    pos += rec;
  }
  return i;
}

static int feeder_submit(struct tasx_ctx *c);
static int server_submit(struct tasx_ctx *c);

int tasx_flush_submit(unsigned ctx_id, uint32_t *ticket)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  int rc;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (c->fd && (rc = feeder_submit(c)) != 0)
    return rc;
  if (c->sv && (rc = server_submit(c)) != 0)
    return rc;
  if (c->npend > 0)
    HIPCHK(hipSetDevice(c->device));
  while (c->npend > 0) {
    const uint32_t t = c->next_ticket + 1;
    const int zc = zerocopy_ok(c, c->npend);
    size_t need = 0;
    const uint32_t cnt = zc ? c->npend : staged_fit(c, &need);
    if (cnt == 0)
      return set_err(-EINVAL, "flush: frame of %zu B exceeds the staging slot", need);
    /* the slot's previous flush (t - NSLOT) must be complete */
    if ((rc = flush_wait(c, t - NSLOT)) != 0)
      return rc;
    if ((rc = flush_launch(c, t, cnt, zc)) != 0)
      return rc;
  }
  if (ticket)
    *ticket = c->next_ticket;
  return 0;
}

int tasx_flush_poll(unsigned ctx_id, uint32_t ticket)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!ticket_le(ticket, c->next_ticket))
    return set_err(-EINVAL, "flush ticket %u not submitted (last %u)", ticket, c->next_ticket);
  const int done = flush_reap(c, ticket);
  if (c->sv && c->sv_err)
    return server_err(c);
  if (!done && c->sv) {
    const int rc = server_alive(c);
    if (rc)
      return rc;
  }
  return done;
}

int tasx_flush_wait(unsigned ctx_id, uint32_t ticket)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!ticket_le(ticket, c->next_ticket))
    return set_err(-EINVAL, "flush ticket %u not submitted (last %u)", ticket, c->next_ticket);
  return flush_wait(c, ticket);
}

int tasx_flush(unsigned ctx_id)
{
  uint32_t t;
  int rc = tasx_flush_submit(ctx_id, &t);
  return rc ? rc : tasx_flush_wait(ctx_id, t);
}

/* ---------------------------------------------------------------------- */
/* Shared feeder: one thread per GPU serves the zero-copy flushes of every
 * attached context with one launch per sweep.  A fast-path core hands its
 * batch over by copying the frame pointers into its own single-producer /
 * single-consumer queue (no lock, no HIP call); the feeder gathers every
 * queue, writes the descriptors (frame start, 14 + total_length) into pinned
 * memory, launches tcp4_tas14_kernel<hints,offs> over all of them (in place,
 * absolute device addresses) and, when the sweep's completion word arrives,
 * publishes each context's last ticket.  Two sweeps are in flight: the next
 * is gathered while one runs.  The launch and completion round trip (~13 us)
 * is paid once per sweep by the feeder's core, not once per batch by each
 * fast-path core. */

#define FQ 8u            /* batches queued per context */
#define FB_MAX 1024u     /* frames per queued batch */
#define SWEEP_MAX 32768u /* frames per launch */
#define SWEEP_REC 256u   /* (context, ticket) records per sweep */
#define NSWEEP 2u     /* sweeps in flight (4 measured no better: profiles/r02) */
#define NSWEEP_MAX 4u /* a power of two: sweep s uses buffer s % nsweep across the uint32 wrap */
#define MAX_DEVICES 64

struct fbatch {
  uint32_t ticket, n;
  uint8_t *ip[FB_MAX];
};

struct fsweep {
  uint64_t *h_off, *d_off;   /* frame start, absolute device address */
  uint32_t *h_flen, *d_flen; /* 14 + total_length */
  uint32_t n, nrec;
  uint16_t rec_ctx[SWEEP_REC];
  uint32_t rec_ticket[SWEEP_REC];
};

struct feeder {
  int device;
  int running; /* cleared by tasx_feeder_stop */
  int failed;  /* a HIP error in the feeder thread (sticky) */
  uint32_t attached; /* bit i: context i is served */
  uint32_t gathers;  /* gather passes done (a detaching context waits for two) */
  pthread_t thr;
  hipStream_t st;
  uint32_t *h_done, *d_done; /* one completion word per sweep buffer */
  uint32_t *d_count;         /* per sweep buffer: blocks finished (device memory) */
  uint32_t nsweep;           /* NSWEEP */
  struct fsweep sw[NSWEEP_MAX];
  uint64_t sweeps, frames;   /* statistics */
};

static struct feeder *g_feeder[MAX_DEVICES];
static pthread_mutex_t g_feeder_mu = PTHREAD_MUTEX_INITIALIZER;

static int feeder_error(const struct tasx_ctx *c)
{
  return __atomic_load_n(&c->fd->failed, __ATOMIC_ACQUIRE);
}

/* every frame in the context's registered region with its 14-byte lead and
 * the slack of whole-chunk reads (zerocopy_ok) */
static int feeder_ok(const struct tasx_ctx *c, uint32_t n)
{
  if (!zerocopy_ok(c, n))
    return 0;
  for (uint32_t i = 0; i < n; i++)
    if (c->pend_ip[i] < c->zc_host + TASX_TAS_IP_OFF)
      return 0;
  return 1;
}

/* hand the open batch to the feeder (frames outside the region: after the
 * context's feeder tickets complete, the local path takes them) */
static int feeder_submit(struct tasx_ctx *c)
{
  int rc;
  while (c->npend > 0) {
    if (!feeder_ok(c, c->npend))
      return flush_wait(c, c->next_ticket); /* in ticket order before the local flushes */
    /* A flush this context launched itself (a batch outside the region) must
     * complete first: the feeder's completion of a later ticket moves
     * done_ticket past it (flush_reap), which would skip copying its staged
     * results into its frames and free its slot while the GPU still uses it. */
    if (!ticket_le(c->local_last, c->done_ticket) && (rc = flush_wait(c, c->local_last)) != 0)
      return rc;
    const uint32_t cnt = c->npend < FB_MAX ? c->npend : FB_MAX;
    /* the slot is reused once the feeder has taken its previous batch AND
     * completed it: until then its frame pointers are what ctx_settle hands
     * back should the feeder fail */
    uint32_t k = 0;
    struct fbatch *b = &c->fq[c->fq_head % FQ];
    while (c->fq_head - __atomic_load_n(&c->fq_tail, __ATOMIC_ACQUIRE) >= FQ ||
           !ticket_le(b->ticket, __atomic_load_n(&c->fd_done, __ATOMIC_ACQUIRE))) {
      if ((++k & 4095u) == 0 && feeder_error(c))
        return set_err(-EIO, "flush: the feeder thread failed");
    }
    b->ticket = ++c->next_ticket;
    b->n = cnt;
    memcpy(b->ip, c->pend_ip, (size_t) cnt * sizeof(*b->ip));
    __atomic_store_n(&c->fq_head, c->fq_head + 1, __ATOMIC_RELEASE);
    c->n_feeder_flushes++;
    if (cnt < c->npend) {
      memmove(c->pend_ip, c->pend_ip + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_ip));
      memmove(c->pend_l4, c->pend_l4 + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_l4));
    }
    c->npend -= cnt;
  }
  return 0;
}

/* take every queued batch that fits into sweep `w` */
static void feeder_gather(struct feeder *F, struct fsweep *w)
{
  const uint32_t att = __atomic_load_n(&F->attached, __ATOMIC_ACQUIRE);
  for (unsigned id = 0; id < TASX_MAX_CTX; id++) {
    if (!(att & (1u << id)))
      continue;
    struct tasx_ctx *c = &g_ctx[id];
    uint32_t tail = c->fq_tail;
    const uint32_t head = __atomic_load_n(&c->fq_head, __ATOMIC_ACQUIRE), tail0 = tail;
    while (tail != head && w->nrec < SWEEP_REC) {
      const struct fbatch *b = &c->fq[tail % FQ];
      if (w->n + b->n > SWEEP_MAX)
        break;
      for (uint32_t i = 0; i < b->n; i++) {
        const uint8_t *ip = b->ip[i];
        const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
        w->h_off[w->n + i] = (uint64_t) (uintptr_t) (c->zc_dev + (ip - TASX_TAS_IP_OFF - c->zc_host));
        w->h_flen[w->n + i] = TASX_TAS_IP_OFF + (tl < 20 ? 20 : tl);
      }
      w->n += b->n;
      w->rec_ctx[w->nrec] = (uint16_t) id;
      w->rec_ticket[w->nrec] = b->ticket;
      w->nrec++;
      tail++;
    }
    if (tail != tail0)
      __atomic_store_n(&c->fq_tail, tail, __ATOMIC_RELEASE); /* the slots are free again */
  }
}

static int feeder_launch(struct feeder *F, struct fsweep *w, uint32_t seq)
{
  tasx_tcp4_params p;
  memset(&p, 0, sizeof(p));
  p.base = NULL; /* absolute device addresses in off[] */
  p.off = w->d_off;
  p.flen = w->d_flen;
  p.n = w->n;
  p.ip_off = TASX_TAS_IP_OFF;
  p.l4_off = TASX_TAS_L4_OFF;
  p.flags = TASX_F_INPLACE;
  if (tasx_launch_tcp4(&p, 0, F->st) != 0)
    return -1;
  return post_done(F->d_done + DONE_STRIDE * (seq % F->nsweep), seq, F->st);
}

static void *feeder_main(void *arg)
{
  struct feeder *F = arg;
  uint32_t launched = 0, published = 0, idle = 0;
  if (hipSetDevice(F->device) != hipSuccess) {
    __atomic_store_n(&F->failed, 1, __ATOMIC_RELEASE);
    return NULL;
  }
  for (;;) {
    int did = 0;
    /* publish completed sweeps, oldest first */
    while (published != launched) {
      const uint32_t s = published + 1;
      struct fsweep *w = &F->sw[s % F->nsweep];
      if (__atomic_load_n(F->h_done + DONE_STRIDE * (s % F->nsweep), __ATOMIC_ACQUIRE) != s)
        break;
      for (uint32_t r = 0; r < w->nrec; r++)
        __atomic_store_n(&g_ctx[w->rec_ctx[r]].fd_done, w->rec_ticket[r], __ATOMIC_RELEASE);
      __atomic_fetch_add(&F->frames, (uint64_t) w->n, __ATOMIC_RELAXED);
      __atomic_fetch_add(&F->sweeps, (uint64_t) 1, __ATOMIC_RELAXED);
      w->n = w->nrec = 0;
      published = s;
      did = 1;
    }
    /* gather into a free sweep buffer and launch it */
    if (launched - published < F->nsweep) {
      struct fsweep *w = &F->sw[(launched + 1) % F->nsweep];
      feeder_gather(F, w);
      __atomic_fetch_add(&F->gathers, 1u, __ATOMIC_RELEASE);
      if (w->nrec > 0) {
        if (feeder_launch(F, w, launched + 1) != 0) {
          __atomic_store_n(&F->failed, 1, __ATOMIC_RELEASE);
          return NULL;
        }
        launched++;
        did = 1;
      }
    }
    if (did) {
      idle = 0;
      continue;
    }
    if (!__atomic_load_n(&F->running, __ATOMIC_ACQUIRE) && published == launched)
      return NULL;
    if ((++idle & 4095u) == 0) {
      if (published != launched) { /* a sweep in flight: is the stream healthy? */
        const hipError_t e = hipStreamQuery(F->st);
        if (e != hipSuccess && e != hipErrorNotReady) {
          __atomic_store_n(&F->failed, 1, __ATOMIC_RELEASE);
          return NULL;
        }
      } else {
        sched_yield();
      }
    }
  }
}

static void feeder_free(struct feeder *F)
{
  for (unsigned k = 0; k < NSWEEP_MAX; k++) {
    if (F->sw[k].h_off)
      hipHostFree(F->sw[k].h_off);
    if (F->sw[k].h_flen)
      hipHostFree(F->sw[k].h_flen);
  }
  if (F->h_done)
    hipHostFree(F->h_done);
  if (F->d_count)
    hipFree(F->d_count);
  if (F->st)
    hipStreamDestroy(F->st);
  free(F);
}

int tasx_feeder_start(int device)
{
  int ndev = 0, rc = 0;
  hipError_t e;
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "feeder: device %d out of range", device);
  if ((e = hipGetDeviceCount(&ndev)) != hipSuccess)
    return hip_err(e, "hipGetDeviceCount");
  if (device >= ndev)
    return set_err(-ENODEV, "device %d not present (%d GPUs)", device, ndev);
  pthread_mutex_lock(&g_feeder_mu);
  if (g_feeder[device]) {
    pthread_mutex_unlock(&g_feeder_mu);
    return set_err(-EINVAL, "feeder for device %d already running", device);
  }
  struct feeder *F = calloc(1, sizeof(*F));
  if (!F) {
    pthread_mutex_unlock(&g_feeder_mu);
    return set_err(-ENOMEM, "feeder: out of host memory");
  }
  F->device = device;
  F->running = 1;
  F->nsweep = NSWEEP;
  if ((e = hipSetDevice(device)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&F->st, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipHostMalloc((void **) &F->h_done, 4u * DONE_STRIDE * NSWEEP_MAX, hipHostMallocCoherent)) != hipSuccess ||
      (e = hipHostGetDevicePointer((void **) &F->d_done, F->h_done, 0)) != hipSuccess ||
      (e = hipMalloc((void **) &F->d_count, 4u * DONE_STRIDE * NSWEEP_MAX)) != hipSuccess ||
      (e = hipMemset(F->d_count, 0, 4u * DONE_STRIDE * NSWEEP_MAX)) != hipSuccess)
    rc = hip_err(e, "feeder allocation");
  for (unsigned k = 0; !rc && k < F->nsweep; k++) {
    struct fsweep *w = &F->sw[k];
    if ((e = hipHostMalloc((void **) &w->h_off, 8u * SWEEP_MAX, 0)) != hipSuccess ||
        (e = hipHostMalloc((void **) &w->h_flen, 4u * SWEEP_MAX, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &w->d_off, w->h_off, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **) &w->d_flen, w->h_flen, 0)) != hipSuccess)
      rc = hip_err(e, "feeder sweep buffers");
  }
  if (!rc) {
    memset(F->h_done, 0, 4u * DONE_STRIDE * NSWEEP_MAX);
    if (pthread_create(&F->thr, NULL, feeder_main, F) != 0)
      rc = set_err(-ENOMEM, "feeder: pthread_create failed");
  }
  if (rc) {
    feeder_free(F);
    pthread_mutex_unlock(&g_feeder_mu);
    return rc;
  }
  g_feeder[device] = F;
  pthread_mutex_unlock(&g_feeder_mu);
  return 0;
}

int tasx_feeder_stop(int device)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "feeder: device %d out of range", device);
  pthread_mutex_lock(&g_feeder_mu);
  struct feeder *F = g_feeder[device];
  if (!F) {
    pthread_mutex_unlock(&g_feeder_mu);
    return set_err(-EINVAL, "no feeder running for device %d", device);
  }
  if (__atomic_load_n(&F->attached, __ATOMIC_ACQUIRE) != 0) {
    pthread_mutex_unlock(&g_feeder_mu);
    return set_err(-EBUSY, "feeder for device %d still serves contexts", device);
  }
  int rc = free_guard_enter("tasx_feeder_stop");
  if (rc) {
    pthread_mutex_unlock(&g_feeder_mu);
    return rc;
  }
  __atomic_store_n(&F->running, 0, __ATOMIC_RELEASE);
  pthread_join(F->thr, NULL);
  const int failed = F->failed;
  g_feeder[device] = NULL;
  hipSetDevice(device);
  hipStreamSynchronize(F->st);
  feeder_free(F);
  free_guard_exit();
  pthread_mutex_unlock(&g_feeder_mu);
  return failed ? set_err(-EIO, "the feeder thread for device %d had failed", device) : 0;
}

int tasx_feeder_stats(int device, uint64_t *sweeps, uint64_t *frames)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-EINVAL, "no feeder running for device %d", device);
  pthread_mutex_lock(&g_feeder_mu); /* not freed by a concurrent stop meanwhile */
  const struct feeder *F = g_feeder[device];
  if (F) { /* a snapshot of counters the feeder keeps updating */
    if (sweeps)
      *sweeps = __atomic_load_n(&F->sweeps, __ATOMIC_RELAXED);
    if (frames)
      *frames = __atomic_load_n(&F->frames, __ATOMIC_RELAXED);
  }
  pthread_mutex_unlock(&g_feeder_mu);
  return F ? 0 : set_err(-EINVAL, "no feeder running for device %d", device);
}

int tasx_ctx_use_feeder(unsigned ctx_id, int on)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  int rc;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  const unsigned id = (unsigned) (c - g_ctx);
  if (on) {
    if (c->fd)
      return 0;
    if (!c->zc_host)
      return set_err(-EINVAL, "ctx %u has no frame region (tasx_ctx_register_frames)", ctx_id);
    if ((rc = flush_wait(c, c->next_ticket)) != 0)
      return rc;
    struct fbatch *fq = calloc(FQ, sizeof(*fq));
    if (!fq)
      return set_err(-ENOMEM, "feeder queue: out of host memory");
    /* look the feeder up and attach under the lock tasx_feeder_stop takes */
    pthread_mutex_lock(&g_feeder_mu);
    struct feeder *F = c->device < MAX_DEVICES ? g_feeder[c->device] : NULL;
    if (F) {
      for (uint32_t q = 0; q < FQ; q++) /* free slots: their "previous batch" is complete */
        fq[q].ticket = c->next_ticket;
      c->fq = fq;
      c->fq_head = c->fq_tail = 0;
      c->fd_done = c->next_ticket;
      c->fd = F;
      __atomic_or_fetch(&F->attached, 1u << id, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_feeder_mu);
    if (!F) {
      free(fq);
      return set_err(-EINVAL, "no feeder running for device %d (tasx_feeder_start)", c->device);
    }
    return 0;
  }
  if (!c->fd)
    return 0;
  /* every ticket handed over completes first; the feeder then never reads the queue again */
  if ((rc = flush_wait(c, c->next_ticket)) != 0)
    return rc;
  struct feeder *F = c->fd;
  __atomic_and_fetch(&F->attached, ~(1u << id), __ATOMIC_RELEASE);
  /* a gather pass that read the old mask may still look at the queue's
   * indices: wait until two more passes have started and ended */
  const uint32_t g0 = __atomic_load_n(&F->gathers, __ATOMIC_ACQUIRE);
  while (__atomic_load_n(&F->gathers, __ATOMIC_ACQUIRE) - g0 < 2u && !__atomic_load_n(&F->failed, __ATOMIC_ACQUIRE))
    sched_yield();
  c->fd = NULL;
  free(c->fq);
  c->fq = NULL;
  return 0;
}

int tasx_ctx_feeder_flushes(unsigned ctx_id, uint32_t *feeder_flushes)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (feeder_flushes)
    *feeder_flushes = c->n_feeder_flushes;
  return 0;
}

/* ---------------------------------------------------------------------- */
/* Flush server (ABI 6): one persistent kernel per GPU (server_kernels.hip)
 * serves every attached context.  A context's tasx_flush_submit() writes each
 * batch of up to TASX_SRV_FB frames into the next slot of its own ring in
 * coherent pinned memory -- the entries (frame offset in its registered
 * region | ip.total_length | tag), then the region word, then the header
 * (release) -- and returns: no HIP call, no lock, no launch.  SRV_K
 * workgroups of the kernel poll ring r (workgroup k the positions k mod
 * SRV_K), checksum the frames in place over PCIe and post each slot's done
 * word; tasx_flush_poll/_wait reap those in position order.
 *
 * Epochs (round 6): a launch serves for SRV_PERIOD_US, then leaves at its
 * rings' positions; the server's epoch thread keeps the next launch queued
 * behind the running one on the server's stream (two outstanding, each with
 * an event), so service goes on while any HIP call that waits for all of the
 * device's work -- hipDeviceSynchronize (torch.cuda.synchronize), the frees
 * (torch.cuda.empty_cache), synchronous copies, waits on the null stream --
 * waits for at most the epochs queued when it was made (about two periods)
 * instead of hanging on a kernel that never ends (the
 * round-5 server had a 2 s lease and no end).  A process that is gone queues
 * no further epoch, so the server also ends with it.  The epoch thread makes
 * the server's only routine HIP calls (hipEventQuery, the launches); a call
 * of its that waits longer than SRV_SLOW_MS, or an epoch overdue by as long,
 * is counted and reported once on stderr (tasx_server_epochs has the counts). */

#define SRV_PERIOD_US 5000u
#define SRV_SLOW_MS 50u
#define SRV_HOT_US 200u
#define SRV_STOP_WAIT_MS 5000u
#define SRV_COLD_US 2000u /* idle time from which a ring's header alone is polled */
/* workgroups per ring (tasx_srv_params.k).  Two, so that one polls the
 * ring's next position while the other sums (profiles/r04/r04g), but taking
 * turns at reading frames (the ring's read token, server_device.h): the frame
 * reads a busy server keeps in flight through the XCDs' L2s are what it costs
 * device-resident work on the same GPU (two workgroups reading at once:
 * 1.30-1.53x a batch's time; one per ring 1.12-1.15x, with a lower rate and
 * a longer lone flush; profiles/r06/INDEX.md r06d-r06f). */
#define SRV_K 2u
#define SRV_QUEUED 2u     /* epochs outstanding on the server's stream */

struct fserver {
  int device;
  hipStream_t st;
  uint8_t *h_mem, *d_mem; /* coherent pinned block (tasx_kernels.h TASX_SRV_*) */
  uint32_t *d_tok;        /* device memory: each ring's read token (tasx_srv_params.tok) */
  uint8_t *h_ring, *d_ring; /* the host-written lines (control word, slots): h_mem / d_mem */
  uint32_t attached;      /* bit r: ring r serves a context */
  int keep_run;           /* the epoch thread runs */
  pthread_t keep;
  uint64_t batches, frames; /* submitted by contexts since detached (statistics) */
  uint32_t k;               /* workgroups per ring */
  uint32_t ring_pos[TASX_MAX_CTX]; /* next position of a ring no context is attached to */
  struct grave *graves;            /* contexts destroyed while the server ran: released at stop */
  int aborted; /* tasx_server_abort stopped the kernel (and the epoch thread); read and written atomically:
                * context threads read it (server_gone) outside g_server_mu */
  /* kstate: 0 while the epochs run (or are paused), < 0 -hipError_t when an
   * epoch failed to launch or faulted.  The fast-path cores read this word:
   * their polls make no HIP call (a hipStreamQuery per poll from 8 cores
   * serialised in the runtime's locks, profiles/r05 r05o).  launched: the
   * epoch thread keeps epochs queued (cleared by a pause).  launched, kstate,
   * paused and the epoch queue (ev, qhead, nq, nlaunch) change under kmu. */
  int launched, kstate;
  pthread_mutex_t kmu;
  hipEvent_t ev[SRV_QUEUED];
  uint64_t qhead, nlaunch; /* epochs completed / launched */
  uint32_t nq;             /* outstanding: nlaunch - qhead */
  uint32_t slow_calls, max_wait_ms, warned; /* the epoch thread's waits (tasx_server_epochs) */
  /* tasx_server_pause: the kernel has left at its rings' positions and
   * tasx_server_resume launches it again from them (prm.resume); set before
   * the stop word is written and cleared after the new launch */
  int paused;
  tasx_srv_params prm;
};

struct grave {
  struct tasx_ctx c;
  struct grave *next;
};

static struct fserver *g_server[MAX_DEVICES];
static pthread_mutex_t g_server_mu = PTHREAD_MUTEX_INITIALIZER;
static int server_settle(struct tasx_ctx *c);
static void ctx_settle(struct tasx_ctx *c);
static int unf_seg(struct tasx_ctx *c, const tasx_tx_seg *g);

/* HIP's frees wait for every stream of the device, the server's kernel too:
 * refused (-EBUSY) while any server's kernel runs (a paused one does not),
 * instead of waiting for its stop.  On success g_server_mu stays held until
 * free_guard_exit(), across the free itself: a resume (which takes the same
 * lock to relaunch the kernel) cannot slip in between the check and the free
 * and leave the free waiting for the relaunched kernel. */
static int free_guard_enter(const char *what)
{
  int d, any = 0;
  pthread_mutex_lock(&g_server_mu);
  for (d = 0; d < MAX_DEVICES; d++)
    any |= g_server[d] != NULL && !__atomic_load_n(&g_server[d]->paused, __ATOMIC_ACQUIRE);
  if (!any)
    return 0;
  pthread_mutex_unlock(&g_server_mu);
  return set_err(-EBUSY,
                 "%s: a flush server is running (HIP frees wait for its kernel; tasx_server_pause or "
                 "tasx_server_stop first)",
                 what);
}

static void free_guard_exit(void)
{
  pthread_mutex_unlock(&g_server_mu);
}

/* tasx_ctx_destroy with a server running on the context's device: the
 * context's resources move to the server's list (the slot is free at once);
 * 1 if taken */
static int server_defer_release(struct tasx_ctx *c)
{
  int taken = 0;
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = c->device >= 0 && c->device < MAX_DEVICES ? g_server[c->device] : NULL;
  struct grave *g = S ? malloc(sizeof(*g)) : NULL;
  if (g) {
    memcpy(&g->c, c, sizeof(*c));
    g->next = S->graves;
    S->graves = g;
    memset(c, 0, sizeof(*c));
    taken = 1;
  }
  pthread_mutex_unlock(&g_server_mu);
  return taken;
}


static uint32_t *srv_dline(const struct fserver *S, unsigned r)
{
  return (uint32_t *) (S->h_mem + TASX_SRV_DONE(r));
}

static uint64_t mono_ns(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t) t.tv_sec * 1000000000ull + (uint64_t) t.tv_nsec;
}

/* the epoch thread's report of a long wait (once per server; the counts stay
 * in tasx_server_epochs) */
static void server_slow(struct fserver *S, const char *what, uint64_t ns)
{
  const uint32_t ms = (uint32_t) (ns / 1000000u);
  S->slow_calls++;
  if (ms > S->max_wait_ms)
    S->max_wait_ms = ms;
  if (!S->warned && !getenv("TASX_SERVER_QUIET")) {
    S->warned = 1;
    fprintf(stderr,
            "tasx: flush server (device %d): %s took %u ms -- another thread is in a HIP call that waits for all "
            "of the device's work (hipDeviceSynchronize / torch.cuda.synchronize, a free, a synchronous copy, a "
            "wait on the null stream).  The server's epochs bound that wait to about %u ms each time; "
            "tasx_server_pause() around such calls avoids it (INTEGRATION.md 4f)\n",
            S->device, what, ms, 2u * SRV_PERIOD_US / 1000u);
  }
}

/* launch the next epoch and record its event (kmu held) */
static hipError_t server_launch_epoch(struct fserver *S)
{
  S->prm.resume = S->nlaunch > 0u ? 1u : 0u;
  if (tasx_launch_server(&S->prm, S->st) != 0) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? hipErrorLaunchFailure : e;
  }
  const hipError_t e = hipEventRecord(S->ev[S->nlaunch % SRV_QUEUED], S->st);
  if (e != hipSuccess)
    return e;
  S->nlaunch++;
  S->nq++;
  return hipSuccess;
}

/* The epoch thread: every 200 us, retire the epochs that have completed and
 * queue new ones up to SRV_QUEUED (unless paused or failed). */
static void *server_epochs(void *arg)
{
  struct fserver *S = arg;
  const struct timespec ts = {0, 200 * 1000};
  const uint64_t slow = (uint64_t) SRV_SLOW_MS * 1000000u;
  uint64_t t_head = mono_ns(); /* when the oldest outstanding epoch became the oldest */
  hipSetDevice(S->device);
  while (__atomic_load_n(&S->keep_run, __ATOMIC_ACQUIRE)) {
    pthread_mutex_lock(&S->kmu);
    if (__atomic_load_n(&S->launched, __ATOMIC_ACQUIRE) && __atomic_load_n(&S->kstate, __ATOMIC_RELAXED) == 0) {
      while (S->nq > 0u) {
        const uint64_t t0 = mono_ns();
        const hipError_t e = hipEventQuery(S->ev[S->qhead % SRV_QUEUED]);
        const uint64_t t1 = mono_ns();
        if (t1 - t0 > slow)
          server_slow(S, "hipEventQuery of an epoch", t1 - t0);
        if (e == hipErrorNotReady) {
          /* an epoch lasts SRV_PERIOD_US and its successor waits behind it:
           * the oldest should retire within about two periods */
          if (t1 - t_head > slow + 2000ull * SRV_PERIOD_US)
            server_slow(S, "an epoch past its period", t1 - t_head), t_head = t1;
          break;
        }
        if (e != hipSuccess) {
          __atomic_store_n(&S->kstate, -(int) e, __ATOMIC_RELEASE);
          break;
        }
        S->qhead++;
        S->nq--;
        t_head = t1;
      }
      while (__atomic_load_n(&S->kstate, __ATOMIC_RELAXED) == 0 && S->nq < SRV_QUEUED) {
        const uint64_t t0 = mono_ns();
        const hipError_t e = server_launch_epoch(S);
        const uint64_t t1 = mono_ns();
        if (t1 - t0 > slow)
          server_slow(S, "an epoch's launch", t1 - t0);
        if (e != hipSuccess)
          __atomic_store_n(&S->kstate, -(int) e, __ATOMIC_RELEASE);
      }
    }
    pthread_mutex_unlock(&S->kmu);
    nanosleep(&ts, NULL);
  }
  return NULL;
}

/* process exit with a server still started: stop the kernel first (the
 * runtime's own teardown would otherwise wait for the queued epochs) */
static void server_atexit(void)
{
  for (int d = 0; d < MAX_DEVICES; d++) {
    struct fserver *S = g_server[d];
    if (S) {
      __atomic_store_n(&S->keep_run, 0, __ATOMIC_RELEASE);
      __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 1u, __ATOMIC_RELEASE);
    }
  }
}

static void server_free(struct fserver *S)
{
  pthread_mutex_destroy(&S->kmu);
  for (uint32_t q = 0; q < SRV_QUEUED; q++)
    if (S->ev[q])
      hipEventDestroy(S->ev[q]);
  if (S->h_mem)
    hipHostFree(S->h_mem);
  if (S->d_tok)
    hipFree(S->d_tok);
  if (S->st)
    hipStreamDestroy(S->st);
  free(S);
}

/* 1 when the server has gone for good: aborted, an epoch failed, or stopped
 * with its last launch finished.  A paused server, and one whose epoch thread
 * runs, has not (between two epochs the stream may be idle for a moment). */
static int server_gone(struct fserver *S)
{
  if (__atomic_load_n(&S->aborted, __ATOMIC_ACQUIRE))
    return 1;
  if (__atomic_load_n(&S->paused, __ATOMIC_ACQUIRE))
    return 0;
  if (__atomic_load_n(&S->kstate, __ATOMIC_ACQUIRE) < 0)
    return 1;
  if (__atomic_load_n(&S->keep_run, __ATOMIC_ACQUIRE))
    return 0;
  return hipStreamQuery(S->st) != hipErrorNotReady;
}

/* 0 while the server kernel runs and has flagged no error */
static int server_err(const struct tasx_ctx *c)
{
  return set_err(-EIO, "flush server: a frame of ctx %u changed after submission (its fields were left alone; "
                 "sticky until tasx_ctx_use_server(ctx, 0))", (unsigned) (c - g_ctx));
}

/* 0 while the server kernel runs */
static int server_alive(const struct tasx_ctx *c)
{
  struct fserver *S = c->sv;
  int st = __atomic_load_n(&S->kstate, __ATOMIC_ACQUIRE);
  if (st == 0) {
    if (__atomic_load_n(&S->keep_run, __ATOMIC_ACQUIRE))
      return 0; /* the epoch thread keeps it going */
    /* it has stopped (an abort or a stop under way): ask the runtime */
    const hipError_t e = hipStreamQuery(S->st);
    if (e == hipErrorNotReady)
      return 0;
    st = e == hipSuccess ? 1 : -(int) e;
  }
  if (st == 1)
    return set_err(-EIO, "flush server: the kernel has exited (stopped)");
  return hip_err((hipError_t) -st, "flush server: an epoch");
}

/* 0 while the server kernel runs and has flagged no frame of this context */
static int server_health(const struct tasx_ctx *c)
{
  return c->sv_err ? server_err(c) : server_alive(c);
}

/* the positions finished in order from sv_done_pos (the ring's workgroups
 * finish theirs out of order); the ring's error word (same line) moves into
 * the context's sticky flag */
static void server_reap(struct tasx_ctx *c)
{
  const unsigned id = (unsigned) (c - g_ctx);
  uint32_t *done = srv_dline(c->sv, id);
  uint32_t d = c->sv_done_pos;
  while (d != c->sv_pos && __atomic_load_n(&done[d % TASX_SRV_RING], __ATOMIC_ACQUIRE) == d + 1u)
    d++;
  if (d == c->sv_done_pos)
    return;
  if (__atomic_load_n(&done[TASX_SRV_ERRW], __ATOMIC_ACQUIRE) != 0) {
    c->sv_err = 1;
    __atomic_store_n(&done[TASX_SRV_ERRW], 0u, __ATOMIC_RELAXED);
  }
  const uint32_t t = c->sv_ticket[(d - 1u) % TASX_SRV_RING];
  c->sv_done_pos = d;
  if (!ticket_le(t, c->done_ticket))
    c->done_ticket = t;
}

/* every frame of the open batch is one the server takes: TAS layout in the
 * registered region, 16-byte aligned frame start (ip - 14), total_length in
 * [38, 1522], and the whole chunks it reads inside the region */
static int server_ok(const struct tasx_ctx *c, uint32_t n)
{
  const uintptr_t dend = (uintptr_t) c->zc_dev + c->zc_bytes;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t *ip = c->pend_ip[i];
    if (c->pend_l4[i] != ip + 20 || ip < c->zc_host + TASX_TAS_IP_OFF ||
        ip + 20 > c->zc_host + c->zc_bytes)
      return 0;
    const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
    const uintptr_t fdev = (uintptr_t) (c->zc_dev + (ip - TASX_TAS_IP_OFF - c->zc_host));
    /* the row reads the chunks of [frame, frame + 14 + tl) */
    if (tl < 38u || tl > 1522u || (fdev & 15u) != 0 || fdev + ((14u + tl + 15u) & ~15u) > dend)
      return 0;
  }
  return 1;
}

static int server_submit(struct tasx_ctx *c)
{
  const unsigned id = (unsigned) (c - g_ctx);
  struct fserver *S = c->sv;
  int rc;
  while (c->npend > 0) {
    if (!server_ok(c, c->npend))
      return flush_wait(c, c->next_ticket); /* the local path takes it, after the server's tickets */
    /* a flush this context launched itself completes first (as feeder_submit) */
    if (!ticket_le(c->local_last, c->done_ticket) && (rc = flush_wait(c, c->local_last)) != 0)
      return rc;
    const uint32_t cnt = c->npend < TASX_SRV_FB ? c->npend : TASX_SRV_FB;
    /* the slot's previous batch (position sv_pos - RING) must be finished */
    uint32_t k = 0;
    while (c->sv_pos - c->sv_done_pos >= TASX_SRV_RING) {
      server_reap(c);
      if ((++k & 4095u) == 0 && (rc = server_health(c)) != 0)
        return rc;
    }
    const uint32_t pos = c->sv_pos;
    const uint64_t tag = (uint64_t) ((pos + 1u) & 0xffffu) << 48;
    uint64_t *slot = (uint64_t *) (S->h_ring + TASX_SRV_SLOTP(id, pos));
    const uintptr_t b16 = (uintptr_t) c->zc_dev & ~(uintptr_t) 15;
    const uint8_t *h16 = c->zc_host - ((uintptr_t) c->zc_dev & 15u); /* host view of b16 */
    const uint64_t bytes = c->zc_bytes + ((uintptr_t) c->zc_dev & 15u);
    for (uint32_t i = 0; i < cnt; i++) {
      const uint8_t *ip = c->pend_ip[i];
      const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
      const uint64_t fo = (uint64_t) (ip - TASX_TAS_IP_OFF - h16);
      slot[TASX_SRV_HDR / 8 + i] = fo | (uint64_t) tl << 32 | tag;
    }
    /* the unused entries get this position's tag too: every entry word of a
     * slot then carries either this position's tag or the one of the slot's
     * previous position, so a word the server reads before the host wrote it
     * can never pass for a current one (an entry left unwritten for 2^16
     * positions, or never written, would carry a stale tag that matches) */
    for (uint32_t i = cnt; i < TASX_SRV_FB; i++)
      slot[TASX_SRV_HDR / 8 + i] = tag;
    __atomic_store_n(&slot[1], (uint64_t) b16 | tag, __ATOMIC_RELEASE);
    __atomic_store_n(&slot[0], (uint64_t) cnt | (bytes > 0xffffffffull ? 0xffffffffull : bytes) << 16 | tag,
                     __ATOMIC_RELEASE);
    c->sv_ticket[pos % TASX_SRV_RING] = ++c->next_ticket;
    c->sv_pos = pos + 1u;
    c->n_server_flushes++;
    __atomic_store_n(&c->sv_batches, c->sv_batches + 1u, __ATOMIC_RELAXED);
    __atomic_store_n(&c->sv_frames, c->sv_frames + cnt, __ATOMIC_RELAXED);
    if (cnt < c->npend) {
      memmove(c->pend_ip, c->pend_ip + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_ip));
      memmove(c->pend_l4, c->pend_l4 + cnt, (size_t) (c->npend - cnt) * sizeof(*c->pend_l4));
    }
    c->npend -= cnt;
  }
  return 0;
}

/* segments per TX slot */
static uint32_t srv_segs_max(void)
{
  return TASX_SRV_SEGS;
}

/* TX segment batches through the server: validated up front (nothing is
 * submitted unless every segment is safe to build in place), then packed
 * up to TASX_SRV_SEGS to a slot, consecutive segments with one hdrs_len and
 * room sharing it (tasx_kernels.h) */
int tasx_server_tx_segments(unsigned ctx_id, const tasx_tx_seg *segs, uint32_t n, uint32_t *ticket)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  int rc;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (!c->sv)
    return set_err(-EINVAL, "ctx %u is not attached to a flush server (tasx_ctx_use_server)", ctx_id);
  if (!c->shm_host)
    return set_err(-EINVAL, "ctx %u has no shared-memory region (tasx_ctx_register_shm)", ctx_id);
  if (n > 0 && !segs)
    return set_err(-EINVAL, "tx segments: NULL descriptors");
  const uint32_t ip_off = TASX_TAS_IP_OFF, l4_off = TASX_TAS_L4_OFF;
  for (uint32_t i = 0; i < n; i++) {
    const tasx_tx_seg *g = &segs[i];
    const uint32_t room = g->room & ~TASX_TXSEG_SCRATCH;
    const uint64_t fend = (uint64_t) g->hdrs_len + g->payload;
    /* frame_off first: the sums below cannot wrap once it lies inside the region */
    if (g->frame_off >= c->zc_bytes || (g->frame_off & 15u) != 0 || g->hdrs_len < l4_off + 20u ||
        g->hdrs_len > 240u || room > 0x7fffu || g->tx_base >= (1ull << 32) ||
        g->hdrs_len > c->zc_bytes - g->frame_off)
      return set_err(-EINVAL, "tx segment %u: frame offset, header length or room outside what the server builds",
                     i);
    /* the row reads and writes whole 16-byte chunks of [frame, frame + max(end, room)) and sums up to
     * ip_off + ip.total_length (TAS's own frames: hdrs_len - ip_off + payload, fast_flows.c:897) */
    const uint8_t *ip = c->zc_host + g->frame_off + ip_off;
    const uint64_t tl = ((uint32_t) ip[2] << 8) | ip[3];
    uint64_t span = fend > ip_off + tl ? fend : ip_off + tl;
    if (g->room & TASX_TXSEG_SCRATCH)
      span = span > room ? span : room;
    if (((span + 15u) & ~(uint64_t) 15) > c->zc_bytes - g->frame_off)
      return set_err(-EINVAL, "tx segment %u: frame (or its room) past the registered frame region", i);
  }
  /* a flush this context launched itself completes first (as server_submit) */
  if (!ticket_le(c->local_last, c->done_ticket) && (rc = flush_wait(c, c->local_last)) != 0)
    return rc;
  struct fserver *S = c->sv;
  const unsigned id = (unsigned) (c - g_ctx);
  for (uint32_t i0 = 0; i0 < n;) {
    /* a slot: up to TASX_SRV_SEGS consecutive segments with one hdrs_len and room */
    uint32_t cnt = 1;
    while (i0 + cnt < n && cnt < srv_segs_max() && segs[i0 + cnt].hdrs_len == segs[i0].hdrs_len &&
           segs[i0 + cnt].room == segs[i0].room)
      cnt++;
    uint32_t k = 0;
    while (c->sv_pos - c->sv_done_pos >= TASX_SRV_RING) {
      server_reap(c);
      if ((++k & 4095u) == 0 && (rc = server_health(c)) != 0) {
        /* the segments not handed over go to the unfinished store with the
         * server's (tasx_take_unfinished_segs) */
        for (uint32_t i = i0; i < n; i++)
          (void) unf_seg(c, &segs[i]);
        return rc;
      }
    }
    const uint32_t pos = c->sv_pos;
    const uint64_t tag = (uint64_t) ((pos + 1u) & 0xffffu) << 48;
    uint64_t *slot = (uint64_t *) (S->h_ring + TASX_SRV_SLOTP(id, pos));
    uint64_t *e = slot + TASX_SRV_HDR / 8;
    const tasx_tx_seg *g0 = &segs[i0];
    const uint32_t room16 = (g0->room & 0x7fffu) | ((g0->room & TASX_TXSEG_SCRATCH) ? 0x8000u : 0u);
    e[0] = (uint64_t) (uintptr_t) c->shm_dev | tag;
    e[1] = (uint64_t) (uint32_t) c->shm_bytes | (uint64_t) ip_off << 32 | (uint64_t) l4_off << 40 | tag;
    e[2] = (uint64_t) g0->hdrs_len | (uint64_t) room16 << 16 | tag;
    for (uint32_t j = 0; j < cnt; j++) {
      const tasx_tx_seg *g = &segs[i0 + j];
      uint64_t *w = e + TASX_SRV_SEGW0 + 3 * j;
      w[0] = (uint32_t) g->frame_off | (uint64_t) g->payload << 32 | tag;
      w[1] = g->pos | (uint64_t) (g->tx_len & 0xffffu) << 32 | tag;
      w[2] = (uint32_t) g->tx_base | (uint64_t) (g->tx_len >> 16) << 32 | tag;
    }
    /* every entry word the first poll reads tagged (server_submit); the words
     * past TASX_SRV_FB are read only after the header, which comes after them */
    for (uint32_t w = TASX_SRV_SEGW0 + 3 * cnt; w < TASX_SRV_FB; w++)
      e[w] = tag;
    const uintptr_t b16 = (uintptr_t) c->zc_dev;
    __atomic_store_n(&slot[1], (uint64_t) b16 | tag, __ATOMIC_RELEASE);
    __atomic_store_n(&slot[0], (uint64_t) (cnt | TASX_SRV_SEG) |
                     (uint64_t) (c->zc_bytes > 0xffffffffull ? 0xffffffffull : c->zc_bytes) << 16 | tag,
                     __ATOMIC_RELEASE);
    c->sv_ticket[pos % TASX_SRV_RING] = ++c->next_ticket;
    c->sv_pos = pos + 1u;
    c->n_server_flushes++;
    __atomic_store_n(&c->sv_batches, c->sv_batches + 1u, __ATOMIC_RELAXED);
    __atomic_store_n(&c->sv_frames, c->sv_frames + cnt, __ATOMIC_RELAXED);
    i0 += cnt;
  }
  if (ticket)
    *ticket = c->next_ticket;
  return 0;
}

int tasx_server_start(int device)
{
  int ndev = 0, khz = 0, rc = 0;
  hipError_t e;
  static int atexit_set = 0;
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "server: device %d out of range", device);
  if ((e = hipGetDeviceCount(&ndev)) != hipSuccess)
    return hip_err(e, "hipGetDeviceCount");
  if (device >= ndev)
    return set_err(-ENODEV, "device %d not present (%d GPUs)", device, ndev);
  pthread_mutex_lock(&g_server_mu);
  if (g_server[device]) {
    pthread_mutex_unlock(&g_server_mu);
    return set_err(-EINVAL, "flush server for device %d already running", device);
  }
  struct fserver *S = calloc(1, sizeof(*S));
  if (!S) {
    pthread_mutex_unlock(&g_server_mu);
    return set_err(-ENOMEM, "server: out of host memory");
  }
  S->device = device;
  pthread_mutex_init(&S->kmu, NULL);
  if ((e = hipSetDevice(device)) != hipSuccess ||
      (e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&S->st, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipHostMalloc((void **) &S->h_mem, TASX_SRV_BYTES, hipHostMallocCoherent)) != hipSuccess ||
      (e = hipHostGetDevicePointer((void **) &S->d_mem, S->h_mem, 0)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&S->ev[0], hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&S->ev[1], hipEventDisableTiming)) != hipSuccess ||
      (e = hipMalloc((void **) &S->d_tok, TASX_MAX_CTX * TASX_SRV_TOKW * sizeof(uint32_t))) != hipSuccess ||
      (e = hipMemsetAsync(S->d_tok, 0, TASX_MAX_CTX * TASX_SRV_TOKW * sizeof(uint32_t), S->st)) != hipSuccess)
    rc = hip_err(e, "server allocation");
  if (!rc && khz <= 0)
    rc = set_err(-ENODEV, "server: device %d reports no wall clock", device);
  tasx_srv_params prm;
  if (!rc) {
    memset(S->h_mem, 0, TASX_SRV_BYTES);
    S->h_ring = S->h_mem;
    S->d_ring = S->d_mem;
    prm.mem = S->d_mem;
    prm.ring = S->d_ring;
    prm.period_ticks = (uint64_t) khz * SRV_PERIOD_US / 1000u;
    prm.hot_ticks = (uint64_t) khz * SRV_HOT_US / 1000u;
    prm.cold_ticks = (uint64_t) khz * SRV_COLD_US / 1000u;
    prm.k = SRV_K;
    prm.resume = 0;
    prm.tok = S->d_tok;
    S->k = prm.k;
    S->prm = prm;
    if (prm.k == 0u || TASX_SRV_RING % prm.k != 0u || prm.k > TASX_SRV_KMAX)
      rc = set_err(-EINVAL, "server: %u workgroups per ring (a divisor of %u)", prm.k, TASX_SRV_RING);
  }
  if (!rc) {
    /* the first epoch here (a launch error is the caller's), the rest from
     * the epoch thread */
    if ((e = server_launch_epoch(S)) != hipSuccess) {
      rc = hip_err(e, "server kernel launch");
    } else {
      S->launched = 1;
      S->keep_run = 1;
      if (pthread_create(&S->keep, NULL, server_epochs, S) != 0) {
        S->keep_run = 0;
        __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 1u, __ATOMIC_RELEASE);
        (void) hipStreamSynchronize(S->st); /* the first epoch leaves on the stop word */
        rc = set_err(-ENOMEM, "server: pthread_create failed");
      }
    }
  }
  if (rc) {
    server_free(S);
    pthread_mutex_unlock(&g_server_mu);
    return rc;
  }
  if (!atexit_set) {
    atexit(server_atexit);
    atexit_set = 1;
  }
  g_server[device] = S;
  pthread_mutex_unlock(&g_server_mu);
  return 0;
}

int tasx_server_stop(int device)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "server: device %d out of range", device);
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = g_server[device];
  if (!S) {
    pthread_mutex_unlock(&g_server_mu);
    return set_err(-EINVAL, "no flush server running for device %d", device);
  }
  if (__atomic_load_n(&S->attached, __ATOMIC_ACQUIRE) != 0) {
    pthread_mutex_unlock(&g_server_mu);
    return set_err(-EBUSY, "flush server for device %d still serves contexts", device);
  }
  __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 1u, __ATOMIC_RELEASE);
  if (!__atomic_load_n(&S->aborted, __ATOMIC_ACQUIRE)) {
    __atomic_store_n(&S->keep_run, 0, __ATOMIC_RELEASE);
    pthread_join(S->keep, NULL);
  }
  /* bounded wait for every workgroup to leave */
  hipError_t e = hipErrorNotReady;
  const struct timespec ts = {0, 100 * 1000};
  for (uint32_t t = 0; t < SRV_STOP_WAIT_MS * 10u && (e = hipStreamQuery(S->st)) == hipErrorNotReady; t++)
    nanosleep(&ts, NULL);
  g_server[device] = NULL;
  pthread_mutex_unlock(&g_server_mu);
  if (e == hipErrorNotReady) /* still running: leave its memory mapped (leaked), never free under it */
    return set_err(-EIO, "flush server for device %d did not stop within %u ms", device, SRV_STOP_WAIT_MS);
  while (S->graves) { /* contexts destroyed while it ran */
    struct grave *g = S->graves;
    S->graves = g->next;
    ctx_release(&g->c);
    free(g);
  }
  server_free(S);
  return e == hipSuccess ? 0 : hip_err(e, "flush server kernel");
}

int tasx_server_epochs(int device, uint64_t *epochs, uint32_t *slow_waits, uint32_t *max_wait_ms)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-EINVAL, "no flush server running for device %d", device);
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = g_server[device];
  if (S) {
    pthread_mutex_lock(&S->kmu);
    if (epochs)
      *epochs = S->qhead;
    if (slow_waits)
      *slow_waits = S->slow_calls;
    if (max_wait_ms)
      *max_wait_ms = S->max_wait_ms;
    pthread_mutex_unlock(&S->kmu);
  }
  pthread_mutex_unlock(&g_server_mu);
  return S ? 0 : set_err(-EINVAL, "no flush server running for device %d", device);
}

int tasx_server_stats(int device, uint64_t *batches, uint64_t *frames)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-EINVAL, "no flush server running for device %d", device);
  pthread_mutex_lock(&g_server_mu);
  const struct fserver *S = g_server[device];
  if (S) { /* detached contexts' counts, plus the attached ones' so far */
    uint64_t b = __atomic_load_n(&S->batches, __ATOMIC_RELAXED), f = __atomic_load_n(&S->frames, __ATOMIC_RELAXED);
    for (unsigned id = 0; id < TASX_MAX_CTX; id++)
      if (__atomic_load_n(&S->attached, __ATOMIC_ACQUIRE) & (1u << id)) {
        b += __atomic_load_n(&g_ctx[id].sv_batches, __ATOMIC_RELAXED);
        f += __atomic_load_n(&g_ctx[id].sv_frames, __ATOMIC_RELAXED);
      }
    if (batches)
      *batches = b;
    if (frames)
      *frames = f;
  }
  pthread_mutex_unlock(&g_server_mu);
  return S ? 0 : set_err(-EINVAL, "no flush server running for device %d", device);
}

int tasx_ctx_use_server(unsigned ctx_id, int on)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  int rc;
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  const unsigned id = (unsigned) (c - g_ctx);
  if (on) {
    if (c->sv)
      return 0;
    if (c->fd)
      return set_err(-EBUSY, "ctx %u uses the shared feeder (tasx_ctx_use_feeder 0 first)", ctx_id);
    if (!c->zc_host)
      return set_err(-EINVAL, "ctx %u has no frame region (tasx_ctx_register_frames)", ctx_id);
    if (c->zc_bytes + 16u > 0xffffffffull || (uint64_t) (uintptr_t) c->zc_dev + c->zc_bytes >= (1ull << 48))
      return set_err(-EINVAL, "ctx %u: frame region beyond the server's 32-bit offsets / 48-bit addresses", ctx_id);
    if ((rc = flush_wait(c, c->next_ticket)) != 0)
      return rc;
    pthread_mutex_lock(&g_server_mu);
    struct fserver *S = c->device < MAX_DEVICES ? g_server[c->device] : NULL;
    if (S && server_gone(S)) {
      pthread_mutex_unlock(&g_server_mu);
      return set_err(-EIO, "the flush server for device %d is not running (aborted, or an epoch failed): "
                     "tasx_server_stop it", c->device);
    }
    if (S) {
      c->sv_pos = c->sv_done_pos = S->ring_pos[id]; /* where the ring's workgroups wait */
      c->sv_err = 0;
      /* an error a previous context of this ring left (no batch of the ring is in flight) */
      __atomic_store_n(srv_dline(S, id) + TASX_SRV_ERRW, 0u, __ATOMIC_RELEASE);
      c->sv_batches = c->sv_frames = 0;
      c->sv = S;
      __atomic_or_fetch(&S->attached, 1u << id, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&g_server_mu);
    return S ? 0 : set_err(-EINVAL, "no flush server running for device %d (tasx_server_start)", c->device);
  }
  if (!c->sv)
    return 0;
  /* the server's positions first: a frame it flagged does not stop the detach;
   * a kernel that has gone leaves its positions unfinished: they move to the
   * context's unfinished store (tasx_take_unfinished) and the detach completes */
  if (server_settle(c) != 0) {
    ctx_settle(c); /* the rest of the context too: every ticket complete, pending frames handed back */
    return set_err(-EIO, "ctx %u detached from a flush server whose kernel has gone; %u frame(s) and %u TX "
                   "segment(s) unfinished (tasx_take_unfinished)", ctx_id, c->unf_n - c->unf_pos,
                   c->unf_seg_n - c->unf_seg_pos);
  }
  const int had_err = c->sv_err;
  c->sv_err = 0;
  if ((rc = flush_wait(c, c->next_ticket)) != 0) {
    c->sv_err = had_err;
    return rc;
  }
  pthread_mutex_lock(&g_server_mu); /* the counts move to the server's totals atomically for tasx_server_stats */
  __atomic_fetch_add(&c->sv->batches, c->sv_batches, __ATOMIC_RELAXED);
  __atomic_fetch_add(&c->sv->frames, c->sv_frames, __ATOMIC_RELAXED);
  c->sv->ring_pos[id] = c->sv_pos;
  __atomic_and_fetch(&c->sv->attached, ~(1u << id), __ATOMIC_RELEASE);
  pthread_mutex_unlock(&g_server_mu);
  c->sv = NULL;
  return had_err ? set_err(-EIO, "ctx %u detached from the flush server; a frame changed after submission since "
                           "attach (its fields were left alone)", ctx_id)
                 : 0;
}

int tasx_ctx_server_flushes(unsigned ctx_id, uint32_t *server_flushes)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (server_flushes)
    *server_flushes = c->n_server_flushes;
  return 0;
}

int tasx_server_abort(int device)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "server: device %d out of range", device);
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = g_server[device];
  if (!S) {
    pthread_mutex_unlock(&g_server_mu);
    return set_err(-EINVAL, "no flush server running for device %d", device);
  }
  __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 1u, __ATOMIC_RELEASE);
  if (!__atomic_load_n(&S->aborted, __ATOMIC_ACQUIRE)) {
    __atomic_store_n(&S->keep_run, 0, __ATOMIC_RELEASE);
    pthread_join(S->keep, NULL);
    __atomic_store_n(&S->aborted, 1, __ATOMIC_RELEASE);
  }
  hipError_t e = hipErrorNotReady;
  const struct timespec ts = {0, 100 * 1000};
  for (uint32_t t = 0; t < SRV_STOP_WAIT_MS * 10u && (e = hipStreamQuery(S->st)) == hipErrorNotReady; t++)
    nanosleep(&ts, NULL);
  pthread_mutex_unlock(&g_server_mu);
  if (e == hipErrorNotReady)
    return set_err(-EIO, "flush server for device %d did not stop within %u ms", device, SRV_STOP_WAIT_MS);
  return 0;
}

/* (ABI 9) HIP's frees (hipFree, hipHostFree, hipHostUnregister, and so
 * torch.cuda.empty_cache) wait for every kernel of the device, the server's
 * too (profiles/r05 r05free).  A pause lets them through without detaching
 * anyone: every workgroup leaves at its next poll (a batch it is summing is
 * finished first) and stores the position it polled; contexts keep
 * submitting meanwhile (the slots wait in the rings) and their polls report
 * "not done yet"; tasx_server_resume launches the kernel again at those
 * positions. */
int tasx_server_pause(int device)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "server: device %d out of range", device);
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = g_server[device];
  int rc = 0;
  if (!S)
    rc = set_err(-EINVAL, "no flush server running for device %d", device);
  else if (__atomic_load_n(&S->aborted, __ATOMIC_ACQUIRE))
    rc = set_err(-EIO, "the flush server for device %d was aborted", device);
  else if (S->paused)
    rc = set_err(-EALREADY, "the flush server for device %d is paused already", device);
  if (rc) {
    pthread_mutex_unlock(&g_server_mu);
    return rc;
  }
  /* under kmu: the epoch thread queues nothing more once launched is clear */
  pthread_mutex_lock(&S->kmu);
  const int st = __atomic_load_n(&S->kstate, __ATOMIC_ACQUIRE);
  if (st == 0) {
    __atomic_store_n(&S->paused, 1, __ATOMIC_RELEASE);
    __atomic_store_n(&S->launched, 0, __ATOMIC_RELEASE);
  }
  pthread_mutex_unlock(&S->kmu);
  if (st != 0) {
    pthread_mutex_unlock(&g_server_mu);
    return hip_err((hipError_t) -st, "flush server: an epoch");
  }
  /* every queued epoch leaves at once on the stop word */
  __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 1u, __ATOMIC_RELEASE);
  hipError_t e = hipErrorNotReady;
  const struct timespec ts = {0, 100 * 1000};
  for (uint32_t t = 0; t < SRV_STOP_WAIT_MS * 10u && (e = hipStreamQuery(S->st)) == hipErrorNotReady; t++)
    nanosleep(&ts, NULL);
  pthread_mutex_lock(&S->kmu);
  if (e == hipSuccess) { /* drained: every outstanding epoch has completed */
    S->qhead += S->nq;
    S->nq = 0;
  } else {
    /* still running after the bound, or failed: not paused.  The stop word
     * stays: cleared, workgroups that had already left would leave their
     * rings unserved beside a launch that still runs */
    if (e != hipErrorNotReady)
      __atomic_store_n(&S->kstate, -(int) e, __ATOMIC_RELEASE);
    __atomic_store_n(&S->launched, 1, __ATOMIC_RELEASE);
    __atomic_store_n(&S->paused, 0, __ATOMIC_RELEASE);
  }
  pthread_mutex_unlock(&S->kmu);
  pthread_mutex_unlock(&g_server_mu);
  if (e != hipSuccess)
    return e == hipErrorNotReady
               ? set_err(-EIO, "flush server for device %d did not leave within %u ms", device, SRV_STOP_WAIT_MS)
               : hip_err(e, "flush server kernel");
  return 0;
}

int tasx_server_resume(int device)
{
  if (device < 0 || device >= MAX_DEVICES)
    return set_err(-ENODEV, "server: device %d out of range", device);
  pthread_mutex_lock(&g_server_mu);
  struct fserver *S = g_server[device];
  int rc = 0;
  if (!S)
    rc = set_err(-EINVAL, "no flush server running for device %d", device);
  else if (!S->paused)
    rc = set_err(-EINVAL, "the flush server for device %d is not paused", device);
  else if (__atomic_load_n(&S->aborted, __ATOMIC_ACQUIRE))
    rc = set_err(-EIO, "the flush server for device %d was aborted", device);
  if (rc) {
    pthread_mutex_unlock(&g_server_mu);
    return rc;
  }
  int prev = -1;
  (void) hipGetDevice(&prev);
  hipError_t e = hipSetDevice(S->device);
  __atomic_store_n((uint32_t *) (S->h_ring + TASX_SRV_CTL), 0u, __ATOMIC_RELEASE); /* the stop word */
  pthread_mutex_lock(&S->kmu);
  /* one epoch here (resuming at the positions the last one left), the rest
   * from the epoch thread; on a failed launch the contexts see the error (and
   * settle, tasx_take_unfinished) */
  if (e == hipSuccess)
    e = server_launch_epoch(S);
  __atomic_store_n(&S->kstate, e == hipSuccess ? 0 : -(int) e, __ATOMIC_RELEASE);
  __atomic_store_n(&S->launched, 1, __ATOMIC_RELEASE);
  __atomic_store_n(&S->paused, 0, __ATOMIC_RELEASE);
  pthread_mutex_unlock(&S->kmu);
  pthread_mutex_unlock(&g_server_mu);
  if (prev >= 0)
    (void) hipSetDevice(prev);
  return e == hipSuccess ? 0 : hip_err(e, "flush server relaunch");
}

/* ---------------------------------------------------------------------- */
/* Error recovery (ABI 8): tasx_take_unfinished.  ctx_settle brings every
 * path of the context to rest -- waiting while the path is healthy -- and
 * moves the frames (and TX segments) no GPU work finished into the
 * context's unfinished store; the caller takes them from there and finishes
 * them with TAS's own CPU path.  Nothing here computes a checksum. */

static int unf_frame(struct tasx_ctx *c, uint8_t *ip, uint8_t *l4)
{
  if (c->unf_n == c->unf_cap) {
    const uint32_t cap = c->unf_cap ? 2u * c->unf_cap : 256u;
    tasx_frame_ref *n = realloc(c->unf, (size_t) cap * sizeof(*n));
    if (!n) {
      c->unf_lost++;
      return -ENOMEM;
    }
    c->unf = n;
    c->unf_cap = cap;
  }
  c->unf[c->unf_n++] = (tasx_frame_ref){ip, l4};
  return 0;
}

static int unf_seg(struct tasx_ctx *c, const tasx_tx_seg *g)
{
  if (c->unf_seg_n == c->unf_seg_cap) {
    const uint32_t cap = c->unf_seg_cap ? 2u * c->unf_seg_cap : 64u;
    tasx_tx_seg *n = realloc(c->unf_seg, (size_t) cap * sizeof(*n));
    if (!n) {
      c->unf_lost++;
      return -ENOMEM;
    }
    c->unf_seg = n;
    c->unf_seg_cap = cap;
  }
  c->unf_seg[c->unf_seg_n++] = *g;
  return 0;
}

/* ring position q's batch back from its slot (the host wrote it; the server
 * only reads slots): frames as host pointers, or the TX segments' descriptors */
static int server_slot_unfinished(struct tasx_ctx *c, uint32_t q)
{
  const unsigned id = (unsigned) (c - g_ctx);
  const uint64_t *slot = (const uint64_t *) (c->sv->h_ring + TASX_SRV_SLOTP(id, q));
  const uint64_t *e = slot + TASX_SRV_HDR / 8;
  const uint32_t n = (uint32_t) slot[0] & 0xffffu;
  int rc = 0;
  if (n & TASX_SRV_SEG) {
    const uint32_t hl = (uint32_t) e[2] & 0xffffu, room16 = (uint32_t) (e[2] >> 16) & 0xffffu;
    for (uint32_t j = 0; j < (n & ~TASX_SRV_SEG) && !rc; j++) {
      const uint64_t *w = e + TASX_SRV_SEGW0 + 3 * j;
      tasx_tx_seg g;
      memset(&g, 0, sizeof(g));
      g.frame_off = (uint32_t) w[0];
      g.payload = (uint16_t) (w[0] >> 32);
      g.pos = (uint32_t) w[1];
      g.tx_len = ((uint32_t) (w[1] >> 32) & 0xffffu) | (((uint32_t) (w[2] >> 32) & 0xffffu) << 16);
      g.tx_base = (uint32_t) w[2];
      g.hdrs_len = (uint16_t) hl;
      g.room = (room16 & 0x7fffu) | ((room16 & 0x8000u) ? TASX_TXSEG_SCRATCH : 0u);
      rc = unf_seg(c, &g);
    }
  } else {
    const uint8_t *h16 = c->zc_host - ((uintptr_t) c->zc_dev & 15u); /* host view of the slot's base */
    for (uint32_t i = 0; i < n && !rc; i++) {
      uint8_t *ip = (uint8_t *) h16 + (uint32_t) e[i] + TASX_TAS_IP_OFF;
      rc = unf_frame(c, ip, ip + 20);
    }
  }
  return rc;
}

/* The server part: wait while its kernel runs for the context's positions;
 * if the kernel has gone, the positions it did not finish become unfinished
 * and the context detaches.  Returns 1 when it detached from a gone kernel. */
static int server_settle(struct tasx_ctx *c)
{
  const unsigned id = (unsigned) (c - g_ctx);
  struct fserver *S = c->sv;
  int gone = 0;
  for (uint32_t k = 1; c->sv_done_pos != c->sv_pos; k++) {
    server_reap(c);
    if ((k & 4095u) == 0 && server_gone(S)) {
      server_reap(c);
      gone = c->sv_done_pos != c->sv_pos;
      break;
    }
  }
  if (!gone && server_gone(S))
    gone = 1; /* idle, but nothing will serve this ring again */
  if (gone) {
    const uint32_t *done = srv_dline(S, id);
    for (uint32_t q = c->sv_done_pos; q != c->sv_pos; q++)
      if (__atomic_load_n(&done[q % TASX_SRV_RING], __ATOMIC_ACQUIRE) != q + 1u)
        (void) server_slot_unfinished(c, q); /* finished out of order: done */
    c->sv_done_pos = c->sv_pos;
  }
  if (!gone)
    return 0;
  pthread_mutex_lock(&g_server_mu);
  __atomic_fetch_add(&S->batches, c->sv_batches, __ATOMIC_RELAXED);
  __atomic_fetch_add(&S->frames, c->sv_frames, __ATOMIC_RELAXED);
  S->ring_pos[id] = c->sv_pos;
  __atomic_and_fetch(&S->attached, ~(1u << id), __ATOMIC_RELEASE);
  pthread_mutex_unlock(&g_server_mu);
  c->sv = NULL;
  return 1;
}

/* a stream's queued work drained (or failed), at most 5 s */
static void stream_drain(hipStream_t st)
{
  const struct timespec ts = {0, 100 * 1000};
  for (uint32_t t = 0; t < SRV_STOP_WAIT_MS * 10u && hipStreamQuery(st) == hipErrorNotReady; t++)
    nanosleep(&ts, NULL);
  (void) hipGetLastError();
}

static void ctx_settle(struct tasx_ctx *c)
{
  /* 1. the flush server's positions (a changed frame the server flagged was
   * left alone and is not handed back: the sticky error ends here) */
  if (c->sv)
    (void) server_settle(c);
  c->sv_err = 0;
  /* 2. the feeder's batches: complete, or unfinished if it failed; its slots
   * keep a batch's frames until the batch completes (feeder_submit) */
  if (c->fd) {
    const uint32_t last = c->fq_head ? c->fq[(c->fq_head - 1u) % FQ].ticket : c->fd_done;
    while (!ticket_le(last, __atomic_load_n(&c->fd_done, __ATOMIC_ACQUIRE)) && !feeder_error(c))
      sched_yield();
    if (feeder_error(c)) {
      struct feeder *F = c->fd;
      stream_drain(F->st); /* a sweep still running writes nothing after this */
      const uint32_t fdone = __atomic_load_n(&c->fd_done, __ATOMIC_ACQUIRE);
      for (uint32_t q = c->fq_head >= FQ ? c->fq_head - FQ : 0u; q != c->fq_head; q++) {
        const struct fbatch *b = &c->fq[q % FQ];
        if (!ticket_le(b->ticket, fdone))
          for (uint32_t i = 0; i < b->n; i++)
            (void) unf_frame(c, b->ip[i], b->ip[i] + 20);
      }
      pthread_mutex_lock(&g_feeder_mu);
      __atomic_and_fetch(&F->attached, ~(1u << (unsigned) (c - g_ctx)), __ATOMIC_RELEASE);
      pthread_mutex_unlock(&g_feeder_mu);
      c->fd = NULL;
      free(c->fq);
      c->fq = NULL;
    }
  }
  /* 3. the context's own flushes: wait while its stream works on them */
  if (!ticket_le(c->local_last, c->done_ticket)) {
    stream_drain(c->st[0]);
    for (int s = 0; s < NSLOT; s++) {
      struct flush_slot *f = &c->fl[s];
      const uint32_t t = f->ticket;
      if (f->n == 0 || ticket_le(t, c->done_ticket) || !ticket_le(t, c->local_last))
        continue;
      if (__atomic_load_n(c->h_done + DONE_STRIDE * (uint32_t) s, __ATOMIC_ACQUIRE) == t) {
        if (!f->zerocopy) { /* finished, not yet reaped: its results into its frames */
          const uint16_t *r = c->h_out[s];
          for (uint32_t i = 0; i < f->n; i++) {
            memcpy(f->ip[i] + 10, &r[2 * i], 2);
            memcpy(f->l4[i] + 16, &r[2 * i + 1], 2);
          }
        }
      } else {
        for (uint32_t i = 0; i < f->n; i++)
          (void) unf_frame(c, f->ip[i], f->l4[i]);
      }
    }
  }
  /* 4. frames recorded but never handed to the GPU (a failed submit; a
   * launch that failed before its completion word may still be running) */
  if (c->npend) {
    stream_drain(c->st[0]);
    for (uint32_t i = 0; i < c->npend; i++)
      (void) unf_frame(c, c->pend_ip[i], c->pend_l4[i]);
    c->npend = 0;
  }
  /* every ticket handed out is complete now */
  c->done_ticket = c->local_last = c->next_ticket;
  if (c->fd)
    __atomic_store_n(&c->fd_done, c->next_ticket, __ATOMIC_RELEASE);
  for (int s = 0; s < NSLOT; s++)
    c->fl[s].n = 0;
}

int tasx_take_unfinished(unsigned ctx_id, tasx_frame_ref *frames, uint32_t max)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (max > 0 && !frames)
    return set_err(-EINVAL, "take_unfinished: NULL frames");
  if (c->unf_pos == c->unf_n) { /* nothing left from an earlier settle: settle now */
    c->unf_n = c->unf_pos = 0;
    hipSetDevice(c->device);
    ctx_settle(c);
  }
  uint32_t k = 0;
  while (k < max && c->unf_pos < c->unf_n)
    frames[k++] = c->unf[c->unf_pos++];
  if (k == 0 && c->unf_lost) { /* everything held was handed out; say what was not */
    const uint32_t lost = c->unf_lost;
    c->unf_lost = 0;
    return set_err(-ENOMEM, "ctx %u: %u unfinished frames / segments could not be kept (out of memory)", ctx_id,
                   lost);
  }
  return (int) k;
}

int tasx_take_unfinished_segs(unsigned ctx_id, tasx_tx_seg *segs, uint32_t max)
{
  struct tasx_ctx *c = get_ctx(ctx_id);
  if (!c)
    return set_err(-EINVAL, "ctx %u not initialised", ctx_id);
  if (max > 0 && !segs)
    return set_err(-EINVAL, "take_unfinished_segs: NULL segs");
  uint32_t k = 0;
  while (k < max && c->unf_seg_pos < c->unf_seg_n)
    segs[k++] = c->unf_seg[c->unf_seg_pos++];
  if (c->unf_seg_pos == c->unf_seg_n)
    c->unf_seg_n = c->unf_seg_pos = 0;
  return (int) k;
}

/* ---------------------------------------------------------------------- */
/* memory helpers */

void *tasx_host_alloc(size_t bytes)
{
  void *p = NULL;
  const unsigned flags = 0u;
  hipError_t e = hipHostMalloc(&p, bytes, flags);
  if (e != hipSuccess) {
    hip_err(e, "hipHostMalloc");
    return NULL;
  }
  return p;
}

int tasx_host_free(void *p)
{
  int rc = free_guard_enter("tasx_host_free");
  if (rc)
    return rc;
  const hipError_t e = hipHostFree(p);
  free_guard_exit();
  return e == hipSuccess ? 0 : hip_err(e, "hipHostFree");
}

void *tasx_host_device_pointer(void *p)
{
  void *d = NULL;
  hipError_t e = hipHostGetDevicePointer(&d, p, 0);
  if (e != hipSuccess) {
    hip_err(e, "hipHostGetDevicePointer");
    return NULL;
  }
  return d;
}

int tasx_host_register(void *p, size_t bytes)
{
  HIPCHK(hipHostRegister(p, bytes, hipHostRegisterDefault));
  return 0;
}

int tasx_host_unregister(void *p)
{
  int rc = free_guard_enter("tasx_host_unregister");
  if (rc)
    return rc;
  const hipError_t e = hipHostUnregister(p);
  free_guard_exit();
  return e == hipSuccess ? 0 : hip_err(e, "hipHostUnregister");
}

void *tasx_dev_alloc(int device, size_t bytes)
{
  void *p = NULL;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess)
    e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    hip_err(e, "hipMalloc");
    return NULL;
  }
  return p;
}

int tasx_dev_free(void *p)
{
  int rc = free_guard_enter("tasx_dev_free");
  if (rc)
    return rc;
  const hipError_t e = hipFree(p);
  free_guard_exit();
  return e == hipSuccess ? 0 : hip_err(e, "hipFree");
}

int tasx_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

int tasx_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int tasx_stream_sync(void *stream)
{
  HIPCHK(hipStreamSynchronize((hipStream_t) stream));
  return 0;
}
