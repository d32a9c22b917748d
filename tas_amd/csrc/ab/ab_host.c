/* ab/ab_host.c -- A/B build only (libtasx_ab.so): the knobs and test hooks
 * kept for comparisons, read from the environment once at load time (TASX_TXSEG_DEBUG, which
 * tests switch per case, at every TX launch: ab/ab_txseg.hip), and the
 * A/B exports of include/tasx_ab.h that need the host layer.  A constructor
 * points the product's extension pointer (tasx_ext, tas_amd/csrc/tasx_kernels.h)
 * at these hooks; libtasx.so has no such constructor, so there tasx_ext stays
 * NULL and the product paths alone run. */
#include <stdint.h>
#include <stdlib.h>

#include "../tasx_kernels.h"

TASX_INTERNAL int ab_launch_raw(const tasx_raw_params *p, int variant, void *stream);
TASX_INTERNAL int ab_launch_tcp4(const tasx_tcp4_params *p, int variant, void *stream);
TASX_INTERNAL int ab_launch_verify(const tasx_tcp4_params *p, int variant, void *stream);
TASX_INTERNAL int ab_launch_rx(const tasx_tcp4_params *p, int variant, void *stream);
TASX_INTERNAL int ab_launch_flow_lookup(const tasx_flow_params *p, int variant, void *stream);
TASX_INTERNAL int ab_launch_txseg(const tasx_txseg_params *p, void *stream);
TASX_INTERNAL int ab_launch_server(const tasx_srv_params *p, void *stream);
TASX_INTERNAL int ab_xrun(uint64_t blocks);

static tasx_ext_hooks g_hooks = {
    .max_variant = 57,
    .raw = ab_launch_raw,
    .tcp4 = ab_launch_tcp4,
    .verify = ab_launch_verify,
    .rx = ab_launch_rx,
    .flow = ab_launch_flow_lookup,
    .txseg = ab_launch_txseg,
    .server = ab_launch_server,
    .xrun = ab_xrun,
    .srv_hot_us = -1,
    .srv_cold_us = -1,
};

static uint32_t env_u32(const char *name, uint32_t dflt)
{
  const char *e = getenv(name);
  return e ? (uint32_t) atoi(e) : dflt;
}

__attribute__((constructor)) static void ab_hooks_init(void)
{
  g_hooks.feeder_sweeps = env_u32("TASX_FEEDER_SWEEPS", 0u);   /* 4: four feeder sweeps in flight */
  g_hooks.srv_k = env_u32("TASX_SRV_K", 0u);                   /* server workgroups per ring, 1/2/4/8 */
  g_hooks.srv_segmax = env_u32("TASX_SRV_SEGMAX", 0u);         /* TX segments per server slot (round 4: 20) */
  g_hooks.srv_diag = getenv("TASX_SRV_DIAG") != NULL;          /* the server's timing sums */
  g_hooks.srv_hot_us = getenv("TASX_SRV_HOT_US") ? atoi(getenv("TASX_SRV_HOT_US")) : -1;
  g_hooks.srv_cold_us = getenv("TASX_SRV_COLD_US") ? atoi(getenv("TASX_SRV_COLD_US")) : -1;
  if (env_u32("TASX_HOST_UC", 0u)) { /* frames and shm mapped MTYPE_UC: the L2 never caches them */
    g_hooks.host_reg_flags = 0x80000000u;   /* hipExtHostRegisterUncached */
    g_hooks.host_alloc_flags = 0x10000000u; /* hipHostMallocUncached */
  }
  tasx_ext = &g_hooks;
}

/* the device buffer the wave-timeline variant (4) stamps into */
int tasx_set_diag_buffer(void *dev_buf)
{
  g_hooks.diag = (uint64_t *) dev_buf;
  return 0;
}

int tasx_ab_ctx_set_tickets(unsigned ctx_id, uint32_t start)
{
  return tasx_ctx_set_tickets_internal(ctx_id, start);
}

int tasx_ab_server_diag(int device, unsigned r, double *out)
{
  return tasx_server_diag_internal(device, r, out);
}
