/* ab/ab_host.c -- comparison build only (libtasx_ab.so): the export of
 * include/tasx_ab.h that needs the host layer (the library is the product's
 * own objects plus tas_amd/csrc/ab/; it changes nothing in the product paths). */
#include <stdint.h>

#include "../tasx_kernels.h"

int tasx_ab_ctx_set_tickets(unsigned ctx_id, uint32_t start)
{
  return tasx_ctx_set_tickets_internal(ctx_id, start);
}
