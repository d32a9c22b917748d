/*
 * rte_standin.h -- TEST INFRASTRUCTURE.  A stand-in for the three DPDK 19.11
 * rte_ip.h inlines TAS's tcp_checksums() calls on its CPU path
 * (tas/fast/fast_flows.c:1066-1067), so that tests/c/tas_glue.h's error
 * recovery (finish the frames libtasx hands back)
 * compiles and runs here without DPDK.  In TAS the glue calls DPDK itself;
 * nothing of this file is part of libtasx.
 *
 * DPDK 19.11 semantics: rte_raw_cksum sums
 * little-endian 16-bit words from the buffer start (an odd tail byte as a low
 * byte) and folds twice; rte_ipv4_cksum = raw sum of the 20-byte header,
 * 0xffff kept, else inverted; rte_ipv4_udptcp_cksum = raw sum of the L4 bytes
 * (length from total_length; total_length < 20 -> 0) plus the pseudo-header
 * {src, dst, 0, proto, htons(l4 length)}, one fold, inverted, 0 -> 0xffff.
 */
#ifndef RTE_STANDIN_H_
#define RTE_STANDIN_H_

#include <stdint.h>
#include <stddef.h>

static inline uint32_t standin_words(const uint8_t *b, size_t len, uint32_t sum)
{
  size_t i = 0;
  for (; i + 1 < len; i += 2)
    sum += (uint32_t) b[i] | ((uint32_t) b[i + 1] << 8);
  if (i < len)
    sum += b[i];
  return sum;
}

static inline uint16_t standin_fold(uint32_t sum)
{
  sum = (sum >> 16) + (sum & 0xffffu);
  sum = (sum >> 16) + (sum & 0xffffu);
  return (uint16_t) sum;
}

static inline uint16_t rte_ipv4_cksum(const void *ip_hdr)
{
  const uint16_t c = standin_fold(standin_words((const uint8_t *) ip_hdr, 20, 0));
  return c == 0xffff ? c : (uint16_t) ~c;
}

static inline uint16_t rte_ipv4_udptcp_cksum(const void *ip_hdr, const void *l4_hdr)
{
  const uint8_t *ip = (const uint8_t *) ip_hdr;
  const uint32_t tl = ((uint32_t) ip[2] << 8) | ip[3];
  if (tl < 20)
    return 0;
  const uint32_t l4 = tl - 20;
  const uint8_t ph[12] = {ip[12], ip[13], ip[14], ip[15], ip[16], ip[17], ip[18], ip[19],
                          0, ip[9], (uint8_t) (l4 >> 8), (uint8_t) l4};
  uint32_t c = standin_fold(standin_words((const uint8_t *) l4_hdr, l4, 0));
  c += standin_fold(standin_words(ph, sizeof ph, 0));
  c = ((c & 0xffff0000u) >> 16) + (c & 0xffffu);
  c = (~c) & 0xffffu;
  return (uint16_t) (c == 0 ? 0xffff : c);
}

#endif
