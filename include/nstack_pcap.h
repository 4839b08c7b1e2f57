/*
 * nstack_pcap.h — frame batches on disk: classic libpcap files read into, and
 * written from, the engine's batch layout (a packed byte arena + u64 offsets + u32 lengths, the
 * layout of ether_fcs_batch_* / ether_fcs_verify_*).
 *
 * Supported: pcap with magic 0xA1B2C3D4 (microsecond) and 0xA1B23C4D (nanosecond timestamps), in
 * either byte order, any link type (reported, not interpreted). pcapng is rejected with
 * -EPROTONOSUPPORT. Records keep their captured bytes (incl_len); a record truncated by the
 * capture's snap length is flagged in the optional `truncated` count, since its FCS cannot be
 * checked. Errors are -errno (fcs_last_error() has the text); host code only, no GPU needed.
 */
#ifndef NSTACK_PCAP_H
#define NSTACK_PCAP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Count the records of a pcap file and the bytes their captured data needs (for sizing the
 * arena / offset / length buffers). linktype and truncated may be NULL. Returns 0 or -errno. */
int fcs_pcap_scan(const char *path, uint64_t *frames, uint64_t *bytes, uint32_t *linktype,
                  uint64_t *truncated);

/* Read up to max_frames records: record i's captured bytes go to arena[off[i] .. off[i]+len[i]),
 * packed in file order. Returns the number of records read (>= 0) or -errno (-ENOSPC when the
 * arena is too small for the records that fit max_frames). */
int64_t fcs_pcap_read(const char *path, uint8_t *arena, uint64_t arena_bytes, uint64_t *off,
                      uint32_t *len, uint64_t max_frames);

/* Write n frames as a microsecond pcap (little-endian, snaplen 65535, the given link type;
 * 1 = Ethernet), timestamps 0, 1, 2, ... us. Returns 0 or -errno. */
int fcs_pcap_write(const char *path, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                   uint64_t n, uint32_t linktype);

#ifdef __cplusplus
}
#endif
#endif /* NSTACK_PCAP_H */
