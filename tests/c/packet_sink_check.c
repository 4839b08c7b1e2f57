/* packet_sink_check.c — test infrastructure for fcs_txq_sink_packet (include/nstack_txq.h), the TX
 * queue's AF_PACKET sink, without CAP_NET_RAW.
 *
 * This executable defines sendmmsg and sendto itself (the sink sends a batch of one frame with
 * sendto, exactly ether_send's call); a symbol of the executable comes first in the dynamic
 * linker's global scope, so libnstack_fcs.so's calls bind here instead of to libc (no LD_PRELOAD).
 * The stand-in records every message (fd, flags, msg_name bytes, iovec) and answers from a script,
 * so partial sends and errors reach the sink's per-frame result mapping:
 *
 *     packet_sink_check N IFINDEX SCRIPT
 *
 * SCRIPT is a comma list, one entry per sendmmsg/sendto call: a number k (accept the first k messages),
 * "A" (accept all), "E<errno>" (fail with that errno), "I" (fail with EINTR). Calls past the script
 * accept all. N frames are built as ether_send builds them (src/linux/ether.c:257-261, FCS bytes
 * left zero: the sink does not look at them) with varied destinations, protocols and lengths, and
 * handed to fcs_txq_sink_packet in one call (fd 77). Output, one JSON object per line: each call
 * ({"call": ...}), each accepted message ({"msg": ...}), then the per-frame results ({"res": [...]}).
 * No GPU call is made. */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>

#include "../../include/nstack_txq.h"

static const char *g_script;
static int g_call, g_sent;

static const char *script_entry(int k) {   /* entry k of the comma list, or NULL */
    static char buf[32];
    const char *s = g_script;
    for (int i = 0; s && *s; i++) {
        const char *e = strchr(s, ',');
        const size_t n = e ? (size_t)(e - s) : strlen(s);
        if (i == k) {
            snprintf(buf, sizeof buf, "%.*s", (int)(n < sizeof buf - 1 ? n : sizeof buf - 1), s);
            return buf;
        }
        s = e ? e + 1 : NULL;
    }
    return NULL;
}

static void hex(const void *p, size_t n) {
    for (size_t i = 0; i < n; i++) printf("%02x", ((const uint8_t *)p)[i]);
}

int sendmmsg(int fd, struct mmsghdr *m, unsigned int vlen, int flags) {
    const char *e = script_entry(g_call);
    printf("{\"call\": %d, \"fd\": %d, \"vlen\": %u, \"flags\": %d, \"entry\": \"%s\"}\n", g_call, fd, vlen, flags,
           e ? e : "A");
    g_call++;
    unsigned int take = vlen;
    if (e && e[0] == 'E') {
        errno = atoi(e + 1);
        return -1;
    }
    if (e && e[0] == 'I') {
        errno = EINTR;
        return -1;
    }
    if (e && e[0] != 'A') {
        const unsigned int k = (unsigned int)atoi(e);
        take = k < vlen ? k : vlen;
    }
    for (unsigned int i = 0; i < take; i++) {
        const struct msghdr *h = &m[i].msg_hdr;
        size_t len = 0;
        for (size_t j = 0; j < h->msg_iovlen; j++) len += h->msg_iov[j].iov_len;
        printf("{\"msg\": %d, \"namelen\": %u, \"name\": \"", g_sent, (unsigned)h->msg_namelen);
        hex(h->msg_name, h->msg_namelen);
        printf("\", \"iovlen\": %zu, \"len\": %zu, \"head\": \"", (size_t)h->msg_iovlen, len);
        hex(h->msg_iov[0].iov_base, h->msg_iov[0].iov_len < 14 ? h->msg_iov[0].iov_len : 14);
        printf("\", \"control\": %zu}\n", (size_t)h->msg_controllen);
        m[i].msg_len = (unsigned int)len;
        g_sent++;
    }
    return (int)take;
}

ssize_t sendto(int fd, const void *buf, size_t len, int flags, const struct sockaddr *addr, socklen_t alen) {
    const char *e = script_entry(g_call);
    printf("{\"call\": %d, \"fd\": %d, \"vlen\": 1, \"flags\": %d, \"entry\": \"%s\", \"kind\": \"sendto\"}\n",
           g_call, fd, flags, e ? e : "A");
    g_call++;
    if (e && e[0] == 'E') {
        errno = atoi(e + 1);
        return -1;
    }
    if (e && e[0] == 'I') {
        errno = EINTR;
        return -1;
    }
    printf("{\"msg\": %d, \"namelen\": %u, \"name\": \"", g_sent, (unsigned)alen);
    hex(addr, alen);
    printf("\", \"iovlen\": 1, \"len\": %zu, \"head\": \"", len);
    hex(buf, len < 14 ? len : 14);
    printf("\", \"control\": 0}\n");
    g_sent++;
    return (ssize_t)len;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s N IFINDEX SCRIPT\n", argv[0]);
        return 2;
    }
    const uint32_t n = (uint32_t)atoi(argv[1]);
    struct fcs_txq_packet_ctx ctx = {77, atoi(argv[2])};
    g_script = argv[3];
    static const uint16_t protos[4] = {0x0800, 0x0806, 0x86DD, 0x88CC};
    uint8_t **frames = calloc(n, sizeof *frames);
    uint32_t *sizes = calloc(n, sizeof *sizes);
    int *res = calloc(n, sizeof *res);
    for (uint32_t i = 0; i < n; i++) {
        const size_t bsize = (size_t)((i * 397u) % 1501u);
        const size_t frame_size = 14 + (bsize > 56 ? bsize : 56) + 4;   /* ether.c:222-224 */
        uint8_t *f = calloc(1, frame_size);
        const uint8_t dst[6] = {(uint8_t)(0x02 | (i & 0xF0)), (uint8_t)i, (uint8_t)(i >> 8), 0xA5, (uint8_t)(i * 7),
                                (uint8_t)(255 - i)};
        const uint8_t src[6] = {0x02, 0x42, 0xAC, 0x11, 0x00, 0x02};
        memcpy(f, dst, 6);                                 /* :257 */
        memcpy(f + 6, src, 6);                             /* :258 */
        f[12] = (uint8_t)(protos[i & 3] >> 8);             /* :259 htons(proto) */
        f[13] = (uint8_t)protos[i & 3];
        for (size_t k = 0; k < bsize; k++) f[14 + k] = (uint8_t)(k * 31 + i);   /* :260; pad stays 0 (:261) */
        frames[i] = f;
        sizes[i] = (uint32_t)frame_size;
        res[i] = -12345;
    }
    fcs_txq_sink_packet(&ctx, frames, sizes, res, n);
    printf("{\"res\": [");
    for (uint32_t i = 0; i < n; i++) printf("%s%d", i ? ", " : "", res[i]);
    printf("], \"sizes\": [");
    for (uint32_t i = 0; i < n; i++) printf("%s%u", i ? ", " : "", sizes[i]);
    printf("]}\n");
    for (uint32_t i = 0; i < n; i++) free(frames[i]);
    free(frames);
    free(sizes);
    free(res);
    return 0;
}
