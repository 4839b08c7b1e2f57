/*
 * dropin_caller.c — the link-level drop-in test of ether_fcs.
 *
 * A C caller written against the reference's own prototype, declared verbatim as
 * /root/reference/src/nstack_ether.h:80 declares it, with no engine header included. It is linked
 * with -lnstack_fcs in place of the reference's ether_fcs.o (/root/reference/Makefile:13,
 * OBJS_core; link line :42-43): the symbol must resolve to libnstack_fcs.so.
 *
 *   dropin_caller ARENA_FILE < "off len" lines   ->   one "%08x" FCS per line on stdout
 *
 * tests/test_dropin_link.py checks the link on the CPU and (GPU box) the FCS of every golden
 * vector against tests/golden/vectors.json.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

uint32_t ether_fcs(const void *data, size_t bsize);

int main(int argc, char **argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s ARENA_FILE < 'off len' lines\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *arena = malloc(size > 0 ? (size_t)size : 1);
    if (!arena || (size > 0 && fread(arena, 1, (size_t)size, f) != (size_t)size)) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(f);
    unsigned long long off, len;
    while (scanf("%llu %llu", &off, &len) == 2) {
        if (off > (unsigned long long)size || len > (unsigned long long)size - off) {
            fprintf(stderr, "frame [%llu, +%llu) outside the %ld-byte arena\n", off, len, size);
            return 2;
        }
        printf("%08x\n", (unsigned)ether_fcs(arena + off, (size_t)len));
    }
    free(arena);
    return 0;
}
