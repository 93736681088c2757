/* Command-line driver for the CPU oracle (test infrastructure only).
 *   hm_oracle_cli hash <msg> <nonce>
 *   hm_oracle_cli scan <msg> <lo> <hi> [threads]
 * Prints "<hash> <nonce>" like the reference client's printResult
 * (cmu440/bitcoin/client/client.go:61-63 prints "Result <hash> <nonce>"). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
uint64_t oracle_hash(const uint8_t *msg, size_t len, uint64_t nonce);
void oracle_scan(const uint8_t *msg, size_t len, uint64_t lo, uint64_t hi, int threads,
                 uint64_t *h, uint64_t *n);
int main(int argc, char **argv) {
    if (argc >= 4 && !strcmp(argv[1], "hash")) {
        uint64_t h = oracle_hash((const uint8_t *)argv[2], strlen(argv[2]),
                                 strtoull(argv[3], NULL, 10));
        printf("%llu\n", (unsigned long long)h);
        return 0;
    }
    if (argc >= 5 && !strcmp(argv[1], "scan")) {
        uint64_t h, n;
        int th = argc >= 6 ? atoi(argv[5]) : 1;
        oracle_scan((const uint8_t *)argv[2], strlen(argv[2]), strtoull(argv[3], NULL, 10),
                    strtoull(argv[4], NULL, 10), th, &h, &n);
        printf("Result %llu %llu\n", (unsigned long long)h, (unsigned long long)n);
        return 0;
    }
    fprintf(stderr, "usage: %s hash <msg> <nonce> | scan <msg> <lo> <hi> [threads]\n", argv[0]);
    return 2;
}
