/* Pure C11 client of include/hbec.h: proves the boundary is a C ABI (no C++
 * or torch types) and exercises the host-only entry points a Go/cgo caller
 * binds.  Built and run by tests/test_abi.py::test_pure_c_client. */
#include <stdio.h>
#include <string.h>

#include "hbec.h"

int main(void) {
    hbec_codec* c = NULL;
    if (hbec_new(4, 2, &c) != HBEC_OK) return 1;
    uint8_t m[6 * 4];
    if (hbec_matrix(c, m) != HBEC_OK) return 2;
    /* parity rows of klauspost's default 4+2 matrix */
    static const uint8_t want[8] = {27, 28, 18, 20, 28, 27, 20, 18};
    if (memcmp(m + 16, want, 8) != 0) return 3;
    if (hbec_data_shards(c) != 4 || hbec_parity_shards(c) != 2) return 4;
    uint8_t present[6] = {0, 0, 1, 1, 1, 1};
    int surv[4], outs[6], nout = 0;
    uint8_t rows[6 * 4];
    if (hbec_decode_rows(c, present, 0, surv, outs, &nout, rows) != HBEC_OK) return 5;
    static const uint8_t drows[8] = {208, 107, 104, 210, 107, 208, 210, 104};
    if (nout != 2 || memcmp(rows, drows, 8) != 0 || surv[0] != 2) return 6;
    hbec_free(c);
    if (hbec_new(0, 2, &c) != HBEC_ERR_INV_SHARD_NUM) return 7;
    if (hbec_new(200, 57, &c) != HBEC_ERR_MAX_SHARD_NUM) return 8;
    if (hbec_ec_shard_length(1001, 4) != 251 || hbec_ec_shard_length(-5, 4) != 0) return 9;
    char algo[32];
    int k, p, chunk;
    if (hbec_parse_ec_scheme("reedsolomon/4/2/1048576", algo, sizeof algo, &k, &p, &chunk) != HBEC_OK) return 10;
    if (strcmp(algo, "reedsolomon") || k != 4 || p != 2 || chunk != 1048576) return 11;
    if (hbec_parse_ec_scheme("1/2/16", algo, sizeof algo, &k, &p, &chunk) != HBEC_ERR_SCHEME) return 12;
    int64_t s, e;
    hbec_range_chunk_align(60, 81, 10, 2, &s, &e);
    if (s != 30 || e != 50) return 13;
    printf("abi ok v%d: %s\n", hbec_version(), hbec_strerror(HBEC_ERR_SHARD_SIZE));
    return 0;
}
