/* Pure C11 client of include/hbec.h: proves the boundary is a C ABI (no C++
 * or torch types) and exercises the entry points a Go/cgo caller binds.
 * Built and run by tests/test_abi.py::test_pure_c_client (host-only checks)
 * and, with the argument "gpu", by tests/test_gpu_parity.py (encode and
 * reconstruct through the single-pointer databuf entries, the way the cgo
 * shim of INTEGRATION.md calls them, against known answers). */
#include <stdio.h>
#include <string.h>

#include "hbec.h"

/* Encode / Reconstruct / ReconstructData through hbec_*_databuf on
 * ecSplit-shaped databufs (ecutils.go:31-35,55-59), checked against:
 *  - the "TESTING" 3+2 stripe (ecobj_test.go:144-206 object; parity rows of
 *    klauspost's default matrix, tests/golden/vectors.json),
 *  - klauspost TestOneEncode (5+5, reedsolomon_test.go). */
static int gpu_checks(void) {
    hbec_codec* c = NULL;
    if (hbec_new(3, 2, &c) != HBEC_OK) return 101;
    uint8_t buf[5 * 3] = {'T', 'E', 'S', 'T', 'I', 'N', 'G', 0, 0};
    static const uint8_t par[6] = {71, 12, 29, 62, 166, 76};
    if (hbec_encode_databuf(c, buf, 3) != HBEC_OK) return 102;
    if (memcmp(buf + 9, par, 6) != 0) return 103;
    uint8_t full[15];
    memcpy(full, buf, 15);
    int ok = 0;
    if (hbec_verify_databuf(c, buf, 3, &ok) != HBEC_OK || ok != 1) return 104;
    /* ecReconstruct: shards 0 and 4 lost, rebuilt in their slots */
    memset(buf, 0xEE, 3);
    memset(buf + 12, 0xEE, 3);
    const uint8_t present[5] = {0, 1, 1, 1, 0};
    if (hbec_reconstruct_databuf(c, buf, 3, present, 0) != HBEC_OK) return 105;
    if (memcmp(buf, full, 15) != 0) return 106;
    /* ecGlue: ReconstructData rebuilds data slots only */
    memset(buf, 0xEE, 3);
    memset(buf + 12, 0xEE, 3);
    if (hbec_reconstruct_databuf(c, buf, 3, present, 1) != HBEC_OK) return 107;
    if (memcmp(buf, full, 12) != 0 || buf[12] != 0xEE) return 108;
    buf[0] ^= 1;
    if (hbec_verify_databuf(c, buf, 3, &ok) != HBEC_OK || ok != 0) return 109;
    hbec_free(c);
    if (hbec_new(5, 5, &c) != HBEC_OK) return 110;
    uint8_t one[10 * 2] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9};
    static const uint8_t want55[10] = {12, 13, 10, 11, 14, 15, 90, 91, 94, 95};
    if (hbec_encode_databuf(c, one, 2) != HBEC_OK) return 111;
    if (memcmp(one + 10, want55, 10) != 0) return 112;
    hbec_free(c);
    printf("databuf gpu ok\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "gpu") == 0) return gpu_checks();
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
    int64_t k, p, chunk;
    if (hbec_parse_ec_scheme("reedsolomon/4/2/1048576", algo, sizeof algo, &k, &p, &chunk) != HBEC_OK) return 10;
    if (strcmp(algo, "reedsolomon") || k != 4 || p != 2 || chunk != 1048576) return 11;
    if (hbec_parse_ec_scheme("1/2/16", algo, sizeof algo, &k, &p, &chunk) != HBEC_ERR_SCHEME) return 12;
    int64_t s, e;
    hbec_range_chunk_align(60, 81, 10, 2, &s, &e);
    if (s != 30 || e != 50) return 13;
    /* databuf entry points: argument checks answer before any device work */
    if (hbec_new(4, 2, &c) != HBEC_OK) return 14;
    uint8_t db[6 * 16] = {0};
    const uint8_t none[6] = {0, 0, 0, 0, 0, 0}, three[6] = {1, 1, 1, 0, 0, 0}, all[6] = {1, 1, 1, 1, 1, 1};
    if (hbec_encode_databuf(c, db, 0) != HBEC_ERR_SHARD_NO_DATA) return 15;
    if (hbec_reconstruct_databuf(c, db, 16, none, 0) != HBEC_ERR_SHARD_NO_DATA) return 16;
    if (hbec_reconstruct_databuf(c, db, 16, three, 0) != HBEC_ERR_TOO_FEW_SHARDS) return 17;
    if (hbec_reconstruct_databuf(c, db, 16, all, 0) != HBEC_OK) return 18;
    if (hbec_encode_databuf(c, NULL, 16) != HBEC_ERR_INVALID_ARG) return 19;
    hbec_free(c);
    printf("abi ok v%d: %s\n", hbec_version(), hbec_strerror(HBEC_ERR_SHARD_SIZE));
    return 0;
}
