"""Generate tests/golden/*.json from the CPU oracle (oracle/oracle.py).

    python tests/golden/make_golden.py

kats.json holds the upstream klauspost/Backblaze known-answer tests and the
reference-pinned ecutils/ecobj KATs (hand-restated from the reference's and
upstream's test files, cited per entry); vectors.json holds oracle-generated
vectors.  The reference (Go) cannot run here, so
these vectors are pinned through the KATs the oracle reproduces.
"""
from __future__ import annotations

import hashlib
import itertools
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import oracle as O  # noqa: E402

OUT = Path(__file__).resolve().parent


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def kats():
    return {
        "source": "upstream klauspost/reedsolomon galois_test.go, matrix_test.go, reedsolomon_test.go "
                  "(Backblaze JavaReedSolomon vectors) and reference objectserver tests",
        "gal_mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
        "gal_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
        "invert": [
            {"in": [[56, 23, 98], [3, 100, 200], [45, 201, 123]],
             "out": [[175, 133, 33], [130, 13, 245], [112, 35, 126]]},
            {"in": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
             "out": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122], [0, 0, 1, 0, 0],
                     [0, 0, 0, 1, 0]]},
        ],
        "one_encode": {"k": 5, "m": 5, "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
                       "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]},
        # reference objectserver/ecutils_test.go:9-21
        "shard_length": [[1000, 4, 250], [0, 4, 0], [-12340, 4, 0], [1001, 4, 251], [1001, 5, 201],
                         [1007, 10, 101]],
        # reference objectserver/ecobj_test.go:360-379
        "range_chunk_align": [[60, 81, 10, 2, 30, 50], [61, 80, 10, 2, 30, 40], [60, 81, 10, 3, 20, 30],
                              [0, 81, 10, 3, 0, 30]],
        # reference objectserver/ecobj_test.go:317-330
        "parse_ec_scheme": {"ok": [["reedsolomon/1/2/16", "reedsolomon", 1, 2, 16]],
                            "err": ["1/2/16", "reedsolomon/1/2/X"]},
        # reference objectserver/ecobj_test.go:144-206: 7 bytes, 3+2 -> 3-byte shards
        "stabilize_lengths": {"body": "TESTING", "k": 3, "m": 2, "chunk": 100, "shard_len": 3},
        # RFC 1321 appendix A.5 test suite (MD5, the ShardHash function)
        "md5_rfc1321": [
            ["", "d41d8cd98f00b204e9800998ecf8427e"],
            ["a", "0cc175b9c0f1b6a831c399e269772661"],
            ["abc", "900150983cd24fb0d6963f7d28e17f72"],
            ["message digest", "f96b697d7cb7938d525a2f31aaf161d0"],
            ["abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"],
            ["ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", "d174ab98d277d9f5a5611c2c9f419d9f"],
            ["1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"],
        ],
        # reference objectserver/auditor_test.go:585-612: the ShardHash the
        # auditor accepts for a shard file holding "testcontents", and rejects
        # for "asdftestcontents"
        "shard_hash": {"hash": "d3ac5112fe464b81184352ccba743001", "match": "testcontents",
                       "mismatch": "asdftestcontents"},
    }


def vectors():
    v = {"seed": O.HBEC_SEED}
    # (2) TESTING 3+2
    files = O.ec_split(3, 2, b"TESTING", 100)
    v["testing_3_2"] = {"files": [list(f) for f in files]}
    # (7) ShardHash of every shard file of a multi-stripe split (4+2, chunk 1 KiB)
    body = bytes(O.object_bytes(3, 10000))
    v["shard_hashes_4_2_chunk1k"] = {"object": 3, "len": 10000, "chunk": 1024,
                                     "hashes": O.ec_split_hashes(4, 2, body, 1024)}
    # parity rows of the configs
    v["parity_rows"] = {f"{k}+{m}": O.Encoder(k, m).parity for k, m in [(2, 1), (3, 2), (4, 2), (8, 3), (10, 4)]}
    # (3) seeded objects: digests of every shard
    seeded = []
    for k, m, size, idx in [(4, 2, 1 << 20, 0), (4, 2, 1 << 20, 4095), (8, 3, 1 << 20, 0), (8, 3, 4096, 0),
                            (8, 3, 4096, 1)]:
        obj = O.object_bytes(idx, size)
        s = size // k
        shards = [obj[j * s:(j + 1) * s].copy() for j in range(k)] + [np.zeros(s, np.uint8) for _ in range(m)]
        O.Encoder(k, m).encode(shards)
        seeded.append({"k": k, "m": m, "size": size, "index": idx, "object_sha256": sha(obj),
                       "shard_sha256": [sha(x) for x in shards],
                       "parity_head": [list(map(int, x[:64])) for x in shards[k:]],
                       "parity_tail": [list(map(int, x[-64:])) for x in shards[k:]]})
    v["seeded"] = seeded
    # (4) every erasure pattern with <= m missing on a 4 KiB object
    patterns = []
    for k, m in [(4, 2), (8, 3)]:
        obj = O.object_bytes(7, 4096)
        s = 4096 // k
        full = [obj[j * s:(j + 1) * s].copy() for j in range(k)] + [np.zeros(s, np.uint8) for _ in range(m)]
        O.Encoder(k, m).encode(full)
        full_sha = [sha(x) for x in full]
        rows = []
        for e in range(1, m + 1):
            for missing in itertools.combinations(range(k + m), e):
                enc = O.Encoder(k, m)
                sh = [x.copy() if i not in missing else np.zeros(0, np.uint8) for i, x in enumerate(full)]
                enc.reconstruct(sh)
                assert [sha(x) for x in sh] == full_sha
                present = [0 if i in missing else 1 for i in range(k + m)]
                surv, inv = enc.decode_matrix(present)
                rows.append({"missing": list(missing), "survivors": surv,
                             "data_rows": [inv[i] for i in missing if i < k]})
        patterns.append({"k": k, "m": m, "index": 7, "size": 4096, "shard_sha256": full_sha, "patterns": rows})
    v["erasures"] = patterns
    # (5) padding cases and (6) multi-stripe: ecSplit shard files
    splits = []
    for k, m, size, chunk in [(4, 2, 1, 1 << 20), (4, 2, 7, 1 << 20), (3, 2, 7, 100), (4, 2, 1001, 1 << 20),
                              (4, 2, 4097, 1 << 20), (4, 2, (1 << 20) + 1, 1 << 20), (8, 3, 4097, 1 << 20),
                              (4, 2, 10000, 1024), (8, 3, 100000, 4096), (4, 2, 0, 1 << 20)]:
        obj = O.object_bytes(size, size).tobytes()
        files = O.ec_split(k, m, obj, chunk)
        assert O.ec_glue(k, m, files, chunk, size) == obj
        splits.append({"k": k, "m": m, "size": size, "chunk": chunk, "object_seed_index": size,
                       "file_len": [len(f) for f in files], "file_sha256": [sha(f) for f in files],
                       "small_files": [list(f) for f in files] if size <= 1001 else None})
    v["ec_split"] = splits
    return v


def main():
    (OUT / "kats.json").write_text(json.dumps(kats(), indent=1) + "\n")
    (OUT / "vectors.json").write_text(json.dumps(vectors()) + "\n")
    print("wrote", OUT / "kats.json", OUT / "vectors.json")


if __name__ == "__main__":
    main()
