"""Full-size oracle comparison for the BASELINE configs (test helper).

Every object's parity from the GPU is compared byte for byte with the CPU
oracle's encode of the same object (oracle/gf_oracle.c through
oracle/coracle.py, the klauspost restatement), not a sample: the parity a
klauspost Encoder writes for every object is what objectserver/ecutils.go:59
stores.  Device tensors are streamed to pinned host chunks, so host memory
stays at one chunk however large the batch.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import coracle as CO


def encode_parity_matches(k: int, m: int, objs: torch.Tensor, parity: torch.Tensor, chunk: int = 1024) -> int:
    """objs [n, k*S] and parity [n, m*S] (uint8, on the GPU): compare every
    object's parity with CO.encode_batch of its data.  Returns the number of
    objects compared; raises AssertionError naming the first bad object."""
    n, ln = objs.shape
    assert parity.shape == (n, m * (ln // k))
    threads = CO.cpu_threads()
    h_obj = torch.empty((min(chunk, n), ln), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty((min(chunk, n), parity.shape[1]), dtype=torch.uint8, pin_memory=True)
    for o0 in range(0, n, chunk):
        c = min(chunk, n - o0)
        h_obj[:c].copy_(objs[o0:o0 + c], non_blocking=True)
        h_par[:c].copy_(parity[o0:o0 + c], non_blocking=True)
        torch.cuda.synchronize()
        want, _ = CO.encode_batch(k, m, h_obj[:c].numpy(), threads=threads)
        got = h_par[:c].numpy()
        if not np.array_equal(got, want):
            bad = int(np.nonzero((got != want).any(axis=1))[0][0])
            raise AssertionError(f"parity of object {o0 + bad} differs from the oracle")
    return n


def rows_match(got: torch.Tensor, want: torch.Tensor, chunk_bytes: int = 1 << 30) -> bool:
    """Byte equality of two same-shape GPU tensors (rebuilt vs original),
    compared on the GPU in chunks of rows."""
    assert got.shape == want.shape
    rows = max(1, chunk_bytes // max(1, got.shape[-1]))
    for r0 in range(0, got.shape[0], rows):
        if not torch.equal(got[r0:r0 + rows], want[r0:r0 + rows]):
            return False
    return True
